"""Wall-clock A/B of whole scan calls (the bench's step without its loop):
build a workload (argv[1]) once, then for each library (argv[2:]) the best of
8 device-resident scan calls, two alternating rounds.
    python tools/wall_ab.py c3 libclyscan.so libexp_X.so"""
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402
from bench import make_workload, timed_scans  # noqa: E402
from couloydb_amd import Scanner  # noqa: E402

cfg = sys.argv[1]
libs = sys.argv[2:]
wl = make_workload(cfg, torch)
for rep in range(2):
    for lib in libs:
        sc = Scanner(0, lib=lib)
        best, kscan, need, res = timed_scans(sc, wl.dev_files, wl.d_out.data_ptr(), wl.out_cap, reps=8)
        print("%s %s rep %d wall %.3f ms  k_scan %.3f  GiB/s %.1f" % (cfg, lib, rep, best * 1e3, kscan,
                                                                     wl.bytes / best / 2**30), flush=True)
        sc.close()
