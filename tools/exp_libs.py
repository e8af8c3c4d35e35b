"""k_scan time of alternative builds of libclyscan (same source, other compiler
options): python tools/exp_libs.py lib1.so lib2.so ... -> one line per library
(C2, five scans each; the product build libclyscan.so first)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from bench import make_workload  # noqa: E402
from couloydb_amd import Scanner  # noqa: E402

wl = make_workload("c2", torch)
for rnd in range(2):
    for lib in ["libclyscan.so"] + sys.argv[1:]:
        sc = Scanner(0, lib=lib)
        ts = []
        for it in range(5):
            first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
            ts.append(st.scan_ms)
        print("round %d %-22s k_scan min %.3f ms  all %s" % (rnd, lib, min(ts), " ".join("%.3f" % t for t in ts)),
              flush=True)
        sc.close()
