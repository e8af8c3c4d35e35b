"""Per-phase cycle breakdown of k_scan (profiling build libclyscan_prof.so) on a
bench workload: python tools/phase_prof.py [c1|c2|c3]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from bench import make_workload  # noqa: E402
from couloydb_amd import Scanner  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
wl = make_workload(cfg, torch)
sc = Scanner(0, lib="libclyscan_prof.so")
sc.lib.cly_dbg_prof.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
sc.lib.cly_dbg_stats.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
dnames = ["wait job", "stage", "filter+spec", "resolve(guess)", "wait ent", "crc", "wait fin", "redo", "emit",
          "locate+summary"]
cnames = ["wait summaries", "take ticket", "compose+SPEC", "look-back", "final+FULL"]
for it in range(3):
    first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
    pr = (ctypes.c_uint64 * 24)()
    sc.lib.cly_dbg_prof(sc.ctx, pr)
    s4 = (ctypes.c_uint32 * 4)()
    sc.lib.cly_dbg_stats(sc.ctx, s4)
    nsub = st.n_chunks
    nunits = sum((ln + 73727) // 73728 for (_, ln, _) in wl.dev_files)
    print("iter %d: k_scan %.3f ms, %d sub-tiles, %d units, redo_units %d redo_subs %d grid %d" % (
        it, st.scan_ms, nsub, nunits, s4[0], s4[1], s4[2]), flush=True)
    tot = sum(pr[i] for i in range(10))
    for i, n in enumerate(dnames):
        print("   data  %-16s %9.0f cyc/sub-tile  %5.1f%%" % (n, pr[i] / nsub, 100.0 * pr[i] / max(tot, 1)), flush=True)
    tot = sum(pr[12 + i] for i in range(5))
    for i, n in enumerate(cnames):
        print("   coord %-16s %9.0f cyc/unit      %5.1f%%" % (n, pr[12 + i] / nunits, 100.0 * pr[12 + i] / max(tot, 1)),
              flush=True)
