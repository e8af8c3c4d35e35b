"""Per-phase cycle breakdown of k_scan / k_fix (profiling build
libclyscan_prof.so) on a bench workload: python tools/phase_prof.py [c1|c2|c3]"""
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
names = ["stage", "filter+spec", "resolve", "crc+summary", "stage tuples", "desc"]
for it in range(3):
    first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
    pr = (ctypes.c_uint64 * 24)()
    sc.lib.cly_dbg_prof(sc.ctx, pr)
    s4 = (ctypes.c_uint32 * 4)()
    sc.lib.cly_dbg_stats(sc.ctx, s4)
    nsub = st.n_chunks
    print("iter %d: k_scan %.3f ms, link+place+fin %.3f ms, %d sub-tiles, %d fixes, passes %d, grid %d" % (
        it, st.scan_ms, st.resolve_ms, nsub, s4[0], st.passes, s4[2]), flush=True)
    for base, kname, n in ((0, "scan", nsub), (8, "fix", max(s4[0], 1))):
        tot = sum(pr[base + i] for i in range(6))
        for i, nm in enumerate(names):
            print("   %-4s %-14s %9.0f cyc/sub-tile  %5.1f%%" % (kname, nm, pr[base + i] / n, 100.0 * pr[base + i] / max(tot, 1)),
                  flush=True)
