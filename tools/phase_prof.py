"""Per-phase cycle breakdown of k_scan (profiling build libclyscan_prof.so,
make -C couloydb_amd/csrc prof) on a bench workload:
    python tools/phase_prof.py [c1|c2|c3|c4|c5]
Cycles are s_memtime ticks summed over tiles (lane 0 of each wave), per tile."""
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
names = ["A: spec+walk+agree+LOCAL", "look-back", "agree+inputs+INCL", "C: fast CRC stream", "C: exact lanes", "fold"]
for it in range(3):
    first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
    pr = (ctypes.c_uint64 * 12)()
    sc.lib.cly_dbg_prof(sc.ctx, pr)
    ntile = st.n_chunks // 64
    tot = sum(pr[i] for i in range(6))
    print("iter %d: k_scan %.3f ms, fin %.3f ms, %d tiles, passes %d" % (it, st.scan_ms, st.resolve_ms, ntile, st.passes),
          flush=True)
    for i, nm in enumerate(names):
        print("   %-26s %10.0f cyc/tile  %5.1f%%" % (nm, pr[i] / max(ntile, 1), 100.0 * pr[i] / max(tot, 1)), flush=True)
    print("   look-back per tile: %.2f backward windows, %.2f forward windows, %.2f LOCAL spins, %.3f bad-guess waits (%.2f spins)" % (
        pr[6] / ntile, pr[7] / ntile, pr[8] / ntile, pr[9] / ntile, pr[10] / ntile), flush=True)
