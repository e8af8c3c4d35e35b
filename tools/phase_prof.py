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
sc.lib.cly_dbg_phases.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
names = {1: "ticket+setup", 2: "stage+spec+guess", 3: "resolve+publish SPEC", 4: "CRC (guessed chain)",
         5: "look-back", 6: "redo+publish FULL", 7: "emit", 8: "summary"}
for it in range(3):
    first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
    ph = (ctypes.c_uint64 * (19 + 32 * 6))()
    sc.lib.cly_dbg_phases(sc.ctx, ph)
    n = st.n_chunks
    tot = sum(ph[k] for k in names)
    print("iter %d: k_scan %.3f ms, %d chunks, avg cycles/chunk %.0f" % (it, st.scan_ms, n, tot / n), flush=True)
    print("   look-back: windows/chunk %.2f  spins/chunk %.2f  slow steps/chunk %.2f  fallbacks %d" % (
        ph[10] / n, ph[11] / n, ph[12] / n, ph[13]), flush=True)
    if it == 2:
        for k in range(min(12, ph[18])):
            v = [ctypes.c_int64(ph[19 + k * 6 + m]).value for m in range(6)]
            print("   fallback c=%d jf=%d req=%d e0=%d X=%d w0=%#x (e0-X=%d, chunk(e0)=%d)" % (
                v[0], v[1], v[2], v[3], v[4], v[5] & 0xffffffffffffffff, v[3] - v[4], v[3] // 7936), flush=True)
    for k, nm in names.items():
        print("   %-26s %10.0f cyc/chunk  %5.1f%%" % (nm, ph[k] / n, 100.0 * ph[k] / max(tot, 1)), flush=True)
