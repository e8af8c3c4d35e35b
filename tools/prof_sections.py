"""Section cycle shares of k_scan's tile body (experiment build CLY_PROF=1):
python tools/prof_sections.py [config] [lib]."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from bench import make_workload  # noqa: E402
from couloydb_amd import Scanner  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
lib = sys.argv[2] if len(sys.argv) > 2 else "libclyscan_prof.so"
wl = make_workload(cfg, torch)
sc = Scanner(0, lib)
sc.lib.cly_dbg_prof.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
out = (ctypes.c_ulonglong * 8)()
for _ in range(2):
    sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
sc.lib.cly_dbg_prof(sc.ctx, out)
N = 5
for _ in range(N):
    sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
    kms = sc.kernel_ms()
sc.lib.cly_dbg_prof(sc.ctx, out)
names = ["load wait+transpose", "stage+guess", "pred_walk", "general pass", "reload+CRC", "tile end"]
tot = sum(out[i] for i in range(6))
blocks = wl.bytes / 4096 * N
for i, n in enumerate(names):
    print("%-22s %6.1f%%  %8.0f cycles/block" % (n, 100.0 * out[i] / tot, out[i] / blocks))
print("guess blocks %.4f per block, general-pass blocks %.4f per block" % (out[6] / blocks, out[7] / blocks))
print("kernel ms", {k: round(v, 3) for k, v in kms.items()})
