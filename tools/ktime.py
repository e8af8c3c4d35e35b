"""Per-kernel times of cly_scan_device (cly_dbg_kernel_ms) on a bench workload:
    python tools/ktime.py [c2|c3|...] [iters]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from bench import make_workload  # noqa: E402
from couloydb_amd import Scanner  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
libs = sys.argv[3].split(",") if len(sys.argv) > 3 else ["libclyscan.so"]
wl = make_workload(cfg, torch)
for lib in libs:
  sc = Scanner(0, lib=lib)
  sc.lib.cly_dbg_kernel_ms.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
  print(lib, sc.lib.cly_build_info().decode(), flush=True)
  for it in range(iters):
    try:
        first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
    except Exception as e:
        print("  error", str(e)[:100], flush=True)
    k = (ctypes.c_double * 6)()
    sc.lib.cly_dbg_kernel_ms(sc.ctx, k)
    print("iter %d: spec %.3f link %.3f crc %.3f fin %.3f locate %.3f | all %.3f ms  passes %d records %d expect %d" % (
        it, k[0], k[1], k[2], k[3], k[4], k[5], 0, 0, wl.expect_records), flush=True)
  sc.close()
