"""Profiling target: build a workload (argv[1], default c2) in HBM and run
cly_scan_device argv[2] times (default 3) with libclyscan (argv[3])."""
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402
from bench import make_workload  # noqa: E402
from couloydb_amd import Scanner  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
lib = sys.argv[3] if len(sys.argv) > 3 else "libclyscan.so"
wl = make_workload(cfg, torch)
sc = Scanner(0, lib=lib)
for _ in range(n):
    first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
torch.cuda.synchronize()
print(cfg, lib, "need", need, "passes", st.passes, sc.kernel_ms(), flush=True)
