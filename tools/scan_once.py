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
if hasattr(sc.lib, "cly_dbg_set"):
    sc.lib.cly_dbg_set(sc.ctx, 4)       # per-kernel markers (link / k_emit / k_fin split)
st = need = None
for _ in range(n):
    try:
        first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
    except Exception as e:  # experiment builds that break the chain: the kernel times still count
        print("scan error:", e, flush=True)
torch.cuda.synchronize()
print(cfg, lib, "need", need, "passes", st.passes if st else None, sc.kernel_ms(), flush=True)
