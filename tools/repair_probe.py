"""Repair-round probe: one scan of a bench workload (argv[1], default c3) with
cly_dbg_set flag 2, which prints each host-driven repair round (tiles listed,
longest walk so far); then the first-round LOCALs of the listed tiles' runs."""
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402
from bench import make_workload  # noqa: E402
from couloydb_amd import Scanner  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
wl = make_workload(cfg, torch)
sc = Scanner(0)
sc.lib.cly_dbg_set(sc.ctx, 2)
first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
torch.cuda.synchronize()
print(cfg, "passes", st.passes, "need", need, sc.kernel_ms(), flush=True)
