"""Per-kernel times (cly_dbg_kernel_ms: k_scan, link, k_emit, k_fin, k_locate,
all) of alternative builds of libclyscan on C2 (or CLY_EXP_CONFIG), with a
tuple/status check of every build against the first one:
python tools/exp_kms.py libclyscan.so libclyscan_x.so ..."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from bench import make_workload  # noqa: E402
from couloydb_amd import Scanner  # noqa: E402

wl = make_workload(os.environ.get("CLY_EXP_CONFIG", "c2"), torch)
ref = None
libs = sys.argv[1:] or ["libclyscan.so"]
for rnd in range(2):
    for lib in libs:
        sc = Scanner(0, lib=lib)
        rows = []
        for it in range(6):
            first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
            k = (ctypes.c_double * 6)()
            sc.lib.cly_dbg_kernel_ms(sc.ctx, k)
            rows.append(list(k))
        torch.cuda.synchronize()
        t64 = wl.d_out[: max(need, 1) * 48].view(torch.int64)
        sig = (tuple(first), tuple((r.status, r.end_offset, r.n_records) for r in res), int(need),
               int(t64.sum().item()), int((t64 * torch.arange(t64.numel(), device=t64.device)).sum().item()))
        if ref is None:
            ref = sig
        best = [min(r[i] for r in rows[1:]) for i in range(6)]
        print("round %d %-26s scan %.3f link %.3f emit %.3f fin %.3f all %.3f  same=%s" %
              (rnd, lib, best[0], best[1], best[2], best[3], best[5], sig == ref), flush=True)
        sc.close()
