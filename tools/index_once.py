"""Index A/B target: build a bench workload (argv[1], default c4) in HBM, scan
it once, then run cly_index_device 5 times with each library named after it
(default libclyscan.so); prints per library the best index_ms, the counters and
a digest of the per-record states (equal digests = identical index states).
    python tools/index_once.py c4 libclyscan.so libexp_fd8e900.so"""
import hashlib
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402
from bench import make_workload  # noqa: E402
from couloydb_amd import Scanner  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
libs = sys.argv[2:] or ["libclyscan.so"]
wl = make_workload(cfg, torch)
for rep in range(2):
    for lib in libs:
        sc = Scanner(0, lib=lib)
        first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
        d_state = torch.empty(max(1, need), dtype=torch.uint8, device="cuda")
        best = None
        for _ in range(5):
            r = sc.index_device(wl.dev_files, wl.d_out.data_ptr(), first, res, d_state.data_ptr())
            best = r.index_ms if best is None else min(best, r.index_ms)
        torch.cuda.synchronize()
        dig = hashlib.sha1(d_state[:need].cpu().numpy().tobytes()).hexdigest()[:16]
        print("%s %s rep %d index_ms %.3f live %d applied %d collisions %d state %s" % (
            cfg, lib, rep, best, r.n_live, r.n_applied, r.n_collisions, dig), flush=True)
        del d_state, sc
        torch.cuda.empty_cache()
