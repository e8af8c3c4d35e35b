"""Profiling target: the C4 workload in HBM, one scan, then cly_merge_device
argv[1] times (default 4) with libclyscan argv[2]; prints the merge times and
a digest of the output files and the hint file (to compare builds)."""
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402
from bench import make_workload, DATA_FILE_SIZE  # noqa: E402
from couloydb_amd import Scanner  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
lib = sys.argv[2] if len(sys.argv) > 2 else "libclyscan.so"
wl = make_workload("c4", torch)
sc = Scanner(0, lib=lib)
first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
ms = []
for _ in range(n):
    rc, lens, m = sc.merge_device(wl.dev_files, wl.d_out.data_ptr(), first, res, wl.live.data_ptr(),
                                  DATA_FILE_SIZE, wl.d_merge.data_ptr(), wl.merge_max_files,
                                  wl.d_hint.data_ptr(), wl.hint_cap)
    if rc != 0:
        raise SystemExit("merge failed: %d" % rc)
    ms.append(round(m.merge_ms, 3))
torch.cuda.synchronize()
out = sum(int(wl.d_merge[k * DATA_FILE_SIZE:k * DATA_FILE_SIZE + lens[k]].to(torch.int64).sum()) * (k + 1)
          for k in range(len(lens)))
hint = int(wl.d_hint[:int(m.hint_bytes)].to(torch.int64).sum())
print("c4 merge", lib, "ms", ms, "files", len(lens), "bytes", sum(lens), "digest", out, hint, flush=True)
