"""Diagnose the c4 workload at a given size: per-file scan status / records / end."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
torch.cuda.set_device(0)
import bench  # noqa: E402
from couloydb_amd import Scanner  # noqa: E402

size = float(sys.argv[1]) if len(sys.argv) > 1 else 32
wl = bench.make_workload("c4", torch, size=int(size * 2**30))
print("files", len(wl.dev_files), "records expected", wl.expect_records, flush=True)
with Scanner(0) as sc:
    first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
    print("need", need, "passes", st.passes, "scan_ms", st.scan_ms, "resolve_ms", st.resolve_ms, flush=True)
    bad = 0
    for i, r in enumerate(res):
        ln = wl.dev_files[i][1]
        if r.status != 0 or r.end_offset != ln or i < 3:
            b = wl.file_bytes(i)
            e = r.end_offset
            print(i, "status", r.status, "n", r.n_records, "end", e, "len", ln,
                  "bytes@end", b[e:e + 24].tobytes().hex() if e < ln else "", flush=True)
            bad += 1
            if bad > 12:
                break
