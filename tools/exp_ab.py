"""k_scan time of alternative builds on one workload: python tools/exp_ab.py c2 lib1.so lib2.so ..."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from bench import make_workload  # noqa: E402
from couloydb_amd import Scanner  # noqa: E402

cfg = sys.argv[1]
wl = make_workload(cfg, torch)
for lib in sys.argv[2:]:
    sc = Scanner(0, lib=lib)
    ts, tot = [], []
    for it in range(5):
        first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
        ts.append(st.scan_ms)
        tot.append(st.total_ms)
        ok = all(r.status == 0 for r in res) and need == wl.expect_records
    print("%-26s k_scan %s ms  total %.3f ms  ok=%s" % (lib, " ".join("%.3f" % t for t in ts), min(tot), ok), flush=True)
    sc.close()
