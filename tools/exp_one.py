"""Run k_scan of one library on the C2 workload a few times (for per-library PMC
passes): python tools/exp_one.py LIB [c2]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from bench import make_workload  # noqa: E402
from couloydb_amd import Scanner  # noqa: E402

lib = sys.argv[1]
wl = make_workload(sys.argv[2] if len(sys.argv) > 2 else "c2", torch)
sc = Scanner(0, lib=lib)
for it in range(2):
    try:
        first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
        print(lib, "k_scan %.3f ms" % st.scan_ms, flush=True)
    except Exception as e:
        print(lib, "error", e, flush=True)
sc.close()
