"""k_scan time of timing-experiment builds (make -C couloydb_amd/csrc exp):
python tools/exp_time.py [c2] -> one line per library."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from bench import make_workload  # noqa: E402
from couloydb_amd import Scanner  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
wl = make_workload(cfg, torch)
for lib, what in [("libclyscan.so", "full"), ("libclyscan_exp1.so", "no tuples"), ("libclyscan_exp2.so", "no CRC"),
                  ("libclyscan_exp3.so", "no tuples, no CRC"), ("libclyscan_exp4.so", "no speculation/chain"),
                  ("libclyscan_exp7.so", "window + descriptor only"),
                  ("libclyscan_exp11.so", "speculation only")]:
    sc = Scanner(0, lib=lib)
    ts = []
    for it in range(3):
        try:
            first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
            ts.append(st.scan_ms)
        except Exception as e:      # experiment builds may not resolve; k_scan time is what counts
            ts.append(float("nan"))
            print(lib, "error", e, flush=True)
    print("%-22s %-24s k_scan %s ms" % (lib, what, " ".join("%.3f" % t for t in ts)), flush=True)
    sc.close()
