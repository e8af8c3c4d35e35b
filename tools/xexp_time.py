"""k_scan time of the round-2 timing-experiment builds (make -C couloydb_amd/csrc xexp)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from bench import make_workload  # noqa: E402
from couloydb_amd import Scanner  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
libs = sys.argv[2].split(",") if len(sys.argv) > 2 else ["libclyscan.so", "libclyscan_x1.so", "libclyscan_x2.so"]
wl = make_workload(cfg, torch)
for lib in libs:
    sc = Scanner(0, lib=lib)
    ts = []
    for it in range(4):
        try:
            first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
            ts.append(st.scan_ms)
        except Exception as e:
            ts.append(float("nan"))
            print(lib, "error", str(e)[:200], flush=True)
    print("%-22s k_scan %s ms" % (lib, " ".join("%.3f" % t for t in ts)), flush=True)
    sc.close()
