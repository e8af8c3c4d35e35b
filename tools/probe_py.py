"""Debug: one fixture through the Python host mirror (cly_scan), with a watchdog dump."""
import faulthandler, os, sys, numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
faulthandler.dump_traceback_later(20, exit=True)
from couloydb_amd import DataFile, Scanner
lib = sys.argv[1] if len(sys.argv) > 1 else "libclyscan.so"
names = sys.argv[2:] or ["anchor"]
with Scanner(0, lib=lib) as sc:
    for n in names:
        d = np.fromfile(os.path.join("tests/golden", n + ".cly"), np.uint8)
        print(n, "scan...", flush=True)
        r = sc.scan([DataFile(d, 1)])
        print(n, r.status, r.end_offset, r.n_records, flush=True)
