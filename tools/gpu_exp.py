"""GPU experiment: scan fixtures in one process with/without the debug trace."""
import ctypes, json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from couloydb_amd import DataFile, Scanner  # noqa: E402
lib, dbg = sys.argv[1], int(sys.argv[2])
names = sys.argv[3:]
gold = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))
sc = Scanner(0, lib=lib)
sc.lib.cly_dbg_enable.argtypes = [ctypes.c_void_p, ctypes.c_int]
if dbg:
    sc.lib.cly_dbg_enable(sc.ctx, dbg)
for n in names:
    data = np.fromfile(os.path.join(ROOT, "tests", "golden", n + ".cly"), dtype=np.uint8)
    try:
        r = sc.scan([DataFile(data, gold[n]["fid"])])
        g = gold[n]
        print(n, "ok" if (r.status[0], r.end_offset[0], r.n_records[0]) == (g["status"], g["end_offset"], g["n_records"]) else "MISMATCH", flush=True)
    except Exception as e:
        print(n, "ERROR", e, flush=True)
