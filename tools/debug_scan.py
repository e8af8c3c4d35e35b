"""Run golden fixtures one by one through a (debug) scan library and diff against
the golden results.  Usage: python tools/debug_scan.py [libname] [fixture ...]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from couloydb_amd import DataFile, Scanner  # noqa: E402

lib = sys.argv[1] if len(sys.argv) > 1 else "libclyscan_dbg.so"
gold = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))
names = sys.argv[2:] or sorted(k for k in gold if not k.startswith("_"))
FIELDS = ["offset", "expiration", "tx_id", "fid", "size", "key_size", "value_size", "type", "data_type",
          "header_size", "txid_len", "crc"]
sc = Scanner(0, lib=lib)
bad = 0
for n in names:
    g = gold[n]
    data = np.fromfile(os.path.join(ROOT, "tests", "golden", n + ".cly"), dtype=np.uint8)
    print("== %s len=%d" % (n, len(data)), flush=True)
    r = sc.scan([DataFile(data, g["fid"])])
    got = [[int(t[f]) for f in FIELDS] for t in r.file_tuples(0)]
    ok = (r.status[0], r.end_offset[0]) == (g["status"], g["end_offset"]) and got == g["tuples"]
    print("   gpu status=%d end=%d n=%d passes=%d | golden status=%d end=%d n=%d  %s" % (
        r.status[0], r.end_offset[0], r.n_records[0], r.stats.passes, g["status"], g["end_offset"],
        g["n_records"], "OK" if ok else "MISMATCH"), flush=True)
    if not ok:
        bad += 1
        for i, (a, b) in enumerate(zip(got, g["tuples"])):
            if a != b:
                print("   first diff at %d: gpu=%s gold=%s" % (i, a, b))
                break
print("mismatches:", bad)
