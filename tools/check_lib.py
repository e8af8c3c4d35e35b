"""Run the golden fixtures (and optional random corpora) through a scan library
(default: libclyscan.so) and diff against the golden results / oracle.
Usage: python tools/check_lib.py [lib] [--corpora N]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from couloydb_amd import DataFile, Scanner  # noqa: E402
from oracle import cly_oracle as co  # noqa: E402
from gpu_util import mixed_corpus  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
lib = args[0] if args else "libclyscan.so"
ncorp = 0
for a in sys.argv[1:]:
    if a.startswith("--corpora="):
        ncorp = int(a.split("=")[1])
gold = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))
names = sorted(k for k in gold if not k.startswith("_"))
FIELDS = ["offset", "expiration", "tx_id", "fid", "size", "key_size", "value_size", "type", "data_type",
          "header_size", "txid_len", "crc"]
sc = Scanner(0, lib=lib)
bad = 0
for n in names:
    g = gold[n]
    data = np.fromfile(os.path.join(ROOT, "tests", "golden", n + ".cly"), dtype=np.uint8)
    try:
        r = sc.scan([DataFile(data, g["fid"])])
    except Exception as e:
        bad += 1
        print("%-20s len=%6d ERROR %s" % (n, len(data), e), flush=True)
        continue
    got = [[int(t[f]) for f in FIELDS] for t in r.file_tuples(0)]
    ok = (r.status[0], r.end_offset[0]) == (g["status"], g["end_offset"]) and got == g["tuples"]
    if not ok:
        bad += 1
        print("%-20s len=%6d got st=%d end=%d n=%d | gold st=%d end=%d n=%d MISMATCH" % (
            n, len(data), r.status[0], r.end_offset[0], r.n_records[0], g["status"], g["end_offset"], g["n_records"]))
        for i, (a, b) in enumerate(zip(got, g["tuples"])):
            if a != b:
                print("   first diff at %d: got=%s gold=%s" % (i, a, b))
                break
print("fixtures: %d mismatches of %d" % (bad, len(names)))
cb = 0
for seed in range(ncorp):
    files = []
    for j in range(3):
        data = mixed_corpus(seed * 7 + j, [40_000, 300_000, 1_500_000][j], corrupt=(seed % 4 == 3) * (j + 1))
        files.append(DataFile(np.frombuffer(data, np.uint8).copy(), 1000 + j))
    try:
        r = sc.scan(files)
    except Exception as e:
        cb += 3
        print("corpus seed %d ERROR %s" % (seed, e), flush=True)
        continue
    for i, f in enumerate(files):
        t, st, end = co.scan_file(f.data, f.fid)
        g = r.file_tuples(i)
        ok = (r.status[i], r.end_offset[i]) == (st, end) and len(g) == len(t) and \
            (g.view(np.uint8) == t.view(np.uint8)).all()
        if not ok:
            cb += 1
            print("corpus seed %d file %d: got st=%d end=%d n=%d | oracle st=%d end=%d n=%d" % (
                seed, i, r.status[i], r.end_offset[i], len(g), st, end, len(t)))
print("corpora: %d mismatches of %d files" % (cb, 3 * ncorp))
