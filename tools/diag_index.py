"""Diagnose an index mismatch: scan tuples of a typed corpus vs the oracle,
then the index states vs the restatement, with record details."""
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from tests.gpu_util import INDEX_NOW, index_states, typed_corpus  # noqa: E402
from tests.test_merge import oracle_scan, split_files  # noqa: E402
from couloydb_amd import DataFile, Scanner  # noqa: E402

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 2
lib = sys.argv[2] if len(sys.argv) > 2 else "libclyscan.so"
b = typed_corpus(100 + seed, n_ops=1500 + 500 * seed, garbage=seed % 2 == 1)
arrays, tts, _ = oracle_scan(split_files(b, 1 + seed % 3, random.Random(seed)))
s = Scanner(0, lib)
s.set_clock(INDEX_NOW)
r = s.scan([DataFile(a.copy(), i) for i, a in enumerate(arrays)])
for i, tt in enumerate(tts):
    g = r.file_tuples(i)
    same = len(g) == len(tt) and (g.view(np.uint8) == tt.view(np.uint8)).all()
    print("file", i, "len", len(arrays[i]), "n", len(tt), len(g), "same", same, "status", r.status[i])
    if not same:
        for k in range(min(len(g), len(tt))):
            if g[k].tobytes() != tt[k].tobytes():
                print(" first diff", k, "\n  gpu", g[k], "\n  ora", tt[k])
                break
want = index_states(arrays, tts)
got, ir = s.index([DataFile(a.copy(), i) for i, a in enumerate(arrays)])
bad = np.nonzero(got != want)[0]
print("index bad", bad[:20], "n_coll", ir.n_collisions)
allt = np.concatenate(tts)
for k in bad[:6]:
    t = allt[k]
    F = arrays[int(t["fid"])]
    o, h, ks = int(t["offset"]), int(t["header_size"]), int(t["key_size"])
    print(k, "gpu", got[k], "want", want[k], "fid", t["fid"], "off", o, "type", t["type"], "dt", t["data_type"],
          "tx", t["tx_id"], "key", bytes(F[o + h:o + h + ks]))
