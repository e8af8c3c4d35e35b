"""Debug: the false-start corpus of tests/test_gpu_parity.py scanned on the GPU,
first differing tuple against the oracle (usage: python tools/dbg_false_starts.py [seed] [lib])."""
import random
import sys

import numpy as np
import torch

torch.zeros(1, device="cuda")               # (the HIP runtime up before the scanner's context)

sys.path.insert(0, "tests/golden")
sys.path.insert(0, ".")
import make_golden as mg  # noqa: E402
from couloydb_amd import DataFile, Scanner  # noqa: E402
from oracle import cly_oracle as co  # noqa: E402

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 0
lib = sys.argv[2] if len(sys.argv) > 2 else "libclyscan.so"
rng = random.Random(seed)
b = bytearray()
i = 0
while len(b) < 600_000:
    vlen = rng.choice([150, 276, 300, 777, 2000])
    key = mg.key_tx(mg.test_key(i), 0)
    hdr_len = len(mg.encode_record(key, b"")) - len(key)
    o = rng.randrange(0, vlen - 40)
    start_v = len(b) + hdr_len + len(key)
    rec_end = start_v + vlen
    fpos = start_v + o
    ks = 10
    body_len = rec_end - fpos
    for hsz in range(9, 20):
        vs = body_len - hsz - ks
        fh = rng.randbytes(4) + bytes([rng.randrange(5), rng.randrange(5)]) + mg.put_varint(ks) + \
            mg.put_varint(vs) + mg.put_varint(0)
        if len(fh) == hsz:
            break
    v = bytearray(rng.randbytes(vlen))
    v[o:o + len(fh)] = fh
    b += mg.encode_record(key, bytes(v))
    i += 1
data = np.frombuffer(bytes(b), np.uint8).copy()
sc = Scanner(0, lib=lib)
r = sc.scan([DataFile(data, 4)])
t, st, end = co.scan_file(data, 4)
g = r.file_tuples(0)
print("gpu", r.status[0], r.end_offset[0], len(g), "oracle", st, end, len(t), "passes", r.stats.passes)
n = min(len(g), len(t))
for k in range(n):
    if g[k].tobytes() != t[k].tobytes():
        print("first diff", k, "gpu", g[k], "oracle", t[k])
        for j in range(max(0, k - 3), min(n, k + 3)):
            print(j, "g", g[j]["offset"], g[j]["size"], "o", t[j]["offset"], t[j]["size"])
        break
# the tuples around the reported failure: device path, every emitted tuple
from couloydb_amd import TUPLE_DTYPE  # noqa: E402
d = torch.from_numpy(np.concatenate([data, np.zeros(4096, np.uint8)])).cuda()
cap = len(data) // 9 + 16
dout = torch.empty(cap * 48, dtype=torch.uint8, device="cuda")
first, res, st2, need = sc.scan_device([(d.data_ptr(), len(data), 4)], dout.data_ptr(), cap)
allt = dout[: need * 48].cpu().numpy().view(TUPLE_DTYPE)
print("device path: status", res[0].status, "n", res[0].n_records, "need", need)
k = int(res[0].n_records)
for j in range(max(0, k - 2), min(len(allt), k + 4)):
    print(j, "gpu", allt[j], "\n   oracle", t[j] if j < len(t) else None)
bad = [j for j in range(min(len(allt), len(t))) if allt[j].tobytes() != t[j].tobytes()]
print("differing tuples", len(bad), bad[:10])
