"""Turn a device dump (tools/find_bad_guess.py) into a replayable data file:
find the true record chain in the dump with the oracle, then prepend one filler
record so every byte keeps its original offset modulo CHUNK.  Writes
<dump>.cly and prints the oracle result."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import cly_oracle as co  # noqa: E402

CHUNK = 7936


def true_start(d):
    best = (-1, 0)
    for off in range(0, 600):
        t, st, end = co.scan_file(d[off:], 0)
        if off + end > best[0] or (off + end == best[0] and len(t) > best[1]):
            best = (off + end, len(t), off)
    return best[2]


def filler(n):
    """One well-formed record of exactly n bytes (n >= 16)."""
    L = co.lib()
    for vl in range(max(0, n - 40), n + 1):
        key = b"\x00FILLER000"
        tmp = np.zeros(64 + vl, np.uint8)
        m = L.clyo_encode_record(tmp.ctypes.data, 0, 0, key, len(key), b"\x5a" * vl, vl, 0)
        if m == n:
            return tmp[:m]
    raise ValueError(n)


def build(path, file_lo):
    d = np.fromfile(path, dtype=np.uint8)
    b0 = true_start(d)
    need = (file_lo + b0) % CHUNK
    while need < 20:
        need += CHUNK
    out = np.concatenate([filler(need), d[b0:]])
    t, st, end = co.scan_file(out, 0)
    out[:end].tofile(path + ".cly")          # cut the torn tail
    return b0, need, len(t), end


if __name__ == "__main__":
    for arg in sys.argv[1:]:
        p, lo = arg.split(":")
        print(p, build(p, int(lo)))
