"""Host-side synthetic data files for tests and diagnostics (C2/C3 shapes),
built with the oracle's EncodeLogRecord restatement (test infrastructure)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import cly_oracle as co  # noqa: E402


def zipf_lengths(n, rng, s=1.1, nmax=65473):
    ranks = np.arange(1, nmax + 1, dtype=np.float64)
    cdf = np.cumsum(ranks ** (-s))
    cdf /= cdf[-1]
    return (63 + np.searchsorted(cdf, rng.random(n)) + 1).astype(np.int64)


def make_file(value_lens, seed=1, key_base=0, limit=None):
    """Concatenated records key 0x00||%09d, random values of the given lengths."""
    rng = np.random.default_rng(seed)
    L = co.lib()
    total = int(sum(int(v) + 40 for v in value_lens))
    buf = np.zeros(total, np.uint8)
    off = 0
    for i, vl in enumerate(value_lens):
        key = b"\x00" + b"%09d" % (key_base + i)
        val = rng.integers(0, 256, int(vl), dtype=np.uint8).tobytes()
        tmp = np.zeros(26 + len(key) + len(val), np.uint8)
        n = L.clyo_encode_record(tmp.ctypes.data, 0, 0, key, len(key), val, len(val), 0)
        if limit is not None and off + n > limit:
            break
        buf[off:off + n] = tmp[:n]
        off += n
    return buf[:off]
