"""Helpers shared by the GPU tests and the bench (input builders, comparison)."""
import os
import random
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden as mg  # noqa: E402

FIELDS = mg.FIELDS


def fixed_records_file(n, value_len, seed=1, key_base=0, zero_values=False):
    """C1/C2-shape data file: key 0x00||%09d(i), value_len random (or key||zeros) bytes."""
    rng = np.random.default_rng(seed)
    hdr = mg.encode_record(mg.key_tx(mg.test_key(0), 0), b"\0" * value_len)[4:4 + 6 + 4]
    # header after the crc: type, dtype, varint(10), varint(vlen), varint(0)
    body = bytes([0, 0]) + mg.put_varint(10) + mg.put_varint(value_len) + mg.put_varint(0)
    hl = 4 + len(body)
    rs = hl + 10 + value_len
    out = np.zeros((n, rs), dtype=np.uint8)
    out[:, 4:hl] = np.frombuffer(body, np.uint8)
    keys = np.array([list(b"\x00" + mg.test_key(key_base + i)) for i in range(n)], dtype=np.uint8)
    out[:, hl:hl + 10] = keys
    if zero_values:
        out[:, hl + 10:hl + 19] = keys[:, 1:]
    else:
        out[:, hl + 10:] = rng.integers(0, 256, size=(n, value_len), dtype=np.uint8)
    for i in range(n):
        c = zlib.crc32(out[i, 4:].tobytes())
        out[i, 0:4] = np.frombuffer(c.to_bytes(4, "little"), np.uint8)
    del hdr
    return out.reshape(-1)


def mixed_corpus(seed, target_bytes, corrupt=0, tail=True):
    """Records of mixed shapes (tx ids, all types/dtypes, tombstones, header-like
    values, embedded records, long values spanning chunks)."""
    rng = random.Random(seed)
    b = bytearray()
    i = 0
    while len(b) < target_bytes:
        kind = rng.random()
        tx = 0 if rng.random() < 0.7 else rng.randrange(1, 1 << 62)
        if kind < 0.45:
            v = rng.randbytes(rng.choice([0, 1, 3, 7, 20, 64, 255, 256, 300, 1000]))
        elif kind < 0.6:
            v = bytes(rng.randrange(0, 5) for _ in range(rng.randrange(0, 120)))
        elif kind < 0.7:
            v = b"".join(mg.encode_record(mg.key_tx(mg.test_key(rng.randrange(10**9)), 0), rng.randbytes(rng.randrange(0, 30)))
                         for _ in range(rng.randrange(1, 6)))
        elif kind < 0.78:
            v = bytes(rng.randrange(0, 1 << 14))                                   # zero run
        elif kind < 0.8:
            v = rng.randbytes(rng.randrange(2000, 70000))                          # spans chunks
        else:
            v = rng.randbytes(rng.randrange(0, 64))
        typ = rng.choice([0, 0, 0, 0, 1, 2, 3, 4])
        dt = rng.choice([0, 0, 0, 1, 2, 3, 4])
        exp = rng.choice([0, 0, 0, -1, 1 << 40, 1_697_000_000_000_000_000])
        b += mg.encode_record(mg.key_tx(mg.test_key(i), tx), v, typ, dt, exp)
        i += 1
    for _ in range(corrupt):
        k = rng.randrange(len(b))
        b[k] ^= 1 << rng.randrange(8)
    if tail:
        t = rng.random()
        if t < 0.3:
            b += bytes(rng.randrange(1, 5000))
        elif t < 0.5:
            b += rng.randbytes(rng.randrange(1, 30))
        elif t < 0.6:
            del b[len(b) - rng.randrange(1, 40):]
    return bytes(b)


def compare(gpu_tuples, gpu_status, gpu_end, oracle_tuples, oracle_status, oracle_end, label=""):
    """Bit-exact comparison with a readable first difference."""
    assert gpu_status == oracle_status, "%s status gpu=%d oracle=%d (end gpu=%d oracle=%d, n gpu=%d oracle=%d)" % (
        label, gpu_status, oracle_status, gpu_end, oracle_end, len(gpu_tuples), len(oracle_tuples))
    assert gpu_end == oracle_end, "%s end_offset gpu=%d oracle=%d" % (label, gpu_end, oracle_end)
    assert len(gpu_tuples) == len(oracle_tuples), "%s n gpu=%d oracle=%d" % (label, len(gpu_tuples), len(oracle_tuples))
    if len(gpu_tuples):
        g = np.asarray(gpu_tuples).view(np.uint8).reshape(-1, 48)
        o = np.asarray(oracle_tuples).view(np.uint8).reshape(-1, 48)
        bad = np.nonzero((g != o).any(axis=1))[0]
        assert bad.size == 0, "%s first differing tuple %d: gpu=%s oracle=%s" % (
            label, bad[0], gpu_tuples[bad[0]], oracle_tuples[bad[0]])
