"""CPU tests: the oracle (C restatement) against the committed golden vectors
and against the independent Python restatement (tests/golden/make_golden.py)."""
import json
import os
import random
import sys
import tempfile
import zlib

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
sys.path.insert(0, GOLD)
import make_golden as mg  # noqa: E402

from oracle import cly_oracle as co  # noqa: E402

with open(os.path.join(GOLD, "golden.json")) as _f:
    GOLDEN = json.load(_f)
FIXTURES = sorted(k for k in GOLDEN if not k.startswith("_"))
FIELDS = mg.FIELDS


def load_fixture(name):
    with open(os.path.join(GOLD, name + ".cly"), "rb") as f:
        return f.read()


def tuples_as_lists(t):
    return [[int(r[f]) for f in FIELDS] for r in t]


def test_crc32_known_answers():
    for hexin, want in GOLDEN["_vectors"]["crc32_check"]:
        b = bytes.fromhex(hexin)
        assert co.crc32(b) == want == zlib.crc32(b)
    assert co.crc32(b"123456789") == 0xCBF43926          # Go crc32.ChecksumIEEE check value


def test_varint_vectors():
    for hexin, v, n in GOLDEN["_vectors"]["varint"]:
        assert co.varint(bytes.fromhex(hexin)) == (v, n), hexin


def test_anchor_record():
    # db.Put("000000001","000000001") -> EncodeLogRecord
    rec = co.encode_record(b"\x00000000001", b"000000001")
    assert rec.hex() == GOLDEN["_vectors"]["anchor_hex"]
    assert rec.hex() == "c634de65000014120000303030303030303031303030303030303031"


@pytest.mark.parametrize("name", FIXTURES)
def test_oracle_matches_golden(name):
    g = GOLDEN[name]
    data = load_fixture(name)
    assert len(data) == g["len"]
    t, st, end = co.scan_file(data, g["fid"])
    assert st == g["status"]
    assert end == g["end_offset"]
    assert tuples_as_lists(t) == g["tuples"]


@pytest.mark.parametrize("name", FIXTURES)
def test_python_restatement_matches_committed(name):
    g = GOLDEN[name]
    st, end, tuples = mg.scan(load_fixture(name), g["fid"])
    assert (st, end, tuples) == (g["status"], g["end_offset"], g["tuples"])


def random_corpus(rng, n_records, corrupt=False):
    """Mixed-shape file from the Python writer (both restatements must agree)."""
    b = bytearray()
    for i in range(n_records):
        kind = rng.random()
        tx = 0 if rng.random() < 0.7 else rng.randrange(1, 1 << 62)
        if kind < 0.6:
            v = bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 1, 7, 64, 255, 256, 300])))
        elif kind < 0.8:
            v = bytes(rng.randrange(0, 5) for _ in range(rng.randrange(0, 90)))   # header-like bytes
        else:
            v = mg.encode_record(mg.key_tx(mg.test_key(i), 0), b"x" * rng.randrange(0, 20))  # embedded
        typ = rng.choice([0, 0, 0, 1, 2, 3, 4])
        dt = rng.choice([0, 0, 1, 2, 3, 4])
        b += mg.encode_record(mg.key_tx(mg.test_key(i), tx), v, typ, dt, rng.choice([0, 0, -1, 1 << 40]))
    if corrupt and b:
        k = rng.randrange(len(b))
        b[k] ^= 1 << rng.randrange(8)
    tail = rng.choice([b"", bytes(rng.randrange(1, 40)), bytes(rng.getrandbits(8) for _ in range(rng.randrange(1, 30)))])
    return bytes(b) + tail


@pytest.mark.parametrize("seed", range(40))
def test_oracle_vs_python_random(seed):
    rng = random.Random(seed)
    data = random_corpus(rng, rng.randrange(0, 60), corrupt=seed % 3 == 0)
    st, end, tuples = mg.scan(data, 7)
    t, st2, end2 = co.scan_file(data, 7)
    assert (st2, end2) == (st, end)
    assert tuples_as_lists(t) == tuples


def test_faithful_baseline_same_result():
    data = load_fixture("c1_shape")
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "000000000.cly")
        with open(p, "wb") as f:
            f.write(data)
        n, st, end = co.scan_path_faithful(p)
    g = GOLDEN["c1_shape"]
    assert (n, st, end) == (g["n_records"], g["status"], g["end_offset"])
    for name in ("bitflip", "tail_5", "torn_kv", "zero_tail", "varint_overflow", "empty"):
        with tempfile.TemporaryDirectory() as d:
            p = os.path.join(d, "x.cly")
            with open(p, "wb") as f:
                f.write(load_fixture(name))
            n, st, end = co.scan_path_faithful(p)
        g = GOLDEN[name]
        assert (n, st, end) == (g["n_records"], g["status"], g["end_offset"]), name


def test_mt_baseline_counts():
    arrs = [np.frombuffer(load_fixture(n), np.uint8).copy() for n in ("c1_shape", "txn_hash", "zero_values")]
    total = co.scan_files_mt(arrs, [0, 1, 2], 3)
    assert total == sum(GOLDEN[n]["n_records"] for n in ("c1_shape", "txn_hash", "zero_values"))
