"""CPU tests of the kernel logic: the per-chunk algorithm of the HIP scan
(couloydb_amd/csrc/scan_core.h — speculation, chain resolution, decoupled
look-back, CRC phases, straddle checks) run by the CPU emulator
tests/emu/libclyscan_emu*.so (test infrastructure, never the product path),
bit-exact against the golden fixtures and the oracle.  GPU parity of the
compiled kernel itself is tests/test_gpu_parity.py."""
import json
import os

import numpy as np
import pytest

from couloydb_amd import DataFile, Scanner
from oracle import cly_oracle as co

from .gpu_util import FIELDS, compare, fixed_records_file, mixed_corpus

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
EMU = os.path.join(HERE, "emu")
with open(os.path.join(GOLD, "golden.json")) as _f:
    GOLDEN = json.load(_f)
FIXTURES = sorted(k for k in GOLDEN if not k.startswith("_"))


def _emu(name):
    path = os.path.join(EMU, name)
    if not os.path.exists(path):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", EMU])
    return path


@pytest.fixture(scope="module", params=["libclyscan_emu.so", "libclyscan_emu_small.so"])
def emu(request):
    s = Scanner(0, lib=_emu(request.param))
    yield s
    s.close()


def fixture_file(name):
    with open(os.path.join(GOLD, name + ".cly"), "rb") as f:
        return DataFile(np.frombuffer(f.read(), np.uint8).copy(), GOLDEN[name]["fid"])


def test_fixtures_each(emu):
    for name in FIXTURES:
        g = GOLDEN[name]
        r = emu.scan([fixture_file(name)])
        assert (r.status[0], r.end_offset[0], r.n_records[0]) == (g["status"], g["end_offset"], g["n_records"]), name
        assert [[int(t[f]) for f in FIELDS] for t in r.file_tuples(0)] == g["tuples"], name


def test_fixtures_one_call(emu):
    files = [fixture_file(n) for n in FIXTURES]
    r = emu.scan(files)
    for i, n in enumerate(FIXTURES):
        g = GOLDEN[n]
        assert (r.status[i], r.end_offset[i]) == (g["status"], g["end_offset"]), n
        assert [[int(t[f]) for f in FIELDS] for t in r.file_tuples(i)] == g["tuples"], n


@pytest.mark.parametrize("seed", range(8))
def test_mixed_corpora(emu, seed):
    files = []
    for j in range(3):
        data = mixed_corpus(seed * 7 + j, [40_000, 300_000, 900_000][j], corrupt=(seed % 4 == 3) * (j + 1))
        files.append(DataFile(np.frombuffer(data, np.uint8).copy(), 1000 + j))
    r = emu.scan(files)
    for i, f in enumerate(files):
        t, st, end = co.scan_file(f.data, f.fid)
        compare(r.file_tuples(i), r.status[i], r.end_offset[i], t, st, end, "seed %d file %d" % (seed, i))


def test_jittered_schedule(monkeypatch):
    """Random delays before descriptor publication: chunks see predecessors
    that have only their speculative descriptor (every look-back path)."""
    monkeypatch.setenv("CLY_EMU_JITTER", "1")
    monkeypatch.setenv("CLY_EMU_THREADS", "16")
    with Scanner(0, lib=_emu("libclyscan_emu_small.so")) as s:
        for seed in range(3):
            data = mixed_corpus(100 + seed, 400_000, corrupt=seed)
            f = DataFile(np.frombuffer(data, np.uint8).copy(), 7)
            r = s.scan([f, fixture_file("big_record"), fixture_file("zero_values")])
            t, st, end = co.scan_file(f.data, 7)
            compare(r.file_tuples(0), r.status[0], r.end_offset[0], t, st, end, "jitter %d" % seed)
            g = GOLDEN["zero_values"]
            assert (r.status[2], r.end_offset[2], r.n_records[2]) == (g["status"], g["end_offset"], g["n_records"])


@pytest.mark.parametrize("shape", ["c1_slice", "zero_values", "tiny"])
def test_shapes(emu, shape):
    if shape == "c1_slice":
        data = fixed_records_file(3000, 1024, seed=11)
    elif shape == "zero_values":
        data = fixed_records_file(800, 1033, seed=12, zero_values=True)
    else:
        data = fixed_records_file(20000, 0, seed=13)
    r = emu.scan([DataFile(data, 0)])
    t, st, end = co.scan_file(data, 0)
    compare(r.file_tuples(0), r.status[0], r.end_offset[0], t, st, end, shape)


def test_chunk_boundary_tails(emu):
    base = fixed_records_file(400, 300, seed=3)
    for chunk in (1792, 31744):
        k = (len(base) // chunk) * chunk - 7
        for extra in (0, 3, 7, 8):
            for cut in (0, 1, 5, 6, 13):
                data = base[:k + extra] if k + extra <= len(base) else base
                data = np.concatenate([data, np.zeros(cut, np.uint8)]) if cut % 2 else data[: len(data) - cut]
                f = DataFile(np.ascontiguousarray(data), 5)
                r = emu.scan([f])
                t, st, end = co.scan_file(f.data, 5)
                compare(r.file_tuples(0), r.status[0], r.end_offset[0], t, st, end, "chunk %d +%d cut %d" % (chunk, extra, cut))


# Chunks captured on the GPU whose first lane holds a false candidate whose
# chain merges into the true one: the speculative guess lands before the true
# first record (tools/find_bad_guess.py + tools/replay_dump.py).
FALSE_MERGE = ["false_merge_a", "false_merge_b"]


def _golden_bytes(name):
    return np.fromfile(os.path.join(GOLD, name + ".cly"), dtype=np.uint8)


@pytest.mark.parametrize("name", FALSE_MERGE)
def test_false_merge_fixtures(emu, name):
    d = _golden_bytes(name)
    r = emu.scan([DataFile(d, 3)])
    t, st, end = co.scan_file(d, 3)
    compare(r.file_tuples(0), r.status[0], r.end_offset[0], t, st, end, name)


@pytest.mark.parametrize("seq", [False, True])
def test_wrong_guess_recovery(monkeypatch, seq):
    """The wrong-guess chunk publishes its resolved descriptor late: every
    successor's look-back walks through its speculative descriptor, fails the
    final check and recovers through that chunk's own resolved words."""
    monkeypatch.setenv("CLY_EMU_THREADS", "32")
    monkeypatch.setenv("CLY_EMU_DELAY_FULL", "2")
    if seq:
        monkeypatch.setenv("CLY_EMU_SEQ_LB", "1")
    d = np.concatenate([_golden_bytes("false_merge_a"), fixed_records_file(4000, 256, seed=9)])
    with Scanner(0, lib=_emu("libclyscan_emu.so")) as s:
        r = s.scan([DataFile(d, 0)])
    t, st, end = co.scan_file(d, 0)
    compare(r.file_tuples(0), r.status[0], r.end_offset[0], t, st, end, "recovery")
