"""Merge rewrite (db.merge, merge.go:90-143).

CPU: the oracle's C restatement (oracle/cly_oracle.c clyo_merge) against the
independent pure-Python restatement (tests/gpu_util.py py_merge) on String-key
workloads with overwrites, deletes and transactions, on every golden fixture
(all records live) and on mixed corpora with random live masks.
GPU (-m gpu): the HIP merge (cly_merge / cly_merge_device through the C-ABI)
against the oracle, byte for byte: merge data files, hint-index file, counters.
The reference ships no merge byte vectors: parity with the Go
binary is pinned through the restatements only."""
import json
import os
import random

import numpy as np
import pytest

from oracle import cly_oracle as co

from .gpu_util import merge_corpus, mg, mixed_corpus, py_merge, string_live_mask

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
with open(os.path.join(GOLD, "golden.json")) as _f:
    GOLDEN = json.load(_f)
FIXTURES = sorted(k for k in GOLDEN if not k.startswith("_"))


def split_files(b, nfiles, rng):
    """Cut a record stream into data files at record boundaries (as appendLogRecord rotates)."""
    _, _, recs = mg.scan(b, 0)
    cuts = sorted(rng.sample(range(1, len(recs)), min(nfiles - 1, max(0, len(recs) - 1)))) if len(recs) > 1 else []
    offs = [0] + [recs[c][0] for c in cuts] + [len(b)]
    return [b[offs[i]:offs[i + 1]] for i in range(len(offs) - 1)]


def oracle_scan(files):
    arrays = [np.frombuffer(f, np.uint8) for f in files]
    tts, sts = [], []
    for fid, a in enumerate(arrays):
        t, st, _ = co.scan_file(a, fid)
        tts.append(t)
        sts.append(st)
    return arrays, tts, sts


def flat(tts):
    tuples = np.concatenate(tts) if tts else np.zeros(0, co.TUPLE_DTYPE)
    tf = np.concatenate([np.full(len(t), i, np.uint32) for i, t in enumerate(tts)]) if tts else np.zeros(0, np.uint32)
    return tuples, tf


def check_oracle(files, live, dfs):
    arrays, tts, _ = oracle_scan(files)
    tuples, tf = flat(tts)
    rc, outs, hint, r = co.merge(arrays, tuples, tf, live, dfs)
    assert rc == 0
    p_outs, p_hint = py_merge(arrays, tts, live, dfs)
    assert outs == p_outs
    assert hint == p_hint
    assert r.n_live == int(np.count_nonzero(live)) and r.n_out_files == len(p_outs)
    return outs, hint, r


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("dfs", [1200, 4096, 1 << 20])
def test_oracle_merge_string_workload(seed, dfs):
    rng = random.Random(seed)
    b = merge_corpus(seed, n_keys=200 + 50 * seed)
    files = split_files(b, 1 + seed % 4, rng)
    arrays, tts, _ = oracle_scan(files)
    live = string_live_mask(arrays, tts)
    _, _, r = check_oracle(files, live, dfs)
    assert r.n_reencoded > 0 or seed % 2          # committed tx records get a NO_TX_ID key


@pytest.mark.parametrize("seed", range(4))
def test_oracle_merge_mixed_random_live(seed):
    rng = np.random.default_rng(seed)
    b = mixed_corpus(100 + seed, 60_000, tail=False)
    files = split_files(b, 3, random.Random(seed))
    arrays, tts, _ = oracle_scan(files)
    live = (rng.random(sum(len(t) for t in tts)) < 0.6).astype(np.uint8)
    check_oracle(files, live, 1 << 16)


def test_oracle_merge_fixtures_all_live():
    for name in FIXTURES:
        g = GOLDEN[name]
        if g["status"] < 0:
            continue
        with open(os.path.join(GOLD, name + ".cly"), "rb") as f:
            b = f.read()
        arrays, tts, _ = oracle_scan([b])
        tuples, tf = flat(tts)
        live = np.ones(len(tuples), np.uint8)
        if len(tuples) and (tuples["txid_len"] == 0xFF).any():
            rc, _, _, _ = co.merge(arrays, tuples, tf, live, 1 << 20)
            assert rc == -3, name
            continue
        check_oracle([b], live, 1 << 20)


def test_oracle_merge_rotation_exact_fit():
    # records of 276 B, data file of exactly 3 records: rotation when WriteOff+size > DataFileSize
    recs = b"".join(mg.encode_record(mg.key_tx(mg.test_key(i), 0), bytes(256)) for i in range(10))
    live = np.ones(10, np.uint8)
    outs, hint, r = check_oracle([recs], live, 3 * 276)
    assert [len(o) for o in outs] == [828, 828, 828, 276]
    assert r.n_reencoded == 0 and outs[0] == recs[:828]


def test_oracle_merge_record_larger_than_file():
    recs = mg.encode_record(mg.key_tx(mg.test_key(1), 0), bytes(500))
    arrays, tts, _ = oracle_scan([recs])
    tuples, tf = flat(tts)
    rc, _, _, _ = co.merge(arrays, tuples, tf, np.ones(1, np.uint8), 100)
    assert rc == -12


# ---------------------------------------------------------------- GPU --------
@pytest.fixture(scope="module")
def scanner():
    from couloydb_amd import Scanner
    s = Scanner(0)
    yield s
    s.close()


def gpu_vs_oracle(scanner, files, live, dfs):
    from couloydb_amd import DataFile
    arrays, tts, _ = oracle_scan(files)
    tuples, tf = flat(tts)
    rc, outs, hint, r = co.merge(arrays, tuples, tf, live, dfs)
    assert rc == 0
    m = scanner.merge([DataFile(a.copy(), i) for i, a in enumerate(arrays)], live, dfs)
    assert m.n_out_files == r.n_out_files and m.n_live == r.n_live and m.n_reencoded == r.n_reencoded
    for k, (g, o) in enumerate(zip(m.files, outs)):
        assert len(g) == len(o), "file %d length gpu=%d oracle=%d" % (k, len(g), len(o))
        if g != o:
            d = next(i for i in range(len(g)) if g[i] != o[i])
            raise AssertionError("merge file %d differs at byte %d" % (k, d))
    assert m.hint == hint
    return m


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("dfs", [1200, 4096, 1 << 20])
def test_gpu_merge_string_workload(scanner, seed, dfs):
    rng = random.Random(seed)
    b = merge_corpus(seed, n_keys=200 + 50 * seed)
    files = split_files(b, 1 + seed % 4, rng)
    arrays, tts, _ = oracle_scan(files)
    gpu_vs_oracle(scanner, files, string_live_mask(arrays, tts), dfs)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_gpu_merge_mixed_random_live(scanner, seed):
    rng = np.random.default_rng(seed)
    b = mixed_corpus(100 + seed, 200_000, tail=False)
    files = split_files(b, 3, random.Random(seed))
    arrays, tts, _ = oracle_scan(files)
    live = (rng.random(sum(len(t) for t in tts)) < 0.6).astype(np.uint8)
    gpu_vs_oracle(scanner, files, live, 1 << 16)


@pytest.mark.gpu
def test_gpu_merge_fixtures_all_live(scanner):
    from couloydb_amd import DataFile, ScanError
    for name in FIXTURES:
        g = GOLDEN[name]
        with open(os.path.join(GOLD, name + ".cly"), "rb") as f:
            b = f.read()
        arrays, tts, _ = oracle_scan([b])
        tuples, _ = flat(tts)
        live = np.ones(len(tuples), np.uint8)
        if g["status"] < 0:
            with pytest.raises(ScanError) as ei:          # merge.go:94-99 returns the scan's error
                scanner.merge([DataFile(np.frombuffer(b, np.uint8).copy(), 0)], live, 1 << 20)
            assert ei.value.code == g["status"], name
            continue
        if len(tuples) and (tuples["txid_len"] == 0xFF).any():
            with pytest.raises(ScanError) as ei:
                scanner.merge([DataFile(np.frombuffer(b, np.uint8).copy(), 0)], live, 1 << 20)
            assert ei.value.code == -3, name
            continue
        gpu_vs_oracle(scanner, [b], live, 1 << 20)


@pytest.mark.gpu
def test_gpu_merge_rotation_and_verbatim(scanner):
    recs = b"".join(mg.encode_record(mg.key_tx(mg.test_key(i), 0), bytes(256)) for i in range(5000))
    live = (np.arange(5000) % 3 != 0).astype(np.uint8)
    m = gpu_vs_oracle(scanner, [recs], live, 64 * 276 + 100)
    assert m.n_reencoded == 0 and m.n_out_files > 50


@pytest.mark.gpu
def test_gpu_merge_big_records_and_empty(scanner):
    rng = random.Random(7)
    recs = b"".join(mg.encode_record(mg.key_tx(mg.test_key(i), i % 3), rng.randbytes(rng.randrange(0, 70000)))
                    for i in range(60))
    gpu_vs_oracle(scanner, [recs], np.ones(60, np.uint8), 1 << 20)
    gpu_vs_oracle(scanner, [recs], np.zeros(60, np.uint8), 1 << 20)


@pytest.mark.gpu
@pytest.mark.parametrize("kmax", [3, 60, 400])
def test_gpu_merge_hint_key_lengths(scanner, kmax):
    """Hint records of realKeys from 0 bytes up to kmax (k_mhint: the LDS stage
    of a workgroup's records, and the direct path when they exceed it), with
    txId prefixes of 1-3 bytes (re-encoded records) and without."""
    rng = random.Random(kmax)
    recs = []
    for i in range(3000):
        key = rng.randbytes(rng.randrange(0, kmax + 1))
        recs.append(mg.encode_record(mg.key_tx(key, rng.choice([0, 0, 5, 300, 70000])), rng.randbytes(rng.randrange(0, 40))))
    b = b"".join(recs)
    live = (np.random.default_rng(kmax).random(3000) < 0.8).astype(np.uint8)
    gpu_vs_oracle(scanner, split_files(b, 2, rng), live, 1 << 16)


@pytest.mark.gpu
def test_gpu_merge_device_c4_shape():
    """BASELINE config 4's shape (puts, k%4==0 overwritten, k%4==2 deleted: 50 %
    of the records dead) at 600 MiB with the reference's 256 MiB data files,
    through the device-resident entry, against the oracle byte for byte."""
    import torch
    import bench
    from couloydb_amd import Scanner, TUPLE_DTYPE
    wl = bench.make_workload("c4", torch, size=600 << 20)
    with Scanner(0) as sc:
        first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
        assert all(r.status == 0 for r in res) and need == wl.expect_records
        rc, lens, m = sc.merge_device(wl.dev_files, wl.d_out.data_ptr(), first, res, wl.live.data_ptr(),
                                      bench.DATA_FILE_SIZE, wl.d_merge.data_ptr(), wl.merge_max_files,
                                      wl.d_hint.data_ptr(), wl.hint_cap)
        assert rc == 0 and m.n_live == wl.n_live and m.n_reencoded == 0
    arrays = [wl.file_bytes(i) for i in range(len(wl.dev_files))]
    tts = [co.scan_file(a, wl.dev_files[i][2])[0] for i, a in enumerate(arrays)]
    tuples, tf = flat(tts)
    got = wl.d_out[: need * 48].cpu().numpy().view(TUPLE_DTYPE)
    assert (got.view(np.uint8) == tuples.view(np.uint8)).all()
    rc, outs, hint, r = co.merge(arrays, tuples, tf, wl.live_np, bench.DATA_FILE_SIZE)
    assert rc == 0 and r.n_out_files == m.n_out_files == len(lens)
    for k in range(len(lens)):
        o = wl.d_merge[k * bench.DATA_FILE_SIZE:k * bench.DATA_FILE_SIZE + lens[k]].cpu().numpy().tobytes()
        assert o == outs[k], k
    assert wl.d_hint[:m.hint_bytes].cpu().numpy().tobytes() == hint


# ------------------------------------------------ hint-index load (§8f row 2) --
def py_decode_pos(v):
    """DecodeLogRecordPos restated (data/logRecord.go:126-134)."""
    f, n = mg.varint(v)
    if n < 0:
        return None
    o, _ = mg.varint(v[n:])
    return f & 0xFFFFFFFF, o


POS_EDGE = [b"", bytes([0]), bytes([2, 0x80, 1]), bytes([3]), bytes([0xff] * 11), bytes([0x80] * 3),
            bytes([4]) + bytes([0xff] * 11), bytes([0xfe, 0xff, 0xff, 0xff, 0x1f, 0x88, 0x04])]


def test_oracle_decode_pos_edges():
    for v in POS_EDGE:
        rc, f, o = co.decode_pos(v)
        want = py_decode_pos(v)
        assert (rc == -3) == (want is None), v.hex()
        if want is not None:
            assert (f, o) == want, v.hex()


def test_oracle_hint_of_merge_roundtrip():
    b = merge_corpus(3, n_keys=400)
    arrays, tts, _ = oracle_scan(split_files(b, 2, random.Random(3)))
    live = string_live_mask(arrays, tts)
    tuples, tf = flat(tts)
    rc, outs, hint, r = co.merge(arrays, tuples, tf, live, 4096)
    assert rc == 0
    ht, st, end = co.scan_file(np.frombuffer(hint, np.uint8), 0)
    assert st == 0 and end == len(hint) and len(ht) == r.n_live
    rc, fids, offs = co.hint_positions(np.frombuffer(hint, np.uint8), ht)
    assert rc == 0
    for t, f, o in zip(ht, fids, offs):
        # every position points at a merged record whose realKey is the hint key
        hk = hint[int(t["offset"]) + int(t["header_size"]):][:int(t["key_size"])]
        m = np.frombuffer(outs[f], np.uint8)
        rec, _, _ = co.scan_file(m[o:], 0)
        k0 = int(rec[0]["header_size"])
        assert outs[f][o + k0:o + k0 + int(rec[0]["key_size"])] == b"\x00" + hk


def hint_file_with(values):
    return b"".join(mg.encode_record(mg.test_key(i), v) for i, v in enumerate(values))


@pytest.mark.gpu
def test_gpu_hint_scan(scanner):
    from couloydb_amd import DataFile, ScanError
    b = merge_corpus(5, n_keys=3000)
    arrays, tts, _ = oracle_scan(split_files(b, 3, random.Random(5)))
    live = string_live_mask(arrays, tts)
    tuples, tf = flat(tts)
    rc, outs, hint, r = co.merge(arrays, tuples, tf, live, 1 << 16)
    files = [np.frombuffer(hint, np.uint8).copy(), np.frombuffer(hint_file_with(POS_EDGE[:4] + POS_EDGE[5:6]), np.uint8).copy()]
    with open(os.path.join(GOLD, "hint_index.cly"), "rb") as f:
        files.append(np.frombuffer(f.read(), np.uint8).copy())
    for h in files:
        t, st, end = co.scan_file(h, 0)
        rc, fids, offs = co.hint_positions(h, t)
        assert rc == 0
        gt, gp, gst, gend = scanner.load_hint(DataFile(h, 0))
        assert (gst, gend) == (st, end) and len(gt) == len(t)
        assert (gt.view(np.uint8) == t.view(np.uint8)).all()
        assert (gp["fid"] == fids).all() and (gp["offset"] == offs).all()
    # a value whose first varint overflows: the reference panics at that record
    bad = np.frombuffer(hint_file_with([bytes([2, 4]), bytes([6, 8]), bytes([0xff] * 11), bytes([2, 2])]), np.uint8).copy()
    with pytest.raises(ScanError) as ei:
        scanner.load_hint(DataFile(bad, 0))
    assert ei.value.code == -3 and "after 2 records" in str(ei.value)


@pytest.mark.gpu
@pytest.mark.slow
def test_gpu_merge_c4_4gib_properties():
    """C4 shape at 4 GiB (16 data files of 256 MiB): scan -> device index ->
    merge -> rescans.  Size-independent properties: the index's live bytes are
    the workload's; the merge output decodes cleanly into exactly the live
    records, in order, with NO_TX_ID keys and the same values (verbatim copies:
    the output sizes/CRCs equal the inputs'); the hint file decodes to one
    position per live record, pointing at that record."""
    import torch
    import bench
    from couloydb_amd import POS_DTYPE, Scanner, TUPLE_DTYPE
    wl = bench.make_workload("c4", torch, size=4 << 30)
    with Scanner(0) as sc:
        first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
        assert all(r.status == 0 for r in res) and need == wl.expect_records
        d_state = torch.empty(need, dtype=torch.uint8, device="cuda")
        ir = sc.index_device(wl.dev_files, wl.d_out.data_ptr(), first, res, d_state.data_ptr())
        assert ir.n_live == wl.n_live and (d_state.cpu().numpy() == wl.live_np).all()
        rc, lens, m = sc.merge_device(wl.dev_files, wl.d_out.data_ptr(), first, res, d_state.data_ptr(),
                                      bench.DATA_FILE_SIZE, wl.d_merge.data_ptr(), wl.merge_max_files,
                                      wl.d_hint.data_ptr(), wl.hint_cap)
        assert rc == 0 and m.n_live == wl.n_live and m.n_reencoded == 0
        stride = int(m.out_stride)
        mfiles = [(wl.d_merge.data_ptr() + k * stride, lens[k], k) for k in range(len(lens))]
        cap = m.n_live + 1024
        d2 = torch.empty(cap * 48, dtype=torch.uint8, device="cuda")
        f2, r2, _, n2 = sc.scan_device(mfiles, d2.data_ptr(), cap)
        assert n2 == m.n_live and all(r.status == 0 and r.end_offset == lens[k] for k, r in enumerate(r2))
        merged = d2[:n2 * 48].cpu().numpy().view(TUPLE_DTYPE)
        d3 = torch.empty(cap * 48, dtype=torch.uint8, device="cuda")
        f3, r3, _, n3 = sc.scan_device([(wl.d_hint.data_ptr(), m.hint_bytes, 0)], d3.data_ptr(), cap)
        assert n3 == m.n_live and r3[0].status == 0
        d_pos = torch.empty(n3 * 16, dtype=torch.uint8, device="cuda")
        rc2 = sc.lib.cly_hint_positions_device(sc.ctx, wl.d_hint.data_ptr(), d3.data_ptr(), n3, d_pos.data_ptr(),
                                               None, None)
        assert rc2 == 0
        pos = d_pos.cpu().numpy().view(POS_DTYPE)
    src = wl.d_out[:need * 48].cpu().numpy().view(TUPLE_DTYPE)[wl.live_np != 0]
    for f in ("size", "key_size", "value_size", "crc", "type", "data_type", "expiration"):
        assert (merged[f] == src[f]).all(), f
    assert (merged["tx_id"] == 0).all() and (merged["txid_len"] == 1).all()
    assert (pos["fid"] == merged["fid"]).all() and (pos["offset"] == merged["offset"]).all()


@pytest.mark.gpu
def test_gpu_merge_repeated_calls_exact_scratch():
    """Regression test of the round-1 fault (a second cly_merge_device call in
    one process faulted in k_mplan while the scratch came from hipMallocAsync):
    one context, exact-size scratch (CLY_MERGE_EXACT, no slack), merges of
    growing and shrinking inputs back to back, each equal to the oracle."""
    import subprocess
    import sys
    code = r'''
import random, sys
import numpy as np
sys.path.insert(0, %r)
from tests.test_merge import gpu_vs_oracle, split_files, oracle_scan
from tests.gpu_util import merge_corpus, string_live_mask
from couloydb_amd import Scanner
with Scanner(0) as sc:
    for k, n in enumerate([120, 900, 60, 1500, 300, 1500]):
        b = merge_corpus(40 + k, n_keys=n)
        files = split_files(b, 1 + k %% 3, random.Random(k))
        arrays, tts, _ = oracle_scan(files)
        gpu_vs_oracle(sc, files, string_live_mask(arrays, tts), 4096 if k %% 2 else 1 << 20)
print("ok")
''' % os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, CLY_MERGE_EXACT="1")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0 and out.stdout.strip().endswith("ok"), out.stderr[-2000:]
