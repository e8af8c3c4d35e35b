"""Index rebuild (db.loadIndex, db.go:511-651) on the
device: per record the state of the indexes after the load (String/ListMeta
workloads here; the composite Hash/List/Set keys in test_index_keys.py).

CPU: the literal restatement (tests/gpu_util.py index_states, a map of tx
buffers as db.go keeps it) against the independent liveness restatement used
for merge (string_live_mask) on String workloads.  GPU (-m gpu): cly_index /
cly_index_device against index_states, byte for byte, incl. forced key-hash
collisions (CLY_IX_HASH_MASK) and the C4 shape through the device entry."""
import os
import random

import numpy as np
import pytest

from oracle import cly_oracle as co

from .gpu_util import INDEX_NOW, index_states, merge_corpus, mixed_corpus, string_live_mask
from .test_merge import oracle_scan, split_files


def test_ttl_sweep_restatement():
    """db.go:639-651: after the load, a String key whose last put has an
    expiration set and not after now is deleted; keys without one, with a later
    one, or deleted afterwards are untouched; ListMeta keys have no TTL."""
    import make_golden as mg
    now = 1_000
    recs = [(b"a", 0, mg.STRING), (b"b", 999, mg.STRING), (b"c", 1_000, mg.STRING), (b"d", 1_001, mg.STRING),
            (b"e", 5, mg.STRING), (b"e", 0, mg.STRING), (b"f", 0, mg.STRING), (b"f", 5, mg.STRING),
            (b"g", -1, mg.STRING), (b"h", 5, mg.LISTMETA)]
    F = b"".join(mg.encode_record(mg.key_tx(k, 0), b"v", mg.NORMAL, dt, exp) for k, exp, dt in recs)
    arr = np.frombuffer(F, np.uint8).copy()
    tt, _, _ = co.scan_file(arr, 0)
    st = index_states([arr], [tt], now_ns=now)
    # swept winners are state 4 (CLY_IX_EXPIRED: db.Del appends their tombstones)
    #         a  b  c  d  e(old) e  f(old) f  g  h
    assert list(st) == [1, 4, 4, 1, 0, 1, 0, 4, 4, 1]


def test_index_restatements_agree():
    for seed in range(6):
        b = merge_corpus(seed, n_keys=150 + 40 * seed)
        arrays, tts, _ = oracle_scan(split_files(b, 1 + seed % 3, random.Random(seed)))
        st = index_states(arrays, tts, now_ns=None)
        live = string_live_mask(arrays, tts)
        strings = np.concatenate([t["data_type"] == 0 for t in tts])
        assert ((st == 1) & strings).sum() == live.sum()
        assert (((st == 1) & strings) == (live == 1)).all()


@pytest.fixture(scope="module")
def scanner():
    from couloydb_amd import Scanner
    s = Scanner(0)
    s.set_clock(INDEX_NOW)
    yield s
    s.close()


def gpu_vs_restatement(scanner, files):
    from couloydb_amd import DataFile, ScanError
    from .index_keys import GoPanic
    arrays, tts, _ = oracle_scan(files)
    dfs = [DataFile(a.copy(), i) for i, a in enumerate(arrays)]
    try:
        want = index_states(arrays, tts)
    except GoPanic:                      # loadIndex panics: the device reports the decode error
        with pytest.raises(ScanError):
            scanner.index(dfs)
        return None
    got, r = scanner.index(dfs)
    assert len(got) == len(want)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, "first differing record %d: gpu=%d want=%d" % (bad[0], got[bad[0]], want[bad[0]])
    assert r.n_live == int(((want == 1) | (want == 3)).sum()) and r.n_loadonly == int((want == 3).sum())
    assert r.n_host == 0
    return r


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_gpu_index_workload(scanner, seed):
    b = merge_corpus(seed, n_keys=300 + 100 * seed, rounds=4)
    gpu_vs_restatement(scanner, split_files(b, 1 + seed % 4, random.Random(seed)))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("dts", [(0, 0, 0, 1, 2, 3, 4), (0, 0, 0, 3, 5, 6)])
def test_gpu_index_mixed(scanner, seed, dts):
    """Mixed corpora: with Hash/List/Set records over %09d keys loadIndex's key
    decode panics (the device must report it); without them, states compare."""
    b = mixed_corpus(200 + seed, 300_000, tail=False, dts=dts)
    gpu_vs_restatement(scanner, split_files(b, 3, random.Random(seed)))


@pytest.mark.gpu
def test_gpu_index_forced_collisions(scanner, monkeypatch):
    monkeypatch.setenv("CLY_IX_HASH_MASK", "f")
    b = merge_corpus(11, n_keys=500, rounds=3)
    r = gpu_vs_restatement(scanner, split_files(b, 2, random.Random(11)))
    assert r.n_collisions > 0


@pytest.mark.gpu
@pytest.mark.parametrize("tx_frac,mask", [(0.0, None), (0.0, "f"), (0.3, None), (0.3, "f")])
def test_gpu_index_key_lengths(scanner, monkeypatch, tx_frac, mask):
    """Keys of 0..40 bytes (the 16-B key signature is exact up to 15 bytes; longer
    keys sharing their first 15 bytes need the byte comparison), without tx
    records (scan order = application order) and with them, with the natural
    hash and with a 4-bit one that puts most keys in one group."""
    from .gpu_util import varlen_key
    if mask:
        monkeypatch.setenv("CLY_IX_HASH_MASK", mask)
    b = merge_corpus(21, n_keys=600, rounds=4, tx_frac=tx_frac, key_fn=varlen_key)
    gpu_vs_restatement(scanner, split_files(b, 3, random.Random(21)))


@pytest.mark.gpu
def test_gpu_index_device_c4_shape():
    """C4 shape (k%4==0 overwritten, k%4==2 deleted) at 600 MiB through the
    device entry: the index's live records are exactly the workload's live mask."""
    import torch
    import bench
    from couloydb_amd import Scanner
    wl = bench.make_workload("c4", torch, size=600 << 20)
    with Scanner(0) as sc:
        first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
        d_state = torch.empty(need, dtype=torch.uint8, device="cuda")
        r = sc.index_device(wl.dev_files, wl.d_out.data_ptr(), first, res, d_state.data_ptr())
    got = d_state.cpu().numpy()
    assert (got == wl.live_np).all() and r.n_live == wl.n_live and r.n_host == 0 and r.n_loadonly == 0


def test_c_load_index_restatement():
    """oracle clyo_load_index (the CPU baseline of the index-load time) against
    the literal restatement: live String / ListMeta keys, swept keys, WriteOff."""
    import make_golden as mg
    for seed in range(6):
        b = merge_corpus(seed, n_keys=150 + 40 * seed)
        arrays, tts, _ = oracle_scan(split_files(b, 1 + seed % 3, random.Random(seed)))
        st = index_states(arrays, tts)
        dts = np.concatenate([t["data_type"] for t in tts])
        rc, r = co.load_index(arrays, list(range(len(arrays))), INDEX_NOW)
        assert rc == 0
        assert r.records == len(st)
        assert r.str_keys == int(((st == 1) & (dts == mg.STRING)).sum())
        assert r.listmeta_keys == int(((st == 1) & (dts == mg.LISTMETA)).sum())
        assert r.expired == int((st == 4).sum())
        assert r.write_off == len(arrays[-1])
    # Hash / List / Set records are outside this restatement
    from .gpu_util import typed_corpus
    arr = np.frombuffer(typed_corpus(1), np.uint8).copy()
    rc, _ = co.load_index([arr], [0], INDEX_NOW)
    assert rc == co.LI_UNSUPPORTED
