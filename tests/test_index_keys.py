"""The composite index keys (Hash/List/Set on the device).

CPU: the Python restatement (tests/index_keys.py) pinned by known answers of
the reference's writers (encodeListKey/GobEncode of integer seqs round-trip,
hashMemberKey); the product's key derivation (couloydb_amd/csrc/ixkey.h, the
same code the device index runs, exported by libclyscan.so as cly_index_key)
against the restatement on the keys typed_corpus writes and on random and
adversarial byte strings, including every gob form a list seq can take; the
literal loadIndex restatement's composite semantics on small hand cases.
GPU (-m gpu): cly_index / cly_index_device against index_states on typed
corpora (all five data types, tx commit/rollback, records without a txId whose
load and merge keys differ, forced hash collisions), the load/merge panics,
and the merge of such files against the restatement."""
import collections
import random
import struct
import zlib

import numpy as np
import pytest

from oracle import cly_oracle as co

from . import index_keys as ik
from .gpu_util import INDEX_NOW, index_states, mg, seq_variant, typed_corpus
from .test_merge import oracle_scan, split_files


def pr_of(dtype, data):
    """index_keys.index_key in cly_index_key's (P, R) form."""
    k = ik.index_key(dtype, data)
    if k is None:
        return None
    if dtype in (mg.STRING, mg.LISTMETA):
        return b"", k[1]
    if dtype == mg.HASH:
        return struct.pack("<I", len(k[1])), k[1] + k[2]
    if dtype == mg.LIST:
        return bytes([len(k[2])]) + k[2], k[1]
    return k[2], k[1]


def test_gob_known_answers():
    # big.NewFloat(1).GobEncode(): version 1, ToNearestEven|Exact|finite, prec 53, exp 1, mantissa 0x8000...
    assert ik.gob_encode_int(1) == bytes([1, 0x0a, 0, 0, 0, 53, 0, 0, 0, 1, 0x80, 0, 0, 0, 0, 0, 0, 0])
    assert ik.gob_encode_int(-3) == bytes([1, 0x0b, 0, 0, 0, 53, 0, 0, 0, 2, 0xc0, 0, 0, 0, 0, 0, 0, 0])
    assert ik.gob_encode_int(0) == bytes([1, 0x08, 0, 0, 0, 53])
    for v in list(range(-300, 300)) + [1 << 52, -(1 << 52) + 1, 123456789]:
        g = ik.gob_encode_int(v)
        assert ik.seq_key(g) == g                    # decode -> encode is the identity on the writer's form
    assert ik.seq_key(b"") == bytes([1, 0x08, 0, 0, 0, 0])                 # Float{}: prec 0
    assert ik.seq_key(b"\x01\x0a\x00") == bytes([1, 0x08, 0, 0, 0, 53])   # too short: NewFloat(0)
    g = bytearray(ik.gob_encode_int(5))
    g[1] |= 0x10 | 0x20                               # Above, ToNearestAway: reset by SetPrec
    assert ik.seq_key(bytes(g)) == ik.gob_encode_int(5)
    # prec 64 with the rounding bit and a sticky bit: rounds up (inexact -> acc Above)
    g = bytearray(ik.gob_encode_int(1))
    g[2:6] = (64).to_bytes(4, "big")
    g[10:18] = ((1 << 63) | (1 << 10) | 1).to_bytes(8, "big")
    out = ik.seq_key(bytes(g))
    assert out[1] == 0x12 and out[10:18] == ((1 << 63) | (1 << 11)).to_bytes(8, "big")


def test_hash_member_key_known_answer():
    # consistent.HashKey: big-endian CRC-32/IEEE of EncodeByteSlices(key, member)
    want = zlib.crc32(b"\x06\x02" + b"key" + b"m") & 0xFFFFFFFF
    assert ik.hash_member_key(b"key", b"m") == want.to_bytes(4, "big")


def test_decode_panics():
    with pytest.raises(ik.GoPanic):
        ik.decode_byte_slices(b"000000123")          # key size 24 > len
    assert ik.decode_byte_slices(b"") == (b"", b"")
    assert ik.decode_byte_slices(b"\x80\x80") == (b"", b"\x80\x80")     # short varints: (0, 0)
    with pytest.raises(ik.GoPanic):
        ik.decode_byte_slices(b"\x80" * 9 + b"\x02")  # overflow: index < 0
    with pytest.raises(ik.GoPanic):
        ik.decode_list_key(b"\x08\x00\x00ab")        # seq (4 bytes) past the end
    assert ik.decode_list_key(b"\x00\x00\x00key") == (b"key", b"")


def _lib():
    from couloydb_amd import _abi
    return _abi.load_scan_lib()


def _check_same(lib, dtype, data):
    from couloydb_amd import index_key
    try:
        want = pr_of(dtype, data)
    except ik.GoPanic:
        with pytest.raises(ValueError):
            index_key(lib, dtype, data)
        return "panic"
    assert index_key(lib, dtype, data) == want, (dtype, data.hex())
    return "ok"


def test_product_keys_vs_restatement_corpus():
    """Every key typed_corpus writes, decoded both ways (stored key and realKey)."""
    lib = _lib()
    b = typed_corpus(3, n_ops=600, garbage=True)
    arr = np.frombuffer(b, np.uint8)
    tt, st, _ = co.scan_file(arr.copy(), 0)
    assert st == 0
    seen = {"ok": 0, "panic": 0}
    for t in tt:
        o, h, ks = int(t["offset"]), int(t["header_size"]), int(t["key_size"])
        key = b[o + h:o + h + ks]
        _, n = mg.varint(key)
        for d in (key, key[n:]):
            seen[_check_same(lib, int(t["data_type"]), d)] += 1
    assert seen["ok"] > 1000 and seen["panic"] > 0


def test_product_keys_vs_restatement_fuzz():
    lib = _lib()
    rng = random.Random(7)
    pool = [b"", b"\x00", b"\x80", b"\xff" * 11, b"\x80" * 9 + b"\x01", b"\x80" * 9 + b"\x02", b"\x02a", b"\x7f"]
    for _ in range(4000):
        c = rng.random()
        if c < 0.3:
            d = rng.randbytes(rng.randrange(0, 40))
        elif c < 0.6:                                     # plausible slices with odd varints
            a, m = rng.randbytes(rng.randrange(0, 6)), rng.randbytes(rng.randrange(0, 6))
            d = mg.put_varint(len(a) + rng.choice([0, 0, 1, -1, 50])) + mg.put_varint(rng.randrange(-5, 300)) + a + m
        elif c < 0.9:                                     # list keys with every gob form
            s, p, n = (seq_variant(rng.randrange(-40, 40), rng) for _ in range(3))
            d = (mg.put_varint(len(s) + rng.choice([0, 0, 0, 1, -1])) + mg.put_varint(len(p)) + mg.put_varint(len(n)) +
                 s + p + n + rng.randbytes(rng.randrange(0, 6)))
        else:
            d = rng.choice(pool) + rng.randbytes(rng.randrange(0, 4))
        for dt in (mg.HASH, mg.LIST, mg.SET, mg.STRING, 7):
            _check_same(lib, dt, d)


def test_gob_canon_fuzz():
    """Random gob buffers through the List key: the product's canonical seq
    encoding equals the math/big restatement (rounding, carries, exponent
    overflow to inf, long mantissas)."""
    lib = _lib()
    rng = random.Random(11)
    for _ in range(6000):
        n = rng.choice([0, 1, 5, 6, 7, 9, 10, 11, 14, 18, 18, 18, 26, 34])
        g = bytearray(rng.randbytes(n))
        if n >= 2 and rng.random() < 0.8:
            g[0] = 1
            if rng.random() < 0.7:
                g[1] = (g[1] & ~0x06) | 0x02                # finite
        if n >= 6 and rng.random() < 0.6:
            g[2:6] = rng.choice([0, 1, 24, 53, 54, 63, 64, 65, 200, 0xFFFFFFFF]).to_bytes(4, "big")
        if n >= 10 and rng.random() < 0.2:
            g[6:10] = rng.choice([0x7FFFFFFF, 0x7FFFFFFE, 0x80000000]).to_bytes(4, "big")
        if n >= 18 and rng.random() < 0.3:
            g[10:18] = b"\xff" * 8
        d = mg.put_varint(len(g)) + b"\x00\x00" + bytes(g) + b"k"
        _check_same(lib, mg.LIST, d)


def test_index_states_composite_cases():
    """Hand cases of the literal restatement: last writer per (key, field),
    HDel, the same entry through non-canonical encodings, a record without a
    txId (its stored key decodes to another entry: state 3), rollback."""
    def rec(key, dt, typ=mg.NORMAL, tx=0, value=b"v"):
        return mg.encode_record(mg.key_tx(key, tx), value, typ, dt, 0)
    h = lambda k, f, nc=False: (mg.put_varint(len(k)) + (b"\x80\x00" if nc else mg.put_varint(len(f))) + k + f)
    F = b"".join([
        rec(h(b"k", b"f"), mg.HASH, tx=1),                # 0 overwritten by 2
        rec(h(b"k", b"g"), mg.HASH, tx=1),                # 1 deleted by 3
        rec(h(b"k", b"f", nc=True), mg.HASH, tx=1),       # 2 same entry (k, f): wins
        rec(h(b"k", b"g"), mg.HASH, mg.DELETED, tx=1),    # 3
        rec(mg.TX_COMMIT_KEY, mg.STRING, mg.TXN_COMMIT, tx=1),
        rec(h(b"k", b"x"), mg.HASH, tx=2),                # 5 rolled back
        rec(mg.TX_ROLLBACK_KEY, mg.STRING, mg.TXN_ROLLBACK, tx=2),
        rec(h(b"s", b"m"), mg.SET, tx=0),                 # 7 no txId: loads as ("", ...), merge looks up (s, crc)
        rec(ik.encode_list_key(0, -1, 1, b"L"), mg.LIST, tx=3),   # 8
        rec(mg.TX_COMMIT_KEY, mg.STRING, mg.TXN_COMMIT, tx=3),
    ])
    arr = np.frombuffer(F, np.uint8).copy()
    tt, _, _ = co.scan_file(arr, 0)
    st = index_states([arr], [tt], now_ns=INDEX_NOW)
    assert list(st) == [0, 0, 1, 0, 0, 0, 0, 3, 1, 0]


def test_typed_corpus_restatement_runs():
    """The typed corpora load without a panic and hold every state."""
    for seed in range(4):
        b = typed_corpus(seed, n_ops=500)
        arrays, tts, _ = oracle_scan(split_files(b, 2, random.Random(seed)))
        st = index_states(arrays, tts)
        assert (st == 1).sum() > 20 and (st == 3).sum() > 0 and (st == 0).sum() > 20
        dts = np.concatenate([t["data_type"] for t in tts])
        assert set(np.unique(dts[st != 0])) >= {0, 1, 2, 3, 4}


# ---- GPU --------------------------------------------------------------------
@pytest.fixture(scope="module")
def scanner():
    from couloydb_amd import Scanner
    s = Scanner(0)
    s.set_clock(INDEX_NOW)
    yield s
    s.close()


def _gpu_vs(scanner, b, nfiles, seed):
    from couloydb_amd import DataFile
    arrays, tts, _ = oracle_scan(split_files(b, nfiles, random.Random(seed)))
    mp = []
    want = index_states(arrays, tts, merge_panics=mp)
    got, r = scanner.index([DataFile(a.copy(), i) for i, a in enumerate(arrays)])
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, "first differing record %d: gpu=%d want=%d" % (bad[0], got[bad[0]], want[bad[0]])
    assert r.n_live == int(((want == 1) | (want == 3)).sum()) and r.n_loadonly == int((want == 3).sum())
    assert r.n_merge_panic == len(mp) and r.n_host == 0
    return r


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_gpu_index_typed(scanner, seed):
    _gpu_vs(scanner, typed_corpus(100 + seed, n_ops=1500 + 500 * seed, garbage=seed % 2 == 1), 1 + seed % 3, seed)


@pytest.mark.gpu
@pytest.mark.parametrize("mask", ["f", "3ff"])
def test_gpu_index_typed_collisions(scanner, monkeypatch, mask):
    monkeypatch.setenv("CLY_IX_HASH_MASK", mask)
    r = _gpu_vs(scanner, typed_corpus(77, n_ops=2000, n_keys=30), 2, 77)
    assert r.n_collisions > 0


@pytest.mark.gpu
def test_gpu_index_load_panic(scanner):
    """A committed Hash record whose key does not decode: loadIndex panics ->
    the device index reports CLY_ERR_VARINT; the restatement raises."""
    from couloydb_amd import DataFile, ScanError
    F = (mg.encode_record(mg.key_tx(b"zz", 9), b"v", mg.NORMAL, mg.HASH, 0) +
         mg.encode_record(mg.key_tx(mg.TX_COMMIT_KEY, 9), b"", mg.TXN_COMMIT, mg.STRING, 0))
    arr = np.frombuffer(F, np.uint8).copy()
    tt, _, _ = co.scan_file(arr, 0)
    with pytest.raises(ik.GoPanic):
        index_states([arr], [tt])
    with pytest.raises(ScanError):
        scanner.index([DataFile(arr, 0)])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
def test_gpu_merge_typed_from_device_states(scanner, seed):
    """merge.go over typed corpora with the device index's states as the live
    bytes as they are (LOADONLY records must be dropped): byte-equal to the
    oracle's merge over the restatement's merge liveness (state 1)."""
    from couloydb_amd import DataFile
    from .test_merge import flat
    files = split_files(typed_corpus(300 + seed, n_ops=1200), 2, random.Random(seed))
    arrays, tts, _ = oracle_scan(files)
    want = index_states(arrays, tts)
    got, _ = scanner.index([DataFile(a.copy(), i) for i, a in enumerate(arrays)])
    assert (got == want).all() and (want == 3).any()
    tuples, tf = flat(tts)
    rc, outs, hint, r = co.merge(arrays, tuples, tf, (want == 1).astype(np.uint8), 4096)
    assert rc == 0
    m = scanner.merge([DataFile(a.copy(), i) for i, a in enumerate(arrays)], got, 4096)
    assert m.n_live == r.n_live and [bytes(x) for x in m.files] == [bytes(x) for x in outs] and m.hint == hint


@pytest.mark.gpu
def test_gpu_load_driver_composite_lookups(scanner, tmp_path):
    """cly_db_open over typed corpus files: every entry of the restated
    indexes (String, ListMeta, Hash (key, field), List (key, seq gob bytes),
    Set (key, member)) is found at its record's position through the loader's
    lookups, and the entry counts match."""
    from .index_keys import decode_byte_slices
    from .test_reference_restart import write_dir
    files = split_files(typed_corpus(500, n_ops=1500, n_keys=20), 3, random.Random(5))
    write_dir(tmp_path, files)
    arrays, tts, _ = oracle_scan(files)
    ix = {}
    index_states(arrays, tts, out_index=ix)
    counts = collections.Counter(k[0] for k in ix)
    with scanner.open_db(str(tmp_path)) as db:
        st = db.stats
        assert (st.str_keys, st.listmeta_keys, st.hash_fields, st.list_items, st.set_members) == \
            (counts[mg.STRING], counts[mg.LISTMETA], counts[mg.HASH], counts[mg.LIST], counts[mg.SET])
        for ik, (key, fid, off, tx) in ix.items():
            dt = ik[0]
            if dt == mg.STRING:
                p = db.pos(ik[1])
            elif dt == mg.LISTMETA:
                p = db.listmeta_pos(ik[1])
            elif dt == mg.HASH:
                p = db.hpos(ik[1], ik[2])
            elif dt == mg.LIST:
                p = db.lpos(ik[1], ik[2])
            else:
                _, n = mg.varint(key)
                k, m = decode_byte_slices(key if tx == 0 else key[n:])      # the load key's member
                p = db.spos(k, m)
            assert (p.fid, p.offset) == (fid, off), (ik, fid, off)
        with pytest.raises(KeyError):
            db.hpos(b"no such key", b"f0")


@pytest.mark.gpu
def test_gpu_entries_in_btree_order(scanner, tmp_path):
    """The enumeration in the reference BTree's order (meta/btree.go:64-66,
    bytes.Compare; MemTable.Iterator): String and ListMeta entries (sorted on
    the device during the open) equal Python's sorted() of the restated
    index's keys with the same positions; Hash / List / Set entries equal
    sorted() of their (key, sub) pairs."""
    from couloydb_amd import _abi
    from .test_reference_restart import write_dir
    files = split_files(typed_corpus(501, n_ops=1500, n_keys=20), 3, random.Random(6))
    write_dir(tmp_path, files)
    arrays, tts, _ = oracle_scan(files)
    ix = {}
    index_states(arrays, tts, out_index=ix)
    with scanner.open_db(str(tmp_path)) as db:
        for kind, dt in ((_abi.IT_STRING, mg.STRING), (_abi.IT_LISTMETA, mg.LISTMETA)):
            got = [(e[0], (e[2].fid, e[2].offset)) for e in db.entries(kind)]
            want = sorted((ik[1], (v[1], v[2])) for ik, v in ix.items() if ik[0] == dt)
            assert got == want, kind
        for kind, dt in ((_abi.IT_HASH, mg.HASH), (_abi.IT_LIST, mg.LIST), (_abi.IT_SET, mg.SET)):
            got = [(e[0], e[1], (e[2].fid, e[2].offset)) for e in db.entries(kind)]
            want = sorted((ik[1], ik[2], (v[1], v[2])) for ik, v in ix.items() if ik[0] == dt)
            assert got == want, kind


@pytest.mark.gpu
def test_gpu_string_order_long_keys(scanner, tmp_path):
    """The device key sort's refinement rounds: keys of 0-40 bytes sharing
    long prefixes (15-byte round-0 window, then 7-byte rounds), keys that are
    prefixes of others, zero bytes at the window edges, a txId-prefixed
    committed write and overwrites/deletes; the String enumeration equals
    sorted() of the live keys, every position the last writer's."""
    from couloydb_amd import _abi
    from .test_reference_restart import write_dir
    rng = random.Random(11)
    stems = [b"", b"user:profile:00", b"user:profile:00\x00", b"user:profile:0000000:",
             b"a" * 22, b"a" * 23, b"\x00" * 16, b"zz"]
    keys = set()
    while len(keys) < 3000:
        st = rng.choice(stems)
        tail = bytes(rng.choice(b"\x00\x01ab\xff") for _ in range(rng.randrange(0, 20)))
        k = (st + tail)[:rng.choice([40, 15, 16, 22, 23, 29, 30, 40])]
        if k:
            keys.add(k)
    keys = sorted(keys)
    rng.shuffle(keys)
    b = bytearray()
    live = {}
    for r, k in enumerate(keys + keys[:500]):
        if r % 7 == 3:
            b += mg.encode_record(mg.key_tx(k, 0), b"", mg.DELETED)
            live.pop(k, None)
        else:
            live[k] = len(b)
            b += mg.encode_record(mg.key_tx(k, 0), b"v%d" % r)
    tx = 9
    k = b"user:profile:00\x00\x00\x00\x00\x00\x00\x00\x00tx"
    off = len(b)
    b += mg.encode_record(mg.key_tx(k, tx), b"t")
    b += mg.encode_record(mg.key_tx(mg.TX_COMMIT_KEY, tx), b"", mg.TXN_COMMIT)
    live[k] = off
    write_dir(tmp_path, [bytes(b)])
    with scanner.open_db(str(tmp_path)) as db:
        got = [(e[0], e[2].offset) for e in db.entries(_abi.IT_STRING)]
        assert got == sorted(live.items())
        assert db.stats.order_rounds >= 2
