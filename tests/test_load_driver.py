"""The open path of NewCouloyDB through the device load driver (cly_db_open,
include/clyload.h) beyond the plain data directory:

  - a directory a merge left (merge.go:90-163 + loadMergeFiles): merged data
    files, the old files the reference leaves in place, newer data files,
    hint-index and merge-finished -> every lookup equals the restatement of
    loadIndexFromHintFile + loadIndex (merge.go:257-287, db.go:487-655);
  - the TTL sweep's db.Del tombstones (db.go:639-651, 186-215): the expired
    keys, the tombstone bytes appended to the active file, WriteOff after;
  - loadDataFile's directory listing (db.go:442-470): strconv.Atoi stems;
  - getLogRecordByPos statuses (db.go:680-704).

CPU tests cover the restatement helpers; the -m gpu tests call the library."""
import collections
import os
import random

import numpy as np
import pytest

from oracle import cly_oracle as co

from .gpu_util import INDEX_NOW, hint_entries, index_states, mg, typed_corpus
from .test_merge import flat, oracle_scan, split_files
from .test_reference_restart import TTL_EXP, ttl_files, write_dir


def merged_dir(seed, tmp_path, new_ops=600):
    """A data directory as NewCouloyDB finds it after db.merge + loadMergeFiles:
    old files 0..M-1 of a typed corpus (M = nowMergeFile: the merge rotated the
    active file to fid M); the merge rewrote the live records (merge.go's
    lookup: the restated index's state 1) into files 0..k-1 and wrote
    hint-index and merge-finished {0x07: "M"}; loadMergeFiles renamed them into
    the directory (files 0..k-1 replaced; k..M-1 stay, the reference removes
    none); after the merge, more writes went to files M, M+1, ...
    Returns (dir files {fid: bytes}, hint bytes)."""
    rng = random.Random(seed)
    old = split_files(typed_corpus(900 + seed, n_ops=1500, n_keys=25), 4, rng)
    arrays, tts, _ = oracle_scan(old)
    st = index_states(arrays, tts)
    tuples, tf = flat(tts)
    rc, merged, hint, r = co.merge(arrays, tuples, tf, (st == 1).astype(np.uint8), 8192)
    assert rc == 0 and len(merged) >= 1
    M = len(old)
    files = {i: bytes(b) for i, b in enumerate(old)}
    for k, b in enumerate(merged):
        files[k] = bytes(b)
    newer = split_files(typed_corpus(1900 + seed, n_ops=new_ops, n_keys=25), 2, rng)
    for j, b in enumerate(newer):
        files[M + j] = bytes(b)
    with open(os.path.join(tmp_path, "hint-index"), "wb") as f:
        f.write(hint)
    with open(os.path.join(tmp_path, "merge-finished"), "wb") as f:
        f.write(mg.encode_record(mg.MERGE_FIN_KEY, str(M).encode()))
    for fid, b in files.items():
        with open(os.path.join(tmp_path, "%09d.cly" % fid), "wb") as f:
            f.write(b)
    return files, hint


def restated_index(files, hint, now_ns=INDEX_NOW):
    fids = sorted(files)
    arrays = [np.frombuffer(files[f], np.uint8) for f in fids]
    tts = []
    for f, a in zip(fids, arrays):
        t, s, _ = co.scan_file(a, f)
        tts.append(t)
    ix = {}
    index_states(arrays, tts, now_ns=now_ns, out_index=ix, preload=hint_entries(hint))
    return ix


def test_hint_entries_decode():
    """The restated hint reader over a merge's hint file: one entry per live
    record, each naming the merged record of that realKey."""
    rng = random.Random(1)
    old = split_files(typed_corpus(77, n_ops=300, n_keys=10), 2, rng)
    arrays, tts, _ = oracle_scan(old)
    st = index_states(arrays, tts)
    tuples, tf = flat(tts)
    rc, merged, hint, r = co.merge(arrays, tuples, tf, (st == 1).astype(np.uint8), 4096)
    ents = hint_entries(hint)
    assert len(ents) == r.n_live == int((st == 1).sum())
    for key, fid, off in ents:
        t = mg.read_log_record(merged[fid], off)[1]
        assert bytes(merged[fid][off + t["header_size"] + 1:off + t["header_size"] + t["key_size"]]) == key


def test_restated_preload_order():
    """A data-file Put or Del of a String key overrides its hint entry; a hint
    entry the data files never touch stays (under its stored key)."""
    hint = mg.encode_record(b"a", b"\x00\x10") + mg.encode_record(b"b", b"\x02\x20") + \
        mg.encode_record(b"c", b"\x02\x40")
    F = mg.encode_record(mg.key_tx(b"a", 0), b"v1") + mg.encode_record(mg.key_tx(b"b", 0), b"", mg.DELETED)
    files = {0: F}
    ix = restated_index(files, hint)
    assert ix[(mg.STRING, b"a")][1:3] == (0, 0)
    assert (mg.STRING, b"b") not in ix
    assert ix[(mg.STRING, b"c")] == (b"c", 1, 32, 0)


@pytest.fixture(scope="module")
def scanner():
    from couloydb_amd import Scanner
    s = Scanner(0)
    yield s
    s.close()


def check_lookups(db, ix):
    from .index_keys import decode_byte_slices
    counts = collections.Counter(k[0] for k in ix)
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
            k, m = decode_byte_slices(key if tx == 0 else key[n:])
            p = db.spos(k, m)
        assert (p.fid, p.offset) == (fid, off), (ik, fid, off)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
def test_gpu_open_after_merge(scanner, tmp_path, seed):
    """cly_db_open over a merged directory: hint entries first, then every data
    file (merged, old, newer) in fid order; every lookup and count equals the
    restatement; a String lookup of a composite record's realKey finds its
    hint entry (merge.go:283 puts every hint key into the String index)."""
    from couloydb_amd import _abi
    files, hint = merged_dir(seed, tmp_path)
    ix = restated_index(files, hint)
    scanner.set_clock(INDEX_NOW)
    with scanner.open_db(str(tmp_path)) as db:
        assert db.stats.hint_records == len(hint_entries(hint)) > 0
        assert db.stats.n_files == len(files)
        check_lookups(db, ix)
        ents = {e[0]: e[2] for e in db.entries(_abi.IT_STRING)}
        assert len(ents) == sum(1 for k in ix if k[0] == mg.STRING)
        for (dt, *rest), (key, fid, off, tx) in ix.items():
            if dt == mg.STRING:
                assert ents[rest[0]] == (fid, off)


@pytest.mark.gpu
def test_gpu_open_merge_finished_checks(scanner, tmp_path):
    """merge-finished must hold a readable record with an integer value
    (getNonMergeFileId); without data files it is not read at all."""
    from couloydb_amd import ScanError, _abi
    write_dir(tmp_path, [mg.encode_record(mg.key_tx(b"k", 0), b"v")])
    mf = os.path.join(tmp_path, "merge-finished")
    for content, code in [(b"", _abi.ERR_MERGE_FIN), (mg.encode_record(mg.MERGE_FIN_KEY, b"x1"), _abi.ERR_MERGE_FIN),
                          (mg.encode_record(mg.MERGE_FIN_KEY, b"-3"), None),
                          (bytearray(mg.encode_record(mg.MERGE_FIN_KEY, b"7")), _abi.ERR_CRC)]:
        if isinstance(content, bytearray):
            content[-1] ^= 1
        with open(mf, "wb") as f:
            f.write(bytes(content))
        if code is None:
            with scanner.open_db(str(tmp_path)) as db:
                assert db.get(b"k") == b"v"
        else:
            with pytest.raises(ScanError) as e:
                scanner.open_db(str(tmp_path))
            assert e.value.code == code
    os.remove(os.path.join(tmp_path, "000000000.cly"))
    with open(mf, "wb") as f:
        f.write(b"")
    with scanner.open_db(str(tmp_path)) as db:                   # no data files: loadIndex returns first
        assert db.stats.n_files == 0


@pytest.mark.gpu
def test_gpu_ttl_sweep_tombstones(scanner, tmp_path):
    """TestDB_TTL_Restart reloaded after the expiration: the key is swept,
    its tombstone {0x00 || key, LogRecordDeleted} goes to the active file
    (db.Del -> appendLogRecord) and WriteOff advances by its size; with
    apply_sweep the bytes land on disk, and the next open sees the tombstone
    (nothing left to sweep, the key still absent)."""
    from couloydb_amd import _abi
    files, v = ttl_files()
    write_dir(tmp_path, files)
    key = mg.test_key(0)
    tomb = mg.encode_record(mg.key_tx(key, 0), b"", mg.DELETED)
    scanner.set_clock(TTL_EXP)
    with scanner.open_db(str(tmp_path)) as db:
        st = db.stats
        assert st.n_expired == 1 and st.write_off_loaded == len(files[0])
        assert st.write_off == len(files[0]) + len(tomb) and st.active_fid == 0
        assert [e[0] for e in db.entries(_abi.IT_EXPIRED)] == [key]
        with pytest.raises(KeyError):
            db.get(key)
    with open(os.path.join(tmp_path, "000000000.cly"), "rb") as f:
        assert f.read() == files[0]                               # nothing written without apply_sweep
    with scanner.open_db(str(tmp_path), apply_sweep=True) as db:
        assert db.stats.write_off == len(files[0]) + len(tomb)
    with open(os.path.join(tmp_path, "000000000.cly"), "rb") as f:
        assert f.read() == files[0] + tomb
    with scanner.open_db(str(tmp_path)) as db:
        assert db.stats.n_expired == 0 and db.stats.write_off == len(files[0]) + len(tomb)
        with pytest.raises(KeyError):
            db.get(key)
    scanner.set_clock(0)


@pytest.mark.gpu
def test_gpu_ttl_sweep_rotation(scanner, tmp_path):
    """Sweep tombstones that do not fit the active file open fid+1
    (WriteOff + size > DataFileSize, db.go:376-385)."""
    recs = [mg.encode_record(mg.key_tx(mg.test_key(i), 0), b"x" * 40, mg.NORMAL, mg.STRING, 5) for i in range(6)]
    F = b"".join(recs)
    write_dir(tmp_path, [F])
    tomb = len(mg.encode_record(mg.key_tx(mg.test_key(0), 0), b"", mg.DELETED))
    dfs = len(F) + 2 * tomb + 1
    scanner.set_clock(10)
    with scanner.open_db(str(tmp_path), data_file_size=dfs, apply_sweep=True) as db:
        st = db.stats
        assert st.n_expired == 6 and st.sweep_files == 1
        assert st.active_fid == 1 and st.write_off == 4 * tomb
    assert os.path.getsize(os.path.join(tmp_path, "000000000.cly")) == len(F) + 2 * tomb
    assert os.path.getsize(os.path.join(tmp_path, "000000001.cly")) == 4 * tomb
    scanner.set_clock(0)


@pytest.mark.gpu
def test_gpu_dir_listing_atoi(scanner, tmp_path):
    """loadDataFile's listing: stems by strconv.Atoi ("+1" and "0001" name fid
    1, read from 000000001.cly, once per listing: sort.Ints keeps the four
    fid-1 entries, db.go:449-464); a stem Atoi rejects fails the open."""
    from couloydb_amd import ScanError, _abi
    a = mg.encode_record(mg.key_tx(b"a", 0), b"1")
    b = mg.encode_record(mg.key_tx(b"a", 0), b"2")
    with open(os.path.join(tmp_path, "000000000.cly"), "wb") as f:
        f.write(a)
    with open(os.path.join(tmp_path, "000000001.cly"), "wb") as f:
        f.write(b)
    for alias in ("+1.cly", "0001.cly", "1.x.cly"):
        with open(os.path.join(tmp_path, alias), "wb") as f:
            f.write(b"garbage")                                   # never read: fid 1 opens 000000001.cly
    with scanner.open_db(str(tmp_path)) as db:
        assert db.get(b"a") == b"2" and db.stats.n_files == 5 and db.stats.active_fid == 1
    with open(os.path.join(tmp_path, "x7.cly"), "wb") as f:
        f.write(b"")
    with pytest.raises(ScanError) as e:
        scanner.open_db(str(tmp_path))
    assert e.value.code == _abi.ERR_DIR


@pytest.mark.gpu
def test_gpu_value_statuses(scanner, tmp_path):
    """getLogRecordByPos: a Deleted record and an unknown fid are
    ErrKeyNotFound; io.EOF near the file's end; a negative offset errors."""
    from couloydb_amd import LogPos, ScanError, _abi
    F = mg.encode_record(mg.key_tx(b"a", 0), b"va") + mg.encode_record(mg.key_tx(b"b", 0), b"", mg.DELETED)
    write_dir(tmp_path, [F])
    r0 = len(mg.encode_record(mg.key_tx(b"a", 0), b"va"))
    with scanner.open_db(str(tmp_path)) as db:
        assert db.value(LogPos(0, 0)) == b"va"
        with pytest.raises(KeyError):
            db.value(LogPos(0, r0))                               # LogRecordDeleted
        with pytest.raises(KeyError):
            db.value(LogPos(7, 0))                                # no such data file
        for off in (len(F), len(F) - 3):
            with pytest.raises(ScanError) as e:
                db.value(LogPos(0, off))
            assert e.value.code == _abi.DB_EOF
        with pytest.raises(ScanError) as e:
            db.value(LogPos(0, -1))
        assert e.value.code == _abi.ERR_OFFSET


@pytest.mark.gpu
@pytest.mark.parametrize("nctx", [2, 3, 5])
def test_gpu_open_multi_matches_single(scanner, tmp_path, nctx):
    """cly_db_open_multi: the merged directory's files sharded by fid range over
    nctx contexts (all on device 0 here; one per GPU on a node) give the same
    index, counts, WriteOff and entries as the one-context open."""
    from couloydb_amd import Scanner, _abi, open_db_multi
    files, hint = merged_dir(7, tmp_path, new_ops=900)
    ix = restated_index(files, hint)
    scanner.set_clock(INDEX_NOW)
    extra = [Scanner(0) for _ in range(nctx - 1)]
    try:
        for sc in extra:
            sc.set_clock(INDEX_NOW)
        with scanner.open_db(str(tmp_path)) as one, open_db_multi([scanner] + extra, str(tmp_path)) as db:
            assert 1 < db.stats.n_shards <= nctx and one.stats.n_shards == 1
            for f in ("records", "hint_records", "n_files", "write_off", "active_fid", "str_keys", "hash_fields",
                      "list_items", "set_members", "n_expired"):
                assert getattr(db.stats, f) == getattr(one.stats, f), f
            check_lookups(db, ix)
            for kind in range(6):
                assert sorted(db.entries(kind)) == sorted(one.entries(kind)), kind
    finally:
        for sc in extra:
            sc.close()


@pytest.mark.gpu
def test_gpu_open_multi_tx_across_shards(scanner, tmp_path):
    """A transaction whose records end file 1 and whose commit opens file 2 (the
    two shards' boundary) applies; a rolled-back one split the same way does
    not; a tx begun in shard 0 and never finished stays out."""
    from couloydb_amd import Scanner, open_db_multi
    pad = lambda i, n: b"".join(mg.encode_record(mg.key_tx(b"p%d-%d" % (i, j), 0), b"x" * 200) for j in range(n))
    f0 = pad(0, 40) + mg.encode_record(mg.key_tx(b"u", 91), b"never")
    f1 = pad(1, 38) + mg.encode_record(mg.key_tx(b"a", 77), b"va") + mg.encode_record(mg.key_tx(b"b", 78), b"vb") + \
        mg.encode_record(mg.key_tx(b"c", 77), b"vc")
    f2 = mg.encode_record(mg.key_tx(mg.TX_COMMIT_KEY, 77), b"", mg.TXN_COMMIT) + \
        mg.encode_record(mg.key_tx(mg.TX_ROLLBACK_KEY, 78), b"", mg.TXN_ROLLBACK) + pad(2, 40)
    f3 = pad(3, 41)
    write_dir(tmp_path, [f0, f1, f2, f3])
    other = Scanner(0)
    try:
        with open_db_multi([scanner, other], str(tmp_path)) as db:
            assert db.stats.n_shards == 2
            assert db.get(b"a") == b"va" and db.get(b"c") == b"vc"
            for k in (b"b", b"u"):
                with pytest.raises(KeyError):
                    db.get(k)
            assert db.stats.str_keys == 40 + 38 + 40 + 41 + 2
            assert db.stats.write_off == len(f3) and db.stats.active_fid == 3
    finally:
        other.close()


@pytest.mark.gpu
def test_gpu_ttl_sweep_empty_key(scanner, tmp_path):
    """An expired String put whose realKey is empty: the sweep's db.Del("")
    returns ErrKeyIsEmpty (db.go:186-188) and loadIndex returns it
    (db.go:646-649), so NewCouloyDB fails.  A live empty key does not."""
    from couloydb_amd import ScanError, _abi
    F = mg.encode_record(mg.key_tx(b"a", 0), b"1", mg.NORMAL, mg.STRING, 5) + \
        mg.encode_record(mg.key_tx(b"", 0), b"2", mg.NORMAL, mg.STRING, 5)
    write_dir(tmp_path, [F])
    scanner.set_clock(10)
    try:
        with pytest.raises(ScanError) as e:
            scanner.open_db(str(tmp_path))
        assert e.value.code == _abi.ERR_KEY_EMPTY
        scanner.set_clock(3)                                      # not expired yet: no Del
        with scanner.open_db(str(tmp_path)) as db:
            assert db.get(b"") == b"2" and db.stats.n_expired == 0
    finally:
        scanner.set_clock(0)


@pytest.mark.gpu
def test_gpu_open_error_order(scanner, tmp_path):
    """NewCouloyDB's error order (db.go:472-485, merge.go:257-287, db.go:492-499):
    the hint file's first failure (a record that does not read, or a value that
    does not decode, whichever comes first in its loop), then merge-finished,
    then the data files."""
    from couloydb_amd import ScanError, _abi
    good = [mg.encode_record(b"k%d" % i, mg.put_varint(0) + mg.put_varint(10 * i)) for i in range(5)]
    panic = mg.encode_record(b"bad", b"\xff" * 10 + b"\x02")       # DecodeLogRecordPos: varint overflow
    crc_bad = bytearray(mg.encode_record(b"k9", mg.put_varint(0) + mg.put_varint(9)))
    crc_bad[-1] ^= 1
    data_bad = bytearray(mg.encode_record(mg.key_tx(b"x", 0), b"v"))
    data_bad[-1] ^= 1
    write_dir(tmp_path, [bytes(data_bad)])
    mf = os.path.join(tmp_path, "merge-finished")
    hf = os.path.join(tmp_path, "hint-index")
    with open(mf, "wb") as f:
        f.write(b"")                                               # does not read: ERR_MERGE_FIN
    cases = [
        (good[0] + bytes(crc_bad) + good[1], _abi.ERR_CRC),        # hint CRC before merge-finished
        (good[0] + panic + bytes(crc_bad), _abi.ERR_VARINT),       # hint decode panic before its later CRC error
        (good[0] + bytes(crc_bad) + panic, _abi.ERR_CRC),          # ... and after it
        (b"".join(good), _abi.ERR_MERGE_FIN),                      # a good hint: merge-finished next
    ]
    for hint, code in cases:
        with open(hf, "wb") as f:
            f.write(hint)
        with pytest.raises(ScanError) as e:
            scanner.open_db(str(tmp_path))
        assert e.value.code == code, (code, e.value.code)
    with open(mf, "wb") as f:
        f.write(mg.encode_record(mg.MERGE_FIN_KEY, b"0"))
    with pytest.raises(ScanError) as e:                            # then the data file's CRC error
        scanner.open_db(str(tmp_path))
    assert e.value.code == _abi.ERR_CRC


@pytest.mark.gpu
def test_gpu_dir_listing_uint32_fids(scanner, tmp_path):
    """Stems Atoi accepts but uint32() wraps: "-1.cly" is fid 4294967295 (read
    from 4294967295.cly; sort.Ints puts it first, and the spelled-out name
    last, so that file is read twice); lookups into it and into fid 3 both
    resolve."""
    a = mg.encode_record(mg.key_tx(b"a", 0), b"from-max")
    b = mg.encode_record(mg.key_tx(b"b", 0), b"from-3")
    with open(os.path.join(tmp_path, "4294967295.cly"), "wb") as f:
        f.write(a)
    with open(os.path.join(tmp_path, "-1.cly"), "wb") as f:
        f.write(b"never read")
    with open(os.path.join(tmp_path, "000000003.cly"), "wb") as f:
        f.write(b)
    with scanner.open_db(str(tmp_path)) as db:
        assert db.stats.n_files == 3
        assert db.get(b"a") == b"from-max" and db.get(b"b") == b"from-3"
        assert db.stats.active_fid == 0xFFFFFFFF                   # the last in sort.Ints order


@pytest.mark.gpu
def test_gpu_dir_listing_tx_across_repeated_file(scanner, tmp_path):
    """A transaction whose data records sit in a file read at two places of
    the listing ("-1.cly" first, "4294967295.cly" last) and whose commit marker
    sits in a file between them: the first reading buffers the records, the
    marker applies them (loadIndex, db.go:603-627), the second reading buffers
    them again without a marker.  The key is therefore found; a single reading
    at the last place would leave it uncommitted."""
    tx = 77
    data = mg.encode_record(mg.key_tx(b"k", tx), b"in-tx")
    fin = mg.encode_record(mg.key_tx(mg.TX_COMMIT_KEY, tx), b"", mg.TXN_COMMIT)
    with open(os.path.join(tmp_path, "4294967295.cly"), "wb") as f:
        f.write(data)
    with open(os.path.join(tmp_path, "-1.cly"), "wb") as f:
        f.write(b"never read")
    with open(os.path.join(tmp_path, "000000003.cly"), "wb") as f:
        f.write(fin)
    files = [np.frombuffer(b, np.uint8) for b in (data, fin, data)]
    tpf = [co.scan_file(F, fid)[0] for F, fid in zip(files, [0xFFFFFFFF, 3, 0xFFFFFFFF])]
    ix = {}
    index_states(files, tpf, out_index=ix)
    assert (mg.STRING, b"k") in ix                                # the restatement finds the key too
    with scanner.open_db(str(tmp_path)) as db:
        assert db.stats.n_files == 3
        assert db.get(b"k") == b"in-tx"


@pytest.mark.gpu
def test_gpu_data_file_size_clamp(scanner, tmp_path):
    """checkOptions raises DataFileSize below 64 to 64 (db.go:436-438): the
    sweep's rotation with DataFileSize 1 equals the one with 64."""
    recs = [mg.encode_record(mg.key_tx(mg.test_key(i), 0), b"x" * 3, mg.NORMAL, mg.STRING, 5) for i in range(9)]
    write_dir(tmp_path, [b"".join(recs)])
    scanner.set_clock(10)
    try:
        with scanner.open_db(str(tmp_path), data_file_size=1) as db1, \
                scanner.open_db(str(tmp_path), data_file_size=64) as db64:
            assert (db1.stats.active_fid, db1.stats.write_off, db1.stats.sweep_files) == \
                (db64.stats.active_fid, db64.stats.write_off, db64.stats.sweep_files)
            assert db64.stats.sweep_files >= 1
    finally:
        scanner.set_clock(0)


@pytest.mark.gpu
def test_gpu_open_multi_rejects_repeated_context(scanner, tmp_path):
    """A context listed twice would run two scans on one context at once."""
    from couloydb_amd import ScanError, _abi, open_db_multi
    write_dir(tmp_path, [mg.encode_record(mg.key_tx(b"k", 0), b"v")])
    with pytest.raises(ScanError) as e:
        open_db_multi([scanner, scanner], str(tmp_path))
    assert e.value.code == _abi.ERR_ARG


@pytest.mark.gpu
def test_gpu_open_tuple_alloc_exact(scanner, tmp_path):
    """The open's device tuple buffer is sized by the exact record count the
    link finds (records + 16 per shard), not by a bytes/9 bound: checked on a
    C3-shaped corpus (bench.make_workload("c3") at 192 MiB: Zipf value sizes
    64 B-64 KiB), where bytes/9 would be ~40x the records; every String key
    is found at its record."""
    import torch
    import bench
    wl = bench.make_workload("c3", torch, size=192 << 20)
    for i, (_, ln, fid) in enumerate(wl.dev_files):
        wl.file_bytes(i).tofile(str(tmp_path / ("%09d.cly" % fid)))
    with scanner.open_db(str(tmp_path)) as db:
        st = db.stats
        assert st.records == wl.expect_records
        assert st.tuple_slots == st.records + 16 * st.n_shards
        assert st.tuple_slots <= 1.1 * st.records
        assert st.str_keys == st.records
    del wl
    torch.cuda.empty_cache()
