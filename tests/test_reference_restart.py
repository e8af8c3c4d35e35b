"""The reference's own restart tests as the parity pin of scan + index
(VERDICT r1 item 3): each test's write sequence is restated (the writer:
tests/gpu_util.py py_append = appendLogRecord with DataFileSize rotation,
db.go:368-413; txn markers as txn.go:250-283 writes them), the files go to a
directory as `%09d.cly`, and the device index load (cly_db_open:
loadDataFile + loadIndex, db.go:442-655) must give exactly the post-reload
state the test asserts:

  TestDB_Reboot        db_test.go:214-261  10 000 keys, Get == key || 1024 zero bytes, 8 MiB files
  TestDB_TTL_Restart   ttl_test.go:55-88   PutWithExpiration(2 s); after 2 s the reloaded Get fails
  TestTxn_Hash_Restart txnHash_test.go:179-223  HGet(0,0), HGet(1,1) found; HGet(1,2) ErrKeyNotFound
  TestTxn_List_Restart txnList_test.go:104-161  LPush/RPush 0..6; after reload LPop 3, LPop 2, RPop 6
  TestDB_TTL_Reset     ttl_test.go:112-134 (as a reload): PutWithExpiration then Put; the second
                       put's zero expiration resets the TTL (db.go:133-141, loadIndex's
                       expirations map keeps the last put's, db.go:517) -> still there after expiry

CPU: the same files through the oracle scan and the literal loadIndex
restatement (index_states) give the asserted visible String keys.
GPU (-m gpu): cly_db_open on the files."""
import os
import random

import numpy as np
import pytest

from oracle import cly_oracle as co

from .gpu_util import index_states, mg, py_append

FILL = bytes(1024)
REBOOT_DFS = 8 * 1024 * 1024


def write_dir(d, files):
    for fid, b in enumerate(files):
        with open(os.path.join(d, "%09d.cly" % fid), "wb") as f:
            f.write(b)


def reboot_files(order_seed=7):
    """TestDB_Reboot: 10 000 goroutines Put(GetTestKey(id), key || 1024 zero
    bytes), DataFileSize 8 MiB, in a scheduling order (any order gives the
    same final state: the keys are distinct)."""
    ids = list(range(10000))
    random.Random(order_seed).shuffle(ids)
    recs = [(mg.test_key(i), mg.test_key(i) + FILL, mg.NORMAL, mg.STRING, 0) for i in ids]
    files, _ = py_append(recs, 0, False, b"", 0, REBOOT_DFS)
    return files


TTL_EXP = 1_800_000_002_000_000_000           # Put at 1_800_000_000 s + 2 s (UnixNano)


def ttl_files():
    """TestDB_TTL_Restart: PutWithExpiration(GetTestKey(0), RandomBytes(24), 2 s)."""
    v = bytes(random.Random(3).choice(b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789") for _ in range(24))
    files, _ = py_append([(mg.test_key(0), v, mg.NORMAL, mg.STRING, TTL_EXP)], 0, False, b"", 0, 256 << 20)
    return files, v


def hash_files():
    """TestTxn_Hash_Restart's transaction: Begin, HSet(0,0,0), HSet(1,1,1),
    HSet(1,2,2), HDel(1,2), Commit (the golden fixture txn_hash)."""
    with open(os.path.join(os.path.dirname(__file__), "golden", "txn_hash.cly"), "rb") as f:
        return [f.read()]


def list_files():
    """TestTxn_List_Restart's transaction, restated through txn.push
    (txnList.go:96-160: per value a List record keyed encodeListKey(cur, prev,
    next, key), then the ListMeta record encodeListMeta(head, tail); getListMeta
    reads the txn's pending ListMeta, else head 1 / tail 0) between the Begin
    and Commit markers of txn.go:258-283."""
    from .index_keys import encode_list_key, encode_list_meta
    tx = 1_700_000_000_000
    k = mg.test_key(0)
    head, tail = 1, 0
    out = [(mg.TX_BEGIN_KEY, b"", mg.TXN_BEGIN, mg.STRING, 0)]
    for vals, left in (([0], True), ([1], True), ([2, 3], True), ([4], False), ([5, 6], False)):
        for v in vals:
            if left:
                cur = head - 1
                prev, nxt = cur - 1, head
                head = cur
            else:
                cur = tail + 1
                prev, nxt = tail, cur + 1
                tail = cur
            out.append((encode_list_key(cur, prev, nxt, k), mg.test_key(v), mg.NORMAL, mg.LIST, 0))
        out.append((k, encode_list_meta(head, tail), mg.NORMAL, mg.LISTMETA, 0))
    out.append((mg.TX_COMMIT_KEY, b"", mg.TXN_COMMIT, mg.STRING, 0))
    b = b"".join(mg.encode_record(mg.key_tx(key, tx), v, typ, dt, e) for key, v, typ, dt, e in out)
    return [b]


def gob_int(buf):
    """The integer value of a writer's gob-encoded seq (GobDecode of an exact
    integer Float)."""
    if buf[1] & 0x06 == 0:
        return 0
    e = int.from_bytes(buf[6:10], "big")
    v = int.from_bytes(buf[10:18], "big") >> (64 - e)
    return -v if buf[1] & 1 else v


def decode_list_meta(v):
    """decodeListMeta (txnList.go:284-294) -> (head, tail)."""
    hl, i = mg.varint(v)
    _, j = mg.varint(v[i:])
    return gob_int(v[i + j:i + j + hl]), gob_int(v[i + j + hl:])


def ttl_reset_files():
    """TestDB_TTL_Reset's writes: PutWithExpiration(key0, v1, 100 ms), Put(key0, v2)."""
    rng = random.Random(4)
    v1, v2 = rng.randbytes(24), rng.randbytes(24)
    files, _ = py_append([(mg.test_key(0), v1, mg.NORMAL, mg.STRING, TTL_EXP),
                          (mg.test_key(0), v2, mg.NORMAL, mg.STRING, 0)], 0, False, b"", 0, 256 << 20)
    return files, v2


def test_ttl_reset_restatement():
    files, _ = ttl_reset_files()
    a = np.frombuffer(files[0], np.uint8).copy()
    tt, _, _ = co.scan_file(a, 0)
    assert list(index_states([a], [tt], now_ns=TTL_EXP + 10**9)) == [0, 1]


def test_reboot_restatement():
    files = reboot_files()
    assert len(files) == 2                                   # rotation at 8 MiB (db.go:376-385)
    arrays = [np.frombuffer(b, np.uint8).copy() for b in files]
    tts = [co.scan_file(a, i)[0] for i, a in enumerate(arrays)]
    st = index_states(arrays, tts)
    assert int((st == 1).sum()) == 10000
    for a, tt in zip(arrays, tts):
        for t in tt[:50]:
            o, h, ks, vs = int(t["offset"]), int(t["header_size"]), int(t["key_size"]), int(t["value_size"])
            assert bytes(a[o + h + ks:o + h + ks + vs]) == bytes(a[o + h + 1:o + h + ks]) + FILL


def test_ttl_restatement():
    files, _ = ttl_files()
    a = np.frombuffer(files[0], np.uint8).copy()
    tt, _, _ = co.scan_file(a, 0)
    assert list(index_states([a], [tt], now_ns=TTL_EXP)) == [4]          # expired at reload: db.Del (CLY_IX_EXPIRED)
    assert list(index_states([a], [tt], now_ns=TTL_EXP - 1)) == [1]      # still pending: ttl.add


@pytest.fixture(scope="module")
def scanner():
    from couloydb_amd import Scanner
    s = Scanner(0)
    yield s
    s.close()


@pytest.mark.gpu
def test_gpu_reboot(scanner, tmp_path):
    files = reboot_files()
    write_dir(tmp_path, files)
    scanner.set_clock(0)
    with scanner.open_db(str(tmp_path)) as db:
        assert db.stats.n_files == 2 and db.stats.str_keys == 10000 and db.stats.records == 10000
        assert db.stats.active_fid == 1 and db.stats.write_off == len(files[1])
        for i in range(10000):
            k = mg.test_key(i)
            assert db.get(k) == k + FILL
        with pytest.raises(KeyError):
            db.get(b"not exist!")


@pytest.mark.gpu
def test_gpu_ttl_restart(scanner, tmp_path):
    files, v = ttl_files()
    write_dir(tmp_path, files)
    scanner.set_clock(TTL_EXP)                   # time.Sleep(2 s) then NewCouloyDB
    with scanner.open_db(str(tmp_path)) as db:
        with pytest.raises(KeyError):
            db.get(mg.test_key(0))
    scanner.set_clock(TTL_EXP - 1_000_000_000)  # reloaded before the expiration: still there
    with scanner.open_db(str(tmp_path)) as db:
        assert db.get(mg.test_key(0)) == v
    scanner.set_clock(0)


@pytest.mark.gpu
def test_gpu_txn_hash_restart(scanner, tmp_path):
    write_dir(tmp_path, hash_files())
    with scanner.open_db(str(tmp_path)) as db:
        assert db.hget(mg.test_key(0), mg.test_key(0)) == mg.test_key(0)
        assert db.hget(mg.test_key(1), mg.test_key(1)) == mg.test_key(1)
        with pytest.raises(KeyError):
            db.hget(mg.test_key(1), mg.test_key(2))
        assert db.stats.hash_fields == 2 and db.stats.str_keys == 0


@pytest.mark.gpu
def test_gpu_load_rejects_corruption(scanner, tmp_path):
    """NewCouloyDB fails with ErrInvalidCRC when a record is corrupt."""
    from couloydb_amd import ErrInvalidCRC
    files = reboot_files()
    b = bytearray(files[0])
    b[5000] ^= 0x40
    write_dir(tmp_path, [bytes(b), files[1]])
    with pytest.raises(ErrInvalidCRC):
        scanner.open_db(str(tmp_path))


def test_list_restatement():
    from .index_keys import decode_list_key
    files = list_files()
    a = np.frombuffer(files[0], np.uint8).copy()
    tt, st, _ = co.scan_file(a, 0)
    assert st == 0 and len(tt) == 7 + 5 + 2
    states = index_states([a], [tt])
    assert int((states == 1).sum()) == 7 + 1                 # 7 list items + the last ListMeta
    # the list order head..tail by following next from the ListMeta head
    meta = [t for t in tt if t["data_type"] == mg.LISTMETA][-1]
    o, h, ks, vs = (int(meta[x]) for x in ("offset", "header_size", "key_size", "value_size"))
    head, tail = decode_list_meta(files[0][o + h + ks:o + h + ks + vs])
    assert (head, tail) == (-3, 3)
    by_seq = {}
    for t in tt:
        if t["data_type"] == mg.LIST:
            o, h, ks, vs = (int(t[x]) for x in ("offset", "header_size", "key_size", "value_size"))
            key = files[0][o + h:o + h + ks]
            _, n = mg.varint(key)
            _, seq = decode_list_key(key[n:])
            by_seq[gob_int(seq)] = files[0][o + h + ks:o + h + ks + vs]
    assert [by_seq[i] for i in range(head, tail + 1)] == [mg.test_key(x) for x in (3, 2, 1, 0, 4, 5, 6)]


@pytest.mark.gpu
def test_gpu_txn_list_restart(scanner, tmp_path):
    """After reload: LPop -> key 3, LPop -> key 2, RPop -> key 6 (txn.pop,
    txnList.go:162-232: head/tail from the ListMeta index, the item from the
    List index by the seq's gob encoding, the next head from the item's key)."""
    from .index_keys import decode_list_key, gob_encode_int
    files = list_files()
    write_dir(tmp_path, files)
    scanner.set_clock(0)
    with scanner.open_db(str(tmp_path)) as db:
        assert db.stats.list_items == 7 and db.stats.listmeta_keys == 1
        k = mg.test_key(0)
        head, tail = decode_list_meta(db.value(db.listmeta_pos(k)))

        tt, _, _ = co.scan_file(np.frombuffer(files[0], np.uint8).copy(), 0)
        at = {int(t["offset"]): t for t in tt}

        def pop(seq):
            pos = db.lpos(k, gob_encode_int(seq))
            t = at[pos.offset]
            o, h, ks = pos.offset, int(t["header_size"]), int(t["key_size"])
            key = files[pos.fid][o + h:o + h + ks]
            _, n = mg.varint(key)
            _, s = decode_list_key(key[n:])
            # the prev/next seqs follow seq in the key (encodeListKey)
            ln, idx = [], 0
            for _ in range(3):
                v, i = mg.varint(key[n + idx:])
                ln.append(v)
                idx += i
            rest = key[n + idx + ln[0]:]
            return db.value(pos), (gob_int(rest[:ln[1]]), gob_int(rest[ln[1]:ln[1] + ln[2]]))

        v, (prev, nxt) = pop(head)
        assert v == mg.test_key(3)
        head = nxt
        v, (prev, nxt) = pop(head)
        assert v == mg.test_key(2)
        v, (prev, nxt) = pop(tail)
        assert v == mg.test_key(6)
        with pytest.raises(KeyError):
            db.lpos(k, gob_encode_int(tail + 1))


@pytest.mark.gpu
def test_gpu_ttl_reset_restart(scanner, tmp_path):
    files, v2 = ttl_reset_files()
    write_dir(tmp_path, files)
    scanner.set_clock(TTL_EXP + 10**9)           # reloaded after the first put's expiration
    with scanner.open_db(str(tmp_path)) as db:
        assert db.get(mg.test_key(0)) == v2
    scanner.set_clock(0)
