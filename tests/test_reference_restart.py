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
    assert list(index_states([a], [tt], now_ns=TTL_EXP)) == [0]          # expired at reload: db.Del
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
