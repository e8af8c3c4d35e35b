"""Multi-GPU scan entry (couloydb_amd.multi.MultiScanner): the
file set split by fid ranges over several contexts must give exactly the
single-context scan, tuples in fid order; a transaction whose records and
commit marker fall into different shards still resolves in the index
restatement over the concatenated tuples (db.go:604-627).  Several contexts
on one device stand in for several GPUs (the path is the same)."""
import random

import numpy as np
import pytest

from oracle import cly_oracle as co

from .gpu_util import index_states, mg, mixed_corpus, py_append


def tx_across_files():
    """A transaction's data records at the end of file 0 and its commit marker
    in file 1 (rotation at DataFileSize), then more non-tx records."""
    tx = 1_700_000_000_000_000_123
    recs = [(mg.test_key(i), bytes(200), mg.NORMAL, mg.STRING, 0) for i in range(40)]
    txr = [(mg.test_key(1000 + i), b"t" * 100, mg.NORMAL, mg.STRING, 0) for i in range(10)]
    s0 = sum(len(mg.encode_record(mg.key_tx(k, 0), v, t, d, e)) for k, v, t, d, e in recs)
    s1 = sum(len(mg.encode_record(mg.key_tx(k, tx), v, t, d, e)) for k, v, t, d, e in txr)
    dfs = s0 + s1                  # the tx records fill file 0 exactly: the commit marker opens file 1
    f0, _ = py_append(recs, 0, False, b"", 0, dfs)
    f1, _ = py_append(txr, tx, True, f0[-1], len(f0[-1]), dfs)
    files = f0[:-1] + f1
    tail = [(mg.test_key(2000 + i), b"z" * 50, mg.NORMAL, mg.STRING, 0) for i in range(300)]
    f2, _ = py_append(tail, 0, False, files[-1], len(files[-1]), dfs)
    return files[:-1] + f2


def test_partition_keeps_tx_resolution():
    from couloydb_amd.shard import partition_by_bytes
    files = tx_across_files()
    assert len(files) >= 4
    arrays = [np.frombuffer(b, np.uint8).copy() for b in files]
    tts = [co.scan_file(a, i)[0] for i, a in enumerate(arrays)]
    whole = index_states(arrays, tts)
    for n in (2, 3):
        parts = partition_by_bytes([len(a) for a in arrays], n)
        cat = [tts[i] for lo, hi in parts for i in range(lo, hi)]
        assert (index_states([arrays[i] for lo, hi in parts for i in range(lo, hi)], cat) == whole).all()
    assert int((whole == 1).sum()) == 40 + 10 + 300


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 3])
def test_gpu_multi_equals_single(n):
    from couloydb_amd import DataFile, Scanner
    from couloydb_amd.multi import MultiScanner
    rng = random.Random(n)
    blobs = [mixed_corpus(300 + k, rng.randint(50_000, 400_000), tail=False) for k in range(7)]
    blobs += tx_across_files()
    files = [DataFile(np.frombuffer(b, np.uint8).copy(), i) for i, b in enumerate(blobs)]
    with Scanner(0) as sc:
        one = sc.scan(files)
    with MultiScanner([0] * n) as ms:
        many = ms.scan(files)
    assert many.status == one.status and many.end_offset == one.end_offset and many.n_records == one.n_records
    assert len(many.tuples) == len(one.tuples)
    assert (many.tuples.view(np.uint8) == one.tuples.view(np.uint8)).all()
    for i in range(len(files)):
        assert many.file_tuples(i).tobytes() == one.file_tuples(i).tobytes()
