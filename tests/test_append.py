"""Batched append (the write path: db.appendLogRecord over a batch,
db.go:368-413, as db.Put and WriteBatch.Commit issue it, batch.go:62-118;
SURVEY.md §8f row 4).

CPU: the restatement (tests/gpu_util.py py_append) against the C oracle's
EncodeLogRecord and a scan round trip.  GPU (-m gpu): cly_append_device
against the restatement, byte for byte (files, positions), continuing an
active file, with rotation, an active file that takes nothing, records larger
than a data file, WriteBatch's commit marker and 10-byte records."""
import random

import numpy as np
import pytest

from oracle import cly_oracle as co

from .gpu_util import mg, py_append


def batch(seed, n, vmax=300, tiny=False):
    rng = random.Random(seed)
    out = []
    for i in range(n):
        key = b"k" if tiny else mg.test_key(rng.randrange(10**9))
        value = b"" if tiny else rng.randbytes(rng.choice([0, 1, 7, 64, 256, vmax]))
        out.append((key, value, rng.choice([0, 0, 0, 1]), rng.choice([0, 0, 1, 3]),
                    rng.choice([0, 0, 1_700_000_000_000_000_000, -5])))
    return out


def test_restatement_matches_oracle_encode_and_scans_back():
    recs = batch(1, 400)
    files, pos = py_append(recs, 77, True, b"", 0, 4096)
    # EncodeLogRecord restated twice (Python, C oracle)
    for key, value, typ, dt, exp in recs[:50]:
        assert mg.encode_record(mg.key_tx(key, 77), value, typ, dt, exp) == \
            co.encode_record(mg.key_tx(key, 77), value, typ, dt, exp)
    got = []
    for fid, f in enumerate(files):
        t, st, end = co.scan_file(np.frombuffer(f, np.uint8), fid)
        assert st == 0 and end == len(f) and len(f) <= 4096
        got += [(int(r["fid"]), int(r["offset"])) for r in t]
    assert got == pos and len(pos) == 401


@pytest.fixture(scope="module")
def scanner():
    from couloydb_amd import Scanner
    s = Scanner(0)
    yield s
    s.close()


def gpu_append(scanner, recs, tx_id, commit, active, write_off, dfs):
    import torch
    from couloydb_amd import POS_DTYPE, REC_IN_DTYPE
    blob = b"".join(k + v for k, v, *_ in recs) or b"\0"
    d_blob = torch.tensor(list(blob), dtype=torch.uint8, device="cuda")
    base = d_blob.data_ptr()
    ri = np.zeros(len(recs), REC_IN_DTYPE)
    o = 0
    for i, (k, v, typ, dt, exp) in enumerate(recs):
        ri[i]["key"], ri[i]["key_len"] = base + o, len(k)
        o += len(k)
        ri[i]["value"], ri[i]["value_len"] = base + o, len(v)
        o += len(v)
        ri[i]["type"], ri[i]["data_type"], ri[i]["expiration"] = typ, dt, exp
    d_recs = torch.from_numpy(ri.view(np.uint8)).cuda() if len(recs) else torch.zeros(40, dtype=torch.uint8,
                                                                                        device="cuda")
    want, wpos = py_append(recs, tx_id, commit, active, write_off, dfs)
    nreg = len(want) + 1
    # capacity query: the region stride (DataFileSize, or more for records larger than a file)
    rc, _, q = scanner.append_device(d_recs.data_ptr(), len(recs), tx_id, commit, 5, write_off, dfs, None, 0, None)
    assert rc == -10 and q.n_out_files == len(want)
    stride = int(q.out_stride)
    out = torch.zeros(nreg * stride, dtype=torch.uint8, device="cuda")
    if write_off:
        out[:write_off] = torch.tensor(list(active[:write_off]), dtype=torch.uint8, device="cuda")
    d_pos = torch.zeros((len(recs) + 1) * 16, dtype=torch.uint8, device="cuda")
    rc, lens, r = scanner.append_device(d_recs.data_ptr(), len(recs), tx_id, commit, 5, write_off, dfs,
                                        out.data_ptr(), nreg, d_pos.data_ptr())
    assert rc == 0
    assert r.n_out_files == len(want) and r.final_fid == 5 + len(want) - 1 and r.final_write_off == len(want[-1])
    host = out.cpu().numpy()
    for k, w in enumerate(want):
        g = host[k * stride:k * stride + lens[k]].tobytes()
        assert len(g) == len(w), (k, len(g), len(w))
        if g != w:
            d = next(i for i in range(len(g)) if g[i] != w[i])
            raise AssertionError("region %d differs at byte %d" % (k, d))
    p = d_pos.cpu().numpy().view(POS_DTYPE)[:len(wpos)]
    assert [(int(x["fid"]) - 5, int(x["offset"])) for x in p] == wpos
    return r


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
def test_gpu_append_fresh(scanner, seed):
    gpu_append(scanner, batch(seed, 3000), 0, False, b"", 0, 1 << 20)


@pytest.mark.gpu
def test_gpu_append_continue_and_rotate(scanner):
    active = random.Random(9).randbytes(5000)
    gpu_append(scanner, batch(5, 2000), 0, False, active, 1234, 9000)
    gpu_append(scanner, batch(6, 2000), 12345, True, active, 4096, 9000)


@pytest.mark.gpu
def test_gpu_append_active_file_takes_nothing(scanner):
    active = bytes(8990)
    gpu_append(scanner, batch(7, 500), 3, True, active, 8990, 9000)


@pytest.mark.gpu
def test_gpu_append_records_larger_than_a_file(scanner):
    recs = [(mg.test_key(i), random.Random(i).randbytes(20000 if i % 3 == 0 else 100), 0, 0, 0) for i in range(40)]
    gpu_append(scanner, recs, -77, True, b"", 0, 16384)


@pytest.mark.gpu
def test_gpu_append_tiny_records(scanner):
    gpu_append(scanner, batch(8, 20000, tiny=True), 0, False, b"", 0, 1 << 16)


@pytest.mark.gpu
def test_gpu_append_host_entry(scanner):
    """cly_append (host buffers, the cgo path) against the restatement."""
    active = random.Random(3).randbytes(3000)
    recs = batch(12, 1500)
    want, wpos = py_append(recs, 99, True, active, 2500, 20000)
    regions, pos, r = scanner.append(recs, 99, True, 7, 2500, 20000)
    assert regions[0] == want[0][2500:] and regions[1:] == want[1:]
    assert [(f - 7, o) for f, o in pos] == wpos and r.final_fid == 7 + len(want) - 1
