"""GPU parity tests: the HIP scan (through the C-ABI) against the golden fixtures
and the CPU oracle, bit-exact, plus size-independent properties at the
BASELINE.json config-2 size.  Run on an MI355X: pytest -m gpu."""
import json
import os

import numpy as np
import pytest

from couloydb_amd import DataFile, ScanError, Scanner, TUPLE_DTYPE, _abi
from oracle import cly_oracle as co

from .gpu_util import FIELDS, compare, fixed_records_file, mixed_corpus

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
with open(os.path.join(GOLD, "golden.json")) as _f:
    GOLDEN = json.load(_f)
FIXTURES = sorted(k for k in GOLDEN if not k.startswith("_"))
LIBS = ["libclyscan.so", "libclyscan_small.so"]


def fixture_file(name):
    with open(os.path.join(GOLD, name + ".cly"), "rb") as f:
        return DataFile(np.frombuffer(f.read(), np.uint8).copy(), GOLDEN[name]["fid"])


@pytest.fixture(scope="module", params=LIBS)
def scanner(request):
    s = Scanner(0, lib=request.param)
    yield s
    s.close()


def as_lists(t):
    return [[int(r[f]) for f in FIELDS] for r in t]


@pytest.mark.parametrize("name", FIXTURES)
def test_fixture(scanner, name):
    g = GOLDEN[name]
    r = scanner.scan([fixture_file(name)])
    assert (r.status[0], r.end_offset[0], r.n_records[0]) == (g["status"], g["end_offset"], g["n_records"])
    assert as_lists(r.file_tuples(0)) == g["tuples"]


def test_all_fixtures_one_call(scanner):
    files = [fixture_file(n) for n in FIXTURES]
    r = scanner.scan(files)
    for i, n in enumerate(FIXTURES):
        g = GOLDEN[n]
        assert (r.status[i], r.end_offset[i]) == (g["status"], g["end_offset"]), n
        assert as_lists(r.file_tuples(i)) == g["tuples"], n


def test_records_iterator_matches_readlogrecord(scanner):
    import make_golden as mg
    f = fixture_file("txn_hash")
    r = scanner.scan([f])
    recs = list(r.records(0))
    assert [s for _, s in recs] == [t[4] for t in GOLDEN["txn_hash"]["tuples"]]
    raw = f.data.tobytes()
    off = 0
    for rec, size in recs:
        st, t = mg.read_log_record(raw, off)
        h = t["header_size"]
        assert rec.key == raw[off + h: off + h + t["key_size"]]
        assert rec.value == raw[off + h + t["key_size"]: off + t["size"]]
        assert (rec.type, rec.data_type, rec.expiration) == (t["type"], t["data_type"], t["expiration"])
        off += size
    with pytest.raises(Exception):
        list(scanner.scan([fixture_file("bitflip")]).records(0))


@pytest.mark.parametrize("seed", range(24))
def test_mixed_corpus_vs_oracle(scanner, seed):
    files = []
    for j in range(3):
        data = mixed_corpus(seed * 7 + j, [40_000, 300_000, 1_500_000][j], corrupt=(seed % 4 == 3) * (j + 1))
        files.append(DataFile(np.frombuffer(data, np.uint8).copy(), 1000 + j))
    r = scanner.scan(files)
    for i, f in enumerate(files):
        t, st, end = co.scan_file(f.data, f.fid)
        compare(r.file_tuples(i), r.status[i], r.end_offset[i], t, st, end, "seed %d file %d" % (seed, i))


@pytest.mark.parametrize("shape", ["c1", "zero_values", "tiny"])
def test_shapes_vs_oracle(scanner, shape):
    if shape == "c1":       # BASELINE config 1: one 64 MiB file of 1 KiB values
        data = fixed_records_file(64280, 1024, seed=11)
    elif shape == "zero_values":   # TestDB_Reboot: value = key || 1024 zero bytes
        data = fixed_records_file(8000, 1033, seed=12, zero_values=True)
    else:
        data = fixed_records_file(200000, 0, seed=13)
    f = DataFile(data, 0)
    r = scanner.scan([f])
    t, st, end = co.scan_file(data, 0)
    compare(r.file_tuples(0), r.status[0], r.end_offset[0], t, st, end, shape)


@pytest.mark.parametrize("seed", range(4))
def test_tiny_records_irregular(scanner, seed):
    """Records whose key+value is <= 3 bytes (commit markers: the header, the
    txId varint and the key share the 4-B word of the next record's start)
    among irregular sizes, so that blocks take the general pass: every header
    must be read before the next record's CRC patch lands in the stage."""
    import random

    import make_golden as mg
    rng = random.Random(seed)
    b = bytearray()
    while len(b) < 400_000:
        if rng.random() < 0.6:
            tx = rng.choice([0, 1, 5, 63, 64, 6453, 100_000])
            key = mg.key_tx(bytes([rng.randrange(256)]) if rng.random() < 0.7 else b"", tx)[:3]
            val = rng.randbytes(max(0, rng.randrange(4) - len(key)))
            b += mg.encode_record(key, val, rng.choice([0, 1, 2, 3, 4]), rng.choice([0, 0, 1, 3]), 0)
        else:
            b += mg.encode_record(mg.key_tx(rng.randbytes(rng.randrange(1, 30)), 0),
                                  rng.randbytes(rng.choice([0, 7, 33, 120])), 0, 0, 0)
    data = np.frombuffer(bytes(b), np.uint8).copy()
    f = DataFile(data, 9)
    r = scanner.scan([f])
    t, st, end = co.scan_file(data, 9)
    assert len(t) > 8000 and st == 0
    compare(r.file_tuples(0), r.status[0], r.end_offset[0], t, st, end, "tiny %d" % seed)


def tiny_records(seed, nbytes):
    """Commit / rollback markers, tombstones, empty values and short keys:
    records of 12-30 bytes (hint-index records average 23.6 B)."""
    import random

    import make_golden as mg
    rng = random.Random(seed)
    b = bytearray()
    while len(b) < nbytes:
        r = rng.random()
        if r < 0.25:
            b += mg.encode_record(mg.key_tx(mg.TX_COMMIT_KEY, rng.randrange(1, 1 << 20)), b"", mg.TXN_COMMIT)
        elif r < 0.35:
            b += mg.encode_record(mg.key_tx(mg.TX_ROLLBACK_KEY, rng.randrange(1, 1 << 20)), b"", mg.TXN_ROLLBACK)
        elif r < 0.6:
            b += mg.encode_record(mg.key_tx(b"%d" % rng.randrange(10 ** 6), 0), b"", mg.DELETED)
        else:
            b += mg.encode_record(mg.key_tx(rng.randbytes(rng.randrange(1, 9)), rng.choice([0, 0, 7])),
                                  rng.randbytes(rng.randrange(0, 12)), 0, rng.choice([0, 0, 1, 3]))
    return bytes(b)


def test_spill_tiles_then_long_record(scanner):
    """A tile with more than CAP_T records (its compact list spills into
    chunks) followed by a 5-MiB record and more tiny records: every tuple
    and the CRC verdicts bit-exact against the oracle; a flipped byte deep in
    the long record stops the file at that record (ErrInvalidCRC)."""
    import make_golden as mg
    small = tiny_records(1, 40_000)                           # ~2000 records: several tiles' worth
    big = mg.encode_record(mg.key_tx(b"big", 0), bytes(range(256)) * (5 << 12))
    data = np.frombuffer(small + big + tiny_records(2, 70_000), np.uint8).copy()
    for flip in (None, len(small) + len(big) // 2):
        d = data.copy()
        if flip is not None:
            d[flip] ^= 0x08
        r = scanner.scan([DataFile(d, 3)])
        t, st, end = co.scan_file(d, 3)
        compare(r.file_tuples(0), r.status[0], r.end_offset[0], t, st, end, "spill + long %s" % flip)
        if flip is not None:
            assert st == _abi.ERR_CRC and end == len(small)


def test_tiny_record_file_1gib(scanner):
    """One 1-GiB data file of 12-30-B records (about 45 M: every tile spills;
    the context's first call grows the spill pool and runs again, the second
    does not), bit-exact against the oracle; then a flipped byte in the last
    tile's records gives ErrInvalidCRC at its record."""
    torch = pytest.importorskip("torch")
    base = np.frombuffer(tiny_records(7, 4 << 20), np.uint8)
    arr = np.tile(base, (1 << 30) // len(base))
    n_base = len(co.scan_file(base.copy(), 1)[0])
    d = torch.from_numpy(arr).cuda()
    t, st, end = co.scan_file(arr, 1)
    assert st == 0 and len(t) == n_base * ((1 << 30) // len(base))
    out = torch.empty((len(t) + 64) * 48, dtype=torch.uint8, device="cuda")
    with Scanner(0, lib=scanner.lib_name) as sc:
        for call in range(2):
            first, res, stt, need = sc.scan_device([(d.data_ptr(), len(arr), 1)], out.data_ptr(), len(t) + 64)
            retry = sc.kernel_ms()["retry"]
            assert (retry > 0) if call == 0 else (retry == 0), (call, retry)
        got = out[: need * 48].cpu().numpy().view(TUPLE_DTYPE)
        compare(got[: res[0].n_records], res[0].status, res[0].end_offset, t, st, end, "1 GiB tiny")
        del got
        k = len(t) - 1000
        arr2 = arr.copy()
        arr2[int(t["offset"][k]) + 5] ^= 0x01                 # the record's data type byte
        d.copy_(torch.from_numpy(arr2))
        first, res, stt, need = sc.scan_device([(d.data_ptr(), len(arr2), 1)], out.data_ptr(), len(t) + 64)
        assert res[0].status == _abi.ERR_CRC and res[0].n_records == k and res[0].end_offset == int(t["offset"][k])


@pytest.mark.parametrize("cut", [0, 1, 4, 5, 6, 13, 27, 31])
def test_tails_at_chunk_boundaries(scanner, cut):
    # lengths around chunk multiples for both builds (32 KiB and 2 KiB chunks)
    base = fixed_records_file(400, 300, seed=cut)        # 400 x 320 B
    for chunk in (1792, 31744):
        k = (len(base) // chunk) * chunk - 7
        for extra in (0, 3, 7, 8):
            data = base[:k + extra] if k + extra <= len(base) else base
            data = np.concatenate([data, np.zeros(cut, np.uint8)]) if cut % 2 else data[: len(data) - cut]
            f = DataFile(np.ascontiguousarray(data), 5)
            r = scanner.scan([f])
            t, st, end = co.scan_file(f.data, 5)
            compare(r.file_tuples(0), r.status[0], r.end_offset[0], t, st, end, "cut %d chunk %d +%d" % (cut, chunk, extra))


@pytest.mark.parametrize("name", ["false_merge_a", "false_merge_b"])
def test_false_merge_fixtures(scanner, name):
    """GPU-captured chunks whose speculative guess is a false candidate merging
    into the true chain (the guess is wrong; the chunk re-resolves)."""
    d = np.fromfile(os.path.join(GOLD, name + ".cly"), dtype=np.uint8)
    long = np.concatenate([d, fixed_records_file(20000, 256, seed=9)])
    for data in (d, long):
        f = DataFile(np.ascontiguousarray(data), 3)
        r = scanner.scan([f])
        t, st, end = co.scan_file(f.data, 3)
        compare(r.file_tuples(0), r.status[0], r.end_offset[0], t, st, end, name)


@pytest.mark.parametrize("seed", range(3))
def test_false_starts_chaining_into_true_records(scanner, seed):
    """Every value embeds a well-formed header whose record size ends exactly
    where the next true record starts: a tile whose entry guess takes such a
    false start runs into the true chain (k_refix's suffix shortcut drops the
    false record, k_emit skips its compact entry and corrects the register)."""
    import random

    import make_golden as mg
    rng = random.Random(seed)
    b = bytearray()
    i = 0
    while len(b) < 600_000:
        vlen = rng.choice([150, 276, 300, 777, 2000])
        key = mg.key_tx(mg.test_key(i), 0)
        hdr_len = len(mg.encode_record(key, b"")) - len(key)
        o = rng.randrange(0, vlen - 40)
        start_v = len(b) + hdr_len + len(key)
        rec_end = start_v + vlen
        fpos = start_v + o
        ks = 10
        body_len = rec_end - fpos
        for hsz in range(9, 20):
            vs = body_len - hsz - ks
            fh = rng.randbytes(4) + bytes([rng.randrange(5), rng.randrange(5)]) + mg.put_varint(ks) + \
                mg.put_varint(vs) + mg.put_varint(0)
            if len(fh) == hsz:
                break
        v = bytearray(rng.randbytes(vlen))
        v[o:o + len(fh)] = fh
        b += mg.encode_record(key, bytes(v))
        i += 1
    data = np.frombuffer(bytes(b), np.uint8).copy()
    f = DataFile(data, 4)
    r = scanner.scan([f])
    t, st, end = co.scan_file(data, 4)
    assert st == 0 and len(t) == i
    compare(r.file_tuples(0), r.status[0], r.end_offset[0], t, st, end, "false starts %d" % seed)


@pytest.mark.parametrize("nfalse", [3, 20])
def test_refix_suffix_entry_at_sentinel_offset(scanner, nfalse):
    """a record spanning many tiles ends exactly 0xFFFFF bytes past
    the start of a middle tile that holds a short false chain (embedded
    records).  The true entry of that tile is then tb + 0xFFFFF, the value the
    suffix shortcut gave lanes without a compact entry; it must re-walk the
    tile instead of taking the shortcut."""
    import random

    import make_golden as mg
    tile = 8192 if "small" in scanner.lib_name else 65536
    rng = random.Random(nfalse)
    head = mg.encode_record(mg.key_tx(mg.test_key(0), 0), rng.randbytes(100))
    t = 2                                                     # the middle tile
    tb = t * tile
    key = mg.key_tx(mg.test_key(1), 0)
    vlen = tb + 0xFFFFF - len(head) - len(key)
    for _ in range(3):                                        # the header's length depends on vlen's varint
        hdr = len(mg.encode_record(key, b"")) - 1 + len(mg.put_varint(vlen)) - len(key)
        vlen = tb + 0xFFFFF - len(head) - hdr - len(key)
    vstart = len(head) + hdr + len(key)
    value = bytearray(rng.randbytes(vlen))
    emb = b"".join(mg.encode_record(mg.key_tx(mg.test_key(900 + j), 0), rng.randbytes(rng.randrange(5, 60)))
                   for j in range(nfalse))
    o = tb + 40 - vstart
    value[o:o + len(emb)] = emb
    big = mg.encode_record(key, bytes(value))
    tail = mg.encode_record(mg.key_tx(mg.test_key(2), 0), b"after")
    data = np.frombuffer(head + big + tail, np.uint8).copy()
    assert len(head) + len(big) == tb + 0xFFFFF
    f = DataFile(data, 6)
    r = scanner.scan([f])
    tt, st, end = co.scan_file(data, 6)
    assert st == 0 and len(tt) == 3
    compare(r.file_tuples(0), r.status[0], r.end_offset[0], tt, st, end, "sentinel %d" % nfalse)


def test_bitflips_everywhere_small(scanner):
    base = fixed_records_file(60, 200, seed=5)
    rng = np.random.default_rng(0)
    files = []
    for k in range(40):
        d = base.copy()
        pos = int(rng.integers(0, len(d)))
        d[pos] ^= np.uint8(1 << int(rng.integers(0, 8)))
        files.append(DataFile(d, k))
    r = scanner.scan(files)
    for i, f in enumerate(files):
        t, st, end = co.scan_file(f.data, f.fid)
        compare(r.file_tuples(i), r.status[i], r.end_offset[i], t, st, end, "flip %d" % i)


def _cancel_corpus(seed):
    """A file and record pairs (i, j) for the CRC-cancellation cases: C2-shape
    records, tiny unaligned records, mixed corpora, and big records spanning
    tiles."""
    import random

    import make_golden as mg
    rng = random.Random(seed)
    kind = seed % 4
    if kind == 0:
        data = fixed_records_file(9000, 256, seed=seed).tobytes()             # 2.5 MB, 276-B records
    elif kind == 1:
        b = bytearray()
        for i in range(60000):                                                # 11-14 B records
            b += mg.encode_record(mg.key_tx(bytes([i & 0xFF]), 0), rng.randbytes(i % 4))
        data = bytes(b)
    elif kind == 2:
        data = mixed_corpus(seed * 13, 1_500_000, tail=False)
    else:
        b = bytearray()
        for i in range(120):                                                  # 2 KiB .. 100 KiB values
            b += mg.encode_record(mg.key_tx(mg.test_key(i), 0), rng.randbytes(rng.choice([2000, 30000, 100000])))
        data = bytes(b)
    return data, rng


@pytest.mark.parametrize("seed", range(16))
def test_crc_residues_that_cancel(scanner, seed):
    """Two (or three) records fail their own CRC while their residues cancel in
    any per-file linear fold (stored-CRC deltas d and A^(end_j - end_i) d, or a
    payload flip compensated in a later record's last word).  ReadLogRecord's
    loop stops at the first of them with ErrInvalidCRC (data/dataFile.go:105-109);
    so must the scan.  Pairs: adjacent, a few records apart, across tiles."""
    import make_golden as mg
    data, rng = _cancel_corpus(seed)
    recs = mg.record_bounds_lenient(data)
    n = len(recs)
    files = []
    for k in range(6):
        i = rng.randrange(0, n - 2)
        j = min(n - 1, i + rng.choice([1, 1, 2, 5, 40, n]))
        if j <= i:
            continue
        if seed % 4 == 0 and k % 2:
            d = mg.cancel_payload(data, i, rng.randrange(14, 270), rng.randrange(8), j)
        else:
            d = mg.cancel_stored(data, i, j, rng.randrange(1, 1 << 32))
        if k == 5 and j + 1 < n:                                              # a third record on top
            d = mg.cancel_stored(d, j, rng.randrange(j + 1, n), rng.randrange(1, 1 << 32))
        assert mg.file_fold(d) == 0
        files.append(DataFile(np.frombuffer(d, np.uint8).copy(), 50 + k))
    r = scanner.scan(files)
    for i, f in enumerate(files):
        t, st, end = co.scan_file(f.data, f.fid)
        assert st == _abi.ERR_CRC
        compare(r.file_tuples(i), r.status[i], r.end_offset[i], t, st, end, "cancel seed %d file %d" % (seed, i))


@pytest.mark.slow
def test_config2_device_generated_properties():
    """BASELINE config 2 at full size (16 x 256 MiB, 256-B values), generated in
    HBM: size-independent properties over all files + bit-exact oracle check of
    one whole file."""
    torch = pytest.importorskip("torch")
    from bench import make_workload   # the bench's own input builder
    wl = make_workload("c2", torch)
    with Scanner(0) as sc:
        first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
        # passes > 1: link rounds after tiles whose guessed entry was wrong were
        # re-resolved (results exact either way; the count is a speed property)
        assert 1 <= st.passes <= 8
        assert need == wl.expect_records
        out = wl.d_out[: need * 48].cpu().numpy().view(TUPLE_DTYPE)
    for i, (ptr, ln, fid) in enumerate(wl.dev_files):
        assert res[i].status == 0 and res[i].end_offset == ln
        t = out[first[i]:first[i] + res[i].n_records]
        assert res[i].n_records == ln // 276
        assert (t["size"] == 276).all() and (t["key_size"] == 10).all() and (t["value_size"] == 256).all()
        assert (t["offset"] == np.arange(len(t), dtype=np.int64) * 276).all()
        assert (t["fid"] == fid).all() and (t["txid_len"] == 1).all() and (t["tx_id"] == 0).all()
    # bit-exact against the oracle on file 3 (D2H of the file bytes)
    ptr, ln, fid = wl.dev_files[3]
    host = wl.file_bytes(3)
    t, st_o, end = co.scan_file(host, fid)
    compare(out[first[3]:first[3] + res[3].n_records], res[3].status, res[3].end_offset, t, st_o, end, "c2 file 3")


@pytest.mark.slow
def test_host_entry_pipelined_c2():
    """cly_scan over host buffers of the whole C2 configuration (4 GiB, 16
    files: the pipelined path, several groups): tuples back in host memory
    equal the oracle's, file by file."""
    torch = pytest.importorskip("torch")
    from bench import make_workload
    wl = make_workload("c2", torch)
    files = [DataFile(np.ascontiguousarray(wl.file_bytes(i)), fid) for i, (_, _, fid) in enumerate(wl.dev_files)]
    with Scanner(0) as sc:
        r = sc.scan(files)
    assert sum(r.n_records) == wl.expect_records
    for i, f in enumerate(files):
        assert r.status[i] == 0 and r.end_offset[i] == len(f.data)
        if i in (0, 7, 15):
            t, st, end = co.scan_file(f.data, f.fid)
            compare(r.file_tuples(i), r.status[i], r.end_offset[i], t, st, end, "host c2 file %d" % i)
        else:
            t = r.file_tuples(i)
            assert (t["offset"] == np.arange(len(t), dtype=np.int64) * 276).all() and (t["fid"] == f.fid).all()


def _device_file_checks(torch, wl, first, res, need):
    """Size-independent properties of a device scan, checked on the device:
    per file status io.EOF at its length, records back to back from offset 0
    (offset[i+1] = offset[i] + size[i], the last ending at the file's end),
    the file's fid; and the generator's record count."""
    assert need == wl.expect_records
    t = wl.d_out[: need * 48].view(torch.int64).view(need, 6)
    u32 = wl.d_out[: need * 48].view(torch.int32).view(need, 12)
    off, size, fidv = t[:, 0], u32[:, 7].to(torch.int64) & 0xFFFFFFFF, u32[:, 6].to(torch.int64) & 0xFFFFFFFF
    for i, (ptr, ln, fid) in enumerate(wl.dev_files):
        assert res[i].status == 0 and res[i].end_offset == ln, (i, res[i].status, res[i].end_offset, ln)
        a, n = int(first[i]), int(res[i].n_records)
        o, sz = off[a:a + n], size[a:a + n]
        assert int(o[0]) == 0 and int(o[-1] + sz[-1]) == ln
        assert bool((o[1:] == o[:-1] + sz[:-1]).all())
        assert bool((fidv[a:a + n] == fid).all())


@pytest.mark.slow
def test_config3_device_generated_properties():
    """BASELINE config 3 at full size: 128 files x 256 MiB = 32 GiB, value
    lengths 64 B-64 KiB (Zipf 1.1, 14.6 % >= 4 KiB; tiles inside one record and
    link repairs both occur), generated in HBM: the size-independent
    properties over every file, and three whole files bit-exact against the
    oracle (the first, the one holding the largest record, the last)."""
    torch = pytest.importorskip("torch")
    from bench import make_workload
    wl = make_workload("c3", torch)
    assert len(wl.dev_files) == 128 and wl.bytes > 31.9 * 2**30
    with Scanner(0) as sc:
        first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
    _device_file_checks(torch, wl, first, res, need)
    vs = wl.d_out[: need * 48].view(torch.int32).view(need, 12)[:, 9]
    big = int(torch.argmax(vs).item())
    fbig = max(i for i in range(len(first)) if first[i] <= big)
    for i in sorted({0, fbig, len(wl.dev_files) - 1}):
        ptr, ln, fid = wl.dev_files[i]
        t, st_o, end = co.scan_file(wl.file_bytes(i), fid)
        got = wl.d_out[first[i] * 48:(first[i] + res[i].n_records) * 48].cpu().numpy().view(TUPLE_DTYPE)
        compare(got, res[i].status, res[i].end_offset, t, st_o, end, "c3 file %d" % i)


@pytest.mark.slow
def test_config5_per_gpu_share_properties():
    """BASELINE config 5's per-GPU share (one rank's 32-GiB fid range of the
    256-GiB C2/C3 mix, 128 files), generated in HBM exactly as bench.py --config
    c5 builds it: the size-independent properties over every file, and the
    first file, the file holding the largest record and the last file bit-exact
    against the oracle."""
    torch = pytest.importorskip("torch")
    from bench import make_workload
    wl = make_workload("c5", torch)
    assert 120 <= len(wl.dev_files) <= 136 and wl.bytes > 31.9 * 2**30
    with Scanner(0) as sc:
        first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
    _device_file_checks(torch, wl, first, res, need)
    vs = wl.d_out[: need * 48].view(torch.int32).view(need, 12)[:, 9]
    big = int(torch.argmax(vs).item())
    fbig = max(i for i in range(len(first)) if first[i] <= big)
    for i in sorted({0, fbig, len(wl.dev_files) - 1}):
        ptr, ln, fid = wl.dev_files[i]
        t, st_o, end = co.scan_file(wl.file_bytes(i), fid)
        got = wl.d_out[first[i] * 48:(first[i] + res[i].n_records) * 48].cpu().numpy().view(TUPLE_DTYPE)
        compare(got, res[i].status, res[i].end_offset, t, st_o, end, "c5 file %d" % i)


@pytest.mark.gpu
def test_gpu_host_scan_capacity_needed_exact():
    """cly_scan (the pipelined host path, > 512 MiB so several groups) with a
    too-small out_cap, and with out_cap = 0 as a size query: CLY_ERR_CAPACITY
    and *needed equal to the true record count (never read res[]
    of unscanned files); then the scan with exactly that capacity."""
    import ctypes
    from couloydb_amd import DataFile, Scanner, TUPLE_DTYPE, _abi
    from .gpu_util import fixed_records_file
    a = fixed_records_file(243_000, 256, seed=5)                 # 67 068 000 B
    files = [DataFile(a, i) for i in range(12)]                  # 768 MiB: two pipeline groups
    want = 12 * 243_000
    with Scanner(0) as sc:
        arr = sc._file_array(files)
        first = (ctypes.c_uint64 * 12)()
        res = (_abi.ClyFileResult * 12)()
        need = ctypes.c_uint64()
        for cap in (0, 10, want - 1):
            out = np.zeros(max(cap, 1), dtype=TUPLE_DTYPE)
            for i in range(12):                                  # garbage in res[]: must not be read
                res[i].n_records = 0xDEADBEEF
            rc = sc.lib.cly_scan(sc.ctx, arr, 12, out.ctypes.data, cap, first, res, ctypes.byref(need), None)
            assert rc == _abi.ERR_CAPACITY and need.value == want, (cap, rc, need.value)
        out = np.zeros(want, dtype=TUPLE_DTYPE)
        rc = sc.lib.cly_scan(sc.ctx, arr, 12, out.ctypes.data, want, first, res, ctypes.byref(need), None)
        assert rc == 0 and need.value == want
        assert all(res[i].n_records == 243_000 and res[i].status == 0 for i in range(12))
        assert [first[i] for i in range(12)] == [243_000 * i for i in range(12)]
        assert (out["offset"][:243_000] == np.arange(243_000) * 276).all()
        assert (out["fid"][243_000 * 11:] == 11).all()


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.parametrize("corrupt", [False, True])
def test_gpu_largest_file_offsets_past_2gib(corrupt):
    """One data file of 4.28 GB (the largest this build takes is MAX_FILE_LEN =
    4 GiB - 128 KiB: Options.SetDataFileSizeGB(1..3) files, options.go:70-71):
    record offsets past 2^31 and 2^32 - 2^25 come out as the reference's int64
    offsets, bit-exact against the oracle, and a record whose value byte is
    flipped at ~3.45 GB stops the file there with ErrInvalidCRC."""
    torch = pytest.importorskip("torch")
    base = fixed_records_file(100_000, 256, seed=9)            # 27.6 MB, 276-B records
    arr = np.tile(base, 155)                                   # 4 278 000 000 B, 15.5 M records
    k = 12_500_000
    if corrupt:
        arr[k * 276 + 100] ^= 0x40
    d = torch.from_numpy(arr).cuda()
    n = len(arr) // 276
    out = torch.empty((n + 64) * 48, dtype=torch.uint8, device="cuda")
    with Scanner(0) as sc:
        first, res, st, need = sc.scan_device([(d.data_ptr(), len(arr), 7)], out.data_ptr(), n + 64)
    got = out[: need * 48].cpu().numpy().view(TUPLE_DTYPE)
    t, st_o, end = co.scan_file(arr, 7)
    compare(got[: res[0].n_records], res[0].status, res[0].end_offset, t, st_o, end, "4.28 GB file")
    if corrupt:
        assert res[0].status == _abi.ERR_CRC and res[0].n_records == k
    else:
        assert res[0].status == 0 and res[0].n_records == n and res[0].end_offset == len(arr)
        assert int(got["offset"][-1]) == (n - 1) * 276 > 2**32 - 2**25


def part_file(total, cuts, seed):
    """One data file of `total` bytes: copies of an 8-MB mixed corpus (no tail),
    and at each cut c (a part end of the scan: 2^31 B for libclyscan, 2^28 B for
    the small build) a long record that ends exactly at c (first cut: the next
    record starts a part) or crosses it (the others); records to the end, then
    a zero tail."""
    import random

    import make_golden as mg
    rng = random.Random(seed)
    base = np.frombuffer(mixed_corpus(seed, 8 << 20, tail=False), np.uint8)
    pieces, off, i = [], 0, 10**8
    for j, c in enumerate(list(cuts) + [total]):
        while off + len(base) <= c - 60_000:
            pieces.append(base)
            off += len(base)
        if j == len(cuts):
            break
        key = mg.key_tx(mg.test_key(i), 0)
        i += 1
        want = c - off + (0 if j == 0 else 20_000)                     # the record's size
        vlen = want - 30
        for _ in range(3):                                             # (the value size's varint length)
            vlen = want - (len(mg.encode_record(key, b"\0" * vlen)) - vlen)
        rec = mg.encode_record(key, rng.randbytes(vlen))
        assert len(rec) == want
        pieces.append(np.frombuffer(rec, np.uint8))
        off += len(rec)
    pieces.append(np.zeros(total - off, np.uint8))
    arr = np.concatenate(pieces)
    assert len(arr) == total
    return arr


def _scan_part_file(lib, arr, corrupt_after):
    torch = pytest.importorskip("torch")
    t, st, end = co.scan_file(arr, 3)
    assert st != _abi.ERR_CRC and len(t) > 1000            # (the zero tail ends the file)
    cap = len(t) + 1024                                    # (tuples past a failing record are written too)
    if corrupt_after is not None:
        k = int(np.searchsorted(t["offset"], corrupt_after)) + 17
        arr = arr.copy()
        arr[int(t["offset"][k]) + int(t["size"][k]) - 1] ^= 0x10     # the record's last byte
        t, st, end = co.scan_file(arr, 3)
        assert st == _abi.ERR_CRC and len(t) == k and end > corrupt_after
    d = torch.from_numpy(arr).cuda()
    out = torch.empty(cap * 48, dtype=torch.uint8, device="cuda")
    with Scanner(0, lib=lib) as sc:
        first, res, stt, need = sc.scan_device([(d.data_ptr(), len(arr), 3)], out.data_ptr(), cap)
    got = out[: need * 48].cpu().numpy().view(TUPLE_DTYPE)
    compare(got[: res[0].n_records], res[0].status, res[0].end_offset, t, st, end, "%s %d B" % (lib, len(arr)))
    return res


@pytest.mark.parametrize("corrupt", [False, True])
def test_records_across_part_ends(scanner, corrupt):
    """A 700-MB file over three parts of the small build (2^28-B parts: a
    record ends exactly at the first part end, another crosses the second),
    one part of libclyscan; bit-exact against the oracle, and a CRC failure in
    the third part stops the file at its record."""
    arr = part_file(700_000_000, [1 << 28, 1 << 29], seed=21)
    _scan_part_file(scanner.lib_name, arr, (1 << 29) + 1_000_000 if corrupt else None)


@pytest.mark.slow
@pytest.mark.parametrize("corrupt", [False, True])
def test_gpu_file_past_4gib(corrupt):
    """One 4.6-GB data file (Options.SetDataFileSizeGB(5), options.go:70-71)
    over three 2-GiB parts: a record ends exactly at 2^31, another crosses
    2^32; bit-exact against the oracle (offsets past 2^32 as int64), and a
    flipped byte at ~4.5 GB gives ErrInvalidCRC at its record."""
    arr = part_file(4_600_000_000, [1 << 31, 1 << 32], seed=22)
    res = _scan_part_file("libclyscan.so", arr, 4_500_000_000 if corrupt else None)
    if not corrupt:
        assert res[0].status != _abi.ERR_CRC and res[0].end_offset > 1 << 32


def _tile_bytes(lib):
    info = _abi.load_scan_lib(lib).cly_build_info().decode()
    return int(info.split("TILE=")[1].split()[0])


def test_tiny_record_file_past_link_mask(scanner):
    """A data file of 12-30-B records longer than k_link's LDS bitmasks cover
    (131072 tiles: 8 GiB in the product build, 1 GiB in the 8-KiB-tile build;
    Options.DataFileSize is an int64, options.go:10,70-71): its contradiction
    and anchor bitmasks live in global memory, every contradicted tile is
    listed in the same repair round (no one-tile-per-round fallback), the
    scan finishes in <= 4 link passes, and every tuple is bit-exact against the
    oracle's tuples of the repeated 4-MiB unit (records tile exactly: tuple j
    is the unit's tuple j % n with its offset moved by (j // n) units).""" 
    torch = pytest.importorskip("torch")
    base = np.frombuffer(tiny_records(11, 4 << 20), np.uint8)
    tb, st0, end0 = co.scan_file(base.copy(), 9)
    assert st0 == 0 and end0 == len(base)
    n = len(tb)
    limit = 131072 * _tile_bytes(scanner.lib_name)
    reps = limit // len(base) + 1 + (limit // 8) // len(base)      # 1/8 past the mask
    d = torch.from_numpy(base.copy()).cuda().repeat(reps)
    total = n * reps
    out = torch.empty((total + 64) * 48, dtype=torch.uint8, device="cuda")
    with Scanner(0, lib=scanner.lib_name) as sc:
        first, res, stt, need = sc.scan_device([(d.data_ptr(), d.numel(), 9)], out.data_ptr(), total + 64)
        assert (res[0].status, res[0].n_records, res[0].end_offset, need) == (0, total, d.numel(), total)
        # link rounds: the first, the device repair round, then host-driven
        # rounds that re-resolve every listed tile at once (4 measured on the
        # product build's 9-GiB file; one round per contradicted tile past the
        # mask before round 6 would be thousands)
        assert stt.passes <= 4, stt.passes
        chunk = 1 << 26
        for j0 in range(0, total, chunk):
            j1 = min(total, j0 + chunk)
            got = out[j0 * 48: j1 * 48].cpu().numpy().view(TUPLE_DTYPE)
            j = np.arange(j0, j1, dtype=np.int64)
            exp = tb[j % n].copy()
            exp["offset"] += (j // n) * len(base)
            assert (got.view(np.uint8) == exp.view(np.uint8)).all(), "tuples %d..%d" % (j0, j1)
        # a flipped data-type byte past the LDS bitmasks' reach: ErrInvalidCRC there
        k = total - 1000
        off = int(tb["offset"][k % n]) + (k // n) * len(base)
        d[off + 5] ^= 1
        first, res, stt, need = sc.scan_device([(d.data_ptr(), d.numel(), 9)], out.data_ptr(), total + 64)
        assert (res[0].status, res[0].n_records, res[0].end_offset) == (_abi.ERR_CRC, k, off)


def test_record_past_part_view(scanner):
    """A record of nearly 4 GiB (ValueSize is a uint32, data/logRecord.go:101-106)
    that starts in a part and ends past that part's 4-GiB view, in a file longer
    than the view: the scan cannot read it whole, and says so (CLY_ERR_ARG)
    instead of reporting the torn-record io.EOF ReadLogRecord would not return.
    The same record in a file that ends inside it is a torn tail (CLY_END_TORN),
    as in the reference (the short ReadAt, data/dataFile.go:94-98)."""
    torch = pytest.importorskip("torch")
    import make_golden as mg
    a = mg.encode_record(mg.key_tx(mg.test_key(1), 0), b"v" * 17)
    vs = 0xFFFFFFFF                      # past both builds' views (4 GiB less two tiles)
    key = mg.key_tx(mg.test_key(2), 0)
    hdr = bytes([0x11, 0x22, 0x33, 0x44, 0, 0]) + mg.put_varint(len(key)) + mg.put_varint(vs) + mg.put_varint(0)
    end = len(a) + len(hdr) + len(key) + vs
    for total, want in ((end + 4096, "arg"), (end - 4096, "torn")):
        d = torch.zeros(total, dtype=torch.uint8, device="cuda")
        head = np.frombuffer(a + hdr + key, np.uint8)
        d[: len(head)] = torch.from_numpy(head.copy()).cuda()
        out = torch.empty(64 * 48, dtype=torch.uint8, device="cuda")
        with Scanner(0, lib=scanner.lib_name) as sc:
            if want == "arg":
                with pytest.raises(ScanError) as ei:
                    sc.scan_device([(d.data_ptr(), total, 5)], out.data_ptr(), 64)
                assert ei.value.code == _abi.ERR_ARG
            else:
                first, res, st, need = sc.scan_device([(d.data_ptr(), total, 5)], out.data_ptr(), 64)
                assert (res[0].status, res[0].n_records, res[0].end_offset) == (2, 1, len(a))
        del d
        torch.cuda.empty_cache()
