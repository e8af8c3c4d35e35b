"""Helpers shared by the GPU tests and the bench (input builders, comparison)."""
import os
import random
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden as mg  # noqa: E402

FIELDS = mg.FIELDS


def fixed_records_file(n, value_len, seed=1, key_base=0, zero_values=False):
    """C1/C2-shape data file: key 0x00||%09d(i), value_len random (or key||zeros) bytes."""
    rng = np.random.default_rng(seed)
    hdr = mg.encode_record(mg.key_tx(mg.test_key(0), 0), b"\0" * value_len)[4:4 + 6 + 4]
    # header after the crc: type, dtype, varint(10), varint(vlen), varint(0)
    body = bytes([0, 0]) + mg.put_varint(10) + mg.put_varint(value_len) + mg.put_varint(0)
    hl = 4 + len(body)
    rs = hl + 10 + value_len
    out = np.zeros((n, rs), dtype=np.uint8)
    out[:, 4:hl] = np.frombuffer(body, np.uint8)
    keys = np.array([list(b"\x00" + mg.test_key(key_base + i)) for i in range(n)], dtype=np.uint8)
    out[:, hl:hl + 10] = keys
    if zero_values:
        out[:, hl + 10:hl + 19] = keys[:, 1:]
    else:
        out[:, hl + 10:] = rng.integers(0, 256, size=(n, value_len), dtype=np.uint8)
    for i in range(n):
        c = zlib.crc32(out[i, 4:].tobytes())
        out[i, 0:4] = np.frombuffer(c.to_bytes(4, "little"), np.uint8)
    del hdr
    return out.reshape(-1)


def mixed_corpus(seed, target_bytes, corrupt=0, tail=True):
    """Records of mixed shapes (tx ids, all types/dtypes, tombstones, header-like
    values, embedded records, long values spanning chunks)."""
    rng = random.Random(seed)
    b = bytearray()
    i = 0
    while len(b) < target_bytes:
        kind = rng.random()
        tx = 0 if rng.random() < 0.7 else rng.randrange(1, 1 << 62)
        if kind < 0.45:
            v = rng.randbytes(rng.choice([0, 1, 3, 7, 20, 64, 255, 256, 300, 1000]))
        elif kind < 0.6:
            v = bytes(rng.randrange(0, 5) for _ in range(rng.randrange(0, 120)))
        elif kind < 0.7:
            v = b"".join(mg.encode_record(mg.key_tx(mg.test_key(rng.randrange(10**9)), 0), rng.randbytes(rng.randrange(0, 30)))
                         for _ in range(rng.randrange(1, 6)))
        elif kind < 0.78:
            v = bytes(rng.randrange(0, 1 << 14))                                   # zero run
        elif kind < 0.8:
            v = rng.randbytes(rng.randrange(2000, 70000))                          # spans chunks
        else:
            v = rng.randbytes(rng.randrange(0, 64))
        typ = rng.choice([0, 0, 0, 0, 1, 2, 3, 4])
        dt = rng.choice([0, 0, 0, 1, 2, 3, 4])
        exp = rng.choice([0, 0, 0, -1, 1 << 40, 1_697_000_000_000_000_000])
        b += mg.encode_record(mg.key_tx(mg.test_key(i), tx), v, typ, dt, exp)
        i += 1
    for _ in range(corrupt):
        k = rng.randrange(len(b))
        b[k] ^= 1 << rng.randrange(8)
    if tail:
        t = rng.random()
        if t < 0.3:
            b += bytes(rng.randrange(1, 5000))
        elif t < 0.5:
            b += rng.randbytes(rng.randrange(1, 30))
        elif t < 0.6:
            del b[len(b) - rng.randrange(1, 40):]
    return bytes(b)


def compare(gpu_tuples, gpu_status, gpu_end, oracle_tuples, oracle_status, oracle_end, label=""):
    """Bit-exact comparison with a readable first difference."""
    assert gpu_status == oracle_status, "%s status gpu=%d oracle=%d (end gpu=%d oracle=%d, n gpu=%d oracle=%d)" % (
        label, gpu_status, oracle_status, gpu_end, oracle_end, len(gpu_tuples), len(oracle_tuples))
    assert gpu_end == oracle_end, "%s end_offset gpu=%d oracle=%d" % (label, gpu_end, oracle_end)
    assert len(gpu_tuples) == len(oracle_tuples), "%s n gpu=%d oracle=%d" % (label, len(gpu_tuples), len(oracle_tuples))
    if len(gpu_tuples):
        g = np.asarray(gpu_tuples).view(np.uint8).reshape(-1, 48)
        o = np.asarray(oracle_tuples).view(np.uint8).reshape(-1, 48)
        bad = np.nonzero((g != o).any(axis=1))[0]
        assert bad.size == 0, "%s first differing tuple %d: gpu=%s oracle=%s" % (
            label, bad[0], gpu_tuples[bad[0]], oracle_tuples[bad[0]])


def string_live_mask(file_bytes, tuples_per_file):
    """The index db.loadIndex rebuilds (db.go:582-637: updateIndex for String
    keys, tx records applied at their commit marker, rollback drops), then
    merge.go:104-132's liveness test: a record is live iff the index still
    points at its (fid, offset).  Non-String data types count as dead here (the
    merge kernel takes the mask as given)."""
    index, txbuf = {}, {}

    def apply(rk, t):
        if t["data_type"] != mg.STRING:
            return
        if t["type"] == mg.DELETED:
            index.pop(rk, None)
        else:
            index[rk] = (int(t["fid"]), int(t["offset"]))

    recs = []
    for F, tt in zip(file_bytes, tuples_per_file):
        for t in tt:
            o, h, ks = int(t["offset"]), int(t["header_size"]), int(t["key_size"])
            key = bytes(F[o + h:o + h + ks])
            tx, n = mg.varint(key)
            rk = key[n:] if n > 0 else key
            recs.append((rk, t))
            if tx == 0:
                apply(rk, t)
            elif t["type"] == mg.TXN_BEGIN:
                pass
            elif t["type"] == mg.TXN_COMMIT:
                for r in txbuf.pop(tx, []):
                    apply(*r)
            elif t["type"] == mg.TXN_ROLLBACK:
                txbuf.pop(tx, None)
            else:
                txbuf.setdefault(tx, []).append((rk, t))
    return np.array([1 if (t["data_type"] == mg.STRING and index.get(rk) == (int(t["fid"]), int(t["offset"]))) else 0
                     for rk, t in recs], dtype=np.uint8)


def py_merge(file_bytes, tuples_per_file, live, data_file_size):
    """Independent restatement of merge.go:90-143 (pure Python, small inputs):
    -> ([merge data files], hint file bytes)."""
    outs, hint = [], bytearray()
    wo, i = 0, 0
    for F, tt in zip(file_bytes, tuples_per_file):
        for t in tt:
            if live[i]:
                o, h, ks, vs = int(t["offset"]), int(t["header_size"]), int(t["key_size"]), int(t["value_size"])
                key = bytes(F[o + h:o + h + ks])
                tx, n = mg.varint(key)
                rk = key[n:] if n > 0 else key
                rec = mg.encode_record(mg.put_varint(0) + rk, bytes(F[o + h + ks:o + h + ks + vs]),
                                       int(t["type"]), int(t["data_type"]), int(t["expiration"]))
                if not outs:
                    outs.append(bytearray())
                if wo + len(rec) > data_file_size:
                    outs.append(bytearray())
                    wo = 0
                outs[-1] += rec
                hint += mg.encode_record(rk, mg.put_varint(len(outs) - 1) + mg.put_varint(wo))
                wo += len(rec)
            i += 1
    return [bytes(x) for x in outs], bytes(hint)


def varlen_key(k):
    """Keys of 0..40 bytes: short ones (<= 15 B) repeat across k (more
    overwrites), long ones share their first 15 bytes and differ after."""
    n = k % 41
    if n <= 15:
        return (b"k%014d" % (k % 97))[:n]
    return (b"0123456789abcde" + b"%026d" % k)[:n]


def merge_corpus(seed, n_keys=300, rounds=3, tx_frac=0.3, key_fn=None):
    """A String-key workload with overwrites, deletes, committed and rolled-back
    transactions (the shapes db.Put/Del/WriteBatch produce) -> record bytes."""
    rng = random.Random(seed)
    key_of = key_fn or mg.test_key
    b = bytearray()
    txid = 1000
    for r in range(rounds):
        for k in rng.sample(range(n_keys), n_keys * 2 // 3):
            key = key_of(k)
            if rng.random() < tx_frac:
                txid += 1
                ops = [(key, rng.random() < 0.2)] + [(key_of(rng.randrange(n_keys)), False)
                                                     for _ in range(rng.randrange(0, 3))]
                for kk, dele in ops:
                    b += mg.encode_record(mg.key_tx(kk, txid), b"" if dele else rng.randbytes(rng.randrange(0, 300)),
                                          mg.DELETED if dele else mg.NORMAL, mg.STRING,
                                          rng.choice([0, 0, 1_700_000_000_000_000_000]))
                end = mg.TXN_ROLLBACK if rng.random() < 0.15 else mg.TXN_COMMIT
                b += mg.encode_record(mg.key_tx(b"txn-fin", txid), b"", end, mg.STRING, 0)
            elif rng.random() < 0.2:
                b += mg.encode_record(mg.key_tx(key, 0), b"", mg.DELETED, mg.STRING, 0)
            else:
                b += mg.encode_record(mg.key_tx(key, 0), rng.randbytes(rng.choice([0, 5, 50, 256, 900])),
                                      mg.NORMAL, rng.choice([0, 0, 0, 1, 2, 3, 4]), 0)
    return bytes(b)


INDEX_NOW = 1_800_000_000_000_000_000      # the clock the index tests give loadIndex (UnixNano, 2027)


def index_states(file_bytes, tuples_per_file, now_ns=INDEX_NOW):
    """db.loadIndex (db.go:582-651) restated literally: a map of buffered tx
    records per txId, updateIndex for String and ListMeta keys (with the
    expirations map of String keys), the TTL sweep (a key whose expiration is
    set and not after now is db.Del'd), then per record the state the device
    index reports: 1 = the index points at it, 2 = a Hash/List/Set record the
    host indexes (tx ones only once committed), 0 otherwise."""
    recs = []
    for F, tt in zip(file_bytes, tuples_per_file):
        for t in tt:
            o, h, ks = int(t["offset"]), int(t["header_size"]), int(t["key_size"])
            key = bytes(F[o + h:o + h + ks])
            tx, n = mg.varint(key)
            recs.append((key[n:] if n > 0 else key, t, tx))
    index = {mg.STRING: {}, mg.LISTMETA: {}}
    expirations = {}
    state = [0] * len(recs)
    txrecords = {}

    def update(i):
        rk, t, _ = recs[i]
        dt = int(t["data_type"])
        if dt in (mg.HASH, mg.LIST, mg.SET):
            state[i] = 2
        elif dt in index:
            if int(t["type"]) == mg.DELETED:
                index[dt].pop(rk, None)
                if dt == mg.STRING:
                    expirations.pop(rk, None)
            else:
                index[dt][rk] = i
                if dt == mg.STRING:
                    expirations[rk] = int(t["expiration"])

    for i, (rk, t, tx) in enumerate(recs):
        if tx == 0:
            update(i)
        elif int(t["type"]) == mg.TXN_BEGIN:
            pass
        elif int(t["type"]) == mg.TXN_COMMIT:
            for j in txrecords.pop(tx, []):
                update(j)
        elif int(t["type"]) == mg.TXN_ROLLBACK:
            txrecords.pop(tx, None)
        else:
            txrecords.setdefault(tx, []).append(i)
    # db.go:639-651: `if exp.After(time.Now()) ttl.add else db.Del(key)`
    if now_ns is not None:
        for rk, exp in expirations.items():
            if exp != 0 and not exp > now_ns:
                index[mg.STRING].pop(rk, None)
    for d in index.values():
        for i in d.values():
            state[i] = 1
    return np.array(state, np.uint8)


def py_append(records, tx_id, commit, active, write_off, data_file_size):
    """appendLogRecord over a batch restated (db.go:368-413, batch.go:62-118):
    records = [(key, value, type, dtype, exp)]; active = the active file's bytes
    (its first write_off bytes are kept).  -> ([file bytes, active first], [(fid, off)])."""
    files = [bytearray(active[:write_off])]
    pos = []
    recs = list(records)
    if commit:
        recs.append((b"\x04", b"", mg.TXN_COMMIT, mg.STRING, 0))       # public.TX_COMMIT_KEY
    for key, value, typ, dt, exp in recs:
        rec = mg.encode_record(mg.key_tx(key, tx_id), value, typ, dt, exp)
        if len(files[-1]) + len(rec) > data_file_size:
            files.append(bytearray())
        pos.append((len(files) - 1, len(files[-1])))
        files[-1] += rec
    return [bytes(f) for f in files], pos
