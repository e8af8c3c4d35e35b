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


def mixed_corpus(seed, target_bytes, corrupt=0, tail=True, dts=(0, 0, 0, 1, 2, 3, 4)):
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
        dt = rng.choice(dts)
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
                                      mg.NORMAL, rng.choice([0, 0, 0, 3, 5, 6, 9]), 0)
    return bytes(b)


def _nc_varint(x, rng):
    """binary.PutVarint(x), sometimes in a longer (non-minimal) form that
    binary.Varint still reads as x."""
    b = bytearray(mg.put_varint(x))
    if rng.random() < 0.5 and len(b) < 9:
        b[-1] |= 0x80
        b += b"\x00"
    return bytes(b)


def seq_variant(v, rng):
    """A gob buffer for list seq v: the writer's encoding, or another buffer of
    the kinds GobDecode accepts (mode/accuracy bits, other precisions with or
    without rounding, longer or zero-padded mantissas, the error forms)."""
    from .index_keys import gob_encode_int
    g = bytearray(gob_encode_int(v))
    c = rng.randrange(14)
    if c < 4:
        return bytes(g)
    if c == 4:                                   # accuracy / mode bits (reset by SetPrec)
        g[1] |= rng.choice([0x10, 0x18, 0x20, 0xa0])
    elif c == 5 and len(g) == 18:                # prec 64, low bits that round (or not)
        g[2:6] = (64).to_bytes(4, "big")
        m = int.from_bytes(g[10:18], "big") | rng.choice([0, 0x1, 0x3ff, 0x400, 0x7ff, 0xc00, 0x800])
        g[10:18] = m.to_bytes(8, "big")
    elif c == 6 and len(g) == 18:                # prec 24: no rounding, prec re-set to 53
        g[2:6] = (24).to_bytes(4, "big")
    elif c == 7 and len(g) == 18:                # two-word mantissa / leading zero bytes
        g += bytes([rng.choice([0, 0, 5])]) * rng.choice([1, 8])
        if rng.random() < 0.5:
            g[10:10] = bytes(rng.randrange(1, 9))
    elif c == 8:
        return b""
    elif c == 9:
        return bytes(g[:rng.randrange(1, 6)])   # short: error, NewFloat(0)
    elif c == 10:
        g[0] = 2                                  # unsupported version
    elif c == 11:
        g[1] = (g[1] & ~0x06) | 0x04              # inf form
    elif c == 12 and len(g) == 18:
        return bytes(g[:rng.randrange(6, 10)])   # finite, shorter than 10 bytes
    elif c == 13 and len(g) == 18:               # prec 200, all-ones low mantissa (carry)
        g[2:6] = (200).to_bytes(4, "big")
        g[10:18] = (int.from_bytes(g[10:18], "big") | ((1 << 11) - 1)).to_bytes(8, "big")
        g += b"\xff" * rng.choice([0, 8])
    return bytes(g)


def typed_corpus(seed, n_ops=400, n_keys=12, tx_frac=0.6, nontx_frac=0.15, garbage=False):
    """Records of all five data types as the reference's writers produce them
    (Put/Del; HSet/HDel txnHash.go:9-90; LPush/RPush/LPop/RPop with their
    ListMeta records txnList.go:96-232; SAdd/SRem txnSet.go:11-90) in committed,
    rolled-back and unterminated transactions, plus records without a txId
    (as a merge rewrites them) and equivalent non-canonical encodings of the
    composite keys (longer varints, other gob forms of a list seq).
    garbage=True adds rolled-back Hash/Set/List records whose keys do not decode
    (merge.go would panic on them; loadIndex never decodes them)."""
    from .index_keys import encode_list_meta
    rng = random.Random(seed)
    b = bytearray()
    txid = 5000
    lists = {}                                   # key -> [head, tail]

    def rec(key, value, typ, dt, tx):
        return mg.encode_record(mg.key_tx(key, tx), value, typ, dt, 0)

    def ops_one(tx):
        out = []
        k = b"key%02d" % rng.randrange(n_keys)
        what = rng.randrange(5)
        dele = rng.random() < 0.25
        if what == 0:                            # String / ListMeta by realKey
            out.append(rec(k, b"" if dele else rng.randbytes(rng.randrange(0, 40)), mg.DELETED if dele else mg.NORMAL,
                           rng.choice([mg.STRING, mg.STRING, mg.LISTMETA]), tx))
        elif what == 1:                          # Hash
            f = b"f%d" % rng.randrange(6)
            key = _nc_varint(len(k), rng) + _nc_varint(rng.choice([len(f), len(f), 99, -3]), rng) + k + f
            out.append(rec(key, b"" if dele else rng.randbytes(rng.randrange(0, 20)), mg.DELETED if dele else mg.NORMAL,
                           mg.HASH, tx))
        elif what == 2:                          # Set
            m = b"m%d" % rng.randrange(6)
            key = _nc_varint(len(k), rng) + _nc_varint(rng.choice([len(m), len(m), 7]), rng) + k + m
            out.append(rec(key, b"" if dele else m, mg.DELETED if dele else mg.NORMAL, mg.SET, tx))
        else:                                    # List push / pop + its ListMeta record
            head, tail = lists.get(k, [1, 0])
            left = rng.random() < 0.5
            if dele and head <= tail:
                seq = head if left else tail
                prev, nxt = seq - 1, seq + 1
                if left:
                    head += 1
                else:
                    tail -= 1
                typ, val = mg.DELETED, b""
            else:
                seq = head - 1 if left else tail + 1
                prev, nxt = (seq - 1, head) if left else (tail, seq + 1)
                if left:
                    head = seq
                else:
                    tail = seq
                typ, val = mg.NORMAL, rng.randbytes(rng.randrange(0, 20))
            a, p, n = seq_variant(seq, rng), seq_variant(prev, rng), seq_variant(nxt, rng)
            key = _nc_varint(len(a), rng) + _nc_varint(len(p), rng) + _nc_varint(len(n), rng) + a + p + n + k
            out.append(rec(key, val, typ, mg.LIST, tx))
            lists[k] = [head, tail]
            out.append(rec(k, encode_list_meta(head, tail), mg.NORMAL, mg.LISTMETA, tx))
        return out

    while len(b) < 1 or n_ops > 0:
        n_ops -= 1
        r = rng.random()
        if r < tx_frac:
            txid += 1
            body = []
            for _ in range(rng.randrange(1, 5)):
                body += ops_one(txid)
            end = rng.random()
            if garbage and rng.random() < 0.2:
                body.append(rec(rng.choice([b"zz", b"\x7f\x7f", b"\x02"]), b"", mg.NORMAL,
                                rng.choice([mg.HASH, mg.LIST, mg.SET]), txid))
                end = 0.8                        # rolled back
            if rng.random() < 0.3:
                b += rec(mg.TX_BEGIN_KEY, b"", mg.TXN_BEGIN, mg.STRING, txid)
            for x in body:
                b += x
            if end < 0.7:
                b += rec(mg.TX_COMMIT_KEY, b"", mg.TXN_COMMIT, mg.STRING, txid)
            elif end < 0.9:
                b += rec(mg.TX_ROLLBACK_KEY, b"", mg.TXN_ROLLBACK, mg.STRING, txid)
        elif r < tx_frac + nontx_frac:
            for x in ops_one(0):
                b += x
        else:
            for x in ops_one(0):
                b += x
    return bytes(b)


INDEX_NOW = 1_800_000_000_000_000_000      # the clock the index tests give loadIndex (UnixNano, 2027)


def hint_entries(hint_bytes):
    """loadIndexFromHintFile's reading (merge.go:257-287) restated: the hint
    file's records in order -> [(stored key, fid, offset)] (DecodeLogRecordPos
    of each value, data/logRecord.go:126-134)."""
    out, off = [], 0
    while True:
        st, t = mg.read_log_record(hint_bytes, off)
        if st is not None:
            break
        h, ks = t["header_size"], t["key_size"]
        key = bytes(hint_bytes[off + h:off + h + ks])
        val = bytes(hint_bytes[off + h + ks:off + t["size"]])
        fid, n = mg.varint(val)
        o, _ = mg.varint(val[n:])
        out.append((key, fid & 0xFFFFFFFF, o))
        off += t["size"]
    return out


def index_states(file_bytes, tuples_per_file, now_ns=INDEX_NOW, merge_panics=None, out_index=None, preload=None):
    """db.loadIndex (db.go:582-651) restated literally: a map of buffered tx
    records per txId, updateIndex for the five indexes (String/ListMeta by
    realKey, Hash/List/Set by the composite keys of tests/index_keys.py decoded
    from log.Key: the stored key for a record applied at once, the realKey for
    a committed tx record), the expirations map of String keys and the TTL
    sweep (a key whose expiration is set and not after now is db.Del'd).  Per
    record the state the device index reports: 1 = an index points at it and
    merge.go's lookup (merge.go:101-132, realKey decoded) finds it, 3 = an
    index points at it under a key merge.go does not look up, 4 = the winning
    put of a String key the TTL sweep removes, 0 otherwise.
    Raises index_keys.GoPanic where updateIndex's decode panics; merge_panics
    (a list) receives the records whose merge.go decode panics.  preload: the
    hint file's [(key, fid, offset)] put into the String index before the data
    files (loadIndexFromHintFile); a key the data files Put or Del later is
    theirs (out_index holds (key, fid, offset, 0) for the other ones)."""
    from .index_keys import GoPanic, index_key
    recs = []
    for F, tt in zip(file_bytes, tuples_per_file):
        for t in tt:
            o, h, ks = int(t["offset"]), int(t["header_size"]), int(t["key_size"])
            key = bytes(F[o + h:o + h + ks])
            tx, n = mg.varint(key)
            recs.append((key, key[n:] if n > 0 else key, t, tx))
    index = {}                      # index key -> record (all five indexes, flattened)
    pre = {k: (f, o) for k, f, o in (preload or [])}
    touched = set()                 # String keys a data-file record Put or Del
    expirations = {}
    state = [0] * len(recs)
    txrecords = {}

    def update(i, log_key):
        _, rk, t, _ = recs[i]
        dt = int(t["data_type"])
        if dt in (mg.STRING, mg.LISTMETA):
            ik = (dt, rk)           # updateIndex's key argument: the realKey
        else:
            ik = index_key(dt, log_key)
            if ik is None:
                return
        if dt == mg.STRING:
            touched.add(rk)
        if int(t["type"]) == mg.DELETED:
            index.pop(ik, None)
            if dt == mg.STRING:
                expirations.pop(rk, None)
        else:
            index[ik] = i
            if dt == mg.STRING:
                expirations[rk] = int(t["expiration"])

    for i, (key, rk, t, tx) in enumerate(recs):
        if tx == 0:
            update(i, key)
        elif int(t["type"]) == mg.TXN_BEGIN:
            pass
        elif int(t["type"]) == mg.TXN_COMMIT:
            for j in txrecords.pop(tx, []):
                update(j, recs[j][1])
        elif int(t["type"]) == mg.TXN_ROLLBACK:
            txrecords.pop(tx, None)
        else:
            txrecords.setdefault(tx, []).append(i)
    # db.go:639-651: `if exp.After(time.Now()) ttl.add else db.Del(key)`; the
    # device marks the swept key's winning put 4 (CLY_IX_EXPIRED)
    swept = []
    if now_ns is not None:
        for rk, exp in expirations.items():
            if exp != 0 and not exp > now_ns:
                i = index.pop((mg.STRING, rk), None)
                if i is not None:
                    swept.append(i)
    if out_index is not None:
        out_index.update({(mg.STRING, k): (k, f, o, 0) for k, (f, o) in pre.items() if k not in touched})
        out_index.update({ik: (recs[i][0], int(recs[i][2]["fid"]), int(recs[i][2]["offset"]), recs[i][3])
                          for ik, i in index.items()})
    for ik, i in index.items():
        _, rk, t, _ = recs[i]
        try:
            mk = index_key(int(t["data_type"]), rk)
        except GoPanic:
            mk = None
        state[i] = 1 if mk == ik else 3
    for i in swept:
        state[i] = 4
    if merge_panics is not None:
        for i, (_, rk, t, _) in enumerate(recs):
            if int(t["data_type"]) in (mg.HASH, mg.LIST, mg.SET):
                try:
                    index_key(int(t["data_type"]), rk)
                except GoPanic:
                    merge_panics.append(i)
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
