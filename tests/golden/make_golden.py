#!/usr/bin/env python3
"""Generate the committed golden fixtures for the log-record scan.

TEST INFRASTRUCTURE.  This is an independent Python restatement of the
reference path (it does not use the C oracle):
  * writer side: EncodeLogRecord (data/logRecord.go:57-84), encodeKeyWithTxId
    (batch.go:120-127), bytex.EncodeByteSlices (public/utils/bytex/bytex.go:35-46),
    file rotation in appendLogRecord (db.go:376-385);
  * reader side: ReadLogRecord (data/dataFile.go:64-111) + DecodeLogRecordHeader
    (data/logRecord.go:86-114) + GetLogRecordCRC (data/logRecord.go:136-146) +
    parseLogRecordKey (db.go:706-710), with Go encoding/binary Varint semantics;
  * CRC-32/IEEE from zlib.crc32 (same polynomial/init/xorout as Go's
    crc32.ChecksumIEEE; check value 0xCBF43926).

Run:  python tests/golden/make_golden.py   (rewrites tests/golden/*.cly/*.json)
The reference itself (Go) cannot be run here, so these vectors pin parity to
the restatement, not to the Go binary ("parity unpinned by the reference").
"""
import json
import os
import random
import struct
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))

END_EOF, END_ZERO, END_TORN = 0, 1, 2
ERR_CRC, ERR_TRUNC5, ERR_VARINT, ERR_OFFSET = -1, -2, -3, -4
NORMAL, DELETED, TXN_COMMIT, TXN_ROLLBACK, TXN_BEGIN = 0, 1, 2, 3, 4
STRING, HASH, LIST, LISTMETA, SET = 0, 1, 2, 3, 4
TX_COMMIT_KEY, TX_ROLLBACK_KEY, TX_BEGIN_KEY, MERGE_FIN_KEY = b"\x04", b"\x15", b"\x12", b"\x07"


# ---- Go encoding/binary ---------------------------------------------------
def put_uvarint(ux):
    out = bytearray()
    while ux >= 0x80:
        out.append((ux & 0x7F) | 0x80)
        ux >>= 7
    out.append(ux)
    return bytes(out)


def put_varint(x):
    ux = (x << 1) & 0xFFFFFFFFFFFFFFFF
    if x < 0:
        ux = ~ux & 0xFFFFFFFFFFFFFFFF
    return put_uvarint(ux)


def uvarint(buf):
    x, s = 0, 0
    for i, b in enumerate(buf):
        if i == 10:
            return 0, -(i + 1)
        if b < 0x80:
            if i == 9 and b > 1:
                return 0, -(i + 1)
            return (x | (b << s)) & 0xFFFFFFFFFFFFFFFF, i + 1
        x |= (b & 0x7F) << s
        s += 7
    return 0, 0


def varint(buf):
    ux, n = uvarint(buf)
    x = ux >> 1
    if ux & 1:
        x = ~x & 0xFFFFFFFFFFFFFFFF
    if x >= 1 << 63:
        x -= 1 << 64
    return x, n


def crc32(b):
    return zlib.crc32(b) & 0xFFFFFFFF


# ---- GF(2) arithmetic of the CRC-32 register (fixture construction only) ----
# Register convention: the reflected register Go's crc32.Update keeps; one zero
# byte through it is the linear map A: s -> T0[s & 0xff] ^ (s >> 8), and A^n is
# multiplication by x^(8n) mod P (bit 31 = x^0).
POLY = 0xEDB88320


def gf_mul(a, b):
    p = 0
    for k in range(31, -1, -1):
        if a & (1 << k):
            p ^= b
        b = (b >> 1) ^ POLY if b & 1 else b >> 1
    return p


def gf_x8n(n):
    p, sq = 1 << 31, 1 << 23
    while n:
        if n & 1:
            p = gf_mul(sq, p)
        sq = gf_mul(sq, sq)
        n >>= 1
    return p


def crc_shift(v, n):
    """A^n v: the register v after n zero bytes."""
    return gf_mul(gf_x8n(n), v) if n else v


def _t0(i):
    for _ in range(8):
        i = (i >> 1) ^ POLY if i & 1 else i >> 1
    return i


_T0 = [_t0(i) for i in range(256)]
_T0_INV = {t >> 24: i for i, t in enumerate(_T0)}


def crc_unshift(v, n):
    """A^-n v (the top byte of T0 is a permutation of the index)."""
    for _ in range(n):
        i = _T0_INV[v >> 24]
        v = (((v ^ _T0[i]) << 8) & 0xFFFFFFFF) | i
    return v


def record_bounds(F):
    """(offset, size) of every record the reader returns."""
    out, off = [], 0
    while True:
        st, t = read_log_record(F, off)
        if st is not None:
            return out
        out.append((off, t["size"]))
        off += t["size"]


def file_fold(F):
    """The per-file linear fold of the records' CRC residues, each shifted to the
    end of the file: sum_k A^(E - end_k) (crc32(record k) ^ stored_k).  A GF(2)
    sum, so two non-zero residues can cancel; a verdict taken from this fold
    alone misses such files, while ReadLogRecord checks every record
    (data/dataFile.go:105-109)."""
    recs = record_bounds_lenient(F)
    E = recs[-1][0] + recs[-1][1] if recs else 0
    s = 0
    for off, size in recs:
        res = crc32(F[off + 4: off + size]) ^ struct.unpack_from("<I", F, off)[0]
        if res:
            s ^= crc_shift(res, E - off - size)
    return s


def record_bounds_lenient(F):
    """Record framing only (header sizes), ignoring the CRC: the chain a decoder
    that does not stop at ErrInvalidCRC would walk."""
    out, off = [], 0
    while True:
        hb = F[off:off + 26]
        if len(hb) <= 5:
            return out
        idx = 6
        ks, a = varint(hb[idx:]); idx += a
        vs, b = varint(hb[idx:]); idx += b
        _, c = varint(hb[idx:]); idx += c
        if a <= 0 or b <= 0 or c <= 0:
            return out
        size = idx + (ks & 0xFFFFFFFF) + (vs & 0xFFFFFFFF)
        if off + size > len(F) or (struct.unpack_from("<I", F, off)[0] == 0 and ks == 0 and vs == 0):
            return out
        out.append((off, size))
        off += size


def cancel_stored(F, i, j, delta):
    """XOR delta into record i's stored CRC and A^(end_j - end_i) delta into record
    j's: both records fail their own CRC check, yet their residues cancel in the
    per-file fold.  The reference stops at record i with ErrInvalidCRC."""
    b = bytearray(F)
    recs = record_bounds_lenient(F)
    (oi, si), (oj, sj) = recs[i], recs[j]
    d2 = crc_shift(delta, (oj + sj) - (oi + si))
    struct.pack_into("<I", b, oi, struct.unpack_from("<I", b, oi)[0] ^ delta)
    struct.pack_into("<I", b, oj, struct.unpack_from("<I", b, oj)[0] ^ d2)
    return bytes(b)


def cancel_payload(F, i, pos_i, bit, j):
    """Flip one payload bit of record i (at offset pos_i inside it) and XOR into
    the last 4 payload bytes of record j the word whose CRC syndrome cancels the
    first in the per-file fold (4 bytes at the record end change the register
    by A^4 v, so v = A^-4 of the wanted residue)."""
    b = bytearray(F)
    recs = record_bounds_lenient(F)
    (oi, si), (oj, sj) = recs[i], recs[j]
    before = crc32(bytes(b[oi + 4: oi + si]))
    b[oi + pos_i] ^= 1 << bit
    res_i = crc32(bytes(b[oi + 4: oi + si])) ^ before
    want = crc_shift(res_i, (oj + sj) - (oi + si))
    v = crc_unshift(want, 4)
    w = struct.unpack_from("<I", b, oj + sj - 4)[0] ^ v
    struct.pack_into("<I", b, oj + sj - 4, w)
    return bytes(b)


# ---- writer side -----------------------------------------------------------
def encode_record(key, value, typ=NORMAL, dtype=STRING, exp=0):
    hdr = bytes([typ, dtype]) + put_varint(len(key)) + put_varint(len(value)) + put_varint(exp)
    body = hdr + key + value
    return struct.pack("<I", crc32(body)) + body


def key_tx(key, tx_id):
    return put_varint(tx_id) + key


def enc_slices(a, b):
    return put_varint(len(a)) + put_varint(len(b)) + a + b


def test_key(i):
    return b"%09d" % i


# ---- reader side (exact ReadLogRecord semantics) ---------------------------
def read_log_record(F, off):
    n = len(F)
    hb = 26 if off + 26 <= n else n - off
    buf = F[off:off + hb]
    if hb <= 4:
        return END_EOF, None
    if hb == 5:
        return ERR_TRUNC5, None
    crc = struct.unpack_from("<I", buf, 0)[0]
    typ, dtype = buf[4], buf[5]
    idx = 6
    ks, a = varint(buf[idx:]); idx += a
    if idx < 0:
        return ERR_VARINT, None
    vs, b = varint(buf[idx:]); idx += b
    if idx < 0:
        return ERR_VARINT, None
    exp, c = varint(buf[idx:]); idx += c
    KS, VS = ks & 0xFFFFFFFF, vs & 0xFFFFFFFF
    if crc == 0 and KS == 0 and VS == 0:
        return END_ZERO, None
    kv = KS + VS
    if kv > 0:
        koff = off + idx
        if koff < 0 or koff > n:
            return ERR_OFFSET, None
        if n - koff < kv:
            return END_TORN, None
    if idx < 4:
        return ERR_VARINT, None
    if crc32(F[off + 4: off + idx + kv]) != crc:
        return ERR_CRC, None
    key = F[off + idx: off + idx + KS]
    tx, tn = varint(key)
    if tn < 0:
        tx, tlen = 0, 0xFF
    else:
        tlen = tn
    return None, dict(offset=off, expiration=exp, tx_id=tx, size=idx + kv, key_size=KS,
                      value_size=VS, type=typ, data_type=dtype, header_size=idx,
                      txid_len=tlen, crc=crc)


FIELDS = ["offset", "expiration", "tx_id", "fid", "size", "key_size", "value_size",
          "type", "data_type", "header_size", "txid_len", "crc"]


def scan(F, fid):
    off, tuples = 0, []
    while True:
        st, t = read_log_record(F, off)
        if st is not None:
            return st, off, tuples
        t["fid"] = fid
        tuples.append([t[f] for f in FIELDS])
        off += t["size"]


# ---- fixtures ----------------------------------------------------------------
def fixtures():
    rng = random.Random(0x434C59)
    fx = {}

    # 1. anchor: db.Put("000000001", "000000001")
    fx["anchor"] = encode_record(key_tx(b"000000001", 0), b"000000001")

    # 2. C1 shape (config 1), truncated: key 0x00||%09d, 1 KiB random value
    b = bytearray()
    for i in range(240):
        b += encode_record(key_tx(test_key(i), 0), bytes(rng.getrandbits(8) for _ in range(1024)))
    fx["c1_shape"] = bytes(b)

    # 3. TestTxn_Hash_Restart: Begin, 3x HSet, HDel, Commit (txnHash_test.go:179-223)
    tx = 1_697_000_000_000_000_000 + 17
    b = bytearray()
    b += encode_record(key_tx(TX_BEGIN_KEY, tx), b"", TXN_BEGIN)
    for k, f in [(0, 0), (1, 1), (1, 2)]:
        b += encode_record(key_tx(enc_slices(test_key(k), test_key(f)), tx), test_key(f), NORMAL, HASH)
    b += encode_record(key_tx(enc_slices(test_key(1), test_key(2)), tx), b"", DELETED, HASH)
    b += encode_record(key_tx(TX_COMMIT_KEY, tx), b"", TXN_COMMIT)
    fx["txn_hash"] = bytes(b)

    # 4. TestTxn_List_Restart shape: ListMeta + List records with opaque seq blobs
    tx2 = tx + 5
    b = bytearray()
    b += encode_record(key_tx(TX_BEGIN_KEY, tx2), b"", TXN_BEGIN)
    for i in range(4):
        seq = bytes([1, 2, 0, 0x80 + i, 3 * i])
        lk = put_varint(len(seq)) * 3 + seq * 3 + b"mylist"
        b += encode_record(key_tx(lk, tx2), test_key(i), NORMAL, LIST)
    meta = put_varint(5) + put_varint(5) + bytes(10)
    b += encode_record(key_tx(b"mylist", tx2), meta, NORMAL, LISTMETA)
    b += encode_record(key_tx(TX_COMMIT_KEY, tx2), b"", TXN_COMMIT)
    fx["txn_list"] = bytes(b)

    # 5. TTL record (ttl_test.go:55-88): UnixNano expiration -> 9-byte varint
    b = bytearray()
    b += encode_record(key_tx(test_key(0), 0), b"AbCdEfGhIjKlMnOpQrStUvWx", exp=1_697_000_002_000_000_000)
    b += encode_record(key_tx(test_key(1), 0), b"v", exp=-5)
    fx["ttl"] = bytes(b)

    # 6. WriteBatch (batch.go:62-118): tx records + Commit, no Begin; plus a Set record
    tx3 = tx + 9
    b = bytearray()
    for i in range(5):
        b += encode_record(key_tx(test_key(i), tx3), b"batch-%d" % i)
    b += encode_record(key_tx(test_key(2), tx3), b"", DELETED)
    b += encode_record(key_tx(TX_COMMIT_KEY, tx3), b"", TXN_COMMIT)
    b += encode_record(key_tx(enc_slices(b"myset", b"m1"), 0), b"", NORMAL, SET)
    fx["write_batch"] = bytes(b)

    # 7. rollback
    tx4 = tx + 11
    b = bytearray()
    b += encode_record(key_tx(TX_BEGIN_KEY, tx4), b"", TXN_BEGIN)
    b += encode_record(key_tx(test_key(7), tx4), b"gone")
    b += encode_record(key_tx(TX_ROLLBACK_KEY, tx4), b"", TXN_ROLLBACK)
    fx["rollback"] = bytes(b)

    # 8. TestDB_Reboot shape: value = key || 1024 zero bytes, then a zero tail
    b = bytearray()
    for i in range(60):
        k = test_key(i)
        b += encode_record(key_tx(k, 0), k + bytes(1024))
    fx["zero_values"] = bytes(b)
    zrec = len(b) // 60
    fx["zero_tail"] = bytes(b[: 20 * zrec]) + bytes(3000)
    fx["zero_tail_mid"] = bytes(b[: 20 * zrec - 500]) + bytes(3000)

    # 9. tails (after whole C1-shape records)
    base = fx["c1_shape"][: 3 * 1044]
    for t in range(0, 6):
        fx["tail_%d" % t] = base + bytes([0x5A]) * t
    rec = encode_record(key_tx(b"tailkey", 0), b"tailvalue-0123456789")
    for t in (6, 9, 12, 25):
        fx["torn_header_%d" % t] = base + rec[:t]
    fx["torn_kv"] = base + rec[:-3]
    # empty file
    fx["empty"] = b""

    # 10. one flipped bit -> ERR_CRC (value byte of record 5)
    b = bytearray(fx["c1_shape"][: 10 * 1044])
    b[5 * 1044 + 500] ^= 0x10
    fx["bitflip"] = bytes(b)
    # header corruption: size field of record 3 changed (usually ERR_CRC, may hop)
    b = bytearray(fx["c1_shape"][: 10 * 1044])
    b[3 * 1044 + 7] ^= 0x02
    fx["bitflip_header"] = bytes(b)

    # 11. hint file (data/dataFile.go:114-121) + merge-finished (merge.go:154-168)
    b = bytearray()
    for i in range(50):
        pos = put_varint(i % 3) + put_varint(1044 * i)
        b += encode_record(test_key(i), pos)
    fx["hint_index"] = bytes(b)
    fx["merge_finished"] = encode_record(MERGE_FIN_KEY, b"12")

    # 12. adversarial: values embedding valid encoded records (+ hint payloads)
    b = bytearray()
    inner = b"".join(encode_record(key_tx(test_key(900 + j), 0), b"inner") for j in range(6))
    for i in range(30):
        b += encode_record(key_tx(test_key(i), 0), inner * (1 + i % 3))
    fx["embedded_records"] = bytes(b)

    # varint edge cases in headers (reference semantics, not writer output)
    def raw(hdr_tail, kv=b"", crc=None, typ=0, dt=0):
        body = bytes([typ, dt]) + hdr_tail + kv
        c = crc32(body) if crc is None else crc
        return struct.pack("<I", c) + body
    good = encode_record(key_tx(b"k", 0), b"v")
    # negative key size -> uint32 huge -> torn -> io.EOF
    fx["neg_size"] = good + raw(put_varint(-1) + put_varint(1) + put_varint(0), b"xx")
    # 10-byte varint overflow in the key size -> slice panic
    fx["varint_overflow"] = good + raw(b"\xff" * 9 + b"\x02" + b"\x00\x00", bytes(16))
    # overflow in the value size after a 9-byte key size: index returns to 5 (no panic)
    fx["varint_overflow2"] = good + raw(b"\x81" + b"\x80" * 7 + b"\x00" + b"\xff" * 9 + b"\x02", bytes(40))
    # ks == 0 with crc != 0 is a legal record for the reader
    fx["ks_zero"] = raw(put_varint(0) + put_varint(3) + put_varint(0), b"abc") + good
    # type/dtype outside the enums are legal for the reader
    fx["odd_type"] = raw(put_varint(2) + put_varint(2) + put_varint(0), b"\x00kvv", typ=9, dt=200) + good
    # header-only garbage with a valid CRC over 2 bytes (6-byte file tail)
    fx["six_tail"] = good + raw(b"", b"", typ=1, dt=2)
    # big keys
    fx["big_record"] = encode_record(key_tx(bytes(range(256)) * 4, 0), bytes(rng.getrandbits(8) for _ in range(70000)))

    # 13. CRC residues that cancel in a per-file linear fold: two (or three)
    # records fail their own check, the file's fold of residues is zero.  The
    # reference returns ErrInvalidCRC at the first of them (dataFile.go:105-109).
    c2 = b"".join(encode_record(key_tx(test_key(i), 0), bytes(rng.getrandbits(8) for _ in range(256)))
                  for i in range(300))                                   # C2 shape, 82 800 B: > one 64-KiB tile
    fx["crc_cancel_near"] = cancel_stored(c2, 2, 5, 0x1D)
    fx["crc_cancel_far"] = cancel_stored(c2, 3, 260, 0x80000001)
    fx["crc_cancel_payload"] = cancel_payload(c2, 10, 130, 3, 200)
    three = cancel_stored(c2, 40, 41, 0xDEADBEEF)                        # i, i+1 cancel ...
    fx["crc_cancel_three"] = cancel_stored(three, 41, 250, 0x00C0FFEE)  # ... and a third pair on top
    tiny = bytearray()
    for i in range(2000):                                                # 11-14 B records, unaligned starts
        tiny += encode_record(key_tx(bytes([i & 0xFF]), 0), bytes(rng.getrandbits(8) for _ in range(i % 4)))
    fx["crc_cancel_tiny"] = cancel_stored(bytes(tiny), 700, 701, 0x5A5A5A5A)
    fx["crc_cancel_tiny_far"] = cancel_payload(bytes(tiny), 101, 10, 0, 1903)
    for name in ("crc_cancel_near", "crc_cancel_far", "crc_cancel_payload", "crc_cancel_three",
                 "crc_cancel_tiny", "crc_cancel_tiny_far"):
        assert file_fold(fx[name]) == 0, name                            # the fold passes ...
        assert scan(fx[name], 0)[0] == ERR_CRC, name                     # ... the reference does not
    return fx


def main():
    fx = fixtures()
    manifest = {}
    for i, (name, data) in enumerate(sorted(fx.items())):
        fid = 100 + i
        st, end, tuples = scan(data, fid)
        with open(os.path.join(HERE, name + ".cly"), "wb") as f:
            f.write(data)
        manifest[name] = dict(fid=fid, len=len(data), status=st, end_offset=end,
                              n_records=len(tuples), tuples=tuples)
    vec = dict(
        crc32_check=[["313233343536373839", 0xCBF43926], ["", 0], ["00", crc32(b"\x00")],
                     [fx["anchor"][4:].hex(), crc32(fx["anchor"][4:])]],
        anchor_hex=fx["anchor"].hex(),
        varint=[],
    )
    cases = [b"\x00", b"\x01", b"\x02", b"\x7f", b"\x80\x01", b"\xff\x01", b"\x80", b"",
             put_varint(1 << 31), put_varint(-(1 << 31)), put_varint(1_697_000_000_000_000_017),
             put_varint((1 << 63) - 1), put_varint(-(1 << 63)), b"\xff" * 9 + b"\x01",
             b"\xff" * 9 + b"\x02", b"\xff" * 10 + b"\x00", b"\xff" * 10, b"\x80" * 10 + b"\x01"]
    for c in cases:
        v, n = varint(c)
        vec["varint"].append([c.hex(), v, n])
    manifest["_vectors"] = vec
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(manifest, f, indent=0, sort_keys=True)
    print("wrote %d fixtures (%d bytes)" % (len(fx), sum(len(v) for v in fx.values())))
    for name in sorted(fx):
        m = manifest[name]
        print("  %-20s len=%-7d n=%-4d status=%d end=%d" % (name, m["len"], m["n_records"], m["status"], m["end_offset"]))


if __name__ == "__main__":
    main()
