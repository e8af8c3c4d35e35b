// ixkey.h — the index key of a record, as db.loadIndex's updateIndex
// (db.go:511-575) and db.merge (merge.go:104-126) derive it; shared by the
// device index rebuild (clyindex.hip) and the host load driver (clyload.hip).
//
// A key is (kind, P, R): the data type, a short computed part P (<= 20 bytes)
// and a byte range R of the key as stored:
//   String (0) / ListMeta (3)   P = "",                  R = realKey
//   Hash (1)    decodeFieldKey (txnHash.go:249-251 -> bytex.DecodeByteSlices,
//               public/utils/bytex/bytex.go:46-55): key a, field b, which are
//               adjacent in the stored bytes:  P = LE32(len a), R = a || b
//   List (2)    decodeListKey (txnList.go:314-328): realKey k and the gob
//               encoding of seq re-encoded (seq.GobEncode() after
//               big.NewFloat(0).GobDecode, db.go:537-538):  P = len || seqBuf,
//               R = k
//   Set (4)     decodeMemberKey (txnSet.go:159-161) + hashMemberKey
//               (txnSet.go:149-153: consistent.HashKey = big-endian CRC-32/IEEE
//               of bytex.EncodeByteSlices(key, member),
//               public/utils/consistent/consistent.go:224-243,277-281):
//               P = BE32(crc), R = key
// Two records name the same index entry iff their (kind, P, R) are equal.
//
// The bytes decoded are log.Key: for a record applied at once (no txId) the
// key as stored, txId varint included (db.go:600-602 passes the record itself);
// for a committed tx record its realKey (db.go:620 replaced Key).  merge.go
// always decodes the realKey (merge.go:101).  A decode that panics in Go (a
// negative or out-of-range slice bound) is reported as such.
#pragma once
#include <stdint.h>

#include "scan_core.h"

#define IXK_PMAX 20

struct IxKey {
    uint32_t kind;       // data type 0..4
    uint32_t plen;       // bytes of P
    uint32_t r_off;      // R = bytes [r_off, r_off + r_len) of the decoded input
    uint32_t r_len;
    uint8_t  p[IXK_PMAX];
    bool     panic;      // the Go decode panics
};

// bytex.DecodeByteSlices(data): a = [a0, sep), b = [sep, n)
CLY_DEV bool ixk_slices(const uint8_t* d, uint32_t n, uint32_t& a0, uint32_t& sep) {
    int n1, n2;
    const int64_t v1 = go_varint(d, (int64_t)n, n1);
    if (n1 < 0) return false;                        // data[index:] with index < 0
    int64_t idx = n1;
    go_varint(d + idx, (int64_t)n - idx, n2);
    idx += n2;
    if (idx < 0) return false;                       // data[index:sep]
    if (v1 < 0 || v1 > (int64_t)n - idx) return false;   // sep < index, or data[sep:] with sep > len
    a0 = (uint32_t)idx;
    sep = (uint32_t)(idx + v1);
    return true;
}

// binary.PutVarint(x) into o; returns the bytes written
CLY_DEV int ixk_put_varint(int64_t x, uint8_t* o) {
    uint64_t ux = (uint64_t)x << 1;
    if (x < 0) ux = ~ux;
    int i = 0;
    while (ux >= 0x80) { o[i++] = (uint8_t)(ux | 0x80); ux >>= 7; }
    o[i++] = (uint8_t)ux;
    return i;
}

CLY_DEV uint32_t ixk_crc_bytes(uint32_t c, const uint8_t* p, uint32_t n) {   // c: the running (inverted) register
    for (uint32_t i = 0; i < n; i++) {
        c ^= p[i];
        for (int k = 0; k < 8; k++) c = (c >> 1) ^ (CLY_POLY & (0u - (c & 1u)));
    }
    return c;
}

CLY_DEV void ixk_be32(uint8_t* o, uint32_t v) {
    o[0] = (uint8_t)(v >> 24); o[1] = (uint8_t)(v >> 16); o[2] = (uint8_t)(v >> 8); o[3] = (uint8_t)v;
}

// seq.GobEncode() after seq := big.NewFloat(0); seq.GobDecode(buf) (errors
// ignored), math/big floatmarsh.go of Go >= 1.20 (length checks before the
// fields; a toolchain of go.mod's 1.18 panics on the short finite forms
// instead).  z starts as NewFloat(0): prec 53, ToNearestEven, so a decoded
// value is re-rounded to 53 bits (Float.SetPrec -> round) and its mode and
// accuracy reset; the result is 6, 10 or 18 bytes.  Returns the length.
CLY_DEV uint32_t ixk_gob_canon(const uint8_t* s, uint32_t n, uint8_t* o) {
    o[0] = 1;                                        // floatGobVersion
    if (n == 0) {                                    // *z = Float{}: prec 0
        o[1] = 0x08; o[2] = o[3] = o[4] = o[5] = 0;
        return 6;
    }
    if (n < 6 || s[0] != 1) {                        // error: z stays NewFloat(0)
        o[1] = 0x08; o[2] = o[3] = o[4] = 0; o[5] = 53;
        return 6;
    }
    const uint32_t b = s[1];
    uint32_t form = (b >> 1) & 3, neg = b & 1;
    const uint32_t P = ((uint32_t)s[2] << 24) | ((uint32_t)s[3] << 16) | ((uint32_t)s[4] << 8) | s[5];
    if (form != 1) {                                 // zero / inf: SetPrec(53), acc Exact, mode reset
        o[1] = (uint8_t)(0x08 | (form << 1) | neg); o[2] = o[3] = o[4] = 0; o[5] = 53;
        return 6;
    }
    if (n < 10) {                                    // error before SetPrec: fields as decoded, exp 0, no mantissa
        for (int i = 1; i < 6; i++) o[i] = s[i];
        o[6] = o[7] = o[8] = o[9] = 0;
        return 10;
    }
    int32_t exp = (int32_t)(((uint32_t)s[6] << 24) | ((uint32_t)s[7] << 16) | ((uint32_t)s[8] << 8) | s[9]);
    // mantissa nat = big-endian bytes s[10:n]; words are 8-byte groups aligned to the end
    const uint8_t* m = s + 10;
    const uint32_t L = n - 10;
    uint32_t k = 0;
    while (k < L && m[k] == 0) k++;
    uint32_t acc = 1;                                // (Accuracy + 1): Exact
    bool have = k < L;
    uint64_t top = 0;
    if (have) {
        const uint32_t wi = (L - 1 - k) / 8;         // index of the top word
        const int64_t lo = (int64_t)L - 8 * (int64_t)(wi + 1);     // first byte of the top word (may be < 0)
        for (int64_t q = lo; q < (int64_t)L - 8 * (int64_t)wi; q++) top = (top << 8) | (q >= 0 ? m[q] : 0u);
        if (P > 53) {                                // SetPrec(53) -> round(0), ToNearestEven
            const uint32_t rbit = (uint32_t)(top >> 10) & 1u;
            bool sbit = (top & 0x3ffu) != 0;
            for (uint32_t q = L - 8 * wi; q < L && !sbit; q++) sbit = m[q] != 0;
            const uint64_t lsb = 1ull << 11;
            if (rbit || sbit) {
                const bool inc = rbit && (sbit || (top & lsb));
                acc = (inc != (neg != 0)) ? 2u : 0u;  // Above : Below
                if (inc) {
                    top += lsb;
                    if (top < lsb) {                 // mantissa overflow
                        if (exp == 0x7fffffff) {     // MaxExp: z.form = inf
                            o[1] = (uint8_t)((acc << 3) | (2u << 1) | neg); o[2] = o[3] = o[4] = 0; o[5] = 53;
                            return 6;
                        }
                        exp++;
                        top = (top >> 1) | (1ull << 63);
                    }
                }
            }
            top &= ~(lsb - 1);
        }
    }
    o[1] = (uint8_t)((acc << 3) | (1u << 1) | neg);
    o[2] = o[3] = o[4] = 0; o[5] = 53;
    ixk_be32(o + 6, (uint32_t)exp);
    if (!have) return 10;
    for (int i = 0; i < 8; i++) o[10 + i] = (uint8_t)(top >> (56 - 8 * i));
    return 18;
}

// The index key of a record of data type dt whose decoded input is d[0:n]
// (see above); kind > 4: updateIndex does nothing (returns false, no panic).
CLY_DEV bool ixk_key(uint32_t dt, const uint8_t* d, uint32_t n, IxKey& k) {
    k.kind = dt; k.plen = 0; k.r_off = 0; k.r_len = n; k.panic = false;
    if (dt == 0 || dt == 3) return true;
    if (dt == 1 || dt == 4) {
        uint32_t a0, sep;
        if (!ixk_slices(d, n, a0, sep)) { k.panic = true; return false; }
        if (dt == 1) {
            const uint32_t la = sep - a0;
            k.plen = 4;
            k.p[0] = (uint8_t)la; k.p[1] = (uint8_t)(la >> 8); k.p[2] = (uint8_t)(la >> 16); k.p[3] = (uint8_t)(la >> 24);
            k.r_off = a0; k.r_len = n - a0;
        } else {
            uint8_t hdr[20];
            int h = ixk_put_varint((int64_t)(sep - a0), hdr);
            h += ixk_put_varint((int64_t)(n - sep), hdr + h);
            uint32_t c = ixk_crc_bytes(0xFFFFFFFFu, hdr, (uint32_t)h);
            c = ixk_crc_bytes(c, d + a0, n - a0);
            k.plen = 4;
            ixk_be32(k.p, ~c);
            k.r_off = a0; k.r_len = sep - a0;
        }
        return true;
    }
    if (dt == 2) {
        int n1, n2, n3;
        const int64_t sl = go_varint(d, (int64_t)n, n1);
        int64_t idx = n1;
        if (idx < 0) { k.panic = true; return false; }
        const int64_t pl = go_varint(d + idx, (int64_t)n - idx, n2);
        idx += n2;
        if (idx < 0) { k.panic = true; return false; }
        const int64_t nl = go_varint(d + idx, (int64_t)n - idx, n3);
        idx += n3;
        if (idx < 0 || sl < 0 || pl < 0 || nl < 0 || sl > (int64_t)n || pl > (int64_t)n || nl > (int64_t)n ||
            idx + sl + pl + nl > (int64_t)n) { k.panic = true; return false; }
        k.plen = 1 + ixk_gob_canon(d + idx, (uint32_t)sl, k.p + 1);
        k.p[0] = (uint8_t)(k.plen - 1);
        k.r_off = (uint32_t)(idx + sl + pl + nl);
        k.r_len = n - k.r_off;
        return true;
    }
    return false;
}

// the decoded input of a record: the stored key without a txId, its realKey with one
CLY_DEV void ixk_input(const cly_tuple& t, uint32_t& off, uint32_t& len, bool merge) {
    const uint32_t tl = t.txid_len == 0xFF ? 0u : t.txid_len;
    if (t.tx_id == 0 && !merge) { off = 0; len = t.key_size; }
    else { off = tl; len = t.key_size - tl; }
}

// 64-bit hash of (index kind, key bytes): FNV-1a over 8-byte words folded by a
// mix; the device index sorts on it (clyindex.hip) and the load driver's String
// / ListMeta tables use the same values (downloaded, not recomputed).
CLY_DEV uint64_t ixk_hash(uint32_t kind, const uint8_t* k, uint32_t len) {
    uint64_t h = 0xcbf29ce484222325ull ^ ((uint64_t)kind << 56) ^ len;
    uint32_t q = 0;
    for (; q + 8 <= len; q += 8) {
        uint64_t w = 0;
        for (int b = 0; b < 8; b++) w |= (uint64_t)k[q + b] << (8 * b);
        h = (h ^ w) * 0x100000001b3ull;
        h ^= h >> 29;
    }
    uint64_t w = 0;
    for (int b = 0; q < len; q++, b++) w |= (uint64_t)k[q] << (8 * b);
    h = (h ^ w) * 0x100000001b3ull;
    h ^= h >> 32;
    h *= 0xd6e8feb86659fd93ull;
    h ^= h >> 32;
    return h;
}
