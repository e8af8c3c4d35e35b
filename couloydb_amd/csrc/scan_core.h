// scan_core.h — definitions shared by the kernels of libclyscan (gfx950): the
// exact per-record semantics of the reference and the scan geometry.
//
// Reference semantics restated here: DataFile.ReadLogRecord
// (data/dataFile.go:64-111), DecodeLogRecordHeader (data/logRecord.go:86-114),
// Go's encoding/binary Varint (toolchain >= 1.18, go.mod:3) and
// parseLogRecordKey (db.go:706-710).
//
// Work decomposition of the scan:
//   segment  CLY_SEG = 64 consecutive bytes, owned by one lane for one block
//   block    64 segments = 4 KiB, read by one wave with four coalesced 1-KiB
//            load instructions and transposed so that lane L holds segment L
//   tile     CLY_NBLK consecutive blocks of one file, owned by one wave, which
//            streams them in order; tiles are the unit of the chain link
//            (record counts and chain state between tiles, k_link)
#pragma once
#include <stdint.h>

#include "../../include/clyscan.h"
#include "crc_gf.h"

#define CLY_DEV __host__ __device__ __forceinline__     // host too: clyload.hip's getLogRecordByPos
#define CLY_LDS __attribute__((address_space(3)))

#ifndef CLY_NBLK
#define CLY_NBLK 16           // blocks per tile (the test build uses 2: 8-KiB tiles)
#endif
#define CLY_SEG 64                                // bytes per lane per block
#define CLY_NL 64                                 // lanes (segments) per block
#define CLY_BLK (CLY_NL * CLY_SEG)                // block bytes (4 KiB)
#define CLY_TILE ((int64_t)CLY_NBLK * CLY_BLK)    // tile bytes
static_assert(CLY_NBLK >= 1 && CLY_TILE <= 65536, "tile-relative record offsets are u16");

#define REC_OK 100

// ---------------------------------------------------------------------------
// Go encoding/binary Varint: zigzag over Uvarint; overflow (10th byte > 1, or an
// 11th byte) -> (0, -(i+1)); short buffer -> (0, 0).
template <class BP>
CLY_DEV int64_t go_varint(BP b, int64_t len, int& n) {
    uint64_t x = 0;
    unsigned s = 0;
    const int lim = len < 11 ? (int)len : 11;
    for (int i = 0; i < lim; i++) {
        const uint32_t c = b[i];
        if (i == 10) { n = -11; return 0; }
        if (c < 0x80) {
            if (i == 9 && c > 1) { n = -10; return 0; }
            n = i + 1;
            const uint64_t ux = x | ((uint64_t)c << s);
            const int64_t v = (int64_t)(ux >> 1);
            return (ux & 1) ? ~v : v;
        }
        x |= (uint64_t)(c & 0x7f) << s;
        s += 7;
    }
    n = 0;
    return 0;
}

struct Hdr {
    int32_t  status;    // REC_OK or a terminal status (CLY_END_* / CLY_ERR_* except CRC)
    int32_t  hsz;       // headerSize
    int64_t  size;      // recordSize (REC_OK)
    int64_t  exp;
    uint32_t ks, vs, crc;
    uint32_t type, dt;
    uint32_t key0;      // first key byte when the fast decode saw it, else 0x100
    bool     good;      // a record the writer produces: varints ok, type<=4, dt<=4, ks>=1, vs>=0
};

// ReadLogRecord's header/bounds semantics at position p of a byte window w,
// without the CRC comparison.  nrel = bytes from the window start to the end of
// the file; p_abs = file offset of p.  data/dataFile.go:64-103,
// data/logRecord.go:86-114.  Exact (slow) form: byte loops.
template <class BP>
CLY_DEV Hdr step_hdr(BP w, int64_t p, int64_t nrel, int64_t p_abs) {
    Hdr h;
    h.status = 0; h.hsz = 0; h.size = 0; h.exp = 0; h.ks = 0; h.vs = 0; h.crc = 0; h.type = 0; h.dt = 0;
    h.key0 = 0x100; h.good = false;
    int64_t m = nrel - p;                           // dataFile.go:70-73
    if (m > 26) m = 26;
    if (m <= 4) { h.status = CLY_END_EOF; return h; }       // logRecord.go:87-89
    if (m == 5) { h.status = CLY_ERR_TRUNC5; return h; }    // buf[5] index panic
    const BP b = w + p;
    h.crc = (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
    h.type = b[4];
    h.dt = b[5];
    int64_t idx = 6;
    int na, nb, nc;
    const int64_t ks = go_varint(b + idx, m - idx, na); idx += na;
    if (idx < 0) { h.status = CLY_ERR_VARINT; return h; }
    const int64_t vs = go_varint(b + idx, m - idx, nb); idx += nb;
    if (idx < 0) { h.status = CLY_ERR_VARINT; return h; }
    h.exp = go_varint(b + idx, m - idx, nc); idx += nc;
    h.ks = (uint32_t)ks;
    h.vs = (uint32_t)vs;
    h.hsz = (int32_t)idx;
    if (h.crc == 0 && h.ks == 0 && h.vs == 0) { h.status = CLY_END_ZERO; return h; }   // dataFile.go:85-87
    const int64_t kv = (int64_t)h.ks + (int64_t)h.vs;
    if (kv > 0) {
        if (p_abs + idx < 0) { h.status = CLY_ERR_OFFSET; return h; }
        if (nrel - (p + idx) < kv) { h.status = CLY_END_TORN; return h; }            // short ReadAt
    }
    if (idx < 4) { h.status = CLY_ERR_VARINT; return h; }    // header[4:headerSize] panics
    h.status = REC_OK;
    h.size = idx + kv;
    h.good = na > 0 && nb > 0 && nc > 0 && h.type <= 4 && h.dt <= 4 && ks >= 1 && vs >= 0;
    return h;
}
