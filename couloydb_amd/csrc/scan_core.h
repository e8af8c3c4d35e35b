// scan_core.h — definitions shared by the kernels of libclyscan (gfx950):
// geometry, the exact per-record semantics of the reference, the look-back
// descriptor algebra of units, and the per-file finish (k_fin) helpers.
//
// Reference semantics restated here: DataFile.ReadLogRecord
// (data/dataFile.go:64-111), DecodeLogRecordHeader (data/logRecord.go:86-114),
// GetLogRecordCRC (data/logRecord.go:136-146), parseLogRecordKey (db.go:706-710)
// and the loop "offset += size until io.EOF" of db.loadIndex (db.go:582-637).
//
// Work decomposition:
//   stripe    CLY_SUB bytes, one lane
//   sub-tile  64 stripes (CLY_TS bytes), one data wave; staged in LDS
//   unit      CLY_NDW sub-tiles, one workgroup (CLY_NDW data waves + one
//             coordinator wave); the unit is the granule of the decoupled
//             look-back (one ticket and one descriptor per unit)
#pragma once
#include <stdint.h>

#include "../../include/clyscan.h"
#include "crc_gf.h"

#define CLY_DEV __device__ __forceinline__
#define CLY_NOINL __device__ __noinline__
#define CLY_LDS __attribute__((address_space(3)))

#ifndef CLY_SUB
#define CLY_SUB 144           // stripe bytes: 16 * odd, so 64 lanes' ds_read_b128 of their
                              // stripes hit distinct 4-bank groups (conflict-free)
#endif
#ifndef CLY_NDW
#define CLY_NDW 8             // waves (one sub-tile each) per workgroup
#endif
#define CLY_NT 64
#define CLY_NWD (CLY_SUB / 4)                 // words per stripe
#define CLY_TS (CLY_NT * CLY_SUB)             // sub-tile bytes
#define CLY_HALO 320                          // >= 26 (max header) + 11 (txId varint); the larger halo lets
                                              // exit checks of records up to ~290 B stay in LDS
#define CLY_WIN (CLY_TS + CLY_HALO)
static_assert(CLY_SUB % 16 == 0 && ((CLY_SUB / 16) & 1), "CLY_SUB = 16 * odd");
static_assert(CLY_NWD <= 64, "check masks are 64-bit");
static_assert(CLY_WIN % 16 == 0, "16-B staging");
static_assert(CLY_TS < (1 << 15), "sub-tile-relative entries are 16-bit");

#define REC_OK 100

// ---------------------------------------------------------------------------
// Go encoding/binary Varint (toolchain >= 1.18, go.mod:3): zigzag over Uvarint;
// overflow (10th byte > 1, or an 11th byte) -> (0, -(i+1)); short buffer -> (0, 0).
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
    h.good = false;
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

// ---------------------------------------------------------------------------
// Per-sub-tile summary for k_fin (written by the sub-tile's wave, read after
// the launch).  CRC state convention: the register of crc_gf.h ("init form").
struct ChunkSum {
    int64_t  evt_off;     // file offset of the sub-tile's first event, INT64_MAX none
    uint64_t evt_gidx;    // tuple index at the event, relative to the sub-tile's first record
    int64_t  open_pos;    // file offset of the record open at the sub-tile end (-1 none)
    int32_t  evt_status;
    uint32_t cnt;         // records starting in the sub-tile
    uint32_t open_state;  // its CRC register at the end of the sub-tile
    uint32_t open_crc;    // its stored CRC
    uint32_t head_raw;    // Z_z(raw register over [4, head_len)): z zero bytes appended
    uint32_t head_shift;  // head_len - 4 + z (k_fin multiplies by x^(8*head_shift))
    uint32_t first4;      // first 4 bytes of the sub-tile
    uint32_t head_len;    // bytes before the first boundary
    uint32_t flags;       // SUM_*
    uint32_t head_z;      // z
};
#define SUM_DEAD 1u
#define SUM_CLOSES 2u     // the record entering the sub-tile ends inside it (or at the file end)
#define SUM_OPEN 4u
#define EVT_NONE INT64_MAX

// k_fin helpers: finish the CRC of the record open at the end of sub-tile i by
// walking the heads of the following sub-tiles of the file.  Returns the
// register after head H, times x^(8*zout) (zout zero bytes appended).
CLY_DEV uint32_t fin_advance(uint32_t s, int64_t ocs, const ChunkSum& H, const uint32_t* x8n, int64_t hstart,
                             uint32_t* zout) {
    const int64_t hlen = H.head_len;
    const int64_t l4 = hlen < 4 ? hlen : 4;
    int lo = 0;
    if (ocs > hstart) lo = (int)(ocs - hstart < l4 ? ocs - hstart : l4);
    for (int k = lo; k < l4; k++) s = cly_crc_byte_bitwise(s, (uint8_t)(H.first4 >> (8 * k)));
    *zout = 0;
    if (hlen > 4) { s = cly_multmodp(x8n[H.head_shift], s) ^ H.head_raw; *zout = H.head_z; }
    return s;
}

// Event of sub-tile i of a file (sub-tiles c0 .. c0+nc-1): in-tile event, or
// the CRC failure of its open record.  Returns the file offset (EVT_NONE if none).
CLY_DEV int64_t fin_chunk_event(const ChunkSum* sums, const uint64_t* sub_P, const uint32_t* x8n, int64_t c0,
                                int64_t nc, int64_t i, uint64_t* gidx, int32_t* status) {
    const ChunkSum S = sums[c0 + i];
    const uint64_t P = sub_P[c0 + i];                   // records before the sub-tile
    int64_t off = EVT_NONE;
    uint64_t g = 0;
    int32_t st = 0;
    if (!(S.flags & SUM_DEAD)) {
        off = S.evt_off;
        g = P + S.evt_gidx;
        st = S.evt_status;
        if (S.flags & SUM_OPEN) {
            uint32_t s = S.open_state;
            uint32_t z = 0;
            const int64_t ocs = S.open_pos + 4;
            for (int64_t j = i + 1; j < nc; j++) {
                const ChunkSum H = sums[c0 + j];
                s = fin_advance(s, ocs, H, x8n, j * (int64_t)CLY_TS, &z);
                if (H.flags & SUM_CLOSES) break;
                z = 0;
            }
            if (s != cly_shift(~S.open_crc, z) && (off == EVT_NONE || S.open_pos < off)) {
                off = S.open_pos;
                g = P + S.cnt - 1;
                st = CLY_ERR_CRC;
            }
        }
    }
    *gidx = g;
    *status = st;
    return off;
}
