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
#define CLY_NDW 8             // data waves (= sub-tiles) per unit / workgroup
#endif
#define CLY_NT 64
#define CLY_NWD (CLY_SUB / 4)                 // words per stripe
#define CLY_TS (CLY_NT * CLY_SUB)             // sub-tile bytes
#define CLY_HALO 48                           // >= 26 (max header) + 11 (txId varint) + alignment
#define CLY_WIN (CLY_TS + CLY_HALO)
#define CLY_UNIT ((int64_t)CLY_NDW * CLY_TS)  // unit bytes (look-back granule)
static_assert(CLY_SUB % 16 == 0 && ((CLY_SUB / 16) & 1), "CLY_SUB = 16 * odd");
static_assert(CLY_NWD <= 64, "check masks are 64-bit");
static_assert(CLY_WIN % 16 == 0, "16-B staging");
static_assert(CLY_NDW * CLY_TS < (1 << 18), "unit-relative guess is an 18-bit field");

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
// Unit look-back descriptors: four 64-bit words per unit, each tagged with the
// call's epoch in bits [63:48] (a word with another epoch is "not yet written":
// no per-call memset).  Each word is written once per call.
//   w0: state word, written after w1 (SPEC) and again after w2/w3 (FULL)
//       [47:46] state (1 SPEC, 2 FULL) | 45 first-of-file | 44 term/dead |
//       43 guess valid | [42:25] guess (unit-relative) | [24:0] count
//   w1: SPEC exit (global position = unit*CLY_UNIT + rel)
//   w2: FULL exit
//   w3: FULL records up to and including this unit (global)
#define DS_SPEC 1ull
#define DS_FULL 2ull
#define DS_VAL_MASK ((1ull << 48) - 1)
CLY_DEV uint64_t ds_tag(uint32_t epoch, uint64_t v) { return ((uint64_t)(epoch & 0xffff) << 48) | (v & DS_VAL_MASK); }
CLY_DEV bool ds_ok(uint64_t w, uint32_t epoch) { return (w >> 48) == (epoch & 0xffff); }
CLY_DEV uint64_t ds_pack(uint32_t epoch, uint64_t state, int fof, int term, int gvalid, int64_t grel, uint32_t cnt) {
    return ds_tag(epoch, (state << 46) | ((uint64_t)(fof & 1) << 45) | ((uint64_t)(term & 1) << 44) |
                             ((uint64_t)(gvalid & 1) << 43) | ((uint64_t)(grel & 0x3ffff) << 25) |
                             ((uint64_t)cnt & 0x1ffffff));
}
CLY_DEV uint64_t ds_state(uint64_t w, uint32_t epoch) { return ds_ok(w, epoch) ? (w >> 46) & 3 : 0; }
CLY_DEV int ds_fof(uint64_t w) { return (int)((w >> 45) & 1); }
CLY_DEV int ds_term(uint64_t w) { return (int)((w >> 44) & 1); }
CLY_DEV int ds_gvalid(uint64_t w) { return (int)((w >> 43) & 1); }
CLY_DEV int64_t ds_grel(uint64_t w) { return (int64_t)((w >> 25) & 0x3ffff); }
CLY_DEV uint32_t ds_cnt(uint64_t w) { return (uint32_t)(w & 0x1ffffff); }
static_assert(CLY_UNIT / 9 + 1 < 0x1ffffff, "count field");

struct Desc {
    unsigned long long w[4];
};

// Composition state of the look-back: chain position entering the next unit.
struct LbState {
    int64_t  E;       // global position (valid when !dead)
    uint64_t P;       // records so far (global)
    int32_t  dead;    // chain of the current file ended
    int32_t  _pad;
};

// Apply SPEC descriptor (w0, exit x) of unit j.  False on a mismatch (the
// caller then waits for j's FULL words).
CLY_DEV bool lb_compose_spec(LbState& s, int64_t j, uint64_t w0, uint64_t x) {
    const int64_t cs = j * CLY_UNIT;
    if (ds_fof(w0)) { s.E = cs; s.dead = 0; }
    if (s.dead) return true;
    if (s.E >= cs + CLY_UNIT) return true;              // a record covers unit j
    if (ds_gvalid(w0) && s.E == cs + ds_grel(w0)) {
        s.P += ds_cnt(w0);
        if (ds_term(w0)) s.dead = 1;
        else s.E = (int64_t)x;
        return true;
    }
    return false;
}

// Decoupled look-back (CUB-style, unbounded): walk back from unit c-1 until a
// unit with FULL words, folding every speculative descriptor on the way into an
// O(1) summary of the suffix (units j+1 .. c-1):
//   requirement  on the chain position entering the suffix: none, == e0
//                (EXACT: the first unit's guess must be the true entry) or
//                >= e0 (ATLEAST: the suffix starts with units covered by one
//                record),
//   result       E_c as a function of that position: the identity (only
//                covered units so far), a constant exit, or dead,
//   counts       records of the suffix (pending on the requirement) and of the
//                part after a first-of-file unit (fixed).
// Folding unit j in front: "tight" when its guessed chain exits where the
// suffix requires (requirement becomes == g_j, counts += n_j), otherwise
// "transparent" (j is covered by one record; requirement unchanged).  Both are
// sufficient conditions; the FULL unit's exit checks the final requirement.
// A first-of-file unit's guess (0) is exact: it fixes E_c, and the walk goes
// on for the record count only.  On a failed check lb_forward() composes
// forward from the FULL unit with exact per-unit checks (rare path).
#define LB_REQ_NONE 0
#define LB_REQ_EXACT 1
#define LB_REQ_ATLEAST 2
#define LB_RES_IDENT 0
#define LB_RES_CONST 1
#define LB_RES_DEAD 2
struct LbSum {
    int64_t  e0, rx, cE;
    uint64_t dp, dp_fixed;
    int32_t  req, res, fixed, cdead;
};
// The walk keeps, next to its summary, the unit kreq whose tight fold set the
// current EXACT requirement and the summary just before that fold (prev): if
// the final check fails (usually kreq's guess was wrong), waiting for kreq's
// own FULL words and applying prev finishes the look-back.
struct LbWalk : LbSum {
    LbSum   prev;
    int64_t kreq;             // -1: no tight fold since the last reset
};

CLY_DEV void lb_walk_init(LbWalk& w, int64_t c, int fof) {
    w.e0 = 0; w.rx = 0; w.cE = 0; w.dp = 0; w.dp_fixed = 0;
    w.req = LB_REQ_NONE; w.res = LB_RES_IDENT; w.fixed = 0; w.cdead = 0;
    if (fof) { w.fixed = 1; w.cE = c * CLY_UNIT; }
    w.prev = static_cast<const LbSum&>(w);
    w.kreq = -1;
}

CLY_DEV bool lb_req_ok(const LbSum& w, int64_t E) {
    return w.req == LB_REQ_NONE || (w.req == LB_REQ_EXACT ? E == w.e0 : E >= w.e0);
}

// Fold SPEC descriptor (w0, exit x) of unit j.  False = the walk cannot
// continue consistently (only at a first-of-file unit whose exact chain
// misses the requirement).
CLY_DEV bool lb_fold_spec(LbWalk& w, int64_t j, uint64_t w0, int64_t x) {
    const int64_t cs = j * CLY_UNIT;
    const int term = ds_term(w0);
    const uint32_t n = ds_cnt(w0);
    if (ds_fof(w0)) {
        if (!term && !lb_req_ok(w, x)) return false;
        if (!w.fixed) {
            w.fixed = 1;
            if (term || w.res == LB_RES_DEAD) w.cdead = 1;
            else w.cE = w.res == LB_RES_IDENT ? x : w.rx;
        }
        w.dp_fixed += (term ? 0 : w.dp) + n;
        w.req = LB_REQ_NONE; w.res = LB_RES_IDENT; w.dp = 0;
        w.kreq = -1;
        return true;
    }
    if (ds_gvalid(w0) && (w.req == LB_REQ_NONE || (!term && lb_req_ok(w, x)))) {
        w.prev = static_cast<const LbSum&>(w);
        w.kreq = j;
        if (term) { w.res = LB_RES_DEAD; w.dp = n; }
        else { if (w.res == LB_RES_IDENT) { w.res = LB_RES_CONST; w.rx = x; } w.dp += n; }
        w.req = LB_REQ_EXACT;
        w.e0 = cs + ds_grel(w0);
    } else if (w.req == LB_REQ_NONE) {
        w.req = LB_REQ_ATLEAST;
        w.e0 = cs + CLY_UNIT;
    }
    return true;
}

// Apply FULL words of unit j (exit X, dead, records P up to and including j).
// False = the requirement fails (forward fallback needed).
CLY_DEV bool lb_apply_full_walk(const LbSum& w, int dead, int64_t X, uint64_t P, LbState& out) {
    if (dead) {
        out.dead = w.fixed ? w.cdead : 1;
        out.E = w.fixed ? w.cE : 0;
        out.P = P + w.dp_fixed;
        return true;
    }
    if (!lb_req_ok(w, X)) return false;
    if (w.fixed) { out.dead = w.cdead; out.E = w.cE; }
    else { out.dead = w.res == LB_RES_DEAD; out.E = w.res == LB_RES_IDENT ? X : w.rx; }
    out.P = P + w.dp + w.dp_fixed;
    return true;
}

// Rare path: exact forward composition from the FULL unit jf (or from the
// start when jf < 0) to c, waiting for the FULL words of any unit whose guess
// does not match the chain.  Env supplies ld(j, k) and spin().
template <class Env>
CLY_DEV void lb_forward(Env& env, int64_t c, int fof, int64_t jf, uint32_t epoch, LbState& s) {
    s.E = 0; s.P = 0; s.dead = 0; s._pad = 0;
    if (jf >= 0) {
        uint64_t w0 = env.ld(jf, 0), x = env.ld(jf, 2), p = env.ld(jf, 3);
        while (ds_state(w0, epoch) != DS_FULL || !ds_ok(x, epoch) || !ds_ok(p, epoch)) {
            if (!env.spin()) return;
            w0 = env.ld(jf, 0); x = env.ld(jf, 2); p = env.ld(jf, 3);
        }
        s.dead = ds_term(w0); s.E = (int64_t)(x & DS_VAL_MASK); s.P = p & DS_VAL_MASK;
    }
    for (int64_t k = jf + 1; k < c; k++) {
        uint64_t w0 = env.ld(k, 0);
        while (ds_state(w0, epoch) == 0) { if (!env.spin()) return; w0 = env.ld(k, 0); }
        if (ds_state(w0, epoch) == DS_SPEC) {
            uint64_t x = env.ld(k, 1);
            while (!ds_ok(x, epoch)) { if (!env.spin()) return; x = env.ld(k, 1); }
            if (lb_compose_spec(s, k, w0, x & DS_VAL_MASK)) continue;
        }
        uint64_t x = env.ld(k, 2), p = env.ld(k, 3);
        while (ds_state(w0, epoch) != DS_FULL || !ds_ok(x, epoch) || !ds_ok(p, epoch)) {
            if (!env.spin()) return;
            w0 = env.ld(k, 0); x = env.ld(k, 2); p = env.ld(k, 3);
        }
        s.dead = ds_term(w0); s.E = (int64_t)(x & DS_VAL_MASK); s.P = p & DS_VAL_MASK;
    }
    if (fof) { s.E = c * CLY_UNIT; s.dead = 0; }
}

// Recovery after a failed check: wait for the FULL words of w.kreq and apply
// the summary from before its fold.  False = still inconsistent.
template <class Env>
CLY_DEV bool lb_recover_kreq(Env& env, const LbWalk& w, uint32_t epoch, LbState& out) {
    if (w.kreq < 0) return false;
    const int64_t k = w.kreq;
    uint64_t w0 = env.ld(k, 0), x = env.ld(k, 2), p = env.ld(k, 3);
    while (ds_state(w0, epoch) != DS_FULL || !ds_ok(x, epoch) || !ds_ok(p, epoch)) {
        if (!env.spin()) return false;
        x = env.ld(k, 2); p = env.ld(k, 3); w0 = env.ld(k, 0);
    }
    return lb_apply_full_walk(w.prev, ds_term(w0), (int64_t)(x & DS_VAL_MASK), p & DS_VAL_MASK, out);
}

// One descriptor of the backward walk (words already loaded and ready).
// Returns 0 = continue, 1 = done (out filled), 2 = forward fallback from jf.
CLY_DEV int lb_walk_step(LbWalk& w, int64_t j, uint64_t w0, uint64_t w1, uint64_t w2, uint64_t w3,
                         uint32_t epoch, LbState& out, int64_t& jf) {
    if (ds_state(w0, epoch) == DS_FULL) {
        if (lb_apply_full_walk(w, ds_term(w0), (int64_t)(w2 & DS_VAL_MASK), w3 & DS_VAL_MASK, out)) return 1;
        jf = j;
        return 2;
    }
    if (!lb_fold_spec(w, j, w0, (int64_t)(w1 & DS_VAL_MASK))) {
        jf = -3;              // find the nearest FULL before j, then compose forward
        return 2;
    }
    return 0;
}

// ---------------------------------------------------------------------------
// Per-sub-tile summary for k_fin (written by the sub-tile's wave, read after
// the launch).  CRC state convention: the register of crc_gf.h ("init form").
struct ChunkSum {
    int64_t  evt_off;     // file offset of the sub-tile's first event, INT64_MAX none
    uint64_t evt_gidx;    // tuple index at the event, relative to the unit's first record
    uint64_t p_excl;      // records of the unit before the sub-tile
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
CLY_DEV int64_t fin_chunk_event(const ChunkSum* sums, const uint64_t* unit_P, const uint32_t* x8n, int64_t c0,
                                int64_t nc, int64_t i, uint64_t* gidx, int32_t* status) {
    const ChunkSum S = sums[c0 + i];
    const uint64_t P = unit_P[(c0 + i) / CLY_NDW];     // records before the sub-tile's unit
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
                g = P + S.p_excl + S.cnt - 1;
                st = CLY_ERR_CRC;
            }
        }
    }
    *gidx = g;
    *status = st;
    return off;
}
