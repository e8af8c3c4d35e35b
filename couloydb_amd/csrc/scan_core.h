// scan_core.h — the per-chunk algorithm of libclyscan, written once for two
// executors:
//   * the gfx950 kernel k_scan in clyscan.hip (one 256-lane workgroup per chunk,
//     DevExec: a phase is one lane per thread followed by a barrier), and
//   * tests/emu (CPU emulator, HostExec: a phase is a loop over the lanes), which
//     is test infrastructure that lets the chunk logic be checked against the
//     oracle without a GPU.  The product path never runs the emulator.
//
// What one chunk does:
//   stage     chunk bytes (+64-B halo) into LDS; build the slicing-by-4 CRC tables
//   spec      every lane finds the first plausible record start in its SUB-byte
//             stripe and walks the record chain to the end of the stripe
//   resolve   from an entry position E, join the lanes' walks into the chunk's true
//             record chain; lanes whose walk disagrees are re-walked exactly
//   lookback  decoupled look-back over per-chunk descriptors gives the true entry
//             E and the number of records before the chunk (output slot)
//   crc       CRC-32 of every record: per-lane stripes + a segmented scan for
//             records that span stripes; straddlers across chunks are finished
//             by k_fin from per-chunk head/open CRC registers
//   emit      cly_tuple per record
//
// Reference semantics restated here: DataFile.ReadLogRecord (data/dataFile.go:64-111),
// DecodeLogRecordHeader (data/logRecord.go:86-114), GetLogRecordCRC
// (data/logRecord.go:136-146), parseLogRecordKey (db.go:706-710), and the loop
// "offset += size until io.EOF" of db.loadIndex (db.go:582-637).
#pragma once
#include <stdint.h>

#include "../../include/clyscan.h"
#include "crc_gf.h"

#ifdef __HIPCC__
#define CLY_DEV __device__ __forceinline__
#define CLY_MEM __device__ __forceinline__
#define CLY_NOINL __device__ __noinline__
#else
#define CLY_DEV static inline
#define CLY_MEM inline
#define CLY_NOINL static
#endif
// LDS address space on the device pass: keeps every access to the chunk's
// shared state a ds_* instruction (a generic pointer would compile to flat_*
// loads in the out-of-line lane routines).
#if defined(__HIP_DEVICE_COMPILE__)
#define CLY_LDS __attribute__((address_space(3)))
#else
#define CLY_LDS
#endif
// Codegen note (ROCm 7.2, gfx950): values computed inside a lane-divergent
// loop with several exits and used after it were observed clobbered by the
// register allocator in this (large) kernel.  Lane routines therefore store
// their results to LDS at the exit point inside the loop and are kept out of
// line (CLY_NOINL).

#ifndef CLY_NT
#define CLY_NT 64             // lanes per chunk: one wave processes one chunk
#endif
#ifndef CLY_SUB
#define CLY_SUB 124           // bytes per lane stripe: 31 dwords (odd), so lane k's
                              // stripe starts at LDS bank 31k mod 32 (no conflicts)
#endif
#ifndef CLY_REP
#define CLY_REP 2             // LDS replication of the CRC tables (bank spread)
#endif
#define CLY_CHUNK (CLY_NT * CLY_SUB)
#define CLY_HALO 64           // >= 26 (max header) + 11 (txId varint) past the chunk end
#define CLY_WIN (CLY_CHUNK + CLY_HALO)
#define CLY_NWAVE (CLY_NT / 64)
#define CLY_LBWIN 64          // look-back: descriptors read per round trip (one wave)
#define CLY_TAB_WORDS (4 * 256 * CLY_REP)
static_assert(CLY_NT == 64, "one chunk per wave: CLY_NT is the wave width");
static_assert(CLY_SUB % 4 == 0 && CLY_SUB >= 28, "CLY_SUB must be a multiple of 4");
static_assert(CLY_CHUNK % 16 == 0 && CLY_WIN % 16 == 0, "16-B staging");
static_assert(CLY_CHUNK <= 32767, "chunk-relative positions are int16");

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
    uint8_t  type, dt;
    bool     good;      // a record the writer produces: varints ok, type<=4, dt<=4, ks>=1
};

// ReadLogRecord's header/bounds semantics at window position p, without the
// CRC comparison.  nrel = bytes from the window start to the end of the file;
// p_abs = file offset of p.  data/dataFile.go:64-103, data/logRecord.go:86-114.
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

template <class BP>
CLY_DEV uint32_t le32(BP b) {
    return (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
}

// ---------------------------------------------------------------------------
// CRC on LDS bytes: slicing-by-4 tables T0..T3, replicated CLY_REP times
// (entry i of table t, replica r at dword (t*256 + i)*CLY_REP + r).
struct CrcTab {
    const CLY_LDS uint32_t* t;
    int r;
    CLY_MEM uint32_t at(int tab, uint32_t i) const { return t[((tab << 8) + (int)i) * CLY_REP + r]; }
    CLY_MEM uint32_t byte(uint32_t s, uint32_t b) const { return at(0, (s ^ b) & 0xff) ^ (s >> 8); }
    CLY_MEM uint32_t word(uint32_t s, uint32_t d) const {
        s ^= d;
        return at(3, s & 0xff) ^ at(2, (s >> 8) & 0xff) ^ at(1, (s >> 16) & 0xff) ^ at(0, s >> 24);
    }
};

// Register s advanced over window bytes [lo, hi).
CLY_DEV uint32_t crc_run(const CrcTab& T, uint32_t s, const CLY_LDS uint8_t* w, int lo, int hi) {
    while (lo < hi && (lo & 3)) { s = T.byte(s, w[lo]); lo++; }
    const CLY_LDS uint32_t* w32 = (const CLY_LDS uint32_t*)w;
    while (hi - lo >= 4) { s = T.word(s, w32[lo >> 2]); lo += 4; }
    while (lo < hi) { s = T.byte(s, w[lo]); lo++; }
    return s;
}

// Fill the slicing tables (thread t of nthr builds entries t, t+nthr, ...).
template <class TP>
CLY_DEV void build_tab_lane(TP tab, int t, int nthr) {
    for (int i = t; i < 256; i += nthr) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ CLY_POLY : c >> 1;
        for (int tb = 0; tb < 4; tb++) {
            for (int r = 0; r < CLY_REP; r++) tab[((tb << 8) + i) * CLY_REP + r] = c;
            uint32_t tl = c & 0xff;
            for (int k = 0; k < 8; k++) tl = (tl & 1) ? (tl >> 1) ^ CLY_POLY : tl >> 1;
            c = (c >> 8) ^ tl;
        }
    }
}

// A^(CLY_SUB * 2^lvl) applied through a 4x256 table (built by the host).
CLY_DEV uint32_t shift_tab(const uint32_t* st, int lvl, uint32_t v) {
    const uint32_t* t = st + lvl * 1024;
    return t[v & 0xff] ^ t[256 + ((v >> 8) & 0xff)] ^ t[512 + ((v >> 16) & 0xff)] ^ t[768 + (v >> 24)];
}

// ---------------------------------------------------------------------------
// Shared (LDS) state of one chunk.
struct ChunkCtx {
    const uint8_t* gfile; // the file's bytes in the executor's memory (device: HBM)
    int64_t  cbase;       // file offset of the chunk start
    int64_t  nrel;        // bytes from chunk start to end of file
    int32_t  dlen;        // data bytes in the chunk (<= CHUNK)
    int32_t  win_len;     // bytes staged in the window (<= WIN)
    int32_t  chunk;       // global chunk index
    int32_t  fidx;        // file index
    int32_t  fof;         // first chunk of its file
    int32_t  lof;         // last chunk of its file
    uint32_t fid;
    int32_t  _pad;
};

// Result of resolve(E) for the chunk.
struct ChainRes {
    int32_t  E;           // entry (chunk-relative); >= dlen means no lane is on the chain
    int32_t  k0;          // lane of E (CLY_NT if none)
    int32_t  term;        // chain terminated inside the chunk
    int32_t  tst;         // terminal status
    int64_t  tpos;        // terminal position (rel)
    int64_t  xrel;        // chain exit (rel) when not terminated
    int32_t  cnt;         // records on the chain in this chunk
    int32_t  last;        // start (rel) of the last record (-1 none)
    int32_t  lterm;       // lane holding the terminal (CLY_NT if none)
    int32_t  eof_exit;    // the chain leaves the file's last chunk exactly at the end of the file
};

struct ScanShared {
    uint32_t win[CLY_WIN / 4];                // chunk bytes (+ halo), zero past the file end
    const CLY_LDS uint32_t* tab;              // slicing-by-4 tables (shared by the workgroup)
    // speculation (entry independent)
    uint32_t sp_x[CLY_NT];                    // exit (rel) of the lane's speculative walk
    int16_t  sp_s[CLY_NT];                    // first record of the walk (rel), -1 none
    int16_t  sp_last[CLY_NT];
    uint16_t sp_cnt[CLY_NT];
    uint8_t  sp_vin[CLY_NT];                  // exit checked inside the window
    // chain working set (resolve)
    uint32_t wx[CLY_NT];                      // exit (rel) or terminal position
    int16_t  ws[CLY_NT];                      // first chain position in the stripe, -1 none
    int16_t  wl[CLY_NT];                      // last record start in the stripe
    uint16_t wc[CLY_NT];                      // records starting in the stripe
    int16_t  pk[CLY_NT];                      // last lane <= t with ws >= 0
    int16_t  base[CLY_NT];                    // local index of the stripe's first record
    uint8_t  wterm[CLY_NT];
    int8_t   wtst[CLY_NT];
    // CRC segmented scan
    uint32_t sc_v[2][CLY_NT];
    uint8_t  sc_c[2][CLY_NT];
    uint8_t  sc_c0[CLY_NT];                   // phase-A constness (kept through the scan)


    // scalars
    ChunkCtx C;
    ChainRes R;
    unsigned long long bad;                   // packed (pos << 32 | local idx) of the first CRC failure
    uint32_t head_raw;                        // raw register over [4, head end)
    uint32_t end_state;                       // register at the end of the data
    int32_t  fix_lo, fix_hi, fix_kill;        // resolve fix step (broadcast)
    int32_t  mode;                            // MODE_*
    int32_t  guess;                           // speculated entry (rel), -1 none
    int32_t  crc_mode_done;                   // CRC results are valid for (mode, E)
    int64_t  entry_g;                         // look-back: global entry position
    uint64_t p_excl;                          // records before the chunk (global slot)
    int32_t  in_dead;                         // look-back: chain ended before this chunk

#ifdef CLY_PHASE_PROF
    uint64_t tstamp[10];                      // profiling build: per-phase clock stamps
    uint64_t pacc[10];                        //   summed per wave, flushed at kernel exit
    uint64_t lacc[4];
#endif
    int32_t  fail;                            // internal invariant violated (reported as a device error)
    int32_t  fail_k;
    int32_t  redo_crc;                        // the guessed chain was wrong: CRC again
};

#define MODE_NORMAL 0     // the chain enters (or ends) inside the chunk: R is valid
#define MODE_PASS 1       // one record covers the whole chunk (no boundary)
#define MODE_DEAD 2       // the file's chain ended in an earlier chunk

// ---------------------------------------------------------------------------
// Per-chunk summary for k_fin (written by the chunk, read after the launch).
struct ChunkSum {
    int64_t  evt_off;     // file offset of the chunk's first event, INT64_MAX none
    uint64_t evt_gidx;    // global tuple index at the event
    uint64_t p_excl;      // records before the chunk (global)
    int64_t  open_pos;    // file offset of the record open at the chunk end (-1 none)
    int32_t  evt_status;
    uint32_t cnt;         // records starting in the chunk
    uint32_t open_state;  // its CRC register at the end of the data
    uint32_t open_crc;    // its stored CRC
    uint32_t head_raw;    // raw register over [4, head_len) of the chunk
    uint32_t head_shift;  // x^(8*(head_len-4)) mod P
    uint32_t first4;      // first 4 bytes of the chunk
    uint32_t head_len;    // bytes before the first boundary
    uint32_t flags;       // SUM_*
    uint32_t _pad;
};
#define SUM_DEAD 1u
#define SUM_CLOSES 2u     // the record entering the chunk ends inside it (or at the file end)
#define SUM_OPEN 4u
#define EVT_NONE INT64_MAX

// ---------------------------------------------------------------------------
// Look-back descriptors: four 64-bit words per chunk, each tagged with the
// call's epoch in bits [63:48] (a word with another epoch is "not yet
// written": no per-call memset, and no word is trusted before its own tag
// matches).  Each word is written once per call.
//   w0: state word, written after w1 (SPEC) and again after w2/w3 (FULL)
//       [47:46] state (1 SPEC, 2 FULL) | 45 first-of-file | 44 term/dead |
//       43 guess valid | [42:27] guess (rel) | [26:13] count
//   w1: SPEC exit (global position = chunk*CHUNK + rel)
//   w2: FULL exit
//   w3: FULL records up to and including this chunk (global)
#define DS_SPEC 1ull
#define DS_FULL 2ull
#define DS_VAL_MASK ((1ull << 48) - 1)
CLY_DEV uint64_t ds_tag(uint32_t epoch, uint64_t v) { return ((uint64_t)(epoch & 0xffff) << 48) | (v & DS_VAL_MASK); }
CLY_DEV bool ds_ok(uint64_t w, uint32_t epoch) { return (w >> 48) == (epoch & 0xffff); }
CLY_DEV uint64_t ds_pack(uint32_t epoch, uint64_t state, int fof, int term, int gvalid, int grel, uint32_t cnt) {
    return ds_tag(epoch, (state << 46) | ((uint64_t)(fof & 1) << 45) | ((uint64_t)(term & 1) << 44) |
                             ((uint64_t)(gvalid & 1) << 43) | ((uint64_t)(grel & 0xffff) << 27) |
                             ((uint64_t)(cnt & 0x3fff) << 13));
}
CLY_DEV uint64_t ds_state(uint64_t w, uint32_t epoch) { return ds_ok(w, epoch) ? (w >> 46) & 3 : 0; }
CLY_DEV int ds_fof(uint64_t w) { return (int)((w >> 45) & 1); }
CLY_DEV int ds_term(uint64_t w) { return (int)((w >> 44) & 1); }
CLY_DEV int ds_gvalid(uint64_t w) { return (int)((w >> 43) & 1); }
CLY_DEV int ds_grel(uint64_t w) { return (int)((w >> 27) & 0xffff); }
CLY_DEV uint32_t ds_cnt(uint64_t w) { return (uint32_t)((w >> 13) & 0x3fff); }
static_assert(CLY_CHUNK / 4 + 1 < 0x3fff, "count field");

struct Desc {
    unsigned long long w[4];
};

// Composition state of the look-back: chain position entering the next chunk.
struct LbState {
    int64_t  E;       // global position (valid when !dead)
    uint64_t P;       // records so far (global)
    int32_t  dead;    // chain of the current file ended
    int32_t  _pad;
};

// Apply SPEC descriptor (w0, exit w1) of chunk j.  Returns false on a
// mismatch (the caller then waits for j's FULL words).
CLY_DEV bool lb_compose_spec(LbState& s, int64_t j, uint64_t w0, uint64_t x) {
    const int64_t cs = j * (int64_t)CLY_CHUNK;
    if (ds_fof(w0)) { s.E = cs; s.dead = 0; }
    if (s.dead) return true;
    if (s.E >= cs + CLY_CHUNK) return true;              // a record covers chunk j
    if (ds_gvalid(w0) && s.E == cs + ds_grel(w0)) {
        s.P += ds_cnt(w0);
        if (ds_term(w0)) s.dead = 1;
        else s.E = (int64_t)x;
        return true;
    }
    return false;
}

// ---------------------------------------------------------------------------
// Decoupled look-back (CUB-style, unbounded): walk back from chunk c-1 until a
// chunk with FULL words, folding every speculative descriptor on the way into
// an O(1) summary of the suffix (chunks j+1 .. c-1):
//   requirement  on the chain position entering the suffix: none, == e0
//                (EXACT: the first chunk's guess must be the true entry) or
//                >= e0 (ATLEAST: the suffix starts with chunks covered by one
//                record),
//   result       E_c as a function of that position: the identity (only
//                covered chunks so far), a constant exit, or dead,
//   counts       records of the suffix (pending on the requirement) and of the
//                part after a first-of-file chunk (fixed).
// Folding chunk j in front: "tight" when its guessed chain exits where the
// suffix requires (requirement becomes == g_j, counts += n_j), otherwise
// "transparent" (j is covered by one record; requirement unchanged).  Both are
// sufficient conditions; the FULL chunk's exit checks the final requirement.
// A first-of-file chunk's guess (0) is exact: it fixes E_c, and the walk goes
// on for the record count only.  On a failed check (a wrong guess or a wrong
// tight/transparent choice) lb_forward() composes forward from the FULL chunk
// with exact per-chunk checks (rare path).
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
// The walk keeps, next to its summary, the chunk kreq whose tight fold set the
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
    if (fof) { w.fixed = 1; w.cE = c * (int64_t)CLY_CHUNK; }
    w.prev = static_cast<const LbSum&>(w);
    w.kreq = -1;
}

CLY_DEV bool lb_req_ok(const LbSum& w, int64_t E) {
    return w.req == LB_REQ_NONE || (w.req == LB_REQ_EXACT ? E == w.e0 : E >= w.e0);
}

// Fold SPEC descriptor (w0, exit x) of chunk j.  False = the walk cannot
// continue consistently (only at a first-of-file chunk whose exact chain
// misses the requirement).
CLY_DEV bool lb_fold_spec(LbWalk& w, int64_t j, uint64_t w0, int64_t x) {
    const int64_t cs = j * (int64_t)CLY_CHUNK;
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
        w.e0 = cs + CLY_CHUNK;
    }
    return true;
}

// Apply FULL words of chunk j (exit X, dead, records P up to and including j).
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

// Rare path: exact forward composition from the FULL chunk jf (or from the
// start when jf < 0) to c, waiting for the FULL words of any chunk whose guess
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
    if (fof) { s.E = c * (int64_t)CLY_CHUNK; s.dead = 0; }
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

// Sequential form of the whole look-back (CPU emulator; the GPU form reads 64
// descriptors per round trip and runs the same steps).
template <class Env>
CLY_DEV void lookback_seq(Env& env, int64_t c, int fof, uint32_t epoch, LbState& out) {
    LbWalk w;
    lb_walk_init(w, c, fof);
    int64_t jf = -1;
    int r = 0;
    for (int64_t j = c - 1; j >= 0 && r == 0; j--) {
        uint64_t w0, w1 = 0, w2 = 0, w3 = 0;
        for (;;) {
            w0 = env.ld(j, 0);
            const uint64_t st = ds_state(w0, epoch);
            if (st == DS_SPEC) { w1 = env.ld(j, 1); if (ds_ok(w1, epoch)) break; }
            else if (st == DS_FULL) { w2 = env.ld(j, 2); w3 = env.ld(j, 3); if (ds_ok(w2, epoch) && ds_ok(w3, epoch)) break; }
            if (!env.spin()) { out.E = 0; out.P = 0; out.dead = 1; return; }
        }
        r = lb_walk_step(w, j, w0, w1, w2, w3, epoch, out, jf);
        if (r == 2 && jf == -3) {
            // nearest FULL before j
            jf = -1;
            for (int64_t k = j - 1; k >= 0; k--) {
                uint64_t a0 = env.ld(k, 0);
                while (ds_state(a0, epoch) == 0) { if (!env.spin()) { out.dead = 1; return; } a0 = env.ld(k, 0); }
                if (ds_state(a0, epoch) == DS_FULL) { jf = k; break; }
            }
        }
    }
    if (r == 0) {
        // reached the start of everything: as a FULL with exit 0 and no records
        if (!lb_apply_full_walk(w, 0, 0, 0, out)) { jf = -1; r = 2; }
        else r = 1;
    }
    if (r == 2 && !lb_recover_kreq(env, w, epoch, out)) { env.note_fallback(c, jf); lb_forward(env, c, fof, jf, epoch, out); }
}

// ---------------------------------------------------------------------------
// Lane work.

// Speculative walk of lane t: first candidate q in the stripe whose chain of
// plain records leaves the stripe at an exit that decodes as a plain record
// (checked when its header lies in the window) or is the end of the file.
// SWAR byte masks (bit 7 of each byte): byte <= 4 (type/dtype), and byte
// nonzero and even (first byte of the key-size varint of a record with ks >= 1).
CLY_DEV uint32_t swar_le4(uint32_t W) { return ~(((W | 0x80808080u) - 0x05050505u) | W) & 0x80808080u; }
CLY_DEV uint32_t swar_ks(uint32_t W) {
    const uint32_t nz = ((W & 0x7f7f7f7fu) + 0x7f7f7f7fu) | W;
    return nz & ~(W << 7) & 0x80808080u;
}
CLY_DEV uint32_t funnel(uint32_t hi, uint32_t lo, int sh) {
#ifdef __HIPCC__
    return __builtin_amdgcn_alignbit(hi, lo, sh);
#else
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> sh);
#endif
}
CLY_DEV int ctz32(uint32_t v) {
#ifdef __HIPCC__
    return __builtin_ctz(v);
#else
    return __builtin_ctz(v);
#endif
}

// First q in [q0, b) whose bytes q+4, q+5 are <= 4 and q+6 is nonzero and even
// (word-parallel filter over the LDS window); b if none.
CLY_DEV int next_candidate(const CLY_LDS uint32_t* w32, int q0, int b) {
    int i = (q0 + 4) >> 2;                 // word holding byte q0+4
    uint32_t Li = swar_le4(w32[i]), Ki = swar_ks(w32[i]);
    for (;;) {
        const int qbase = 4 * i - 4;       // candidates of word i: q in [qbase, qbase+4)
        if (qbase >= b) return b;
        const uint32_t Wn = w32[i + 1];
        const uint32_t Ln = swar_le4(Wn), Kn = swar_ks(Wn);
        uint32_t c = Li & funnel(Ln, Li, 8) & funnel(Kn, Ki, 16);
        if (qbase < q0) c &= ~0u << (8 * (q0 - qbase));
        if (c) {
            const int q = qbase + (ctz32(c) >> 3);
            return q < b ? q : b;
        }
        i++;
        Li = Ln;
        Ki = Kn;
    }
}

CLY_NOINL void spec_lane(CLY_LDS ScanShared& S, int t) {
    const CLY_LDS ChunkCtx& C = S.C;
    const CLY_LDS uint8_t* w = (const CLY_LDS uint8_t*)(S.win);
    S.sp_s[t] = -1; S.sp_last[t] = -1; S.sp_cnt[t] = 0; S.sp_vin[t] = 0; S.sp_x[t] = 0;
    const int a = t * CLY_SUB;
    if (a >= C.dlen) return;
    const int b = a + CLY_SUB < C.dlen ? a + CLY_SUB : C.dlen;
    for (int q = next_candidate(S.win, a, b); q < b; q = next_candidate(S.win, q + 1, b)) {
        Hdr h = step_hdr(w, q, C.nrel, C.cbase + q);
        if (!h.good) continue;
        int64_t p = q;
        int c = 1;
        int64_t x = p + h.size;
        bool ok = true;
        while (x < b) {
            const Hdr h2 = step_hdr(w, x, C.nrel, C.cbase + x);
            if (!h2.good) { ok = false; break; }
            p = x;
            c++;
            x = p + h2.size;
        }
        if (!ok) continue;
        uint8_t vin = 1;
        if (x < C.nrel) {
            const int64_t need = C.nrel - x < 26 ? C.nrel - x : 26;
            if (x + need <= C.win_len) {
                const Hdr e = step_hdr(w, x, C.nrel, C.cbase + x);
                if (!e.good) continue;
            } else {
                // exit beyond the window: check its header in global memory
                uint8_t hb[28];
                const uint8_t* gp = C.gfile + C.cbase + x;
                for (int k = 0; k < need; k++) hb[k] = gp[k];
                const Hdr e = step_hdr(hb, 0, C.nrel - x, C.cbase + x);
                if (!e.good) continue;
            }
        }
        // keep the first candidate; a later one with a checked exit replaces
        // one whose exit could not be checked (then the scan stops)
        if (S.sp_s[t] < 0 || vin) {
            S.sp_s[t] = (int16_t)q; S.sp_last[t] = (int16_t)p; S.sp_cnt[t] = (uint16_t)c; S.sp_vin[t] = vin;
            S.sp_x[t] = (uint32_t)x;
        }
        if (vin) return;
    }
}

// Exact walk (ReadLogRecord semantics, any record or terminal) of stripe k
// from position e.
CLY_NOINL void exact_walk(CLY_LDS ScanShared& S, int k, int e) {
    const CLY_LDS ChunkCtx& C = S.C;
    const CLY_LDS uint8_t* w = (const CLY_LDS uint8_t*)(S.win);
    const int a = k * CLY_SUB;
    const int b = a + CLY_SUB < C.dlen ? a + CLY_SUB : C.dlen;
    (void)a;
    S.ws[k] = (int16_t)e;
    int64_t p = e;
    int c = 0, last = -1;
    for (;;) {
        const Hdr h = step_hdr(w, p, C.nrel, C.cbase + p);
        if (h.status != REC_OK) {
            S.wc[k] = (uint16_t)c; S.wl[k] = (int16_t)last; S.wx[k] = (uint32_t)p;
            S.wterm[k] = 1; S.wtst[k] = (int8_t)h.status;
            return;
        }
        c++;
        last = (int)p;
        const int64_t p2 = p + h.size;
        if (p2 >= b) {
            S.wc[k] = (uint16_t)c; S.wl[k] = (int16_t)last; S.wx[k] = (uint32_t)p2;
            S.wterm[k] = 0; S.wtst[k] = 0;
            return;
        }
        p = p2;
    }
}

// ---------------------------------------------------------------------------
// resolve(E): the chunk's record chain from entry E (chunk-relative, < dlen or
// >= dlen for "no lane").  Fills ws/wc/wl/wx/wterm/pk/base and S.R.
template <class EX>
CLY_DEV void resolve(EX& ex, CLY_LDS ScanShared& S, int E) {
    const int dlen = S.C.dlen;
    if (E >= dlen) {
        // only in the file's last chunk: E is the end of the file (ReadLogRecord there: io.EOF)
        ex.all([&](int t) { S.ws[t] = -1; S.wterm[t] = 0; S.pk[t] = -1; S.base[t] = 0; });
        ex.one([&]() {
            const CLY_LDS uint8_t* w = (const CLY_LDS uint8_t*)(S.win);
            CLY_LDS ChainRes& R = S.R;
            R.E = E; R.k0 = CLY_NT; R.cnt = 0; R.last = -1; R.lterm = CLY_NT; R.xrel = E;
            R.tpos = E; R.eof_exit = 0;
            const Hdr h = step_hdr(w, E, S.C.nrel, S.C.cbase + E);
            R.term = h.status != REC_OK;
            R.tst = h.status != REC_OK ? h.status : 0;
        });
        return;
    }
    const int k0 = E / CLY_SUB;
    ex.all([&](int t) {
        if (t < k0 || t * CLY_SUB >= dlen) { S.ws[t] = -1; S.wc[t] = 0; }
        else { S.ws[t] = S.sp_s[t]; S.wx[t] = S.sp_x[t]; S.wc[t] = S.sp_cnt[t]; S.wl[t] = S.sp_last[t]; }
        S.wterm[t] = 0;
    });
    ex.one([&]() {
        if (S.ws[k0] != E) exact_walk(S, k0, E);
        S.fix_lo = k0; S.fix_hi = k0; S.fix_kill = S.wterm[k0] ? k0 : CLY_NT;
    });
    ex.all([&](int t) { if (t > S.fix_kill) S.ws[t] = -1; });
    for (int iter = 0;; iter++) {
        ex.scan_max_incl([&](int t) -> int { return S.ws[t] >= 0 ? t : -1; }, S.pk);
        const int kstar = ex.reduce_min([&](int t) -> int {
            if (t <= k0 || t * CLY_SUB >= dlen) return CLY_NT;
            const int j = S.pk[t - 1];
            if (S.wterm[j]) return CLY_NT;
            const uint32_t X = S.wx[j];
            const int end = (t + 1) * CLY_SUB < dlen ? (t + 1) * CLY_SUB : dlen;
            if (S.ws[t] >= 0) return X != (uint32_t)S.ws[t] ? t : CLY_NT;
            return X < (uint32_t)end ? t : CLY_NT;
        });
        if (kstar >= CLY_NT) break;
        if (iter > CLY_NT + 1) { ex.one([&]() { S.fail = 1; S.fail_k = kstar; }); break; }   // cannot happen: each fix advances
        ex.one([&]() {
            const int j = S.pk[kstar - 1];
            const uint32_t X = S.wx[j];
            const int K = X < (uint32_t)dlen ? (int)(X / CLY_SUB) : CLY_NT;
            S.fix_lo = j;
            S.fix_hi = K;
            S.fix_kill = CLY_NT;
            if (K < CLY_NT && S.ws[K] != (int)X) {
                exact_walk(S, K, (int)X);
                if (S.wterm[K]) S.fix_kill = K;
            }
        });
        ex.all([&](int t) { if ((t > S.fix_lo && t < S.fix_hi) || t > S.fix_kill) S.ws[t] = -1; });
    }
    const int total = ex.scan_add_excl([&](int t) -> int { return S.ws[t] >= 0 ? (int)S.wc[t] : 0; }, S.base);
    ex.one([&]() {
        CLY_LDS ChainRes& R = S.R;
        const int L = S.pk[CLY_NT - 1];
        R.E = E; R.k0 = k0; R.cnt = total;
        R.term = S.wterm[L]; R.tst = S.wtst[L];
        R.lterm = R.term ? L : CLY_NT;
        R.tpos = S.wx[L];
        R.xrel = S.wx[L];
        R.last = S.wl[L];
        R.eof_exit = 0;
        if (!R.term && S.C.lof && R.xrel == S.C.nrel) {
            // the chain leaves the file's last chunk exactly at the end of the
            // file: the next ReadLogRecord there returns io.EOF
            R.term = 1; R.tst = CLY_END_EOF; R.tpos = R.xrel; R.lterm = CLY_NT; R.eof_exit = 1;
        }
    });
}

// ---------------------------------------------------------------------------
// CRC of every record in the chunk for the current mode / chain.
//   per lane: phase A (stripe-local registers), segmented scan over lanes
//   (element (c, v): S -> c ? v : A^SUB S ^ v), phase B (heads that need the
//   register entering the stripe).  Sets S.bad, S.head_raw, S.end_state.
#define OPN_HEAD (-2)
CLY_DEV void note_bad(CLY_LDS ScanShared& S, unsigned long long key) {
#ifdef __HIPCC__
    atomicMin(&S.bad, key);
#else
    if (key < S.bad) S.bad = key;
#endif
}

// Phase A of lane t: registers of the record pieces inside the stripe; writes
// the scan element (sc_v[0][t], sc_c[0][t]).
CLY_NOINL void crc_lane_a(CLY_LDS ScanShared& S, int t) {
    const int dlen = S.C.dlen;
    const int mode = S.mode;
    const CLY_LDS ChainRes& R = S.R;
    const CLY_LDS uint8_t* w = (const CLY_LDS uint8_t*)(S.win);
    CrcTab T{S.tab, t % CLY_REP};
    const int a = t * CLY_SUB;
    const int b = a + CLY_SUB < dlen ? a + CLY_SUB : dlen;
    S.sc_v[0][t] = 0; S.sc_c[0][t] = 1; S.sc_c0[t] = 1;
    if (a >= dlen || mode == MODE_DEAD || (mode == MODE_NORMAL && t > R.lterm)) return;
    const bool on = mode == MODE_NORMAL && S.ws[t] >= 0;
    const int opn = (mode == MODE_PASS || t <= R.k0) ? OPN_HEAD : S.wl[S.pk[t - 1]];
    const int e1 = on ? S.ws[t] : b;
    uint8_t c = 1;
    uint32_t v = 0;
    // head segment [a, e1) of record opn
    if (opn == OPN_HEAD) {
        const int lo = a < 4 ? 4 : a;
        if (t == 0) {
            const uint32_t r = lo < e1 ? crc_run(T, 0u, w, lo, e1) : 0u;
            if (on) S.head_raw = r;
            else { c = 1; v = r; }
        } else if (!on) {
            c = 0; v = crc_run(T, 0u, w, a, b);
        }
        // on && t > 0: phase B
    } else {
        const int cs = opn + 4;
        if (on) {
            if (cs > a || cs >= e1) {
                const uint32_t r = cs < e1 ? crc_run(T, 0xFFFFFFFFu, w, cs, e1) : 0xFFFFFFFFu;
                if (~r != le32(w + opn)) {
                    const int j = S.pk[t - 1];
                    note_bad(S, ((unsigned long long)(uint32_t)opn << 32) | (uint32_t)(S.base[j] + S.wc[j] - 1));
                }
            }
            // else phase B
        } else {
            if (cs >= b) { c = 1; v = 0xFFFFFFFFu; }
            else if (cs > a) { c = 1; v = crc_run(T, 0xFFFFFFFFu, w, cs, b); }
            else { c = 0; v = crc_run(T, 0u, w, a, b); }
        }
    }
    // records starting in the stripe
    if (on) {
        int64_t p = S.ws[t];
        const int n = S.wc[t];
        for (int i = 0; i < n; i++) {
            const Hdr h = step_hdr(w, p, S.C.nrel, S.C.cbase + p);
            const int64_t pe = p + h.size;
            const int cs = (int)p + 4;
            if (pe < b) {
                const uint32_t r = crc_run(T, 0xFFFFFFFFu, w, cs, (int)pe);
                if (~r != h.crc) note_bad(S, ((unsigned long long)(uint32_t)p << 32) | (uint32_t)(S.base[t] + i));
                p = pe;
            } else {
                // the last record is open at the stripe end
                S.sc_v[0][t] = cs < b ? crc_run(T, 0xFFFFFFFFu, w, cs, b) : 0xFFFFFFFFu;
                S.sc_c[0][t] = 1; S.sc_c0[t] = 1;
                return;
            }
        }
        // every record closed inside the stripe: a terminal follows
        S.sc_v[0][t] = 0; S.sc_c[0][t] = 1; S.sc_c0[t] = 1;
        return;
    }
    S.sc_v[0][t] = v; S.sc_c[0][t] = c; S.sc_c0[t] = c;
}

// Phase B of lane t (after the scan; sc_v[fin] holds the inclusive scan).
CLY_NOINL void crc_lane_b(CLY_LDS ScanShared& S, int t, int fin) {
    const int dlen = S.C.dlen;
    const int mode = S.mode;
    const CLY_LDS ChainRes& R = S.R;
    const CLY_LDS uint8_t* w = (const CLY_LDS uint8_t*)(S.win);
    CrcTab T{S.tab, t % CLY_REP};
    const int a = t * CLY_SUB;
    const int b = a + CLY_SUB < dlen ? a + CLY_SUB : dlen;
    const int last_lane = dlen > 0 ? (dlen - 1) / CLY_SUB : 0;
    if (a >= dlen || mode == MODE_DEAD || (mode == MODE_NORMAL && t > R.lterm)) return;
    const bool on = mode == MODE_NORMAL && S.ws[t] >= 0;
    if (t == last_lane) {
        // register at the end of the data (open record / pass-through head)
        if (t > 0 && !S.sc_c0[t] && b - a < CLY_SUB) S.end_state = crc_run(T, S.sc_v[fin][t - 1], w, a, b);
        else S.end_state = S.sc_v[fin][t];
    }
    if (!on || t == 0) return;
    const int opn = t <= R.k0 ? OPN_HEAD : S.wl[S.pk[t - 1]];
    const int e1 = S.ws[t];
    if (opn == OPN_HEAD) {
        S.head_raw = crc_run(T, S.sc_v[fin][t - 1], w, a, e1);
        return;
    }
    const int cs = opn + 4;
    if (cs > a || cs >= e1) return;       // done in phase A
    const uint32_t r = crc_run(T, S.sc_v[fin][t - 1], w, a, e1);
    if (~r != le32(w + opn)) {
        const int j = S.pk[t - 1];
        note_bad(S, ((unsigned long long)(uint32_t)opn << 32) | (uint32_t)(S.base[j] + S.wc[j] - 1));
    }
}

// CRC of every record in the chunk for the current mode / chain: phase A,
// segmented Kogge-Stone scan over lanes (element (c, v): S -> c ? v :
// A^SUB S ^ v), phase B.  Sets S.bad, S.head_raw, S.end_state.
template <class EX>
CLY_DEV void crc_phase(EX& ex, CLY_LDS ScanShared& S, const uint32_t* shift_tabs) {
    ex.one([&]() { S.bad = ~0ull; S.head_raw = 0; S.end_state = 0; });
    ex.all([&](int t) { crc_lane_a(S, t); });
    // levels stop once every element is constant (records shorter than a few
    // stripes: 1-2 levels instead of log2(NT))
    int cur = 0;
    bool all_const = ex.all_and([&](int t) -> int { return S.sc_c[0][t]; });
    for (int lvl = 0, d = 1; d < CLY_NT && !all_const; lvl++, d <<= 1) {
        const int src = cur;
        all_const = ex.all_and([&](int t) -> int {
            uint32_t v = S.sc_v[src][t];
            uint8_t c = S.sc_c[src][t];
            if (t >= d && !c) {
                v ^= shift_tab(shift_tabs, lvl, S.sc_v[src][t - d]);
                c = S.sc_c[src][t - d];
            }
            S.sc_v[src ^ 1][t] = v;
            S.sc_c[src ^ 1][t] = c;
            return c;
        });
        cur ^= 1;
    }
    const int fin = cur;
    ex.all([&](int t) { crc_lane_b(S, t, fin); });
}

// Tuples for the records starting in lane t's stripe.
CLY_NOINL void emit_lane(CLY_LDS ScanShared& S, int t, cly_tuple* out, uint64_t out_cap, unsigned* overflow) {
    if (S.mode != MODE_NORMAL || S.ws[t] < 0) return;
    const CLY_LDS uint8_t* w = (const CLY_LDS uint8_t*)(S.win);
    const int n = S.wc[t];
    uint64_t idx = S.p_excl + (uint64_t)S.base[t];
    int64_t p = S.ws[t];
    for (int i = 0; i < n; i++, idx++) {
        const Hdr h = step_hdr(w, p, S.C.nrel, S.C.cbase + p);
        if (idx < out_cap) {
            cly_tuple tp;
            tp.offset = S.C.cbase + p;
            tp.expiration = h.exp;
            tp.fid = S.C.fid;
            tp.size = (uint32_t)h.size;
            tp.key_size = h.ks;
            tp.value_size = h.vs;
            tp.type = h.type;
            tp.data_type = h.dt;
            tp.header_size = (uint8_t)h.hsz;
            tp.crc = h.crc;
            int tn;
            const int64_t klim = h.ks < 11u ? (int64_t)h.ks : 11;
            const int64_t tx = go_varint(w + p + h.hsz, klim, tn);      // parseLogRecordKey, db.go:706-710
            if (tn < 0) { tp.tx_id = 0; tp.txid_len = 0xFF; }
            else { tp.tx_id = tx; tp.txid_len = (uint8_t)tn; }
            out[idx] = tp;
        } else {
            *overflow = 1;
        }
        p += h.size;
    }
}

// Chunk summary for k_fin (one lane).
// x8n[n] = x^(8n) mod P for n in [0, CLY_CHUNK] (host-built table).
CLY_DEV void write_summary(CLY_LDS ScanShared& S, ChunkSum* sums, const uint32_t* x8n) {
    const CLY_LDS ChunkCtx& C = S.C;
    const CLY_LDS uint8_t* w = (const CLY_LDS uint8_t*)(S.win);
    ChunkSum cs;
    cs.p_excl = S.p_excl;
    cs.evt_off = EVT_NONE;
    cs.evt_gidx = 0;
    cs.evt_status = 0;
    cs.cnt = 0;
    cs.open_pos = -1;
    cs.open_state = 0;
    cs.open_crc = 0;
    cs.first4 = S.win[0];
    cs.head_raw = 0;
    cs.head_len = 0;
    cs.flags = 0;
    cs._pad = 0;
    if (S.mode == MODE_DEAD) {
        cs.flags = SUM_DEAD;
    } else if (S.mode == MODE_PASS) {
        cs.head_len = (uint32_t)C.dlen;
        cs.head_raw = S.end_state;
        if (C.lof) {
            cs.flags |= SUM_CLOSES;                // the covering record ends at the file end
            cs.evt_off = C.cbase + C.dlen;          // io.EOF at the end of the file
            cs.evt_gidx = S.p_excl;
            cs.evt_status = CLY_END_EOF;
        }
    } else {
        const CLY_LDS ChainRes& R = S.R;
        cs.cnt = (uint32_t)R.cnt;
        cs.flags |= SUM_CLOSES;
        cs.head_len = (uint32_t)(R.E < C.dlen ? R.E : C.dlen);
        cs.head_raw = R.E < C.dlen ? S.head_raw : S.end_state;
        if (S.bad != ~0ull) {
            cs.evt_off = C.cbase + (int64_t)(S.bad >> 32);
            cs.evt_gidx = S.p_excl + (S.bad & 0xffffffffull);
            cs.evt_status = CLY_ERR_CRC;
        } else if (R.term) {
            cs.evt_off = C.cbase + R.tpos;
            cs.evt_gidx = S.p_excl + (uint64_t)R.cnt;
            cs.evt_status = R.tst;
        }
        // the last record on the chain is still open at the end of the data
        // unless a terminal follows it inside the chunk
        if ((!R.term || R.eof_exit) && R.cnt > 0 && R.last >= 0) {
            cs.flags |= SUM_OPEN;
            cs.open_pos = C.cbase + R.last;
            cs.open_state = S.end_state;
            cs.open_crc = le32(w + R.last);
        }
    }
    if (cs.head_len > (uint32_t)CLY_CHUNK) { S.fail = 3; cs.head_len = 0; }     // internal error guard
    cs.head_shift = cs.head_len > 4 ? x8n[cs.head_len - 4] : (1u << 31);
    sums[C.chunk] = cs;
}

// ---------------------------------------------------------------------------
// k_fin helpers: finish the CRC of the record open at the end of chunk i by
// walking the heads of the following chunks of the file.
CLY_DEV uint32_t fin_advance(uint32_t s, int64_t ocs, const ChunkSum& H, int64_t hstart) {
    const int64_t hlen = H.head_len;
    const int64_t l4 = hlen < 4 ? hlen : 4;
    int lo = 0;
    if (ocs > hstart) lo = (int)(ocs - hstart < l4 ? ocs - hstart : l4);
    for (int k = lo; k < l4; k++) s = cly_crc_byte_bitwise(s, (uint8_t)(H.first4 >> (8 * k)));
    if (hlen > 4) s = cly_multmodp(H.head_shift, s) ^ H.head_raw;
    return s;
}

// Event of chunk i of a file (chunks c0 .. c0+nc-1): in-chunk event, or the
// CRC failure of its open record.  Returns the file offset (EVT_NONE if none).
CLY_DEV int64_t fin_chunk_event(const ChunkSum* sums, int c0, int nc, int i, uint64_t* gidx, int32_t* status) {
    const ChunkSum S = sums[c0 + i];
    int64_t off = EVT_NONE;
    uint64_t g = 0;
    int32_t st = 0;
    if (!(S.flags & SUM_DEAD)) {
        off = S.evt_off;
        g = S.evt_gidx;
        st = S.evt_status;
        if (S.flags & SUM_OPEN) {
            uint32_t s = S.open_state;
            const int64_t ocs = S.open_pos + 4;
            for (int j = i + 1; j < nc; j++) {
                const ChunkSum H = sums[c0 + j];
                s = fin_advance(s, ocs, H, (int64_t)j * CLY_CHUNK);
                if (H.flags & SUM_CLOSES) break;
            }
            if (~s != S.open_crc && (off == EVT_NONE || S.open_pos < off)) {
                off = S.open_pos;
                g = S.p_excl + S.cnt - 1;
                st = CLY_ERR_CRC;
            }
        }
    }
    *gidx = g;
    *status = st;
    return off;
}

// Per-chunk trace record (written only when a debug buffer is supplied).
struct ChunkDbg {
    int64_t  entry_g;
    uint64_t p_excl;
    int64_t  xrel;
    int64_t  tpos;
    int32_t  mode, guess, E, cnt, term, tst, in_dead, k0;
};

// Per-lane trace (debug builds of the trace only; 8 ints per lane).
CLY_DEV void dbg_lane_fill(const CLY_LDS ScanShared& S, int t, int* o) {
    o[0] = S.sp_s[t]; o[1] = (int)S.sp_x[t]; o[2] = S.sp_cnt[t]; o[3] = S.ws[t];
    o[4] = (int)S.wx[t]; o[5] = S.wc[t]; o[6] = S.pk[t]; o[7] = S.base[t] | (S.wterm[t] << 16) | (S.fail_k << 20);
}

// ---------------------------------------------------------------------------
// The chunk pipeline, common to kernel and emulator.  Env supplies the global
// memory side: publish/lookback of descriptors, ticket, file table.
template <class EX, class Env>
CLY_DEV void chunk_body(EX& ex, CLY_LDS ScanShared& S, Env& env) {
    // ---- stage
    ex.one([&]() { S.fail = 0; env.mark(S, 1); });
    ex.all([&](int t) { env.stage_lane(S, t); env.stage_wait(); });
    // ---- speculation
    ex.all([&](int t) { spec_lane(S, t); });
    // ---- guess the entry: the first lane whose walk left through a checked
    //      exit, else the first lane with any walk (first chunk of a file: 0)
    {
        const int key = ex.reduce_min([&](int t) -> int {
            if (S.sp_s[t] < 0) return 2 * CLY_NT;
            return S.sp_vin[t] ? t : CLY_NT + t;
        });
        ex.one([&]() {
            int g = -1;
            if (S.C.fof) g = 0;
            else if (key < 2 * CLY_NT) g = S.sp_s[key % CLY_NT];
            S.guess = g;
            S.mode = g >= 0 ? MODE_NORMAL : MODE_PASS;
            env.mark(S, 2);
        });
    }
    if (S.guess >= 0) resolve(ex, S, S.guess);
    ex.all([&](int t) { env.dbg_lane(S, t); });
    // ---- publish the speculative descriptor
    const int64_t cg = (int64_t)S.C.chunk * CLY_CHUNK;
    ex.one([&]() {
        const CLY_LDS ChainRes& R = S.R;
        const uint32_t ep = env.epoch;
        if (S.guess >= 0)
            env.publish_spec(S.C.chunk, ds_pack(ep, DS_SPEC, S.C.fof, R.term, 1, S.guess, (uint32_t)R.cnt),
                             ds_tag(ep, (uint64_t)(cg + R.xrel)));
        else
            env.publish_spec(S.C.chunk, ds_pack(ep, DS_SPEC, S.C.fof, 0, 0, 0, 0), ds_tag(ep, 0));
        env.mark(S, 3);
    });
    // ---- CRC under the guessed chain (overlaps the wait for predecessors)
    env.crc(ex, S);
    ex.one([&]() { env.mark(S, 4); });
    // ---- look-back: true entry and output slot
    ex.all([&](int t) { env.lookback(S, t); });
    ex.one([&]() {
        if (!env.spin_ok()) { S.fail = 4; S.in_dead = 1; }
        if (!S.in_dead && S.entry_g < cg) { S.fail = 2; S.in_dead = 1; }   // cannot happen
        env.mark(S, 5);
    });
    // ---- the true chain (re-resolved, and its CRC redone, when the guess was wrong)
    ex.one([&]() { S.redo_crc = 0; });
    if (S.in_dead) {
        ex.one([&]() { S.mode = MODE_DEAD; S.R.cnt = 0; S.R.term = 1; });
    } else if (S.entry_g >= cg + CLY_CHUNK) {
        if (S.mode != MODE_PASS) ex.one([&]() { S.mode = MODE_PASS; S.R.cnt = 0; S.R.term = 0; S.redo_crc = 1; });
    } else {
        const int newE = (int)(S.entry_g - cg);
        if (S.mode != MODE_NORMAL || S.guess != newE) {
            ex.one([&]() { S.mode = MODE_NORMAL; S.redo_crc = 1; });
            resolve(ex, S, newE);
        }
    }
    // ---- publish the resolved descriptor
    ex.one([&]() {
        const CLY_LDS ChainRes& R = S.R;
        uint64_t X;
        int dead;
        uint32_t cnt = 0;
        if (S.mode == MODE_DEAD) { X = 0; dead = 1; }
        else if (S.mode == MODE_PASS) { X = (uint64_t)S.entry_g; dead = 0; }
        else { X = (uint64_t)(cg + R.xrel); dead = R.term; cnt = (uint32_t)R.cnt; }
        const uint32_t ep = env.epoch;
        env.publish_full(S.C.chunk, ds_pack(ep, DS_FULL, S.C.fof, dead, 0, 0, cnt), ds_tag(ep, X),
                         ds_tag(ep, S.p_excl + cnt), S.p_excl + cnt);
        env.mark(S, 6);
    });
    // ---- CRC again when the chain changed (successors already have the FULL words)
    if (S.redo_crc) env.crc(ex, S);
    // ---- tuples, summary
    ex.all([&](int t) { env.emit_lane(S, t); });
    ex.one([&]() {
        env.mark(S, 7);
        ChunkDbg* d = env.dbg_slot(S.C.chunk);
        if (d) {
            d->entry_g = S.entry_g; d->p_excl = S.p_excl; d->xrel = S.R.xrel; d->tpos = S.R.tpos;
            d->mode = S.mode; d->guess = S.guess; d->E = S.R.E; d->cnt = S.R.cnt; d->term = S.R.term;
            d->tst = S.R.tst; d->in_dead = S.in_dead; d->k0 = S.R.k0;
        }
        env.summary(S);
        env.mark(S, 8);
        if (S.fail) env.report_fail(S);
    });
}
