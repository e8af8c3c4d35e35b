// clyscan.hip — MI355X (gfx950) log-record scan for CouloyDB data files.
//
// Product library libclyscan.so: HIP kernels + the C-ABI of include/clyscan.h.
// It restates, for whole files at once, the loop
//     for { rec, size, err := df.ReadLogRecord(offset); ...; offset += size }
// of db.loadIndex (db.go:582-637) / db.merge (merge.go:90-143) /
// loadIndexFromHintFile (merge.go:257-287), with the per-record semantics of
// DataFile.ReadLogRecord (data/dataFile.go:64-111), DecodeLogRecordHeader
// (data/logRecord.go:86-114), GetLogRecordCRC (data/logRecord.go:136-146) and
// parseLogRecordKey (db.go:706-710).  Design and data layout: DESIGN.md.
//
// Pipeline per call (one HIP stream):
//   k_scan    one workgroup per CHUNK bytes of one file (dynamic ticket order).
//             Stages the chunk in LDS, finds record boundaries by per-lane
//             speculative header walks resolved inside the workgroup, verifies
//             every record's CRC-32 with LDS slicing tables and a segmented
//             scan for records spanning lanes, counts records with a decoupled
//             look-back, and writes cly_tuple entries plus a chunk summary.
//   k_check / k_finish: check the chunk-level speculation
//             (each chunk's guessed entry == its predecessor's exit), finishes
//             the CRC of records that straddle chunks, and derives the per-file
//             (n_records, end_offset, status).  A failed check (rare) asks the
//             host for a repair pass that re-runs k_scan with forced entries.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/clyscan.h"
#include "crc_gf.h"

#ifndef CLY_NT
#define CLY_NT 256            // threads per workgroup (4 waves)
#endif
#ifndef CLY_SUB
#define CLY_SUB 128           // bytes per lane (walk sub-segment == CRC stripe)
#endif
#ifndef CLY_REP
#define CLY_REP 2             // LDS replication of the slicing tables (bank spread)
#endif
#define CLY_CHUNK (CLY_NT * CLY_SUB)
#define CLY_HALO 64
#define CLY_WIN (CLY_CHUNK + CLY_HALO)
constexpr int cly_log2(int v) { return v <= 1 ? 0 : 1 + cly_log2(v >> 1); }
#define CLY_SCAN_LEVELS cly_log2(CLY_NT)
static_assert((1 << CLY_SCAN_LEVELS) == CLY_NT, "CLY_NT must be a power of two");
static_assert(CLY_SUB % 16 == 0 && CLY_SUB >= 32, "CLY_SUB must be a multiple of 16");
static_assert(CLY_CHUNK <= 65536, "chunk offsets are kept in 16+ bits");

#define REC_OK 100
#define FORCE_GUESS (-1LL)
#define FORCE_SKIP (-2LL)
#define LB_AGG (1ULL << 62)
#define LB_INC (1ULL << 63)
#define LB_MASK ((1ULL << 62) - 1)

// ---------------------------------------------------------------------------
// Device-side data structures
struct DevFile {                 // 32 B
    const uint8_t* base;         // device pointer to the file's first byte
    uint64_t len;
    uint32_t fid;
    uint32_t first_chunk;        // global index of the file's first chunk
    uint32_t nchunks;
    uint32_t _pad;
};

struct ChunkSum {                // 80 B, written by k_scan, read by k_check / k_finish
    int64_t  entry;              // first chain position used (file offset), -1 none
    int64_t  exit;               // first chain position >= chunk end, or the TERM position
    int64_t  open_pos;           // chain's last record if it is still open at chunk end, else -1
    int64_t  bad_pos;            // first in-chunk CRC failure (file offset) or -1
    uint32_t n_records;
    uint32_t bad_idx;            // local index of that record
    int32_t  term;               // 1 if the chain terminated inside this chunk
    int32_t  term_status;        // CLY_END_* / CLY_ERR_* of the terminal position
    uint32_t open_state;         // CRC register of the open record at chunk end
    uint32_t open_crc;           // its stored CRC
    uint32_t head_raw;           // raw register over [start+4, start+head_len)
    uint32_t first4;             // first 4 bytes of the chunk (little-endian)
    uint32_t head_len;           // bytes before the first boundary (or chunk length)
    uint32_t chunk_len;
    uint32_t head_shift;         // x^(8*(head_len-4)) mod P: advances a register over head_raw's span
    uint32_t _pad;
};
static_assert(sizeof(ChunkSum) == 80, "ChunkSum layout");

struct FileOut {                 // per-file result from k_finish
    uint64_t n_records;
    int64_t  end_offset;
    int32_t  status;
    int32_t  repair;             // 1 = speculation failed before the file end
    uint64_t first_index;        // global tuple index of the file's first record
};

struct Globals {                 // small control block, zeroed per pass
    uint32_t ticket;
    uint32_t repair;             // any file needs a repair pass
    uint32_t lb_timeout;         // look-back spin bound hit (never expected)
    uint32_t overflow;           // tuples beyond out_cap were dropped
    uint64_t total_records;      // inclusive count after the last chunk
    uint32_t dbg_site;           // CLY_DEBUG builds: first out-of-range global index
    uint32_t _pad;
    int64_t  dbg_idx, dbg_lim;
};

#ifdef CLY_DEBUG
__device__ int* g_trace;   // host-mapped progress trace (survives a device fault)
#define TRACE(slot, v) do { if (g_trace) { g_trace[(slot)] = (v); __threadfence_system(); } } while (0)
// Debug builds check every global index; a violation is recorded (site, index,
// limit) and the access is redirected to element 0 instead of faulting.
__device__ __forceinline__ int64_t cly_gidx(int64_t i, int64_t lim, unsigned site, Globals* g) {
    if (i < 0 || i >= lim) {
        if (atomicCAS(&g->dbg_site, 0u, site) == 0u) { g->dbg_idx = i; g->dbg_lim = lim; }
        return 0;
    }
    return i;
}
#define GIDX(i, lim, site) cly_gidx((int64_t)(i), (int64_t)(lim), (site), g)
#else
#define GIDX(i, lim, site) (i)
#define TRACE(slot, v) do { } while (0)
#endif

// ---------------------------------------------------------------------------
// Go encoding/binary Varint (toolchain >= 1.18): zigzag over Uvarint; overflow
// (10th byte > 1, or an 11th byte read) -> (0, -(i+1)); short buffer -> (0, 0).
__device__ __forceinline__ int64_t go_varint(const uint8_t* b, int64_t len, int& n) {
    uint64_t x = 0;
    unsigned s = 0;
    int lim = len < 11 ? (int)len : 11;
    for (int i = 0; i < lim; i++) {
        uint32_t c = b[i];
        if (i == 10) { n = -11; return 0; }
        if (c < 0x80) {
            if (i == 9 && c > 1) { n = -10; return 0; }
            n = i + 1;
            uint64_t ux = x | ((uint64_t)c << s);
            int64_t v = (int64_t)(ux >> 1);
            return (ux & 1) ? ~v : v;
        }
        x |= (uint64_t)(c & 0x7f) << s;
        s += 7;
    }
    n = 0;
    return 0;
}

struct Hdr {
    int32_t  status;    // REC_OK or a terminal status
    int32_t  hsz;       // headerSize
    int64_t  size;      // recordSize (REC_OK)
    int64_t  exp;
    uint32_t ks, vs, crc;
    uint8_t  type, dt;
    bool     good;      // plain record the writer produces: all varints ok, type<=4, dt<=4, ks>=1
};

// Exact ReadLogRecord header/kv semantics at window position p (chunk-relative),
// without the CRC comparison (done separately).  n = file length - chunk start
// (may exceed the window); p_abs = file offset of p (for the negative-offset
// test).  Mirrors data/dataFile.go:64-103 and data/logRecord.go:86-114.
__device__ __forceinline__ Hdr step_hdr(const uint8_t* w, int64_t p, int64_t n, int64_t p_abs) {
    Hdr h;
    h.good = false;
    int64_t m = n - p;
    if (m > 26) m = 26;
    if (m <= 4) { h.status = CLY_END_EOF; return h; }
    if (m == 5) { h.status = CLY_ERR_TRUNC5; return h; }
    const uint8_t* b = w + p;
    h.crc = (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
    h.type = b[4];
    h.dt = b[5];
    int64_t idx = 6;
    int na, nb, nc;
    int64_t ks = go_varint(b + idx, m - idx, na); idx += na;
    if (idx < 0) { h.status = CLY_ERR_VARINT; return h; }
    int64_t vs = go_varint(b + idx, m - idx, nb); idx += nb;
    if (idx < 0) { h.status = CLY_ERR_VARINT; return h; }
    h.exp = go_varint(b + idx, m - idx, nc); idx += nc;
    h.ks = (uint32_t)ks;
    h.vs = (uint32_t)vs;
    h.hsz = (int32_t)idx;
    if (h.crc == 0 && h.ks == 0 && h.vs == 0) { h.status = CLY_END_ZERO; return h; }
    int64_t kv = (int64_t)h.ks + (int64_t)h.vs;
    if (kv > 0) {
        if (p_abs + idx < 0) { h.status = CLY_ERR_OFFSET; return h; }
        if (n - (p + idx) < kv) { h.status = CLY_END_TORN; return h; }
    }
    if (idx < 4) { h.status = CLY_ERR_VARINT; return h; }
    h.status = REC_OK;
    h.size = idx + kv;
    h.good = na > 0 && nb > 0 && nc > 0 && h.type <= 4 && h.dt <= 4 && h.ks >= 1;
    return h;
}

// ---------------------------------------------------------------------------
// CRC helpers on LDS data.  Tables: slicing-by-4 (T0..T3), replicated CLY_REP
// times (entry i of table t for replica r at dword (t*256 + i)*CLY_REP + r).
struct CrcTab {
    const uint32_t* t;
    int r;
    __device__ __forceinline__ uint32_t at(int tab, uint32_t i) const {
        return t[((tab << 8) + (int)i) * CLY_REP + r];
    }
    __device__ __forceinline__ uint32_t byte(uint32_t s, uint32_t b) const {
        return at(0, (s ^ b) & 0xff) ^ (s >> 8);
    }
    __device__ __forceinline__ uint32_t word(uint32_t s, uint32_t d) const {
        s ^= d;
        return at(3, s & 0xff) ^ at(2, (s >> 8) & 0xff) ^ at(1, (s >> 16) & 0xff) ^ at(0, s >> 24);
    }
};

// Register s advanced over window bytes [lo, hi).
__device__ __forceinline__ uint32_t crc_run(const CrcTab& T, uint32_t s, const uint8_t* w, int lo, int hi) {
    while (lo < hi && (lo & 3)) { s = T.byte(s, w[lo]); lo++; }
    const uint32_t* w32 = (const uint32_t*)w;
    while (hi - lo >= 4) { s = T.word(s, w32[lo >> 2]); lo += 4; }
    while (lo < hi) { s = T.byte(s, w[lo]); lo++; }
    return s;
}

// A^(CLY_SUB * 2^lvl) applied through a host-built 4x256 table (global memory).
__device__ __forceinline__ uint32_t shift_tab(const uint32_t* __restrict__ st, int lvl, uint32_t v) {
    const uint32_t* t = st + lvl * 1024;
    return t[v & 0xff] ^ t[256 + ((v >> 8) & 0xff)] ^ t[512 + ((v >> 16) & 0xff)] ^ t[768 + (v >> 24)];
}

// ---------------------------------------------------------------------------
// LDS layout of k_scan
struct LaneInfo {
    int32_t s;        // speculative / confirmed first chain position in the lane's stripe (-1 none)
    int32_t x;        // exit (first chain position >= stripe end) or terminal position
    int32_t last;     // last chain position (record start) inside the stripe
    int32_t prev;     // resolver: last chain position before the stripe (-1: chunk head)
    uint16_t cnt;     // records starting in the stripe
    uint8_t conf;     // resolver: stripe lies on the chain
    uint8_t lterm;    // walk ended at an END_EOF terminal (speculation) / TERM (confirmed)
    int32_t base;     // resolver: local index of the stripe's first record
    int32_t term_st;  // confirmed: terminal status if the chain ends in this stripe
};

struct ScanShared {
    uint32_t win[CLY_WIN / 4];                    // chunk bytes (+ halo)
    uint32_t tab[4 * 256 * CLY_REP];              // slicing-by-4 tables
    LaneInfo lane[CLY_NT];
    uint32_t sc_v[2][CLY_NT];                     // segmented scan: register value
    uint8_t  sc_c[2][CLY_NT];                     //                 1 = constant (reset inside)
    unsigned long long bad;                       // packed (pos << 32 | idx) of the first CRC failure
    uint32_t head_raw;
    int32_t  chunk;                               // global chunk index (ticket)
    int32_t  fidx;                                // file index
    uint64_t out_base;
};

// One lane's speculative walk over its stripe [a, b): first candidate q whose
// chain of plain records leaves the stripe (and whose exit decodes as a plain
// record or END_EOF).  Returns the number of records on that walk.
__device__ void spec_walk(const uint8_t* w, int a, int b, int end_rel, int64_t n, int64_t cbase,
                          LaneInfo& L) {
    L.s = -1; L.x = -1; L.last = -1; L.cnt = 0; L.lterm = 0;
    for (int q = a; q < b; q++) {
        // quick filter: type<=4, dtype<=4, first key-size varint byte != 0
        if (w[q + 4] > 4 || w[q + 5] > 4 || w[q + 6] == 0) continue;
        Hdr h = step_hdr(w, q, n, cbase + q);
        if (!h.good) continue;
        int p = q, c = 0, x = -1;
        bool ok = true;
        uint8_t term = 0;
        for (;;) {
            const int64_t p2 = (int64_t)p + h.size;
            c++;
            if (p2 >= b) { x = (int)(p2 < 0x7fffffff ? p2 : 0x7fffffff); break; }
            h = step_hdr(w, (int)p2, n, cbase + p2);
            if (!h.good) {
                // only a clean end of file is accepted as a speculative exit
                if (h.status == CLY_END_EOF) { x = (int)p2; term = 1; }
                else ok = false;
                break;
            }
            p = (int)p2;
        }
        if (!ok) continue;
        if (!term && x < end_rel) {      // validate the exit position inside the chunk
            Hdr e = step_hdr(w, x, n, cbase + x);
            if (!e.good && e.status != CLY_END_EOF) continue;
        }
        L.s = q; L.x = x; L.cnt = (uint16_t)c; L.lterm = term; L.last = p;
        return;
    }
}

// Exact walk (any record / terminal) from position e inside stripe [a, b).
__device__ void exact_walk(const uint8_t* w, int e, int b, int64_t n, int64_t cbase, LaneInfo& L) {
    int p = e, c = 0, last = -1;
    L.s = e; L.lterm = 0; L.term_st = 0;
    for (;;) {
        Hdr h = step_hdr(w, p, n, cbase + p);
        if (h.status != REC_OK) { L.lterm = 1; L.term_st = h.status; L.x = p; break; }
        c++;
        last = p;
        int64_t p2 = (int64_t)p + h.size;
        if (p2 >= b) { L.x = (int)(p2 < 0x7fffffff ? p2 : 0x7fffffff); break; }
        p = (int)p2;
    }
    L.cnt = (uint16_t)c;
    L.last = last;
}

// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(CLY_NT)
k_scan(const DevFile* __restrict__ files, int nfiles, const uint32_t* __restrict__ file_chunk_prefix,
       int nchunks, const int64_t* __restrict__ forced, const uint32_t* __restrict__ shift_tabs,
       ChunkSum* __restrict__ sums, unsigned long long* __restrict__ lb, uint64_t* __restrict__ out_base,
       cly_tuple* __restrict__ out, uint64_t out_cap, Globals* __restrict__ g) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    ScanShared& S = *reinterpret_cast<ScanShared*>(smem_raw);
    const int tid = threadIdx.x;

    if (tid == 0) {
        int c = (int)atomicAdd(&g->ticket, 1u);
        S.chunk = c;
        // file containing chunk c: last f with prefix[f] <= c
        int lo = 0, hi = nfiles - 1;
        while (lo < hi) {
            int mid = (lo + hi + 1) >> 1;
            if ((int)file_chunk_prefix[GIDX(mid, nfiles + 1, 1)] <= c) lo = mid; else hi = mid - 1;
        }
        S.fidx = lo;
        S.bad = ~0ULL;
        S.head_raw = 0;
    }
    __syncthreads();
    const int chunk = S.chunk;
    if (chunk >= nchunks) return;                    // uniform
    const DevFile F = files[GIDX(S.fidx, nfiles, 2)];
    const int cl = chunk - (int)F.first_chunk;       // chunk index within the file
    const int64_t cbase = (int64_t)cl * CLY_CHUNK;   // file offset of the chunk start
    const int64_t n = (int64_t)F.len - cbase;        // bytes from chunk start to file end
    const int end_rel = (int)(n < CLY_CHUNK ? n : CLY_CHUNK);
    const int win_len = (int)(n < CLY_WIN ? n : CLY_WIN);

    // ---- stage the chunk (+halo) in LDS: 16-B loads, bytewise tail, zero fill
    {
        uint4* w4 = reinterpret_cast<uint4*>(S.win);
        const int nvec = win_len >> 4;
        for (int i = tid; i < CLY_WIN / 16; i += CLY_NT) {
            uint4 v = make_uint4(0, 0, 0, 0);
            if (i < nvec) v = reinterpret_cast<const uint4*>(F.base)[GIDX((cbase >> 4) + i, (F.len + 15) >> 4, 3)];
            else if (i == nvec) {
                uint32_t wv[4] = {0, 0, 0, 0};
                for (int k = 0; k < (win_len & 15); k++) wv[k >> 2] |= (uint32_t)F.base[GIDX(cbase + (i << 4) + k, F.len, 4)] << (8 * (k & 3));
                v = make_uint4(wv[0], wv[1], wv[2], wv[3]);
            }
            w4[i] = v;
        }
    }
    // ---- slicing-by-4 tables, built in place (T0 bitwise; Tk from Tk-1)
    for (int i = tid; i < 256; i += CLY_NT) {
        uint32_t c0 = i;
        for (int k = 0; k < 8; k++) c0 = (c0 & 1) ? (c0 >> 1) ^ CLY_POLY : c0 >> 1;
        uint32_t c = c0;
        for (int t = 0; t < 4; t++) {
            for (int r = 0; r < CLY_REP; r++) S.tab[((t << 8) + i) * CLY_REP + r] = c;
            // next table: one more zero byte
            uint32_t lo = c & 0xff;
            uint32_t tl = lo;
            for (int k = 0; k < 8; k++) tl = (tl & 1) ? (tl >> 1) ^ CLY_POLY : tl >> 1;
            c = (c >> 8) ^ tl;
        }
    }
    __syncthreads();
    const uint8_t* w = reinterpret_cast<const uint8_t*>(S.win);

    // ---- forced entry (repair pass) / chunk 0 of a file always enters at 0
    int64_t fe = forced ? forced[GIDX(chunk, nchunks, 5)] : FORCE_GUESS;
    if (cl == 0) fe = 0;

    // ---- per-lane speculative walks
    const int a = tid * CLY_SUB;
    const int b = min(a + CLY_SUB, end_rel);
    {
        LaneInfo L;
        L.prev = -1; L.conf = 0; L.base = 0; L.term_st = 0;
        if (a < end_rel && fe == FORCE_GUESS) spec_walk(w, a, b, end_rel, n, cbase, L);
        else { L.s = -1; L.x = -1; L.last = -1; L.cnt = 0; L.lterm = 0; }
        S.lane[tid] = L;
    }
    __syncthreads();

    // ---- resolver (one lane): walk the chain across stripes, re-walking
    //      exactly wherever the speculation does not match.
    if (tid == 0) {
        int E;
        if (fe >= 0) E = (int)(fe - cbase);
        else if (fe == FORCE_SKIP) E = -1;
        else {
            E = -1;
            for (int k = 0; k < CLY_NT; k++) if (S.lane[k].s >= 0) { E = S.lane[k].s; break; }
        }
        const int entry = E;
        int last = -1, base = 0, term = 0, term_st = 0, term_pos = -1;
        if (E >= 0 && E >= end_rel && (int64_t)E >= n - 5) {
            // entry at (or within 5 bytes of) the end of the file: exact terminal
            Hdr h = step_hdr(w, E, n, cbase + E);
            term = 1; term_st = h.status; term_pos = E;
        }
        if (E >= 0 && E < end_rel) {
            for (int k = 0; k < CLY_NT; k++) {
                LaneInfo& L = S.lane[k];
                const int la = k * CLY_SUB;
                const int lend = min(la + CLY_SUB, end_rel);
                if (la >= end_rel) { L.conf = 0; L.prev = last; L.base = base; L.cnt = 0; continue; }
                if (term || E >= lend) {      // stripe not on the chain (pass-through or after TERM)
                    L.conf = 0; L.prev = term ? -2 : last; L.base = base; L.cnt = 0;
                    continue;
                }
                // E lies in this stripe
                const bool spec_ok = (L.s == E) && (!L.lterm);
                if (!spec_ok) exact_walk(w, E, lend, n, cbase, L);
                else { L.term_st = 0; }
                L.conf = 1; L.prev = last; L.base = base;
                base += L.cnt;
                if (L.cnt) last = L.last;
                if (L.lterm) { term = 1; term_st = L.term_st; term_pos = L.x; }
                else E = L.x;
            }
        } else {
            for (int k = 0; k < CLY_NT; k++) {
                LaneInfo& L = S.lane[k];
                L.conf = 0; L.prev = -1; L.base = 0; L.cnt = 0;
            }
        }
        const bool has_first = entry >= 0 && entry < end_rel;
        ChunkSum& cs = sums[GIDX(chunk, nchunks, 6)];
        cs.entry = entry >= 0 ? cbase + entry : -1;
        cs.term = term;
        cs.term_status = term_st;
        cs.exit = term ? cbase + term_pos : (has_first ? cbase + E : -1);
        if (term && !has_first) cs.head_len = (uint32_t)end_rel;
        cs.n_records = (uint32_t)base;
        cs.open_pos = (!term && has_first && last >= 0) ? cbase + last : -1;
        cs.chunk_len = (uint32_t)end_rel;
        cs.head_len = (uint32_t)(has_first ? entry : end_rel);
        cs.head_shift = cs.head_len > 4 ? cly_x8n(cs.head_len - 4) : (1u << 31);
        cs.first4 = S.win[0];
        // decoupled look-back: publish this chunk's aggregate now
        unsigned long long v = (unsigned long long)base;
        if (chunk == 0) __hip_atomic_store(&lb[GIDX(chunk, nchunks, 7)], v | LB_INC, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else __hip_atomic_store(&lb[GIDX(chunk, nchunks, 7)], v | LB_AGG, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();

    // ---- CRC, phase A: each lane walks its confirmed records and runs the
    //      CRC register over its stripe; records closed inside the stripe are
    //      compared now; the open record's head waits for the scan (phase B).
    const LaneInfo L = S.lane[tid];
    CrcTab T{S.tab, tid % CLY_REP};
    const bool live_lane = (a < end_rel) && (L.prev != -2);
    int cs_open;                     // CRC range start of the record open at stripe start
    uint32_t init_open;
    if (L.prev >= 0) { cs_open = L.prev + 4; init_open = 0xFFFFFFFFu; }
    else { cs_open = 4; init_open = 0u; }       // chunk head: raw register
    // first boundary in the stripe: first record (conf) or terminal position
    int e1 = b;
    bool has_boundary = false;
    if (live_lane && L.conf) {
        has_boundary = true;
        e1 = L.s;
    }
    uint8_t sc_const = 1;
    uint32_t sc_val = 0;
    bool pending_head = false;          // head [a, e1) needs S_in
    if (live_lane) {
        if (cs_open >= a) {
            // the open record's CRC range starts inside this stripe (or it is the chunk head)
            uint32_t st = init_open;
            int lo = cs_open, hi = has_boundary ? e1 : b;
            if (lo < hi) st = crc_run(T, st, w, lo, hi);
            if (has_boundary) {
                if (L.prev >= 0) {
                    uint32_t stored = (uint32_t)w[L.prev] | ((uint32_t)w[L.prev + 1] << 8) |
                                      ((uint32_t)w[L.prev + 2] << 16) | ((uint32_t)w[L.prev + 3] << 24);
                    if (~st != stored) {
                        unsigned long long key = ((unsigned long long)(uint32_t)L.prev << 32) | (uint32_t)(L.base - 1);
                        atomicMin(&S.bad, key);
                    }
                } else {
                    S.head_raw = st;    // only one lane can own the first boundary
                }
            } else {
                sc_const = 1; sc_val = st;
            }
        } else if (has_boundary) {
            pending_head = true;
        } else {
            sc_const = 0;               // pure middle stripe of one record
            sc_val = crc_run(T, 0u, w, a, b);
        }
        if (has_boundary) {
            // records starting in this stripe
            int p = L.s;
            for (int i = 0; i < (int)L.cnt; i++) {
                Hdr h = step_hdr(w, p, n, cbase + p);
                int64_t pe = (int64_t)p + h.size;       // record end (next boundary)
                const int lo = p + 4;
                if (pe < b) {
                    uint32_t st = crc_run(T, 0xFFFFFFFFu, w, lo, (int)pe);
                    if (~st != h.crc) {
                        unsigned long long key = ((unsigned long long)(uint32_t)p << 32) | (uint32_t)(L.base + i);
                        atomicMin(&S.bad, key);
                    }
                    p = (int)pe;
                } else {
                    // open at stripe end
                    uint32_t st = 0xFFFFFFFFu;
                    if (lo < b) st = crc_run(T, st, w, lo, b);
                    sc_const = 1; sc_val = st;
                    break;
                }
            }
            if (L.lterm && L.cnt == 0) { sc_const = 1; sc_val = 0; }
            if (L.lterm) { sc_const = 1; sc_val = 0; }
            // last record closed exactly at a boundary inside the stripe (terminal)
        }
    } else {
        sc_const = 1; sc_val = 0;
    }
    // ---- segmented Kogge-Stone scan over lanes: element (c, v) maps S ->
    //      c ? v : A^SUB S ^ v.  Inclusive; lane 0 is always constant.
    int cur = 0;
    S.sc_v[0][tid] = sc_val;
    S.sc_c[0][tid] = sc_const;
    __syncthreads();
    {
        uint32_t v = sc_val;
        uint8_t c = sc_const;
        #pragma unroll 1
        for (int lvl = 0; lvl < CLY_SCAN_LEVELS; lvl++) {
            const int d = 1 << lvl;
            if (tid >= d && !c) {
                uint32_t pv = S.sc_v[cur][tid - d];
                uint8_t pc = S.sc_c[cur][tid - d];
                v ^= shift_tab(shift_tabs, lvl, pv);
                c = pc;
            }
            S.sc_v[cur ^ 1][tid] = v;
            S.sc_c[cur ^ 1][tid] = c;
            __syncthreads();
            cur ^= 1;
        }
    }
    // ---- phase B: heads that close the record open at stripe start
    if (pending_head) {
        uint32_t st = S.sc_v[cur][tid - 1];     // register entering this stripe (tid >= 1 here)
        st = crc_run(T, st, w, a, e1);
        if (L.prev >= 0) {
            uint32_t stored = (uint32_t)w[L.prev] | ((uint32_t)w[L.prev + 1] << 8) |
                              ((uint32_t)w[L.prev + 2] << 16) | ((uint32_t)w[L.prev + 3] << 24);
            if (~st != stored) {
                unsigned long long key = ((unsigned long long)(uint32_t)L.prev << 32) | (uint32_t)(L.base - 1);
                atomicMin(&S.bad, key);
            }
        } else {
            S.head_raw = st;
        }
    }
    __syncthreads();

    // ---- chunk summary: CRC fields
    if (tid == 0) {
        ChunkSum& cs = sums[GIDX(chunk, nchunks, 8)];
        const int last_lane = (end_rel > 0) ? (end_rel - 1) / CLY_SUB : 0;
        const uint32_t end_state = S.sc_v[cur][last_lane];
        const bool has_first = cs.entry >= 0;      // a boundary (record or terminal) lies in the chunk
        cs.head_raw = has_first ? S.head_raw : end_state;
        cs.open_state = end_state;
        if (cs.open_pos >= 0) {
            const int op = (int)(cs.open_pos - cbase);
            cs.open_crc = (uint32_t)w[op] | ((uint32_t)w[op + 1] << 8) | ((uint32_t)w[op + 2] << 16) |
                          ((uint32_t)w[op + 3] << 24);
        } else {
            cs.open_crc = 0;
        }
        if (S.bad != ~0ULL) {
            cs.bad_pos = cbase + (int64_t)(S.bad >> 32);
            cs.bad_idx = (uint32_t)(S.bad & 0xffffffffu);
        } else {
            cs.bad_pos = -1;
            cs.bad_idx = 0xffffffffu;
        }
        // ---- decoupled look-back for this chunk's first output slot
        uint64_t prefix = 0;
        if (chunk > 0) {
            int k = chunk - 1;
            uint32_t spins = 0;
            while (k >= 0) {
                unsigned long long v = __hip_atomic_load(&lb[GIDX(k, nchunks, 9)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (v & LB_INC) { prefix += v & LB_MASK; break; }
                if (v & LB_AGG) { prefix += v & LB_MASK; k--; continue; }
                __builtin_amdgcn_s_sleep(2);
                if (++spins > (1u << 22)) { atomicOr(&g->lb_timeout, 1u); break; }
            }
            __hip_atomic_store(&lb[GIDX(chunk, nchunks, 10)], (unsigned long long)(prefix + cs.n_records) | LB_INC,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        out_base[GIDX(chunk, nchunks, 11)] = prefix;
        S.out_base = prefix;
        if (chunk == nchunks - 1) g->total_records = prefix + cs.n_records;
    }
    __syncthreads();

    // ---- emit tuples for the records starting in this lane's stripe
    if (live_lane && L.conf && L.cnt) {
        uint64_t idx = S.out_base + (uint64_t)L.base;
        int p = L.s;
        for (int i = 0; i < (int)L.cnt; i++, idx++) {
            Hdr h = step_hdr(w, p, n, cbase + p);
            if (idx < out_cap) {
                cly_tuple t;
                t.offset = cbase + p;
                t.expiration = h.exp;
                t.fid = F.fid;
                t.size = (uint32_t)h.size;
                t.key_size = h.ks;
                t.value_size = h.vs;
                t.type = h.type;
                t.data_type = h.dt;
                t.header_size = (uint8_t)h.hsz;
                t.crc = h.crc;
                int tn;
                int64_t klim = h.ks < 11u ? (int64_t)h.ks : 11;
                int64_t tx = go_varint(w + p + h.hsz, klim, tn);
                if (tn < 0) { t.tx_id = 0; t.txid_len = 0xFF; }
                else { t.tx_id = tx; t.txid_len = (uint8_t)tn; }
                out[GIDX(idx, out_cap, 12)] = t;
            } else {
                atomicOr(&g->overflow, 1u);
            }
            p = (int)(p + h.size);
        }
    }
}

// ---------------------------------------------------------------------------
// Chain verification + per-file results (two small kernels).
//
// k_check  (one thread per chunk): chunk i of a file "claims" an entry when its
//          speculation started a chain (chunk 0 always claims offset 0).  With
//          P(i) the nearest claiming chunk before i and X its exit, the claims are
//          the true chain iff every chunk satisfies  claim ? X == entry : X >= end
//          (induction from chunk 0).  The thread also derives the chunk's first
//          end event: an in-chunk CRC failure, a terminal, or a CRC failure of the
//          record that straddles into later chunks (finished here from the
//          following chunks' head CRCs).
// k_finish (one block per file): first failing chunk and first event by
//          min-reduction; the event counts only if it and every chunk it relies
//          on lie before the first failure.  Otherwise the host runs a repair
//          pass with forced entries (k_scan forced mode).
#define CHK_NT 256
#define FIN_NT 256
#define MAX_BACK 4096            // bound on the backward search for P(i)
#define EVT_NONE 0
#define EVT_BAD 1                // CRC failure of a record finished inside the chunk
#define EVT_STRADDLE 2           // CRC failure of the record open at the chunk end
#define EVT_TERM 3               // terminal position inside the chunk
#define EVT_UNKNOWN 4            // straddle depends on chunks that failed the check

struct ChunkChk {                // 16 B, written by k_check
    int32_t ok;                  // 1 = consistent with the chain from chunk 0
    int32_t evt;                 // EVT_*
    int32_t dep_end;             // last chunk (local) the event relies on
    int32_t _pad;
};

__device__ __forceinline__ uint32_t crc_bytes_bitwise(uint32_t s, uint32_t word, int lo, int hi) {
    for (int k = lo; k < hi; k++) s = cly_crc_byte_bitwise(s, (uint8_t)(word >> (8 * k)));
    return s;
}

// Advance register s (of a record whose CRC range starts at file offset cs)
// over the first hlen bytes of chunk H (which starts at file offset hstart).
__device__ __forceinline__ uint32_t advance_head(uint32_t s, int64_t cs, const ChunkSum& H, int64_t hstart,
                                                 int64_t hlen) {
    const int64_t l4 = hlen < 4 ? hlen : 4;
    const int lo = (int)(cs > hstart ? (cs - hstart < l4 ? cs - hstart : l4) : 0);
    s = crc_bytes_bitwise(s, H.first4, lo, (int)l4);
    if (hlen > 4) s = cly_multmodp(H.head_shift, s) ^ H.head_raw;   // head_raw spans [hstart+4, hstart+hlen)
    return s;
}

__device__ __forceinline__ bool claims(const ChunkSum& cs, int i) { return i == 0 || cs.entry >= 0; }

__global__ void __launch_bounds__(CHK_NT)
k_check(const DevFile* __restrict__ files, int nfiles, const uint32_t* __restrict__ file_chunk_prefix,
        int nchunks, const ChunkSum* __restrict__ sums, ChunkChk* __restrict__ chk, Globals* __restrict__ g) {
    const int c = blockIdx.x * CHK_NT + threadIdx.x;
    if (c >= nchunks) return;
    int lo = 0, hi = nfiles - 1;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if ((int)file_chunk_prefix[GIDX(mid, nfiles + 1, 30)] <= c) lo = mid; else hi = mid - 1;
    }
    const DevFile F = files[GIDX(lo, nfiles, 31)];
    const int c0 = (int)F.first_chunk, nc = (int)F.nchunks, i = c - c0;
    const ChunkSum cs = sums[GIDX(c, nchunks, 32)];
    ChunkChk r;
    r.ok = 1; r.evt = EVT_NONE; r.dep_end = i; r._pad = 0;
    const bool cl = claims(cs, i);
    if (i > 0) {
        int p = i - 1, steps = 0;
        while (p > 0 && sums[GIDX(c0 + p, nchunks, 33)].entry < 0 && steps < MAX_BACK) { p--; steps++; }
        const ChunkSum ps = sums[GIDX(c0 + p, nchunks, 34)];
        if (!claims(ps, p)) r.ok = 0;                          // search bound hit: let the host repair
        else {
            const int64_t X = ps.term ? INT64_MAX : ps.exit;
            const int64_t end = (int64_t)i * CLY_CHUNK + cs.chunk_len;
            r.ok = cl ? (X == cs.entry) : (X >= end);
        }
    }
    if (cl) {
        if (cs.bad_pos >= 0) r.evt = EVT_BAD;
        else if (cs.term) r.evt = EVT_TERM;
        else if (cs.open_pos >= 0) {
            // the open record's bytes continue through the heads of the following
            // chunks up to the chain exit X (pass-through chunks carry all bytes)
            const int64_t X = cs.exit;
            uint32_t s = cs.open_state;
            const int64_t ocs = cs.open_pos + 4;
            int j = i + 1;
            bool known = true;
            while (j < nc && (int64_t)j * CLY_CHUNK < X) {
                const ChunkSum h = sums[GIDX(c0 + j, nchunks, 35)];
                const int64_t hs = (int64_t)j * CLY_CHUNK;
                const int64_t hl = (X - hs) < (int64_t)h.chunk_len ? (X - hs) : (int64_t)h.chunk_len;
                if (hl != (int64_t)h.head_len) { known = false; break; }   // j's speculation disagrees
                s = advance_head(s, ocs, h, hs, hl);
                j++;
            }
            r.dep_end = j - 1;
            if (!known) { r.evt = EVT_UNKNOWN; r.dep_end = j; }
            else if (~s != cs.open_crc) r.evt = EVT_STRADDLE;
        }
    }
    chk[c] = r;
}

__global__ void __launch_bounds__(FIN_NT)
k_finish(const DevFile* __restrict__ files, int nchunks, const ChunkSum* __restrict__ sums,
         const ChunkChk* __restrict__ chk, const uint64_t* __restrict__ out_base,
         int64_t* __restrict__ forced_out, FileOut* __restrict__ fout, Globals* __restrict__ g) {
    const int f = blockIdx.x;
    const int tid = threadIdx.x;
    const DevFile F = files[f];
    const int c0 = (int)F.first_chunk, nc = (int)F.nchunks;
    const int64_t nlen = (int64_t)F.len;
    __shared__ int red[FIN_NT];

    // first chunk failing the chain check
    int m = nc;
    for (int i = tid; i < nc; i += FIN_NT)
        if (!chk[GIDX(c0 + i, nchunks, 40)].ok) { m = i; break; }
    red[tid] = m;
    __syncthreads();
    for (int d = FIN_NT / 2; d > 0; d >>= 1) {
        if (tid < d && red[tid + d] < red[tid]) red[tid] = red[tid + d];
        __syncthreads();
    }
    const int fail = red[0];
    __syncthreads();
    // first event among chunks before the failure
    m = nc;
    for (int i = tid; i < fail; i += FIN_NT)
        if (chk[GIDX(c0 + i, nchunks, 41)].evt != EVT_NONE) { m = i; break; }
    red[tid] = m;
    __syncthreads();
    for (int d = FIN_NT / 2; d > 0; d >>= 1) {
        if (tid < d && red[tid + d] < red[tid]) red[tid] = red[tid + d];
        __syncthreads();
    }
    const int ev = red[0];
    if (tid != 0) return;
    TRACE(0, 1); TRACE(1, fail); TRACE(2, ev);

    FileOut fo;
    const uint64_t first = out_base[GIDX(c0, nchunks, 42)];
    fo.first_index = first;
    fo.repair = 0;
    bool need_repair = false;
    if (ev < nc) {
        const ChunkChk e = chk[GIDX(c0 + ev, nchunks, 43)];
        const ChunkSum cs = sums[GIDX(c0 + ev, nchunks, 44)];
        const uint64_t ob = out_base[GIDX(c0 + ev, nchunks, 45)];
        if (e.evt == EVT_UNKNOWN || e.dep_end >= fail) need_repair = true;
        else if (e.evt == EVT_BAD) {
            fo.status = CLY_ERR_CRC; fo.end_offset = cs.bad_pos; fo.n_records = ob + cs.bad_idx - first;
        } else if (e.evt == EVT_STRADDLE) {
            fo.status = CLY_ERR_CRC; fo.end_offset = cs.open_pos; fo.n_records = ob + cs.n_records - 1 - first;
        } else {
            fo.status = cs.term_status; fo.end_offset = cs.exit; fo.n_records = ob + cs.n_records - first;
        }
    } else if (fail < nc) {
        need_repair = true;
    } else {
        // every chunk verified and no event: the chain leaves the last claiming chunk at n
        int p = nc - 1;
        while (p > 0 && sums[GIDX(c0 + p, nchunks, 46)].entry < 0) p--;
        const ChunkSum ps = sums[GIDX(c0 + p, nchunks, 47)];
        fo.status = CLY_END_EOF;
        fo.end_offset = ps.exit;
        fo.n_records = out_base[GIDX(c0 + p, nchunks, 48)] + ps.n_records - first;
    }
    if (need_repair) {
        // The chain entered the first failing chunk at the exit of its predecessor.
        // An entry within 5 bytes of the end of the file is a terminal (no data
        // needed); otherwise the host re-runs k_scan with forced entries.
        const int i = fail < ev ? fail : ev;
        int p = i - 1;
        while (p > 0 && sums[GIDX(c0 + p, nchunks, 49)].entry < 0) p--;
        const ChunkSum ps = sums[GIDX(c0 + (p < 0 ? 0 : p), nchunks, 50)];
        const int64_t E = ps.exit;
        if (p >= 0 && !ps.term && E >= nlen - 5 && E < nlen && ps.bad_pos < 0) {
            fo.status = (nlen - E == 5) ? CLY_ERR_TRUNC5 : CLY_END_EOF;
            fo.end_offset = E;
            fo.n_records = out_base[GIDX(c0 + p, nchunks, 51)] + ps.n_records - first;
            need_repair = false;
        } else {
            fo.repair = 1; fo.status = 0; fo.end_offset = 0; fo.n_records = 0;
            atomicOr(&g->repair, 1u);
        }
    }
    TRACE(0, 2);
    fout[f] = fo;
    if (fo.repair) {
        // forced entries: exact where the chain is known, re-speculate after it
        int64_t E = 0;
        bool known = true;
        for (int i = 0; i < nc; i++) {
            const ChunkSum cs = sums[GIDX(c0 + i, nchunks, 52)];
            const int64_t start = (int64_t)i * CLY_CHUNK, end = start + cs.chunk_len;
            int64_t fv;
            if (!known) fv = FORCE_GUESS;
            else if (E < 0 || E >= end) fv = (i == 0) ? 0 : FORCE_SKIP;
            else {
                fv = E;
                if (cs.entry == E) E = cs.term ? -1 : cs.exit;
                else known = false;
            }
            forced_out[GIDX(c0 + i, nchunks, 53)] = fv;
        }
    } else {
        for (int i = 0; i < nc; i++) forced_out[GIDX(c0 + i, nchunks, 54)] = FORCE_GUESS;
    }
    TRACE(0, 3);
}

// ---------------------------------------------------------------------------
// Host side
#define HIPCK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "clyscan: %s failed: %s\n", #x, hipGetErrorString(e_)); return CLY_ERR_DEVICE; } } while (0)

struct cly_ctx {
    int device;
    hipStream_t stream;
    hipEvent_t ev[4];
    // device buffers (grown on demand)
    DevFile* d_files; int cap_files;
    uint32_t* d_prefix;
    ChunkSum* d_sums; int cap_chunks;
    unsigned long long* d_lb;
    uint64_t* d_outbase;
    int64_t* d_forced;
    ChunkChk* d_chk;
    FileOut* d_fout;
    Globals* d_g;
    uint32_t* d_shift;
    // pinned host staging
    DevFile* h_files;
    uint32_t* h_prefix;
    FileOut* h_fout;
    Globals* h_g;
    int* h_trace;               // CLY_DEBUG: host-mapped trace buffer
    // host-path staging
    uint8_t* d_bytes; uint64_t cap_bytes;
    cly_tuple* d_tuples; uint64_t cap_tuples;
};

static void build_shift_tables(uint32_t* h) {
    for (int lvl = 0; lvl < CLY_SCAN_LEVELS; lvl++) {
        const uint64_t L = (uint64_t)CLY_SUB << lvl;
        const uint32_t xm = cly_x8n(L);
        for (int bpos = 0; bpos < 4; bpos++)
            for (uint32_t i = 0; i < 256; i++)
                h[lvl * 1024 + bpos * 256 + i] = cly_multmodp(xm, i << (8 * bpos));
    }
}

extern "C" int cly_ctx_create(int device, cly_ctx** out) {
    if (!out) return CLY_ERR_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev) return CLY_ERR_DEVICE;
    HIPCK(hipSetDevice(device));
    cly_ctx* c = (cly_ctx*)calloc(1, sizeof(cly_ctx));
    c->device = device;
    HIPCK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    for (int i = 0; i < 4; i++) HIPCK(hipEventCreate(&c->ev[i]));
    HIPCK(hipMalloc(&c->d_g, sizeof(Globals)));
    HIPCK(hipHostMalloc(&c->h_g, sizeof(Globals), hipHostMallocDefault));
    const size_t shift_bytes = sizeof(uint32_t) * 1024 * CLY_SCAN_LEVELS;
    HIPCK(hipMalloc(&c->d_shift, shift_bytes));
    uint32_t* hs = (uint32_t*)malloc(shift_bytes);
    build_shift_tables(hs);
    HIPCK(hipMemcpy(c->d_shift, hs, shift_bytes, hipMemcpyHostToDevice));
    free(hs);
#ifdef CLY_DEBUG
    HIPCK(hipHostMalloc(&c->h_trace, 64 * sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
    memset(c->h_trace, 0, 64 * sizeof(int));
    { int* dptr = nullptr; HIPCK(hipHostGetDevicePointer((void**)&dptr, c->h_trace, 0));
      HIPCK(hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &dptr, sizeof(dptr))); }
#endif
    HIPCK(hipFuncSetAttribute((const void*)k_scan, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)sizeof(ScanShared)));
    *out = c;
    return CLY_OK;
}

extern "C" void cly_ctx_destroy(cly_ctx* c) {
    if (!c) return;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    hipFree(c->d_files); hipFree(c->d_prefix); hipFree(c->d_sums); hipFree(c->d_lb);
    hipFree(c->d_outbase); hipFree(c->d_forced); hipFree(c->d_chk); hipFree(c->d_fout); hipFree(c->d_g);
    hipFree(c->d_shift); hipFree(c->d_bytes); hipFree(c->d_tuples);
    hipHostFree(c->h_files); hipHostFree(c->h_prefix); hipHostFree(c->h_fout); hipHostFree(c->h_g);
    for (int i = 0; i < 4; i++) hipEventDestroy(c->ev[i]);
    hipStreamDestroy(c->stream);
    free(c);
}

extern "C" uint64_t cly_scan_capacity(const cly_file* files, int nfiles) {
    uint64_t cap = 0;
    for (int i = 0; i < nfiles; i++) cap += files[i].len / 9 + 1;
    return cap;
}

static int ensure_files(cly_ctx* c, int nfiles) {
    if (nfiles <= c->cap_files) return CLY_OK;
    hipFree(c->d_files); hipFree(c->d_prefix); hipFree(c->d_fout);
    hipHostFree(c->h_files); hipHostFree(c->h_prefix); hipHostFree(c->h_fout);
    int cap = nfiles < 64 ? 64 : nfiles;
    HIPCK(hipMalloc(&c->d_files, sizeof(DevFile) * cap));
    HIPCK(hipMalloc(&c->d_prefix, sizeof(uint32_t) * (cap + 1)));
    HIPCK(hipMalloc(&c->d_fout, sizeof(FileOut) * cap));
    HIPCK(hipHostMalloc(&c->h_files, sizeof(DevFile) * cap, hipHostMallocDefault));
    HIPCK(hipHostMalloc(&c->h_prefix, sizeof(uint32_t) * (cap + 1), hipHostMallocDefault));
    HIPCK(hipHostMalloc(&c->h_fout, sizeof(FileOut) * cap, hipHostMallocDefault));
    c->cap_files = cap;
    return CLY_OK;
}

static int ensure_chunks(cly_ctx* c, int nchunks) {
    if (nchunks <= c->cap_chunks) return CLY_OK;
    hipFree(c->d_sums); hipFree(c->d_lb); hipFree(c->d_outbase); hipFree(c->d_forced); hipFree(c->d_chk);
    int cap = nchunks < 1024 ? 1024 : nchunks;
    HIPCK(hipMalloc(&c->d_chk, sizeof(ChunkChk) * cap));
    HIPCK(hipMalloc(&c->d_sums, sizeof(ChunkSum) * cap));
    HIPCK(hipMalloc(&c->d_lb, sizeof(unsigned long long) * cap));
    HIPCK(hipMalloc(&c->d_outbase, sizeof(uint64_t) * cap));
    HIPCK(hipMalloc(&c->d_forced, sizeof(int64_t) * cap));
    c->cap_chunks = cap;
    return CLY_OK;
}

extern "C" int cly_scan_device(cly_ctx* c, const cly_file* files, int nfiles,
                               cly_tuple* d_out, uint64_t out_cap,
                               uint64_t* file_first, cly_file_result* res,
                               uint64_t* needed, cly_stats* stats, void* stream_v) {
    if (!c || (!files && nfiles) || nfiles < 0 || !res || !file_first) return CLY_ERR_ARG;
    if (nfiles == 0) { if (needed) *needed = 0; return CLY_OK; }
    HIPCK(hipSetDevice(c->device));
    hipStream_t st = stream_v ? (hipStream_t)stream_v : c->stream;
    int rc = ensure_files(c, nfiles);
    if (rc) return rc;
    uint64_t nchunks64 = 0, bytes = 0;
    for (int i = 0; i < nfiles; i++) {
        if (files[i].len >= (1ULL << 32)) return CLY_ERR_ARG;
        if (files[i].len && (((uintptr_t)files[i].base) & 15)) return CLY_ERR_ARG;
        uint32_t nch = files[i].len ? (uint32_t)((files[i].len + CLY_CHUNK - 1) / CLY_CHUNK) : 1;
        c->h_files[i].base = files[i].base;
        c->h_files[i].len = files[i].len;
        c->h_files[i].fid = files[i].fid;
        c->h_files[i].first_chunk = (uint32_t)nchunks64;
        c->h_files[i].nchunks = nch;
        c->h_files[i]._pad = 0;
        c->h_prefix[i] = (uint32_t)nchunks64;
        nchunks64 += nch;
        bytes += files[i].len;
    }
    if (nchunks64 >= (1ULL << 31)) return CLY_ERR_ARG;
    const int nchunks = (int)nchunks64;
    c->h_prefix[nfiles] = (uint32_t)nchunks;
    rc = ensure_chunks(c, nchunks);
    if (rc) return rc;
    HIPCK(hipMemcpyAsync(c->d_files, c->h_files, sizeof(DevFile) * nfiles, hipMemcpyHostToDevice, st));
    HIPCK(hipMemcpyAsync(c->d_prefix, c->h_prefix, sizeof(uint32_t) * (nfiles + 1), hipMemcpyHostToDevice, st));

#ifdef CLY_DEBUG
    fprintf(stderr, "clyscan[debug] nfiles=%d nchunks=%d d_out=%p out_cap=%llu shared=%zu\n", nfiles, nchunks,
            (void*)d_out, (unsigned long long)out_cap, sizeof(ScanShared));
    for (int i = 0; i < nfiles && i < 8; i++)
        fprintf(stderr, "clyscan[debug]   file %d base=%p len=%llu first_chunk=%u nchunks=%u\n", i,
                (const void*)c->h_files[i].base, (unsigned long long)c->h_files[i].len, c->h_files[i].first_chunk,
                c->h_files[i].nchunks);
#endif
    double scan_ms = 0, res_ms = 0;
    uint32_t pass = 0;
    HIPCK(hipEventRecord(c->ev[0], st));
    for (;;) {
        HIPCK(hipMemsetAsync(c->d_lb, 0, sizeof(unsigned long long) * nchunks, st));
        HIPCK(hipMemsetAsync(c->d_g, 0, sizeof(Globals), st));
        HIPCK(hipEventRecord(c->ev[1], st));
        hipLaunchKernelGGL(k_scan, dim3(nchunks), dim3(CLY_NT), sizeof(ScanShared), st,
                           c->d_files, nfiles, c->d_prefix, nchunks, pass ? c->d_forced : nullptr,
                           c->d_shift, c->d_sums, c->d_lb, c->d_outbase, d_out, out_cap, c->d_g);
        HIPCK(hipGetLastError());
#ifdef CLY_DEBUG
        { hipError_t e = hipStreamSynchronize(st);
          fprintf(stderr, "clyscan[debug] k_scan pass %u: %s\n", pass, hipGetErrorString(e));
          if (e != hipSuccess) return CLY_ERR_DEVICE;
          Globals hg; (void)hipMemcpy(&hg, c->d_g, sizeof(Globals), hipMemcpyDeviceToHost);
          if (hg.dbg_site) fprintf(stderr, "clyscan[debug] k_scan OOB site %u idx %lld lim %lld\n", hg.dbg_site,
                                   (long long)hg.dbg_idx, (long long)hg.dbg_lim); }
#endif
        HIPCK(hipEventRecord(c->ev[2], st));
        hipLaunchKernelGGL(k_check, dim3((nchunks + CHK_NT - 1) / CHK_NT), dim3(CHK_NT), 0, st,
                           c->d_files, nfiles, c->d_prefix, nchunks, c->d_sums, c->d_chk, c->d_g);
        HIPCK(hipGetLastError());
        hipLaunchKernelGGL(k_finish, dim3(nfiles), dim3(FIN_NT), 0, st,
                           c->d_files, nchunks, c->d_sums, c->d_chk, c->d_outbase, c->d_forced, c->d_fout, c->d_g);
        HIPCK(hipGetLastError());
#ifdef CLY_DEBUG
        { hipError_t e = hipStreamSynchronize(st);
          fprintf(stderr, "clyscan[debug] k_check+k_finish pass %u: %s\n", pass, hipGetErrorString(e));
          fprintf(stderr, "clyscan[debug] trace:");
          for (int t = 0; t < 8; t++) fprintf(stderr, " %d", c->h_trace[t]);
          fprintf(stderr, "\n");
          if (e != hipSuccess) return CLY_ERR_DEVICE;
          Globals hg; (void)hipMemcpy(&hg, c->d_g, sizeof(Globals), hipMemcpyDeviceToHost);
          if (hg.dbg_site) fprintf(stderr, "clyscan[debug] OOB site %u idx %lld lim %lld\n", hg.dbg_site,
                                   (long long)hg.dbg_idx, (long long)hg.dbg_lim); }
#endif
        HIPCK(hipEventRecord(c->ev[3], st));
        HIPCK(hipMemcpyAsync(c->h_g, c->d_g, sizeof(Globals), hipMemcpyDeviceToHost, st));
        HIPCK(hipMemcpyAsync(c->h_fout, c->d_fout, sizeof(FileOut) * nfiles, hipMemcpyDeviceToHost, st));
        HIPCK(hipStreamSynchronize(st));
        float ms = 0;
        HIPCK(hipEventElapsedTime(&ms, c->ev[1], c->ev[2])); scan_ms += ms;
        HIPCK(hipEventElapsedTime(&ms, c->ev[2], c->ev[3])); res_ms += ms;
        pass++;
        if (c->h_g->lb_timeout) return CLY_ERR_DEVICE;
        if (!c->h_g->repair) break;
        if (pass > 64) return CLY_ERR_NOREPAIR;
    }
    float tot = 0;
    HIPCK(hipEventElapsedTime(&tot, c->ev[0], c->ev[3]));
    uint64_t total = 0;
    for (int i = 0; i < nfiles; i++) {
        file_first[i] = c->h_fout[i].first_index;
        res[i].n_records = c->h_fout[i].n_records;
        res[i].end_offset = c->h_fout[i].end_offset;
        res[i].status = c->h_fout[i].status;
        res[i]._pad = 0;
        total += c->h_fout[i].n_records;
    }
    if (needed) *needed = c->h_g->total_records;
    if (stats) {
        stats->scan_ms = scan_ms; stats->resolve_ms = res_ms; stats->total_ms = tot;
        stats->passes = pass; stats->n_chunks = (uint32_t)nchunks; stats->bytes = bytes; stats->records = total;
    }
    if (c->h_g->overflow || c->h_g->total_records > out_cap) return CLY_ERR_CAPACITY;
    return CLY_OK;
}

extern "C" int cly_scan(cly_ctx* c, const cly_file* files, int nfiles,
                        cly_tuple* out, uint64_t out_cap,
                        uint64_t* file_first, cly_file_result* res,
                        uint64_t* needed, cly_stats* stats) {
    if (!c || (!files && nfiles) || nfiles < 0 || !res || !file_first) return CLY_ERR_ARG;
    if (nfiles == 0) { if (needed) *needed = 0; return CLY_OK; }
    HIPCK(hipSetDevice(c->device));
    // pack files into one device buffer, each at a 4 KiB-aligned offset
    uint64_t total = 0;
    for (int i = 0; i < nfiles; i++) {
        if (files[i].len >= (1ULL << 32)) return CLY_ERR_ARG;
        total += (files[i].len + 4095) & ~4095ULL;
    }
    if (total + 4096 > c->cap_bytes) {
        hipFree(c->d_bytes);
        c->cap_bytes = total + 4096;
        HIPCK(hipMalloc(&c->d_bytes, c->cap_bytes));
    }
    cly_file* df = (cly_file*)malloc(sizeof(cly_file) * nfiles);
    uint64_t off = 0;
    for (int i = 0; i < nfiles; i++) {
        df[i] = files[i];
        df[i].base = c->d_bytes + off;
        if (files[i].len)
            HIPCK(hipMemcpyAsync(c->d_bytes + off, files[i].base, files[i].len, hipMemcpyHostToDevice, c->stream));
        off += (files[i].len + 4095) & ~4095ULL;
    }
    uint64_t cap = cly_scan_capacity(files, nfiles);
    if (cap > c->cap_tuples) {
        hipFree(c->d_tuples);
        c->cap_tuples = cap;
        HIPCK(hipMalloc(&c->d_tuples, sizeof(cly_tuple) * cap));
    }
    uint64_t need = 0;
    int rc = cly_scan_device(c, df, nfiles, c->d_tuples, c->cap_tuples, file_first, res, &need, stats, nullptr);
    free(df);
    if (needed) *needed = need;
    if (rc != CLY_OK) return rc;
    if (need > out_cap) return CLY_ERR_CAPACITY;
    if (need) HIPCK(hipMemcpyAsync(out, c->d_tuples, sizeof(cly_tuple) * need, hipMemcpyDeviceToHost, c->stream));
    HIPCK(hipStreamSynchronize(c->stream));
    return CLY_OK;
}

extern "C" const char* cly_strerror(int code) {
    switch (code) {
        case CLY_END_EOF: return "ok / io.EOF";
        case CLY_END_ZERO: return "io.EOF (zero header)";
        case CLY_END_TORN: return "io.EOF (torn record)";
        case CLY_ERR_CRC: return "invalid crc value, logRecord maybe corrupted";
        case CLY_ERR_TRUNC5: return "5-byte tail: header decode index out of range";
        case CLY_ERR_VARINT: return "varint overflow: header slice bounds out of range";
        case CLY_ERR_OFFSET: return "mmap: invalid ReadAt offset";
        case CLY_ERR_CAPACITY: return "output capacity too small";
        case CLY_ERR_DEVICE: return "HIP device error";
        case CLY_ERR_ARG: return "invalid argument";
        case CLY_ERR_NOREPAIR: return "speculation repair did not converge";
        default: return "unknown status";
    }
}

extern "C" const char* cly_build_info(void) {
#define CLY_STR2(x) #x
#define CLY_STR(x) CLY_STR2(x)
    return "clyscan gfx950 NT=" CLY_STR(CLY_NT) " SUB=" CLY_STR(CLY_SUB) " CHUNK=" CLY_STR(CLY_CHUNK)
           " REP=" CLY_STR(CLY_REP);
}
