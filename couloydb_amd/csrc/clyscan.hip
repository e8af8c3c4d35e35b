// clyscan.hip — MI355X (gfx950) log-record scan for CouloyDB data files.
//
// Product library libclyscan.so: the HIP kernels + the C-ABI of include/clyscan.h.
// It restates, for whole files at once, the loop
//     for { rec, size, err := df.ReadLogRecord(offset); ...; offset += size }
// of db.loadIndex (db.go:582-637) / db.merge (merge.go:90-143) /
// loadIndexFromHintFile (merge.go:257-287), with the per-record semantics of
// DataFile.ReadLogRecord (data/dataFile.go:64-111), DecodeLogRecordHeader
// (data/logRecord.go:86-114), GetLogRecordCRC (data/logRecord.go:136-146) and
// parseLogRecordKey (db.go:706-710).
//
// Layout: every file is cut into chunks of CLY_CH bytes, one
// per lane; 64 consecutive chunks of a file are a tile, one per wave.
//
// k_scan (persistent, tiles in ticket order), per tile:
//   A  each lane finds the first record start of its chunk (SWAR candidate
//      filter over its bytes, then a walk of header gathers that must leave the
//      chunk at a plausible header), and walks its records to the chunk end;
//      the wave makes the lanes' chains agree (lane l+1 starts where lane l's
//      chain leaves), re-walking exactly where they do not;
//   L  decoupled look-back over tile descriptors: the chain state and record
//      count entering the tile; a tile whose guessed entry is wrong re-resolves;
//   C  every lane streams its chunk through a slicing-by-4 CRC register from
//      HBM (16-B loads, 128 B per burst), re-walks its records, writes their
//      tuples straight to their output slots and XORs one combined patch per
//      record into the stream, so that the register of the whole file ends at
//      zero iff every record's CRC matches; the tile's register is folded
//      in-wave.
// k_fin (one workgroup per file): folds the tile registers of the file and
// checks it; k_locate (only when a file fails) finds the first bad record.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <thread>

#include "scan_core.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(4)));
typedef unsigned long long u64;

#define CLY_GL __attribute__((address_space(1)))   // global memory (loads/stores as global_*, not flat_*)
typedef const CLY_GL uint8_t* gbytes;
typedef CLY_GL cly_tuple* gtuples;
#define NONE32 0xFFFFFFFFu       // no position
#define TERM_NONE 127            // the chain leaves the chunk (no terminal inside)
#define LM_NONE 0                // no record starts in the chunk (the chain passes through it)
#define LM_CHAIN 1               // the chain enters the chunk at E (a record start or its terminal)
#define LM_DEAD 2                // the file's chain ended before the chunk
#define LM_OFF 3                 // chunk beyond the end of the file
#define NO_EV 0xFFFFu            // empty event slot
#ifdef CLY_DEBUG
#define DBG(...) do { if ((threadIdx.x & 63) == 0) printf(__VA_ARGS__); } while (0)
#else
#define DBG(...)
#endif

struct DevFile {                 // 32 B
    const uint8_t* base;         // device pointer to the file's first byte (16-B aligned)
    uint64_t len;
    uint32_t fid;
    uint32_t first_tile;         // global index of the file's first tile
    uint32_t ntile;              // tiles of the file (>= 1)
    uint32_t _pad;
};

struct FileInfo {                // per file, zeroed per call (fail_key: all ones)
    uint64_t first_index;        // global tuple index of the file's first record
    uint64_t end_index;          // global index after the file's last record
    uint32_t term_pos;           // terminal position T of the file's chain
    int32_t  term_status;
    uint32_t term_tile;          // global tile index holding T
    uint32_t term_lane;
    uint32_t expect;             // value the folded register must have (see k_fin)
    uint32_t has_term;
    u64      fail_key;           // (offset << 32) | index in file of the first CRC failure (k_locate)
    uint32_t fold;               // k_fin: the folded register
    uint32_t ok;                 // k_fin: fold == expect
};

// Tile descriptor: LOCAL (from the tile's own speculation) and INCL (the true
// state after the tile), each published by its flag word, written last.
struct TileDesc { u64 l[4]; u64 i[4]; };
// l[0]: bit0 published | bit1 the chain ends in the tile | bit2 no chunk of the tile
//       holds a boundary | bit3 first tile of its file | bit4 a record starts in the
//       tile | records << 32
// l[1]: G (the tile's guessed entry: its first boundary) | exit or terminal position << 32
// l[2]: crc_last | P_last << 32 (last record start in the tile and its stored CRC)
// l[3]: the smallest entry that passes the whole tile (tile end, or len + 1 for
//       the tile holding the file's end)
// i[0]: bit0 published | bit1 the file's chain ended | records before the next tile << 16
// i[1]: X (chain position after the tile) | crc_last << 32
// i[2]: P_last (start of the last record before the next tile, NONE32 if none)
#define DF_PUB 1ull
#define DF_TERM 2ull
#define DF_NONE 4ull
#define DF_FOF 8ull
#define DF_REC 16ull

struct Globals {                 // zeroed per call
    uint32_t ticket;
    uint32_t overflow;           // tuples beyond out_cap were dropped
    uint32_t fail;               // internal invariant / spin bound (never expected)
    uint32_t refix;              // tiles whose guessed entry the look-back corrected
    uint32_t slow_lanes;         // lanes that took the exact (slow) CRC path
    uint32_t any_fail;           // a file's CRC fold failed (k_locate needed)
    uint64_t total;              // records over all files
    uint64_t prof[12];           // profiling build (-DCLY_PROF): cycles per phase, summed over tiles; look-back counters
};
#ifdef CLY_PROF
#define PROF_T0() uint64_t prof_t = __builtin_amdgcn_s_memtime()
#define PROF(i) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); if ((threadIdx.x & 63) == 0) atomicAdd((unsigned long long*)&g->prof[i], (unsigned long long)(t_ - prof_t)); prof_t = t_; } while (0)
#else
#define PROF_T0()
#define PROF(i)
#endif
#ifdef CLY_PROF
#define PCNT(i, n) do { if ((threadIdx.x & 63) == 0) atomicAdd((unsigned long long*)&g->prof[i], (unsigned long long)(n)); } while (0)
#else
#define PCNT(i, n)
#endif

// ---------------------------------------------------------------------------
// LDS of k_scan / k_locate (static: compile-time offsets)
//   [0, 65536)     CRC slicing-by-4 tables T0..T3, 16 replicas: dword (i*64 + t*16 + r)
//   [65536, +256)  inverse of a zero-byte step (top byte of T0 -> index)
//   [65792, ...)   nibble tables of A^(CLY_CH * 2^k), k < 7 (8 x 16 words each)
#define LDS_INV 65536
#define LDS_NIB (LDS_INV + 256)
#define NIB_LEVELS 7                     // A^(CLY_CH * 2^k), k < 7 (k = 6: one tile)
#define EVQ 10                   // events per lane in the LDS ring of phase C
#define LDS_EVQ (LDS_NIB + NIB_LEVELS * 128 * 4)          // event rings: [wave][EVQ][64 lanes] x 8 B
#define SCAN_WAVES 16
#define SCAN_LDS (LDS_EVQ + SCAN_WAVES * EVQ * 64 * 8)

__device__ __forceinline__ void init_tables(CLY_LDS uint8_t* smem, const uint32_t* __restrict__ nib) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) {
        uint32_t cv = i;
        for (int k = 0; k < 8; k++) cv = (cv & 1) ? (cv >> 1) ^ CLY_POLY : cv >> 1;
        smem[LDS_INV + (cv >> 24)] = (uint8_t)i;
        for (int t = 0; t < 4; t++) {
            for (int r = 0; r < 16; r++) ((CLY_LDS uint32_t*)smem)[i * 64 + t * 16 + r] = cv;
            uint32_t tl = cv & 0xff;
            for (int k = 0; k < 8; k++) tl = (tl & 1) ? (tl >> 1) ^ CLY_POLY : tl >> 1;
            cv = (cv >> 8) ^ tl;
        }
    }
    for (int i = threadIdx.x; i < NIB_LEVELS * 128; i += blockDim.x) ((CLY_LDS uint32_t*)(smem + LDS_NIB))[i] = nib[i];
    __syncthreads();
}

// One slicing-by-4 step s' = A^4 (s ^ word), bank-conflict-free: lookup i of
// lanes with bit 4 set reads table slot i^1 (16 banks away) with the byte that
// slot takes; table address = (byte << 8) | replica offset by one v_perm.
struct CrcLane { uint32_t oe, oo, s0, s1, s2, s3, r4; };
__device__ __forceinline__ CrcLane crc_lane(int lane) {
    const uint32_t r4 = (uint32_t)(lane & 15) * 4, h = (uint32_t)(lane >> 4) & 1u;
    CrcLane c;
    c.r4 = r4;
    c.oe = r4 + 64 * h;
    c.oo = r4 + 64 * (1 - h);
    c.s0 = 0x0c0c0000u | ((4u + (3u - (0u ^ h))) << 8);
    c.s1 = 0x0c0c0000u | ((4u + (3u - (1u ^ h))) << 8);
    c.s2 = 0x0c0c0000u | ((4u + (3u - (2u ^ h))) << 8);
    c.s3 = 0x0c0c0000u | ((4u + (3u - (3u ^ h))) << 8);
    return c;
}
__device__ __forceinline__ uint32_t crc_word(const CLY_LDS uint8_t* smem, uint32_t x, const CrcLane& c) {
    const uint32_t a0 = __builtin_amdgcn_perm(x, c.oe, c.s0), a1 = __builtin_amdgcn_perm(x, c.oo, c.s1);
    const uint32_t a2 = __builtin_amdgcn_perm(x, c.oe, c.s2), a3 = __builtin_amdgcn_perm(x, c.oo, c.s3);
    return *(const CLY_LDS uint32_t*)(smem + a0) ^ *(const CLY_LDS uint32_t*)(smem + a1) ^
           *(const CLY_LDS uint32_t*)(smem + a2 + 128) ^ *(const CLY_LDS uint32_t*)(smem + a3 + 128);
}
// inverse of one zero-byte step: s = A^-1 s'
__device__ __forceinline__ uint32_t crc_unbyte(const CLY_LDS uint8_t* smem, uint32_t s, uint32_t r4) {
    const uint32_t i = smem[LDS_INV + (s >> 24)];
    const uint32_t t = *(const CLY_LDS uint32_t*)(smem + ((i << 8) | r4));
    return ((s ^ t) << 8) | i;
}
// A^(CLY_CH * 2^lvl) v by nibble tables (entry n*16+k = M (k << 4n))
__device__ __forceinline__ uint32_t nib_mul(const CLY_LDS uint8_t* smem, int lvl, uint32_t v) {
    const CLY_LDS uint32_t* t = (const CLY_LDS uint32_t*)(smem + LDS_NIB) + lvl * 128;
    uint32_t p = 0;
    #pragma unroll
    for (int n = 0; n < 8; n++) p ^= t[n * 16 + ((v >> (4 * n)) & 15u)];
    return p;
}

// ---------------------------------------------------------------------------
// Boundary patch.  A record starting at P (stored CRC c, the record before it
// stored cq) changes the file's byte stream, as seen by the CRC register, by
//   pa on word a = P>>2: the stored-CRC bytes [P, 4a+4) zeroed, and Q = A^-j ~cq
//                  (j = P&3) XORed in, so that the register after word a is zero
//                  iff the record ending at P has a good CRC (none at P = 0);
//   pb on word a+1: the rest of the stored CRC zeroed, 0xFF (the init) on the
//                  record's first region bytes [P+4, 4a+8);
//   pc on word a+2: 0xFF on [4a+8, P+8).
// XORing d into a word equals XORing A^4 d into the register after it, so the
// three are one XOR delta' = A^8 pa ^ A^4 pb ^ pc on word a+2.  The register
// of the whole patched file (everything from the chain's terminal T on zeroed,
// Q of T's predecessor at T) is zero iff every record's CRC matches.
__device__ __forceinline__ uint32_t q_of(const CLY_LDS uint8_t* smem, uint32_t cq, uint32_t j, uint32_t r4) {
    uint32_t q = ~cq;
    for (uint32_t k = 0; k < j; k++) q = crc_unbyte(smem, q, r4);
    return q;
}
__device__ __forceinline__ uint32_t patch_delta(const CLY_LDS uint8_t* smem, const CrcLane& cl, uint32_t P, uint32_t c,
                                                uint32_t cq) {
    const uint32_t j = P & 3, sh = 8 * j;
    uint32_t pa = j ? (c << sh) : c;
    if (P != 0) pa ^= q_of(smem, cq, j, cl.r4);
    const uint32_t pb = (j ? (c >> (32 - sh)) : 0u) ^ (j ? (0xFFFFFFFFu << sh) : 0xFFFFFFFFu);
    const uint32_t pc = j ? ((1u << sh) - 1u) : 0u;
    return crc_word(smem, crc_word(smem, pa, cl) ^ pb, cl) ^ pc;
}

// ---------------------------------------------------------------------------
// Header decode at file position p.  Fast path: 32 bytes gathered from
// [p & ~3, +32) by two 16-B loads, varints of at most 4 bytes ending within
// header bytes 6..13 (every record the writer produces except long
// expirations); otherwise the exact byte-loop form over global memory.
struct Gath { uint32_t w[8]; };
__device__ __forceinline__ bool gath_ok(uint32_t p, uint64_t len) { return (uint64_t)(p & ~3u) + 32 <= len; }
__device__ __forceinline__ void gath_issue(gbytes base, uint32_t p, Gath& g) {
    const CLY_GL u32x4u* q = (const CLY_GL u32x4u*)(base + (p & ~3u));
    const u32x4u a = q[0], b = q[1];
    g.w[0] = a.x; g.w[1] = a.y; g.w[2] = a.z; g.w[3] = a.w;
    g.w[4] = b.x; g.w[5] = b.y; g.w[6] = b.z; g.w[7] = b.w;
}
__device__ __forceinline__ uint32_t alignb(uint32_t hi, uint32_t lo, uint32_t s) {
    return __builtin_amdgcn_alignbyte(hi, lo, s);
}
__device__ __forceinline__ uint32_t pack7(uint32_t s) {
    return (s & 0x7fu) | ((s >> 1) & 0x3f80u) | ((s >> 2) & 0x1fc000u) | ((s >> 3) & 0xfe00000u);
}
__device__ __noinline__ void hdr_slow(gbytes base, uint32_t p, uint64_t len, Hdr& h) {
    h = step_hdr(base, (int64_t)p, (int64_t)len, (int64_t)p);
}
// header bytes 0..15 at p from a gather
__device__ __forceinline__ bool hdr_fast(const Gath& g, uint32_t p, uint64_t len, Hdr& h) {
    const uint64_t m64 = len - p;
    const int m = m64 > 26 ? 26 : (int)m64;
    if (m < 14) return false;
    const uint32_t s = p & 3;
    const uint32_t h0 = alignb(g.w[1], g.w[0], s), h1 = alignb(g.w[2], g.w[1], s), h2 = alignb(g.w[3], g.w[2], s),
                   h3 = alignb(g.w[4], g.w[3], s);
    const uint32_t lo = alignb(h2, h1, 2), hi = alignb(h3, h2, 2);       // bytes 6..9, 10..13
    const uint64_t W = ((uint64_t)hi << 32) | lo;
    const uint64_t T = ~W & 0x8080808080808080ull;
    const uint64_t T2 = T & (T - 1), T3 = T2 & (T2 - 1);
    const int e1 = __builtin_ctzll(T | (1ull << 63)) >> 3;
    const int e2 = __builtin_ctzll(T2 | (1ull << 63)) >> 3;
    const int e3 = __builtin_ctzll(T3 | (1ull << 63)) >> 3;
    const int n1 = e1 + 1, n2 = e2 - e1, n3 = e3 - e2;
    if (!(T3 != 0 && n1 <= 4 && n2 <= 4 && n3 <= 4 && 6 + e3 < m)) return false;
    const uint32_t u1 = pack7((uint32_t)W) & ((1u << (7 * n1)) - 1);
    const uint32_t u2 = pack7((uint32_t)(W >> (8 * n1))) & ((1u << (7 * n2)) - 1);
    const uint32_t u3 = pack7((uint32_t)(W >> (8 * (e2 + 1)))) & ((1u << (7 * n3)) - 1);
    const int32_t v1 = (int32_t)(u1 >> 1) ^ -(int32_t)(u1 & 1);
    const int32_t v2 = (int32_t)(u2 >> 1) ^ -(int32_t)(u2 & 1);
    const int32_t v3 = (int32_t)(u3 >> 1) ^ -(int32_t)(u3 & 1);
    h.crc = h0;
    h.key0 = (((7 + e3) >= 12 ? h3 : h2) >> (8 * ((7 + e3) & 3))) & 0xffu;
    h.type = h1 & 0xff;
    h.dt = (h1 >> 8) & 0xff;
    h.ks = (uint32_t)v1;
    h.vs = (uint32_t)v2;
    h.exp = v3;
    h.hsz = 7 + e3;
    h.size = 0;
    h.good = false;
    if (h.crc == 0 && h.ks == 0 && h.vs == 0) { h.status = CLY_END_ZERO; return true; }
    const int64_t kv = (int64_t)h.ks + (int64_t)h.vs;
    if (kv > 0 && (int64_t)(len - (p + (uint32_t)h.hsz)) < kv) { h.status = CLY_END_TORN; return true; }
    h.status = REC_OK;
    h.size = h.hsz + kv;
    h.good = h.type <= 4 && h.dt <= 4 && v1 >= 1 && v2 >= 0;
    return true;
}
// Header at p; `g` must hold the gather of p when gath_ok(p).
__device__ __forceinline__ Hdr hdr_at(gbytes base, uint32_t p, uint64_t len, const Gath& g) {
    Hdr h;
    if (gath_ok(p, len) && hdr_fast(g, p, len, h)) return h;
    hdr_slow(base, p, len, h);
    return h;
}
__device__ __forceinline__ Hdr hdr_load(gbytes base, uint32_t p, uint64_t len) {
    Gath g;
    if (gath_ok(p, len)) gath_issue(base, p, g);
    return hdr_at(base, p, len, g);
}

// ---------------------------------------------------------------------------
// Per-lane chain of one chunk [cb, ce) (file offsets; the file's last chunk
// also owns position len, where ReadLogRecord returns io.EOF).
struct Chunk {
    gbytes base;
    uint64_t len;
    uint32_t cb, ce;
    bool last;                   // the file's last chunk
    bool on;                     // the chunk exists (cb < len, or the empty file's chunk 0)
};
__device__ __forceinline__ bool in_chunk(const Chunk& K, uint32_t x) {
    return (x >= K.cb && x < K.ce) || (K.last && (uint64_t)x == K.len);
}
struct LaneChain {
    int      mode;               // LM_*
    uint32_t E;                  // first boundary (record start or terminal)
    uint32_t x;                  // exit (>= ce) or terminal position
    int      term;               // terminal status, TERM_NONE if the chain leaves the chunk
    uint32_t cnt;                // records starting in the chunk
    uint32_t last, last_crc;     // last record start and its stored CRC
    uint32_t prev_crc;           // stored CRC of the record before `last` (cnt >= 2)
    uint32_t minsz;              // smallest record size
};
__device__ __forceinline__ void chain_set(LaneChain& L, int mode) {
    L.mode = mode; L.E = NONE32; L.x = 0; L.term = TERM_NONE; L.cnt = 0; L.last = NONE32; L.last_crc = 0;
    L.prev_crc = 0; L.minsz = 0xFFFFFFFFu;
}

// Walk from p: exact (ReadLogRecord semantics, every terminal) or speculative
// (every record must be one the writer produces and the chain must leave the
// chunk at a plausible header, or end at io.EOF at len).  Returns false when a
// speculative chain is rejected.
__device__ __forceinline__ bool walk(const Chunk& K, uint32_t p, bool exact, LaneChain& L) {
    chain_set(L, LM_CHAIN);
    L.E = p;
    for (;;) {
        if (!in_chunk(K, p)) {
            L.x = p;
            if (exact || (uint64_t)p == K.len) return true;
            if ((uint64_t)p > K.len) return false;
            const Hdr e = hdr_load(K.base, p, K.len);
            return (e.status == REC_OK && e.good) || e.status == CLY_END_ZERO;
        }
        const Hdr h = hdr_load(K.base, p, K.len);
        if (h.status != REC_OK) {
            L.x = p; L.term = h.status;
            return exact || (h.status == CLY_END_EOF && (uint64_t)p == K.len);
        }
        if (!exact && !h.good) return false;
        L.cnt++;
        L.prev_crc = L.last_crc;
        L.last = p; L.last_crc = h.crc;
        if ((uint32_t)h.size < L.minsz) L.minsz = (uint32_t)h.size;
        p += (uint32_t)h.size;
    }
}

// SWAR byte masks (bit 7 of each byte): byte <= 4 (type / data type), byte
// nonzero and even (first byte of the key-size varint of a record with ks >= 1).
__device__ __forceinline__ uint32_t swar_le4(uint32_t W) { return ~(((W | 0x80808080u) - 0x05050505u) | W) & 0x80808080u; }
__device__ __forceinline__ uint32_t swar_ks(uint32_t W) {
    const uint32_t nz = ((W & 0x7f7f7f7fu) + 0x7f7f7f7fu) | W;
    return nz & ~(W << 7) & 0x80808080u;
}

// 16-B piece at chunk-relative offset o (bytes past len read as zero; pieces
// wholly past it are not loaded).
__device__ __forceinline__ u32x4 piece(const Chunk& K, uint32_t o) {
    const uint64_t a = (uint64_t)K.cb + o;
    if (a + 16 <= K.len) return *(const CLY_GL u32x4*)(K.base + a);
    u32x4 v = {0u, 0u, 0u, 0u};
    if (a < K.len) {
        v = *(const CLY_GL u32x4*)(K.base + a);
        const uint32_t n = (uint32_t)(K.len - a);          // 1..15 valid bytes
        #pragma unroll
        for (int k = 0; k < 4; k++) {
            const int lo = 4 * k;
            const uint32_t m = (int)n >= lo + 4 ? 0xFFFFFFFFu : ((int)n <= lo ? 0u : ((1u << (8 * (n - lo))) - 1u));
            v[k] &= m;
        }
    }
    return v;
}

// Phase A for one lane: the chain of its chunk under its own guess.
__device__ __noinline__ LaneChain phase_a(const Chunk K) {
    LaneChain L;
    if (!K.on) { chain_set(L, LM_OFF); return L; }
    if (K.cb == 0) { walk(K, 0, true, L); return L; }
    chain_set(L, LM_NONE);
    bool found = false;
    for (int b = 0; b < CLY_NB; b++) {
        if (found) continue;
        uint32_t w[CLY_BW + 4];
        if ((uint64_t)K.cb + (uint32_t)((b + 1) * CLY_BW * 4 + 16) <= K.len) {
            const CLY_GL u32x4* src = (const CLY_GL u32x4*)(K.base + K.cb + (uint32_t)(b * CLY_BW * 4));
            #pragma unroll
            for (int k = 0; k < CLY_BW / 4 + 1; k++) {
                const u32x4 v = src[k];
                w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
            }
        } else {
            #pragma unroll
            for (int k = 0; k < CLY_BW / 4 + 1; k++) {
                const u32x4 v = piece(K, (uint32_t)(b * CLY_BW * 4 + 16 * k));
                w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
            }
        }
        // candidate positions of the burst, one bit each (4 per word)
        uint32_t cmk[CLY_BW / 8];
        #pragma unroll
        for (int k = 0; k < CLY_BW / 8; k++) cmk[k] = 0;
        #pragma unroll
        for (int k = 0; k < CLY_BW; k++) {
            // positions 4k..4k+3: bytes +4, +5 <= 4 and +6 even nonzero
            const uint32_t L1 = swar_le4(w[k + 1]), L2 = swar_le4(w[k + 2]);
            const uint32_t cm = L1 & __builtin_amdgcn_alignbit(L2, L1, 8) & swar_ks(alignb(w[k + 2], w[k + 1], 2));
            const uint32_t nib = ((cm >> 7) & 1u) | ((cm >> 14) & 2u) | ((cm >> 21) & 4u) | ((cm >> 28) & 8u);
            cmk[k >> 3] |= nib << (4 * (k & 7));
        }
        #pragma unroll
        for (int k = 0; k < CLY_BW / 8; k++) {
            uint32_t m = found ? 0u : cmk[k];
            while (m) {
                const uint32_t q = K.cb + (uint32_t)(b * CLY_BW * 4 + 32 * k) + (uint32_t)__builtin_ctz(m);
                m &= m - 1;
                if (q >= K.ce) { m = 0; break; }
                LaneChain T;
                if (walk(K, q, false, T)) { L = T; found = true; m = 0; }
            }
        }
    }
    return L;
}

// ---------------------------------------------------------------------------
// wave helpers
__device__ __forceinline__ int scan_max_incl(int v, int lane) {
    #pragma unroll
    for (int o = 1; o < 64; o <<= 1) { const int u = __shfl_up(v, o, 64); if (lane >= o) v = max(v, u); }
    return v;
}
__device__ __forceinline__ int scan_max_excl(int v, int lane) {
    const int inc = scan_max_incl(v, lane);
    const int up = __shfl_up(inc, 1, 64);
    return lane > 0 ? up : -1;
}
__device__ __forceinline__ uint32_t scan_add_incl(uint32_t v, int lane) {
    #pragma unroll
    for (int o = 1; o < 64; o <<= 1) { const uint32_t u = __shfl_up(v, o, 64); if (lane >= o) v += u; }
    return v;
}
__device__ __forceinline__ uint32_t shfl_u32(uint32_t v, int src) { return (uint32_t)__shfl((int)v, src, 64); }

// In-wave agreement: lane l's chain must start where the chain of the nearest
// chunk before it leaves (the tile's entry X0 for the first lanes; dead0: the
// file's chain ended before the tile).  The lowest disagreeing lane is
// re-walked exactly, until every lane agrees.
__device__ __noinline__ LaneChain resolve(const Chunk K, LaneChain L, int lane, uint32_t X0, bool dead0, Globals* g) {
    for (int iter = 0;; iter++) {
        const bool isC = L.mode == LM_CHAIN;
        const int pk = scan_max_incl(isC ? lane : -1, lane);
        const int pu = __shfl_up(pk, 1, 64);            // (every lane: cross-lane reads outside conditionals)
        const int j = lane > 0 ? pu : -1;
        const uint32_t xj = shfl_u32(L.x, j < 0 ? 0 : j);
        const int tj = __shfl(L.term, j < 0 ? 0 : j, 64);
        const uint32_t Xin = j >= 0 ? xj : X0;
        const bool din = j >= 0 ? tj != TERM_NONE : dead0;
        bool bad = false;
        if (L.mode != LM_OFF) {
            if (din) bad = L.mode != LM_DEAD;
            else if (L.mode == LM_CHAIN) bad = L.E != Xin;
            else if (L.mode == LM_NONE) bad = in_chunk(K, Xin);
            else bad = true;                                   // LM_DEAD under a live chain
        }
        const u64 bm = __ballot(bad);
        if (!bm) return L;
        if (iter > 2 * CLY_NL + 2) { if (lane == 0) atomicOr(&g->fail, 1u); return L; }
        const int k = __ffsll((long long)bm) - 1;
        if (lane == k) {
            if (din) chain_set(L, LM_DEAD);
            else if (!in_chunk(K, Xin)) chain_set(L, LM_NONE);
            else walk(K, Xin, true, L);
        }
    }
}

// ---------------------------------------------------------------------------
// Look-back: the chain state and record count entering a tile.
struct LBState {
    uint64_t count;              // records of all tiles before
    uint32_t X;                  // chain position
    uint32_t crc_last;           // stored CRC of the last record started before (its successor's Q)
    uint32_t P_last;             // that record's start (NONE32: none in this file)
    int      dead;               // the file's chain has ended
};
__device__ __forceinline__ u64 ld_agent(const u64* p) {
    return __hip_atomic_load((const CLY_GL u64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(u64* p, u64 v) {
    __hip_atomic_store((CLY_GL u64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
#define SPIN_MAX (1u << 18)

__device__ __forceinline__ LBState lb_virtual() {
    LBState s;
    s.count = 0; s.X = 0; s.crc_last = 0; s.P_last = NONE32; s.dead = 1;
    return s;
}
__device__ __forceinline__ LBState lb_incl(u64 i0, u64 i1, u64 i2) {
    LBState s;
    s.dead = (i0 & DF_TERM) != 0;
    s.count = i0 >> 16;
    s.X = (uint32_t)i1; s.crc_last = (uint32_t)(i1 >> 32);
    s.P_last = (uint32_t)i2;
    return s;
}
// State after tile u given the state before it and u's LOCAL; false when the
// tile's guess disagrees with the state (then only its INCL can tell).
__device__ __forceinline__ bool lb_local(LBState& s, u64 l0, u64 l1, u64 l2, u64 l3) {
    if (!(l0 & DF_FOF)) {
        if (s.dead) return true;                                    // nothing of the file after its end
        if (l0 & DF_NONE) return s.X >= (uint32_t)l3;              // the chain passes the tile
        if (s.X != (uint32_t)l1) return false;
    }
    s.count += l0 >> 32;
    s.dead = (l0 & DF_TERM) != 0;
    s.X = (uint32_t)(l1 >> 32);
    if (l0 & DF_REC) { s.crc_last = (uint32_t)l2; s.P_last = (uint32_t)(l2 >> 32); }
    else if (l0 & DF_FOF) { s.crc_last = 0; s.P_last = NONE32; }
    return true;
}
__device__ __forceinline__ u64 shfl64(u64 v, int src) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, 64), hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64);
    return ((u64)hi << 32) | lo;
}
__device__ __forceinline__ void bad_spin(Globals* g, uint32_t code) { atomicOr(&g->fail, code); }

__device__ __forceinline__ int scan_max_excl(int v, int lane);

// Look-back of tile t: the nearest published INCL before it, then the
// LOCALs after it composed 64 tiles (one per lane) at a time.  Within a
// window the chain position entering tile m is the exit of the nearest tile
// before it that has a chain (or the window's entering state), "ended" is set
// by the nearest tile whose chain terminates and cleared by the first tile of
// a file; a tile whose guess disagrees with the position it is entered at
// stops the window: its own INCL (published once it has re-resolved) is
// awaited and the window goes on after it.
__device__ __noinline__ LBState look_back(const TileDesc* desc, int64_t t, int lane, Globals* g) {
    int64_t k = -1;
    for (int64_t base = t - 1; base >= 0; base -= 64) {
        const int64_t u = base - lane;
        const bool pub = u >= 0 && (ld_agent(&desc[u].i[0]) & DF_PUB);
        const u64 bm = __ballot(pub);
        PCNT(6, 1);
        if (bm) { k = base - (__ffsll((long long)bm) - 1); break; }
    }
    LBState s = lb_virtual();
    if (k >= 0) s = lb_incl(ld_agent(&desc[k].i[0]), ld_agent(&desc[k].i[1]), ld_agent(&desc[k].i[2]));
    for (int64_t u0 = k + 1; u0 < t; u0 += 64) {
        const int64_t u = u0 + lane;
        const int n = t - u0 < 64 ? (int)(t - u0) : 64;
        int got = lane < n ? 0 : 3;                    // 1 LOCAL, 2 INCL
        u64 w0 = 0;
        for (uint32_t spin = 0;; spin++) {
            if (got == 0) {
                const u64 i0 = ld_agent(&desc[u].i[0]);
                if (i0 & DF_PUB) { got = 2; w0 = i0; }
                else {
                    const u64 l0 = ld_agent(&desc[u].l[0]);
                    if (l0 & DF_PUB) { got = 1; w0 = l0; }
                }
            }
            if (__ballot(got == 0) == 0) break;
            PCNT(8, 1);
            if (spin > SPIN_MAX) { if (lane == 0) bad_spin(g, 2u); return s; }
            __builtin_amdgcn_s_sleep(2);
        }
        PCNT(7, 1);
        u64 w1 = 0, w2 = 0, w3 = 0;
        if (got == 2) { w1 = ld_agent(&desc[u].i[1]); w2 = ld_agent(&desc[u].i[2]); }
        else if (got == 1) { w1 = ld_agent(&desc[u].l[1]); w2 = ld_agent(&desc[u].l[2]); w3 = ld_agent(&desc[u].l[3]); }
        int m_lo = 0;
        for (int round = 0;; round++) {
            // the last INCL at or after m_lo overrides everything before it
            const u64 bi = __ballot(got == 2 && lane >= m_lo);
            if (bi) {
                const int mi = 63 - __clzll((long long)bi);
                s = lb_incl(shfl64(w0, mi), shfl64(w1, mi), shfl64(w2, mi));
                m_lo = mi + 1;
            }
            if (m_lo >= n) break;
            const bool act = lane >= m_lo && lane < n;
            const bool fof = act && (w0 & DF_FOF);
            const bool none = act && !fof && (w0 & DF_NONE);
            const bool chain = act && !none;
            const bool term = chain && (w0 & DF_TERM);
            const uint32_t G = (uint32_t)w1, Xo = (uint32_t)(w1 >> 32), tend = (uint32_t)w3;
            // entering state of each lane
            const int e = scan_max_excl((term || fof) ? lane : -1, lane);
            const int j = scan_max_excl(chain ? lane : -1, lane);
            const int te = __shfl((int)term, e < 0 ? 0 : e, 64);
            const uint32_t xj = shfl_u32(Xo, j < 0 ? 0 : j);
            const bool din = e >= 0 ? te != 0 : s.dead != 0;
            const uint32_t Xin = j >= 0 ? xj : s.X;
            const bool valid = !act || fof || din || (none ? Xin >= tend : Xin == G);
            const u64 bad = __ballot(!valid);
            const int ne = bad ? __ffsll((long long)bad) - 1 : n;      // lanes [m_lo, ne) compose
            const bool in = act && lane < ne;
            const bool applied = in && chain && (fof || !din);
            const bool rec = applied && (fof || (w0 & DF_REC));
            // state after each composed lane (inclusive scans)
            const uint32_t cnt = applied ? (uint32_t)(w0 >> 32) : 0u;
            const uint32_t ci = scan_add_incl(cnt, lane);
            const int ei = scan_max_incl(in && (term || fof) ? lane : -1, lane);
            const int ji = scan_max_incl(in && chain ? lane : -1, lane);
            const int ri = scan_max_incl(rec ? lane : -1, lane);
            const int tei = __shfl((int)term, ei < 0 ? 0 : ei, 64);
            const uint32_t xji = shfl_u32(Xo, ji < 0 ? 0 : ji);
            const u64 w0r = shfl64(w0, ri < 0 ? 0 : ri), w2r = shfl64(w2, ri < 0 ? 0 : ri);
            LBState o = s;
            o.count = s.count + ci;
            if (ei >= 0) o.dead = tei != 0;
            if (ji >= 0) o.X = xji;
            if (ri >= 0) {
                if (w0r & DF_REC) { o.crc_last = (uint32_t)w2r; o.P_last = (uint32_t)(w2r >> 32); }
                else { o.crc_last = 0; o.P_last = NONE32; }
            }
            const int last = ne - 1;
            if (last >= m_lo) {
                s.count = shfl64(o.count, last);
                s.X = shfl_u32(o.X, last);
                s.dead = __shfl(o.dead, last, 64);
                s.crc_last = shfl_u32(o.crc_last, last);
                s.P_last = shfl_u32(o.P_last, last);
            }
            if (!bad) break;
            // the tile at ne guessed wrong: wait for its true state
            const TileDesc* d = &desc[u0 + ne];
            u64 i0 = 0;
            PCNT(9, 1);
            for (uint32_t spin = 0;; spin++) {
                i0 = ld_agent(&d->i[0]);
                if (i0 & DF_PUB) break;
                PCNT(10, 1);
                if (spin > SPIN_MAX) { if (lane == 0) bad_spin(g, 4u); return s; }
                __builtin_amdgcn_s_sleep(2);
            }
            s = lb_incl(i0, ld_agent(&d->i[1]), ld_agent(&d->i[2]));
            m_lo = ne + 1;
            if (m_lo >= n) break;
        }
    }
    return s;
}

// ---------------------------------------------------------------------------
// Inputs of phase C for one lane (after the tile's chain is final).
struct LaneIn {
    uint64_t base;               // global tuple index of the lane's first record
    uint32_t crc_in;             // stored CRC of the record open when the chunk starts
    uint32_t P_in;               // its start (NONE32 none)
    bool     spill;              // P_in's patch reaches into this chunk
};

// The patch of the record start P (stored CRC c, predecessor's cq) on the
// words [wlo, whi) (absolute word indices), combined onto the last of them it
// touches; returns that word (NONE32: none in range).
__device__ __forceinline__ uint32_t patch_part(const CLY_LDS uint8_t* smem, const CrcLane& cl, uint32_t P, uint32_t c,
                                               uint32_t cq, uint32_t wlo, uint32_t whi, uint32_t& delta) {
    const uint32_t j = P & 3, sh = 8 * j, a = P >> 2;
    uint32_t acc = 0, wl = NONE32;
    if (a >= wlo && a < whi) {
        uint32_t pa = j ? (c << sh) : c;
        if (P != 0) pa ^= q_of(smem, cq, j, cl.r4);
        acc = pa; wl = a;
    }
    if (a + 1 >= wlo && a + 1 < whi) {
        const uint32_t pb = (j ? (c >> (32 - sh)) : 0u) ^ (j ? (0xFFFFFFFFu << sh) : 0xFFFFFFFFu);
        acc = wl == NONE32 ? pb : (crc_word(smem, acc, cl) ^ pb);
        wl = a + 1;
    }
    if (j && a + 2 >= wlo && a + 2 < whi) {
        const uint32_t pc = (1u << sh) - 1u;
        acc = wl == NONE32 ? pc : (crc_word(smem, acc, cl) ^ pc);
        wl = a + 2;
    }
    delta = acc;
    return wl;
}

// Tuple of the record at p (header h): 48 B, cly_tuple layout.
__device__ __forceinline__ void put_tuple(gtuples out, uint64_t idx, uint64_t out_cap, const Chunk& K, uint32_t p,
                                          const Hdr& h, uint32_t fid, Globals* g) {
    int tn;
    int64_t tx;
    if (h.key0 < 0x80 && h.ks >= 1) { tn = 1; tx = (int64_t)(h.key0 >> 1) ^ -(int64_t)(h.key0 & 1); }
    else {
        const int64_t klim = h.ks < 11u ? (int64_t)h.ks : 11;
        tx = go_varint(K.base + p + h.hsz, klim, tn);                   // parseLogRecordKey, db.go:706-710
    }
    if (idx >= out_cap) { atomicOr(&g->overflow, 1u); return; }
    const uint64_t off = p, ex = (uint64_t)h.exp, txv = tn < 0 ? 0ull : (uint64_t)tx;
    CLY_GL u32x4* dst = (CLY_GL u32x4*)(out + idx);
    dst[0] = (u32x4){(uint32_t)off, (uint32_t)(off >> 32), (uint32_t)ex, (uint32_t)(ex >> 32)};
    dst[1] = (u32x4){(uint32_t)txv, (uint32_t)(txv >> 32), fid, (uint32_t)h.size};
    dst[2] = (u32x4){h.ks, h.vs,
                     (h.type & 0xff) | ((h.dt & 0xff) << 8) | ((uint32_t)(h.hsz & 0xff) << 16) |
                         ((uint32_t)(tn < 0 ? 0xFF : tn) << 24),
                     h.crc};
}

// ---------------------------------------------------------------------------
// Phase C, uniform path.  Each record start P has one combined patch delta'
// on one word of the stream (patch_part); the walker decodes the lane's
// records (tuples written as it goes) and queues (word, delta') events in a
// per-lane LDS ring, ahead of the stream.  Per 128-B burst the stream loads
// the lane's 32 words, XORs in the burst's events, and runs the register
// through them: the loop body is the plain slicing-by-4 step.
struct Walker {
    uint32_t p, cq, i;
    Gath gt;
};
__device__ __forceinline__ void walker_step(const Chunk& K, Walker& W, uint32_t nrec, uint64_t base, uint32_t fid,
                                            gtuples out, uint64_t out_cap, const CLY_LDS uint8_t* smem,
                                            const CrcLane& cl, uint32_t& w, uint32_t& d, Globals* g) {
    const Hdr h = hdr_at(K.base, W.p, K.len, W.gt);
    put_tuple(out, base + W.i, out_cap, K, W.p, h, fid, g);
    const uint32_t wlo = K.cb >> 2;
    const uint32_t wa = patch_part(smem, cl, W.p, h.crc, W.cq, wlo, wlo + CLY_NW, d);
    w = wa == NONE32 ? NONE32 : wa - wlo;
    W.cq = h.crc;
    W.p += (uint32_t)h.size;
    W.i++;
    if (W.i < nrec && gath_ok(W.p, K.len)) gath_issue(K.base, W.p, W.gt);
}

__device__ __noinline__ uint32_t phase_c_fast(const Chunk K, const LaneChain L, const LaneIn I, bool active, uint32_t fid,
                                              gtuples out, uint64_t out_cap, const CLY_LDS uint8_t* smem,
                                              CLY_LDS u32x2* evq, const CrcLane cl, Globals* g) {
    // ring slot k of this lane: evq[k * 64]  (evq points at the wave's ring + lane)
    uint32_t head = 0, tail = 0;
    const uint32_t wlo = K.cb >> 2;
    if (active && I.spill) {
        uint32_t d;
        const uint32_t w = patch_part(smem, cl, I.P_in, I.crc_in, 0u, wlo, wlo + CLY_NW, d);
        if (w != NONE32) { evq[0] = (u32x2){w - wlo, d}; tail = 1; }
    }
    Walker W;
    W.p = L.E; W.cq = I.crc_in; W.i = 0;
    const uint32_t nrec = (active && L.mode == LM_CHAIN) ? L.cnt : 0u;
    if (nrec && gath_ok(W.p, K.len)) gath_issue(K.base, W.p, W.gt);
    // next event in registers
    uint32_t nw = NONE32, nd = 0;
    uint32_t s = 0;
    const CLY_GL u32x4* src = (const CLY_GL u32x4*)(K.base + K.cb);
    #pragma unroll 1
    for (int b = 0; b < CLY_NB; b++) {
        const uint32_t bend = (uint32_t)(b + 1) * CLY_BW;
        // walker ahead: every event of this and the next burst queued (ring permitting)
        for (;;) {
            const bool need = W.i < nrec && tail - head < EVQ && ((W.p >> 2) - wlo) < bend + CLY_BW;
            if (!__ballot(need)) break;
            if (need) {
                uint32_t w, d;
                walker_step(K, W, nrec, I.base, fid, out, out_cap, smem, cl, w, d, g);
                if (w != NONE32) { evq[(tail % EVQ) * 64] = (u32x2){w, d}; tail++; }
            }
        }
        if (nw == NONE32 && head != tail) { const u32x2 e = evq[(head % EVQ) * 64]; nw = e.x; nd = e.y; head++; }
        u32x4 v[CLY_BW / 4];
        if (active) {
            #pragma unroll
            for (int k = 0; k < CLY_BW / 4; k++) v[k] = src[b * (CLY_BW / 4) + k];
        } else {
            #pragma unroll
            for (int k = 0; k < CLY_BW / 4; k++) v[k] = (u32x4){0u, 0u, 0u, 0u};
        }
        // the burst's events into its words
        while (__ballot(nw < bend)) {
            if (nw < bend) {
                const uint32_t r = nw - (uint32_t)b * CLY_BW;
                #pragma unroll
                for (int k = 0; k < CLY_BW / 4; k++) {
                    v[k].x ^= r == 4u * k ? nd : 0u;
                    v[k].y ^= r == 4u * k + 1 ? nd : 0u;
                    v[k].z ^= r == 4u * k + 2 ? nd : 0u;
                    v[k].w ^= r == 4u * k + 3 ? nd : 0u;
                }
                nw = NONE32;
                if (head != tail) { const u32x2 e = evq[(head % EVQ) * 64]; nw = e.x; nd = e.y; head++; }
            }
        }
        #pragma unroll
        for (int k = 0; k < CLY_BW / 4; k++) {
            s = crc_word(smem, s ^ v[k].x, cl);
            s = crc_word(smem, s ^ v[k].y, cl);
            s = crc_word(smem, s ^ v[k].z, cl);
            s = crc_word(smem, s ^ v[k].w, cl);
        }
    }
    return s;
}

// ---------------------------------------------------------------------------
// Phase C, exact path (the lane holding the chain's terminal, lanes with
// records shorter than 12 bytes, and k_locate): word by word with every
// boundary's byte patches, everything from the terminal T on zeroed.  Starts
// from register s0.  With `observe`, the first record whose check fails
// (register after its end word != 0) is returned in fail_P / fail_i.
struct Bnd { uint32_t P, c, q, start; uint64_t idx; int term; };
__device__ __noinline__ uint32_t exact_lane(const Chunk& K, const LaneChain& L, const LaneIn& I, uint32_t s0, bool emit,
                               bool observe, uint32_t fid, gtuples out, uint64_t out_cap,
                               const CLY_LDS uint8_t* smem, const CrcLane& cl, Globals* g, uint32_t& fail_P,
                               uint64_t& fail_i, uint32_t& expect) {
    uint32_t s = s0;
    fail_P = NONE32; fail_i = 0; expect = 0;
    Bnd bq[4];
    int nb = 0;
    if (I.spill) { bq[0].P = I.P_in; bq[0].c = I.crc_in; bq[0].q = 0; bq[0].term = 0; bq[0].start = NONE32; bq[0].idx = 0; nb = 1; }
    const uint32_t T = (L.mode == LM_CHAIN && L.term != TERM_NONE) ? L.x : NONE32;
    uint32_t wp = L.E, cq = I.crc_in, wi = 0, start = I.P_in;
    uint64_t sidx = I.base - 1;
    const uint32_t nrec = L.mode == LM_CHAIN ? L.cnt : 0u;
    bool tpushed = T == NONE32;
    for (uint32_t w = 0; w < CLY_NW; w++) {
        const uint32_t A = K.cb + 4 * w;
        // queue the boundaries whose first patch word is this one
        for (;;) {
            if (wi < nrec && (wp >> 2) == (A >> 2) && nb < 4) {
                const Hdr h = hdr_load(K.base, wp, K.len);
                if (emit) put_tuple(out, I.base + wi, out_cap, K, wp, h, fid, g);
                Bnd& b = bq[nb++];
                b.P = wp; b.c = h.crc; b.q = wp != 0 ? q_of(smem, cq, wp & 3, cl.r4) : 0u; b.term = 0;
                b.start = start; b.idx = sidx;
                start = wp; sidx = I.base + wi;
                cq = h.crc; wp += (uint32_t)h.size; wi++;
                continue;
            }
            if (!tpushed && wi >= nrec && (T >> 2) == (A >> 2) && nb < 4) {
                Bnd& b = bq[nb++];
                b.P = T; b.c = 0; b.q = T != 0 ? q_of(smem, cq, T & 3, cl.r4) : 0u; b.term = 1;
                b.start = start; b.idx = sidx;
                tpushed = true;
                continue;
            }
            break;
        }
        uint32_t d = 0;
        if ((uint64_t)A < K.len) {
            d = *(const CLY_GL uint32_t*)(K.base + A);
            const uint64_t n = K.len - A;
            if (n < 4) d &= (1u << (8 * n)) - 1u;
        }
        if (T != NONE32 && A + 4 > T) d = A >= T ? 0u : (d & ((1u << (8 * (T - A))) - 1u));
        uint32_t patch = 0;
        for (int k = 0; k < nb; k++) {
            const Bnd& b = bq[k];
            #pragma unroll
            for (int i = 0; i < 4; i++) {
                const uint32_t x = A + i;
                uint32_t m = 0;
                if (!b.term && x >= b.P && x < b.P + 4) m = (d >> (8 * i)) & 0xffu;          // stored CRC zeroed
                if (!b.term && x >= b.P + 4 && x < b.P + 8) m ^= 0xffu;                     // init 0xFF
                patch ^= m << (8 * i);
            }
            if ((b.P >> 2) == (A >> 2)) patch ^= b.q;
        }
        s = crc_word(smem, s ^ d ^ patch, cl);
        if (observe && fail_P == NONE32) {
            for (int k = 0; k < nb; k++)
                if ((bq[k].P >> 2) == (A >> 2) && bq[k].P != 0 && bq[k].start != NONE32 && s != 0) {
                    fail_P = bq[k].start; fail_i = bq[k].idx;
                }
        }
        // retire boundaries whose patch span ended
        int o = 0;
        for (int k = 0; k < nb; k++) if (bq[k].P + 8 > A + 4 && !(bq[k].term && (bq[k].P >> 2) <= (A >> 2))) bq[o++] = bq[k];
        nb = o;
        if (nb == 4) { if (emit) atomicOr(&g->fail, 16u); }
    }
    // the terminal one word past a full chunk (T = len = chunk end): the register
    // after the chunk must equal Q there
    if (!tpushed) {
        expect = T != 0 ? q_of(smem, cq, 0, cl.r4) : 0u;
        if (observe && fail_P == NONE32 && s != expect && start != NONE32) { fail_P = start; fail_i = sidx; }
    }
    return s;
}

// ---------------------------------------------------------------------------
// One tile: phase A, agreement, look-back, phase C, fold.
__device__ __forceinline__ int find_file(const uint32_t* __restrict__ tprefix, int nfiles, uint32_t t) {
    int lo = 0, hi = nfiles - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (tprefix[mid] <= t) lo = mid; else hi = mid - 1;
    }
    return lo;
}
__device__ __forceinline__ Chunk make_chunk(const DevFile& F, uint32_t tt, int lane) {
    Chunk K;
    K.base = (gbytes)F.base; K.len = F.len;
    const uint64_t cb = (uint64_t)tt * CLY_TILE + (uint64_t)lane * CLY_CH;
    K.cb = (uint32_t)cb;
    K.ce = (uint32_t)(cb + CLY_CH < F.len ? cb + CLY_CH : F.len);
    K.last = cb + CLY_CH >= F.len;
    K.on = cb < F.len || cb == 0;
    if (!K.on) { K.cb = 0xFFFFFFF0u; K.ce = 0xFFFFFFF0u; }
    return K;
}
// Lane inputs from the final chain and the state entering the tile.
__device__ __forceinline__ LaneIn lane_inputs(const Chunk& K, const LaneChain& L, const LBState& S, int lane,
                                             uint32_t& tile_cnt) {
    LaneIn I;
    const uint32_t cnt = (L.mode == LM_CHAIN) ? L.cnt : 0u;
    const uint32_t incl = scan_add_incl(cnt, lane);
    tile_cnt = shfl_u32(incl, 63);
    I.base = S.count + (incl - cnt);
    const int pr = scan_max_incl(cnt > 0 ? lane : -1, lane);
    const int pu = __shfl_up(pr, 1, 64);
    const int j = lane > 0 ? pu : -1;
    const uint32_t lc = shfl_u32(L.last_crc, j < 0 ? 0 : j), lp = shfl_u32(L.last, j < 0 ? 0 : j);
    I.crc_in = j >= 0 ? lc : S.crc_last;
    I.P_in = j >= 0 ? lp : S.P_last;
    I.spill = K.on && (L.mode == LM_CHAIN || L.mode == LM_NONE) && I.P_in != NONE32 && I.P_in + 8 > K.cb &&
              I.P_in < K.cb;
    return I;
}
// Fold of the lanes' registers: sum over l of A^(CLY_CH (63 - l)) r_l (lane 0).
__device__ __forceinline__ uint32_t tile_fold(const CLY_LDS uint8_t* smem, uint32_t r, int lane) {
    #pragma unroll
    for (int lvl = 0; lvl < 6; lvl++) {
        const int d = 1 << lvl;
        const uint32_t o = (uint32_t)__shfl_down((int)r, d, 64);
        const uint32_t sh = nib_mul(smem, lvl, r);
        if ((lane & (2 * d - 1)) == 0) r = sh ^ o;
    }
    return r;
}

// Phase A of one tile: the lanes' chains under their own guesses, made to
// agree, and the tile's LOCAL descriptor.
struct TileA { LaneChain L; uint32_t G; };
__device__ __noinline__ TileA tile_a(const Chunk K, uint32_t t, uint32_t tt, uint64_t flen, int lane, TileDesc* desc,
                                     Globals* g) {
    const bool fof = tt == 0;
    TileA A;
    A.L = phase_a(K);
    A.G = NONE32;
    {
        const u64 bm = __ballot(A.L.mode == LM_CHAIN);
        if (bm) A.G = shfl_u32(A.L.E, __ffsll((long long)bm) - 1);
    }
    A.L = resolve(K, A.L, lane, fof ? 0u : A.G, false, g);
    const LaneChain& L = A.L;
    const u64 bc = __ballot(L.mode == LM_CHAIN), br = __ballot(L.mode == LM_CHAIN && L.cnt > 0);
    const uint32_t c = L.mode == LM_CHAIN ? L.cnt : 0u;
    const uint32_t tile_cnt = shfl_u32(scan_add_incl(c, lane), 63);
    const int lc = bc ? 63 - __clzll((long long)bc) : 0, lr = br ? 63 - __clzll((long long)br) : 0;
    const uint32_t X = shfl_u32(L.x, lc);
    const int term = __shfl(L.term, lc, 64);
    const uint32_t crc = shfl_u32(L.last_crc, lr), Pl = shfl_u32(L.last, lr);
    if (lane == 0) {
        const uint64_t tstart = (uint64_t)tt * CLY_TILE;
        const uint32_t tend = tstart + CLY_TILE >= flen ? (uint32_t)(flen + 1) : (uint32_t)(tstart + CLY_TILE);
        TileDesc* d = &desc[t];
        st_agent(&d->l[1], (u64)A.G | ((u64)X << 32));
        st_agent(&d->l[2], (u64)crc | ((u64)Pl << 32));
        st_agent(&d->l[3], (u64)tend);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        u64 f0 = DF_PUB | ((u64)tile_cnt << 32);
        if (bc && term != TERM_NONE) f0 |= DF_TERM;
        if (!bc) f0 |= DF_NONE;
        if (fof) f0 |= DF_FOF;
        if (br) f0 |= DF_REC;
        st_agent(&d->l[0], f0);
    }
    return A;
}
__device__ __forceinline__ uint32_t take_tile(Globals* g, int lane) {
    uint32_t t = 0;
    if (lane == 0) t = atomicAdd(&g->ticket, 1u);
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)shfl_u32(t, 0));
}

__global__ void __launch_bounds__(64 * SCAN_WAVES, 4)
k_scan(const DevFile* __restrict__ files, int nfiles, const uint32_t* __restrict__ tprefix, uint32_t ntiles,
       TileDesc* desc, uint32_t* treg, FileInfo* finfo, const uint32_t* __restrict__ nib, cly_tuple* out_,
       uint64_t out_cap, Globals* g, uint32_t* dump) {
    gtuples out = (gtuples)out_;
    __shared__ __attribute__((aligned(16))) unsigned char smem_raw[SCAN_LDS];
    CLY_LDS uint8_t* smem = (CLY_LDS uint8_t*)smem_raw;
    init_tables(smem, nib);
    const int lane = threadIdx.x & 63;
    const CrcLane cl = crc_lane(lane);
    CLY_LDS u32x2* evq = (CLY_LDS u32x2*)(smem + LDS_EVQ) + (threadIdx.x >> 6) * (EVQ * 64) + lane;
    // Tiles are software-pipelined per wave: phase A of the wave's next tile
    // (and its LOCAL) comes before phase C of the current one, so the
    // look-back of the next tile finds its predecessors published.
    uint32_t t = take_tile(g, lane);
    if (t >= ntiles) return;
    int f = find_file(tprefix, nfiles, t);
    DevFile F = files[f];
    uint32_t tt = t - F.first_tile;
    Chunk K = make_chunk(F, tt, lane);
    TileA A = tile_a(K, t, tt, F.len, lane, desc, g);
    for (;;) {
        PROF_T0();
        const bool fof = tt == 0;
        LaneChain L = A.L;
        // ---- L: the true state entering the tile
        LBState S = look_back(desc, (int64_t)t, lane, g);
        PROF(1);
        if (fof) { S.dead = 0; S.X = 0; S.crc_last = 0; S.P_last = NONE32; }
        if (!fof && (S.dead || S.X != A.G) && lane == 0) atomicAdd(&g->refix, 1u);
        L = resolve(K, L, lane, S.dead ? 0u : S.X, S.dead != 0, g);
        uint32_t tile_cnt;
        const LaneIn I = lane_inputs(K, L, S, lane, tile_cnt);
        if (dump) {
            // debug dump (CLY_DUMP): the final chain of every lane
            uint32_t* o = dump + ((uint64_t)t * 64 + lane) * 8;
            o[0] = (uint32_t)L.mode; o[1] = L.E; o[2] = L.x; o[3] = (uint32_t)L.term; o[4] = L.cnt;
            o[5] = S.X | (S.dead ? 0x80000000u : 0u); o[6] = A.G; o[7] = (uint32_t)f;
        }
        {
            // INCL descriptor
            LBState o = S;
            o.count += tile_cnt;
            const u64 bc = __ballot(L.mode == LM_CHAIN), br = __ballot(L.mode == LM_CHAIN && L.cnt > 0);
            if (bc) {
                const int lc = 63 - __clzll((long long)bc);
                o.X = shfl_u32(L.x, lc);
                o.dead = __shfl(L.term, lc, 64) != TERM_NONE;
            }
            if (br) {
                const int lr = 63 - __clzll((long long)br);
                o.crc_last = shfl_u32(L.last_crc, lr);
                o.P_last = shfl_u32(L.last, lr);
            }
            if (lane == 0) {
                TileDesc* d = &desc[t];
                st_agent(&d->i[1], (u64)o.X | ((u64)o.crc_last << 32));
                st_agent(&d->i[2], (u64)o.P_last);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                st_agent(&d->i[0], DF_PUB | (o.dead ? DF_TERM : 0ull) | (o.count << 16));
                if (fof) finfo[f].first_index = S.count;
                if (t == ntiles - 1) g->total = o.count;
            }
        }
        PROF(2);
        // ---- A of the next tile
        const uint32_t tn = take_tile(g, lane);
        int fn = f;
        DevFile Fn = F;
        uint32_t ttn = 0;
        Chunk Kn = K;
        TileA An = A;
        if (tn < ntiles) {
            fn = find_file(tprefix, nfiles, tn);
            Fn = files[fn];
            ttn = tn - Fn.first_tile;
            Kn = make_chunk(Fn, ttn, lane);
            An = tile_a(Kn, tn, ttn, Fn.len, lane, desc, g);
        }
        PROF(0);
        // ---- C: CRC stream, tuples
        const bool term_lane = L.mode == LM_CHAIN && L.term != TERM_NONE;
        const bool slow = L.mode == LM_CHAIN && !term_lane && L.minsz < 12;
        const bool fast = (L.mode == LM_CHAIN && !term_lane && !slow) || L.mode == LM_NONE;
        uint32_t r = phase_c_fast(K, L, I, fast, F.fid, out, out_cap, smem, evq, cl, g);
        PROF(3);
        if (term_lane || slow) {
            uint32_t fp, ex;
            uint64_t fi;
            r = exact_lane(K, L, I, 0u, true, false, F.fid, out, out_cap, smem, cl, g, fp, fi, ex);
            if (slow) atomicAdd(&g->slow_lanes, 1u);
            if (term_lane) {
                FileInfo* fo = &finfo[f];
                fo->term_pos = L.x; fo->term_status = L.term; fo->term_tile = t; fo->term_lane = (uint32_t)lane;
                fo->expect = ex; fo->end_index = I.base + L.cnt; fo->has_term = 1;
            }
        }
        if (!fast && !term_lane && !slow) r = 0;
        PROF(4);
        r = tile_fold(smem, r, lane);
        PROF(5);
        if (lane == 0) treg[t] = r;
        if (tn >= ntiles) break;
        t = tn; f = fn; F = Fn; tt = ttn; K = Kn; A = An;
    }
}

// ---------------------------------------------------------------------------
// k_fin: per file, the fold of its tile registers up to the terminal's tile
// must equal A^(CLY_CH (63 - terminal lane)) expect.
__device__ __forceinline__ uint32_t xpow_mul(const uint32_t* __restrict__ pw, uint64_t m, uint32_t v) {
    for (int k = 0; m; k++, m >>= 1) if (m & 1) v = cly_multmodp(pw[k], v);
    return v;
}
#define FIN_NT 256
__global__ void __launch_bounds__(FIN_NT)
k_fin(const DevFile* __restrict__ files, FileInfo* finfo, const uint32_t* __restrict__ treg,
      const uint32_t* __restrict__ nib, const uint32_t* __restrict__ pw, Globals* g) {
    __shared__ uint32_t tab[NIB_LEVELS * 128];
    __shared__ uint32_t part[FIN_NT];
    __shared__ uint32_t plen[FIN_NT];
    for (int i = threadIdx.x; i < NIB_LEVELS * 128; i += FIN_NT) tab[i] = nib[i];
    __syncthreads();
    const int f = blockIdx.x;
    const DevFile F = files[f];
    FileInfo* fo = &finfo[f];
    const uint32_t has = fo->has_term;
    if (!has) {
        if (threadIdx.x == 0) { atomicOr(&g->fail, 32u); fo->ok = 0; }
        return;
    }
    const uint32_t n = fo->term_tile - F.first_tile + 1;
    const uint32_t per = (n + FIN_NT - 1) / FIN_NT;
    const uint32_t lo = threadIdx.x * per, hi = lo + per < n ? lo + per : n;
    uint32_t s = 0;
    for (uint32_t i = lo; i < hi; i++) {
        uint32_t p = 0;
        #pragma unroll
        for (int k = 0; k < 8; k++) p ^= tab[6 * 128 + k * 16 + ((s >> (4 * k)) & 15u)];
        s = p ^ treg[F.first_tile + i];
    }
    part[threadIdx.x] = s;
    plen[threadIdx.x] = hi > lo ? hi - lo : 0;
    __syncthreads();
    for (int d = 1; d < FIN_NT; d <<= 1) {
        if ((threadIdx.x & (2 * d - 1)) == 0) {
            part[threadIdx.x] = xpow_mul(pw, plen[threadIdx.x + d], part[threadIdx.x]) ^ part[threadIdx.x + d];
            plen[threadIdx.x] += plen[threadIdx.x + d];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        // A^(CLY_CH (63 - lane)) expect
        uint32_t e = fo->expect;
        const uint32_t m = 63 - fo->term_lane;
        for (int lvl = 0; lvl < 6; lvl++) {
            if (m & (1u << lvl)) {
                uint32_t p = 0;
                for (int k = 0; k < 8; k++) p ^= tab[lvl * 128 + k * 16 + ((e >> (4 * k)) & 15u)];
                e = p;
            }
        }
        fo->fold = part[0];
        fo->ok = part[0] == e;
        fo->fail_key = ~0ull;
        if (part[0] != e) atomicOr(&g->any_fail, 1u);
    }
}

// ---------------------------------------------------------------------------
// k_locate (only after a failed fold): every tile of a failing file up to its
// terminal re-derives its chain from the published states, the register
// entering each chunk, and walks its records' checks from there; the first
// failing record of the file wins (atomicMin on offset << 32 | index).
__global__ void __launch_bounds__(512, 4)
k_locate(const DevFile* __restrict__ files, int nfiles, const uint32_t* __restrict__ tprefix, uint32_t ntiles,
         const TileDesc* desc, const uint32_t* __restrict__ treg, FileInfo* finfo, const uint32_t* __restrict__ nib,
         Globals* g) {
    __shared__ __attribute__((aligned(16))) unsigned char smem_raw[SCAN_LDS];
    CLY_LDS uint8_t* smem = (CLY_LDS uint8_t*)smem_raw;
    init_tables(smem, nib);
    const int lane = threadIdx.x & 63;
    const CrcLane cl = crc_lane(lane);
    for (uint32_t t = blockIdx.x * 8 + (threadIdx.x >> 6); t < ntiles; t += gridDim.x * 8) {
        const int f = find_file(tprefix, nfiles, t);
        const DevFile F = files[f];
        FileInfo* fo = &finfo[f];
        if (fo->ok || t > fo->term_tile) continue;
        const uint32_t tt = t - F.first_tile;
        const bool fof = tt == 0;
        const Chunk K = make_chunk(F, tt, lane);
        LBState S;
        if (fof) { S = lb_virtual(); S.dead = 0; S.X = 0; S.count = fo->first_index; }
        else S = lb_incl(desc[t - 1].i[0], desc[t - 1].i[1], desc[t - 1].i[2]);
        if (S.dead) continue;
        LaneChain L = phase_a(K);
        L = resolve(K, L, lane, S.X, false, g);
        uint32_t tile_cnt;
        const LaneIn I = lane_inputs(K, L, S, lane, tile_cnt);
        // register entering the tile
        uint32_t st = 0;
        for (uint32_t i = F.first_tile; i < t; i++) st = nib_mul(smem, 6, st) ^ treg[i];
        const bool live = L.mode == LM_CHAIN || L.mode == LM_NONE;
        uint32_t fp, ex;
        uint64_t fi;
        uint32_t r = live ? exact_lane(K, L, I, 0u, false, false, F.fid, nullptr, 0, smem, cl, g, fp, fi, ex) : 0u;
        // exclusive fold over the lanes, plus A^(CLY_CH l) st
        uint32_t v = r;
        #pragma unroll
        for (int lvl = 0; lvl < 6; lvl++) {
            const int d = 1 << lvl;
            const uint32_t u = (uint32_t)__shfl_up((int)v, d, 64);
            const uint32_t sh = nib_mul(smem, lvl, u);
            if (lane >= d) v ^= sh;
        }
        uint32_t sin = (uint32_t)__shfl_up((int)v, 1, 64);
        if (lane == 0) sin = 0;
        uint32_t se = st;
        for (int lvl = 0; lvl < 6; lvl++) if (lane & (1 << lvl)) se = nib_mul(smem, lvl, se);
        sin ^= se;
        if (live) {
            exact_lane(K, L, I, sin, false, true, F.fid, nullptr, 0, smem, cl, g, fp, fi, ex);
            if (fp != NONE32) atomicMin(&fo->fail_key, ((u64)fp << 32) | (u64)(fi - fo->first_index));
        }
    }
}

// ---------------------------------------------------------------------------
// Host side
#define HIPCK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "clyscan: %s failed: %s\n", #x, hipGetErrorString(e_)); return CLY_ERR_DEVICE; } } while (0)

struct cly_ctx {
    int device;
    hipStream_t stream;
    hipEvent_t ev[4];
    DevFile* d_files; uint32_t* d_tprefix; FileInfo* d_finfo; int cap_files;
    DevFile* h_files; uint32_t* h_tprefix; FileInfo* h_finfo;
    TileDesc* d_desc; uint32_t* d_treg; int64_t cap_tiles;
    Globals* d_g; Globals* h_g;
    uint32_t* d_nib;             // nibble tables of A^(CLY_CH 2^k), k < NIB_LEVELS
    uint32_t* d_pw;              // x^(8 CLY_TILE 2^k) mod P, k < 40
    int scan_grid;
    uint8_t* d_bytes; uint64_t cap_bytes;          // host-path staging
    cly_tuple* d_tuples; uint64_t cap_tuples;
    void* merge_scratch;         // clymerge.hip's buffers (grow-only)
};
extern "C" void cly_merge_scratch_free(void* p);

extern "C" int cly_ctx_create(int device, cly_ctx** out) {
    if (!out) return CLY_ERR_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev) return CLY_ERR_DEVICE;
    HIPCK(hipSetDevice(device));
    cly_ctx* c = (cly_ctx*)calloc(1, sizeof(cly_ctx));
    if (!c) return CLY_ERR_DEVICE;
    c->device = device;
    HIPCK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    for (int i = 0; i < 4; i++) HIPCK(hipEventCreate(&c->ev[i]));
    HIPCK(hipMalloc(&c->d_g, sizeof(Globals)));
    HIPCK(hipHostMalloc(&c->h_g, sizeof(Globals), hipHostMallocDefault));
    {
        uint32_t hn[NIB_LEVELS * 128];
        for (int lvl = 0; lvl < NIB_LEVELS; lvl++) {
            const uint32_t xm = cly_x8n((uint64_t)CLY_CH << lvl);
            for (int nb = 0; nb < 8; nb++)
                for (uint32_t v = 0; v < 16; v++) hn[lvl * 128 + nb * 16 + v] = cly_multmodp(xm, v << (4 * nb));
        }
        HIPCK(hipMalloc(&c->d_nib, sizeof(hn)));
        HIPCK(hipMemcpy(c->d_nib, hn, sizeof(hn), hipMemcpyHostToDevice));
        uint32_t hp[40];
        hp[0] = cly_x8n((uint64_t)CLY_TILE);
        for (int k = 1; k < 40; k++) hp[k] = cly_multmodp(hp[k - 1], hp[k - 1]);
        HIPCK(hipMalloc(&c->d_pw, sizeof(hp)));
        HIPCK(hipMemcpy(c->d_pw, hp, sizeof(hp), hipMemcpyHostToDevice));
    }
    {
        int per_cu = 0, ncu = 0;
        HIPCK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_scan, 64 * SCAN_WAVES, 0));
        HIPCK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device));
        if (per_cu < 1) per_cu = 1;
        if (per_cu > 1) per_cu = 1;
        c->scan_grid = per_cu * ncu;
    }
    *out = c;
    return CLY_OK;
}

extern "C" void cly_ctx_destroy(cly_ctx* c) {
    if (!c) return;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    hipFree(c->d_files); hipFree(c->d_tprefix); hipFree(c->d_finfo); hipFree(c->d_desc); hipFree(c->d_treg);
    hipFree(c->d_g); hipFree(c->d_nib); hipFree(c->d_pw); hipFree(c->d_bytes); hipFree(c->d_tuples);
    hipHostFree(c->h_files); hipHostFree(c->h_tprefix); hipHostFree(c->h_finfo); hipHostFree(c->h_g);
    cly_merge_scratch_free(c->merge_scratch);
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
    hipFree(c->d_files); hipFree(c->d_tprefix); hipFree(c->d_finfo);
    hipHostFree(c->h_files); hipHostFree(c->h_tprefix); hipHostFree(c->h_finfo);
    c->d_files = nullptr; c->d_tprefix = nullptr; c->d_finfo = nullptr;
    c->h_files = nullptr; c->h_tprefix = nullptr; c->h_finfo = nullptr;
    c->cap_files = 0;
    const int cap = nfiles < 64 ? 64 : nfiles;
    HIPCK(hipMalloc(&c->d_files, sizeof(DevFile) * cap));
    HIPCK(hipMalloc(&c->d_tprefix, sizeof(uint32_t) * (cap + 1)));
    HIPCK(hipMalloc(&c->d_finfo, sizeof(FileInfo) * cap));
    HIPCK(hipHostMalloc(&c->h_files, sizeof(DevFile) * cap, hipHostMallocDefault));
    HIPCK(hipHostMalloc(&c->h_tprefix, sizeof(uint32_t) * (cap + 1), hipHostMallocDefault));
    HIPCK(hipHostMalloc(&c->h_finfo, sizeof(FileInfo) * cap, hipHostMallocDefault));
    c->cap_files = cap;
    return CLY_OK;
}

static int ensure_tiles(cly_ctx* c, int64_t ntiles) {
    if (ntiles <= c->cap_tiles) return CLY_OK;
    hipFree(c->d_desc); hipFree(c->d_treg);
    c->d_desc = nullptr; c->d_treg = nullptr; c->cap_tiles = 0;
    const int64_t cap = ntiles < 1024 ? 1024 : ntiles;
    HIPCK(hipMalloc(&c->d_desc, sizeof(TileDesc) * cap));
    HIPCK(hipMalloc(&c->d_treg, sizeof(uint32_t) * cap));
    c->cap_tiles = cap;
    return CLY_OK;
}

extern "C" int cly_scan_device(cly_ctx* c, const cly_file* files, int nfiles, cly_tuple* d_out, uint64_t out_cap,
                               uint64_t* file_first, cly_file_result* res, uint64_t* needed, cly_stats* stats,
                               void* stream_v) {
    if (!c || (!files && nfiles) || nfiles < 0 || !res || !file_first) return CLY_ERR_ARG;
    if (nfiles == 0) { if (needed) *needed = 0; return CLY_OK; }
    HIPCK(hipSetDevice(c->device));
    hipStream_t st = stream_v ? (hipStream_t)stream_v : c->stream;
    int rc = ensure_files(c, nfiles);
    if (rc) return rc;
    int64_t ntiles = 0;
    uint64_t bytes = 0;
    for (int i = 0; i < nfiles; i++) {
        if (files[i].len >= 0xFFFFFFFFull) return CLY_ERR_ARG;
        if (files[i].len && (((uintptr_t)files[i].base) & 15)) return CLY_ERR_ARG;
        const uint64_t nt = files[i].len ? (files[i].len + CLY_TILE - 1) / CLY_TILE : 1;
        c->h_files[i].base = files[i].base;
        c->h_files[i].len = files[i].len;
        c->h_files[i].fid = files[i].fid;
        c->h_files[i].first_tile = (uint32_t)ntiles;
        c->h_files[i].ntile = (uint32_t)nt;
        c->h_files[i]._pad = 0;
        c->h_tprefix[i] = (uint32_t)ntiles;
        ntiles += (int64_t)nt;
        bytes += files[i].len;
    }
    if (ntiles >= (1LL << 31)) return CLY_ERR_ARG;
    c->h_tprefix[nfiles] = (uint32_t)ntiles;
    rc = ensure_tiles(c, ntiles);
    if (rc) return rc;
    HIPCK(hipMemcpyAsync(c->d_files, c->h_files, sizeof(DevFile) * nfiles, hipMemcpyHostToDevice, st));
    HIPCK(hipMemcpyAsync(c->d_tprefix, c->h_tprefix, sizeof(uint32_t) * (nfiles + 1), hipMemcpyHostToDevice, st));
    HIPCK(hipMemsetAsync(c->d_desc, 0, sizeof(TileDesc) * ntiles, st));
    HIPCK(hipMemsetAsync(c->d_finfo, 0, sizeof(FileInfo) * nfiles, st));
    HIPCK(hipMemsetAsync(c->d_g, 0, sizeof(Globals), st));
    int grid = c->scan_grid;
    if ((int64_t)grid * SCAN_WAVES > ntiles) grid = (int)((ntiles + SCAN_WAVES - 1) / SCAN_WAVES);
    HIPCK(hipEventRecord(c->ev[0], st));
    // debug: CLY_DUMP=<path> appends every lane's final chain (8 u32 per lane) of each call
    const char* dump_path = getenv("CLY_DUMP");
    uint32_t* d_dump = nullptr;
    if (dump_path) HIPCK(hipMalloc(&d_dump, sizeof(uint32_t) * 8 * 64 * ntiles));
    hipLaunchKernelGGL(k_scan, dim3(grid), dim3(64 * SCAN_WAVES), 0, st, c->d_files, nfiles, c->d_tprefix, (uint32_t)ntiles,
                       c->d_desc, c->d_treg, c->d_finfo, c->d_nib, d_out, out_cap, c->d_g, d_dump);
    HIPCK(hipGetLastError());
    HIPCK(hipEventRecord(c->ev[1], st));
    hipLaunchKernelGGL(k_fin, dim3(nfiles), dim3(FIN_NT), 0, st, c->d_files, c->d_finfo, c->d_treg, c->d_nib, c->d_pw,
                       c->d_g);
    HIPCK(hipGetLastError());
    HIPCK(hipEventRecord(c->ev[2], st));
    HIPCK(hipMemcpyAsync(c->h_g, c->d_g, sizeof(Globals), hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    bool located = false;
    if (c->h_g->any_fail && !c->h_g->fail) {
        hipLaunchKernelGGL(k_locate, dim3(c->scan_grid), dim3(512), 0, st, c->d_files, nfiles, c->d_tprefix, (uint32_t)ntiles,
                           c->d_desc, c->d_treg, c->d_finfo, c->d_nib, c->d_g);
        HIPCK(hipGetLastError());
        located = true;
    }
    HIPCK(hipEventRecord(c->ev[3], st));
    HIPCK(hipMemcpyAsync(c->h_finfo, c->d_finfo, sizeof(FileInfo) * nfiles, hipMemcpyDeviceToHost, st));
    HIPCK(hipMemcpyAsync(c->h_g, c->d_g, sizeof(Globals), hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    if (d_dump) {
        const size_t nb = sizeof(uint32_t) * 8 * 64 * ntiles;
        uint32_t* h = (uint32_t*)malloc(nb);
        if (h && hipMemcpy(h, d_dump, nb, hipMemcpyDeviceToHost) == hipSuccess) {
            FILE* fd = fopen(dump_path, "ab");
            if (fd) { fwrite(h, 1, nb, fd); fclose(fd); }
        }
        free(h);
        hipFree(d_dump);
    }
    float ms_scan = 0, ms_fin = 0, ms_loc = 0;
    HIPCK(hipEventElapsedTime(&ms_scan, c->ev[0], c->ev[1]));
    HIPCK(hipEventElapsedTime(&ms_fin, c->ev[1], c->ev[2]));
    HIPCK(hipEventElapsedTime(&ms_loc, c->ev[2], c->ev[3]));
    if (c->h_g->fail) {
        fprintf(stderr, "clyscan: internal error (code %#x)\n", c->h_g->fail);
        return CLY_ERR_DEVICE;
    }
    uint64_t total = 0;
    for (int i = 0; i < nfiles; i++) {
        const FileInfo& fi = c->h_finfo[i];
        file_first[i] = fi.first_index;
        if (fi.ok) {
            res[i].n_records = fi.end_index - fi.first_index;
            res[i].end_offset = fi.term_pos;
            res[i].status = fi.term_status;
        } else {
            if (fi.fail_key == ~0ull) { fprintf(stderr, "clyscan: internal error (file %d: no failing record)\n", i); return CLY_ERR_DEVICE; }
            res[i].n_records = fi.fail_key & 0xffffffffull;
            res[i].end_offset = (int64_t)(fi.fail_key >> 32);
            res[i].status = CLY_ERR_CRC;
        }
        res[i]._pad = 0;
        total += res[i].n_records;
    }
    if (needed) *needed = c->h_g->total;
    if (stats) {
        stats->scan_ms = ms_scan; stats->resolve_ms = ms_fin + ms_loc; stats->total_ms = ms_scan + ms_fin + ms_loc;
        stats->passes = 1 + (c->h_g->refix ? 1 : 0) + (located ? 1 : 0);
        stats->n_chunks = (uint32_t)(ntiles * CLY_NL); stats->bytes = bytes; stats->records = total;
    }
    if (c->h_g->overflow || c->h_g->total > out_cap) return CLY_ERR_CAPACITY;
    return CLY_OK;
}

// Host-memory entry.  Inputs of at least PIPE_MIN bytes go through a
// pipeline: the files are split into groups of >= PIPE_GROUP bytes (whole
// files); a copy thread moves group g+1 host->device while group g is scanned
// and its tuples travel device->host (PCIe is full duplex), so the H2D stream
// of the file bytes sets the pace.  On CLY_ERR_CAPACITY every group is still
// scanned (nothing copied back) so that *needed is the exact record count.
#define PIPE_MIN (256ull << 20)
#define PIPE_GROUP (512ull << 20)
extern "C" int cly_scan(cly_ctx* c, const cly_file* files, int nfiles, cly_tuple* out, uint64_t out_cap,
                        uint64_t* file_first, cly_file_result* res, uint64_t* needed, cly_stats* stats) {
    if (!c || (!files && nfiles) || nfiles < 0 || !res || !file_first) return CLY_ERR_ARG;
    if (nfiles == 0) { if (needed) *needed = 0; return CLY_OK; }
    HIPCK(hipSetDevice(c->device));
    uint64_t total = 0;
    for (int i = 0; i < nfiles; i++) {
        if (files[i].len >= 0xFFFFFFFFull) return CLY_ERR_ARG;
        total += (files[i].len + 4095) & ~4095ULL;
    }
    if (total + 4096 > c->cap_bytes) {
        hipFree(c->d_bytes);
        c->d_bytes = nullptr; c->cap_bytes = 0;
        HIPCK(hipMalloc(&c->d_bytes, total + 4096));
        c->cap_bytes = total + 4096;
    }
    const uint64_t cap = cly_scan_capacity(files, nfiles) + 16 * (uint64_t)nfiles + 16;
    if (cap > c->cap_tuples) {
        hipFree(c->d_tuples);
        c->d_tuples = nullptr; c->cap_tuples = 0;
        HIPCK(hipMalloc(&c->d_tuples, sizeof(cly_tuple) * cap));
        c->cap_tuples = cap;
    }
    cly_file* df = (cly_file*)malloc(sizeof(cly_file) * nfiles);
    uint64_t* goff = (uint64_t*)malloc(sizeof(uint64_t) * (nfiles + 1));   // device byte offset of each file
    int* gstart = (int*)malloc(sizeof(int) * (nfiles + 1));
    if (!df || !goff || !gstart) { free(df); free(goff); free(gstart); return CLY_ERR_DEVICE; }
    {
        uint64_t off = 0;
        for (int i = 0; i < nfiles; i++) {
            df[i] = files[i];
            df[i].base = c->d_bytes + off;
            goff[i] = off;
            off += (files[i].len + 4095) & ~4095ULL;
        }
        goff[nfiles] = off;
    }
    int ng = 0;
    {
        uint64_t acc = 0;
        gstart[ng++] = 0;
        for (int i = 0; i < nfiles; i++) {
            acc += files[i].len;
            if (total >= PIPE_MIN && acc >= PIPE_GROUP && i + 1 < nfiles) { gstart[ng++] = i + 1; acc = 0; }
        }
        gstart[ng] = nfiles;
    }
    // the copy thread: group after group, each fully on the device before `ready` moves on
    std::atomic<int> ready(0), copy_err(0);
    std::thread copier([&]() {
        if (hipSetDevice(c->device) != hipSuccess) { copy_err = 1; ready = ng; return; }
        for (int g = 0; g < ng; g++) {
            for (int i = gstart[g]; i < gstart[g + 1]; i++)
                if (files[i].len && hipMemcpy(c->d_bytes + goff[i], files[i].base, files[i].len,
                                              hipMemcpyHostToDevice) != hipSuccess) copy_err = 1;
            ready.store(g + 1, std::memory_order_release);
        }
    });
    int rc = CLY_OK;
    uint64_t tbase = 0, o = 0, need = 0;
    bool over = false;
    cly_stats st_acc;
    memset(&st_acc, 0, sizeof(st_acc));
    for (int g = 0; g < ng && (rc == CLY_OK || rc == CLY_ERR_CAPACITY); g++) {
        while (ready.load(std::memory_order_acquire) <= g) std::this_thread::yield();
        if (copy_err) { rc = CLY_ERR_DEVICE; break; }
        const int f0 = gstart[g], nf = gstart[g + 1] - gstart[g];
        const uint64_t gcap = cly_scan_capacity(files + f0, nf) + 16;
        uint64_t slots = 0;
        cly_stats sg;
        const int r = cly_scan_device(c, df + f0, nf, c->d_tuples + tbase, gcap, file_first + f0, res + f0, &slots, &sg,
                                      nullptr);
        if (r == CLY_ERR_CAPACITY) { over = true; need += slots; rc = CLY_ERR_CAPACITY; tbase += gcap; continue; }
        if (r != CLY_OK) { rc = r; break; }
        st_acc.scan_ms += sg.scan_ms; st_acc.resolve_ms += sg.resolve_ms; st_acc.total_ms += sg.total_ms;
        st_acc.passes = st_acc.passes > sg.passes ? st_acc.passes : sg.passes;
        st_acc.n_chunks += sg.n_chunks; st_acc.bytes += sg.bytes; st_acc.records += sg.records;
        // tuples of the group's files back to host memory (per file: the slots may hold
        // tuples past an ErrInvalidCRC), while the next group is still coming in
        for (int i = f0; i < f0 + nf; i++) {
            need += res[i].n_records;
            if (over || need > out_cap) { over = true; rc = CLY_ERR_CAPACITY; continue; }
            if (res[i].n_records &&
                hipMemcpyAsync(out + o, c->d_tuples + tbase + file_first[i], sizeof(cly_tuple) * res[i].n_records,
                               hipMemcpyDeviceToHost, c->stream) != hipSuccess) { rc = CLY_ERR_DEVICE; break; }
            file_first[i] = o;
            o += res[i].n_records;
        }
        tbase += gcap;
    }
    if (rc != CLY_OK && rc != CLY_ERR_CAPACITY) ready.store(ng);
    copier.join();                                // no return before this: the copier must be joined
    if (hipStreamSynchronize(c->stream) != hipSuccess && rc == CLY_OK) rc = CLY_ERR_DEVICE;
    free(df); free(goff); free(gstart);
    if (stats) *stats = st_acc;
    if (needed) *needed = need;
    return rc;
}

// Context accessors for the merge / index entries (clymerge.hip, clyindex.hip); not in the public header.
extern "C" hipStream_t cly_ctx_stream_internal(cly_ctx* c) { return c->stream; }
extern "C" int cly_ctx_device_internal(cly_ctx* c) { return c->device; }
extern "C" void** cly_ctx_merge_slot_internal(cly_ctx* c) { return &c->merge_scratch; }

// Profiling build only: the phase cycle counters of the last call.
extern "C" int cly_dbg_prof(cly_ctx* c, uint64_t* out12) {
    for (int i = 0; i < 12; i++) out12[i] = c->h_g->prof[i];
    return 12;
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
        case CLY_ERR_NOREPAIR: return "internal: chain resolution failed";
        default: return "unknown status";
    }
}

#ifndef CLY_SRC_HASH
#define CLY_SRC_HASH "unknown"
#endif
extern "C" const char* cly_build_info(void) {
    static char buf[200];
    snprintf(buf, sizeof(buf), "clyscan gfx950 lane-chunk CH=%d TILE=%lld LDS=%d src=%s", CLY_CH, (long long)CLY_TILE,
             (int)SCAN_LDS, CLY_SRC_HASH);
    return buf;
}
