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
// One call, all on one stream, no inter-workgroup waiting inside a kernel:
//   k_spec   per tile: each lane finds the first record start of its chunk
//            (SWAR candidate filter, then a walk of header gathers that must
//            leave the chunk at a plausible header) and walks its records to
//            the chunk end; the wave makes the lanes' chains agree under the
//            tile's own guess of its entry; lane chains + the tile's LOCAL out;
//   k_link   per file: the chain state entering every tile (record count,
//            position, the record open at the tile start) from the LOCALs;
//            tiles whose guess the state contradicts are listed;
//   k_refix  (only for listed tiles) re-resolves them from the true entry,
//            then k_link again;
//   k_fbase  tuple index of each file's first record;
//   k_crc    per tile: every lane streams its chunk through a slicing-by-4 CRC
//            register (16-B loads, 128 B per burst) while a walker decodes its
//            records one gather ahead, writes their tuples straight to their
//            output slots and adds one shifted patch per record to the lane's
//            register, so that the register of the whole file ends at zero iff
//            every record's CRC matches; the tile's register is folded in-wave;
//   k_fin    per file: folds the tile registers up to the terminal's and checks
//            that the fold is zero;
//   k_locate (only when a file fails) finds the first bad record exactly.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

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

// Tile LOCAL (from the tile's own speculation), written by k_spec / k_refix:
// l[0]: bit1 the chain ends in the tile | bit2 no chunk of the tile holds a
//       boundary | bit3 first tile of its file | bit4 a record starts in the
//       tile | records << 32
// l[1]: G (the tile's guessed entry: its first boundary) | exit or terminal position << 32
// l[2]: crc_last | P_last << 32 (last record start in the tile and its stored CRC)
// l[3]: the smallest entry that passes the whole tile (tile end, or len + 1 for
//       the tile holding the file's end)
struct TileLocal { u64 l[4]; };
#define DF_PUB 1ull
#define DF_TERM 2ull
#define DF_NONE 4ull
#define DF_FOF 8ull
#define DF_REC 16ull
#define DF_OVF 32ull             // the tile's record starts are not stored (more than POS_CAP)
#define POS_CAP 2048             // stored record starts per tile (u16, tile-relative)

#define LINK_ROUNDS 3            // link rounds launched per call without a host wait (more: host loop)
struct Globals {                 // zeroed per call
    uint32_t nfix[LINK_ROUNDS];  // tiles listed by k_link round r for k_refix round r + 1
    uint32_t overflow;           // tuples beyond out_cap were dropped
    uint32_t fail;               // internal invariant (never expected)
    uint32_t refix;              // tiles re-resolved over all rounds
    uint32_t rounds;             // link rounds
    uint32_t any_fail;           // a file's CRC fold failed (k_locate needed)
    uint64_t total;              // records over all files
};
// ---------------------------------------------------------------------------
// LDS of k_crc / k_locate (static: compile-time offsets)
//   [0, 65536)     CRC slicing-by-4 tables T0..T3, 16 replicas: dword (i*64 + t*16 + r)
//   [65536, +256)  inverse of a zero-byte step (top byte of T0 -> index)
//   LDS_NIB        nibble tables of A^(CLY_CH * 2^k), k < 7 (8 x 16 words each)
//   LDS_SH         nibble tables of A^(v 16^d) (v < 16, d < 4: a byte shift by one hex
//                  digit each), then A^65536 and A^(COAL_BLK - 64)
#define LDS_INV 65536
#define COAL_BLK 4096                    // k_crc's coalesced block (64 lanes x 64 B)
#define LDS_NIB (LDS_INV + 256)
#define NIB_LEVELS 7                     // A^(CLY_CH * 2^k), k < 7 (k = 6: one tile)
#define NSH 66                           // shift tables (the last: A^(COAL_BLK - 64))
#define LDS_SH (LDS_NIB + NIB_LEVELS * 128 * 4)
#define NTAB ((NIB_LEVELS + NSH) * 128)  // words of nibble tables (copied from the context's buffer)
#define SCAN_LDS (LDS_SH + NSH * 128 * 4)

__device__ __forceinline__ void init_tables(CLY_LDS uint8_t* smem, const uint32_t* __restrict__ nib, int ntab = NTAB) {
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
    for (int i = threadIdx.x; i < ntab; i += blockDim.x) ((CLY_LDS uint32_t*)(smem + LDS_NIB))[i] = nib[i];
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
__device__ __forceinline__ void gath_issue_at(gbytes a, Gath& g) {     // a: 4-aligned, 32 readable bytes
    const CLY_GL u32x4u* q = (const CLY_GL u32x4u*)a;
    const u32x4u x = q[0], y = q[1];
    g.w[0] = x.x; g.w[1] = x.y; g.w[2] = x.z; g.w[3] = x.w;
    g.w[4] = y.x; g.w[5] = y.y; g.w[6] = y.z; g.w[7] = y.w;
}
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
__device__ __noinline__ Hdr hdr_slow(gbytes base, uint32_t p, uint64_t len) {
    return step_hdr(base, (int64_t)p, (int64_t)len, (int64_t)p);
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
    return hdr_slow(base, p, len);
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
    uint32_t tb;                 // file offset of the tile's first byte
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
    uint32_t pk[4];              // the first PK_N record starts, tile-relative u16 pairs (k_spec)
};
#define PK_N 8
__device__ __forceinline__ void chain_set(LaneChain& L, int mode) {
    L.mode = mode; L.E = NONE32; L.x = 0; L.term = TERM_NONE; L.cnt = 0; L.last = NONE32; L.last_crc = 0;
    L.prev_crc = 0; L.minsz = 0xFFFFFFFFu;
    L.pk[0] = L.pk[1] = L.pk[2] = L.pk[3] = 0;
}
// record start `rel` (tile-relative) as the chain's record number cnt (constant indices only)
__device__ __forceinline__ void pk_put(LaneChain& L, uint32_t cnt, uint32_t rel) {
    const uint32_t v = (rel & 0xFFFFu) << (16 * (cnt & 1));
    const uint32_t q = cnt >> 1;                 // value selects, not indexed stores
    L.pk[0] = L.pk[0] | (q == 0 ? v : 0u);
    L.pk[1] = L.pk[1] | (q == 1 ? v : 0u);
    L.pk[2] = L.pk[2] | (q == 2 ? v : 0u);
    L.pk[3] = L.pk[3] | (q == 3 ? v : 0u);
}

// Walk from p: exact (ReadLogRecord semantics, every terminal) or speculative
// (every record must be one the writer produces and the chain must leave the
// chunk at a plausible header, or end at io.EOF at len).  Returns false when a
// speculative chain is rejected.
__device__ __forceinline__ bool walk_(const Chunk& K, uint32_t p, bool exact, LaneChain& L) {
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
        pk_put(L, L.cnt, p - K.tb);
        L.cnt++;
        L.prev_crc = L.last_crc;
        L.last = p; L.last_crc = h.crc;
        if ((uint32_t)h.size < L.minsz) L.minsz = (uint32_t)h.size;
        p += (uint32_t)h.size;
    }
}

__device__ __forceinline__ bool walk(const Chunk& K, uint32_t p, bool exact, LaneChain& L) {
    return walk_(K, p, exact, L);
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

// First candidate record start at or after chunk offset `from` (SWAR filter:
// the type and data-type bytes are <= 4), NONE32 if none starts in the chunk.
// The four candidate bits of a word are gathered by one multiply: bits 7, 15,
// 23, 31 times 1 + 2^7 + 2^14 + 2^21 land in bits 28..31.
__device__ __forceinline__ uint32_t first_cand(const Chunk& K, uint32_t from) {
    for (uint32_t b = from / (CLY_BW * 4); b < (uint32_t)CLY_NB; b++) {
        uint32_t w[CLY_BW + 4];
        if ((uint64_t)K.cb + (b + 1) * CLY_BW * 4 + 16 <= K.len) {
            const CLY_GL u32x4* src = (const CLY_GL u32x4*)(K.base + K.cb + b * CLY_BW * 4);
            #pragma unroll
            for (int k = 0; k < CLY_BW / 4 + 1; k++) {
                const u32x4 v = src[k];
                w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
            }
        } else {
            #pragma unroll
            for (int k = 0; k < CLY_BW / 4 + 1; k++) {
                const u32x4 v = piece(K, b * CLY_BW * 4 + 16 * k);
                w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
            }
        }
        uint32_t cmk[CLY_BW / 8];
        #pragma unroll
        for (int k = 0; k < CLY_BW / 8; k++) cmk[k] = 0;
        #pragma unroll
        for (int k = 0; k < CLY_BW; k++) {
            // positions 4k..4k+3: bytes +4 (type) and +5 (data type) <= 4
            const uint32_t L1 = swar_le4(w[k + 1]), L2 = swar_le4(w[k + 2]);
            const uint32_t cm = L1 & __builtin_amdgcn_alignbit(L2, L1, 8);
            cmk[k >> 3] |= ((cm * 0x204081u) >> 28) << (4 * (k & 7));
        }
        const uint32_t base = b * CLY_BW * 4;
        #pragma unroll
        for (int k = 0; k < CLY_BW / 8; k++) {
            const uint32_t lo = base + 32 * k;
            uint32_t m = cmk[k];
            if (from > lo) m = from - lo >= 32 ? 0u : (m & (0xFFFFFFFFu << (from - lo)));
            if (m) {
                const uint32_t q = K.cb + lo + (uint32_t)__builtin_ctz(m);
                return q < K.ce ? q : NONE32;
            }
        }
    }
    return NONE32;
}

// Phase A for one lane: the chain of its chunk under its own guess (the first
// candidate whose speculative walk holds).
__device__ __forceinline__ LaneChain phase_a(const Chunk K) {
    LaneChain L;
    if (!K.on) { chain_set(L, LM_OFF); return L; }
    if (K.cb == 0) { walk(K, 0, true, L); return L; }
    chain_set(L, LM_NONE);
    uint32_t from = 0;
    for (int it = 0; it < CLY_CH; it++) {
        const uint32_t q = first_cand(K, from);
        if (q == NONE32) break;
        LaneChain T;
        if (walk(K, q, false, T)) { L = T; break; }
        from = q + 1 - K.cb;
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
__device__ __forceinline__ LaneChain resolve(const Chunk K, LaneChain L, int lane, uint32_t X0, bool dead0, Globals* g) {
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
// ---------------------------------------------------------------------------
// Chain state between tiles (k_link) and the per-lane chains (k_spec -> k_crc).
struct LBState {
    uint64_t count;              // records before (file-relative in TileIn, absolute in k_crc)
    uint32_t X;                  // chain position
    uint32_t crc_last;           // stored CRC of the last record started before (its successor's Q)
    uint32_t P_last;             // that record's start (NONE32: none in this file)
    int      dead;               // the file's chain has ended
};
// TileIn (k_link): the true state entering a tile, 32 B:
//   w[0..1] count (file-relative), w[2] X, w[3] dead | fix << 1, w[4] crc_last, w[5] P_last
struct TileIn { uint32_t w[8]; };
#define TI_DEAD 1u
#define TI_FIX 2u
__device__ __forceinline__ LBState ti_load(const TileIn* p) {
    const u32x4 a = ((const u32x4*)p)[0], b = ((const u32x4*)p)[1];
    LBState s;
    s.count = ((uint64_t)a.y << 32) | a.x; s.X = a.z; s.dead = (a.w & TI_DEAD) != 0; s.crc_last = b.x; s.P_last = b.y;
    return s;
}
__device__ __forceinline__ void ti_store(TileIn* p, const LBState& s, bool fix) {
    ((u32x4*)p)[0] = (u32x4){(uint32_t)s.count, (uint32_t)(s.count >> 32), s.X, (s.dead ? TI_DEAD : 0u) | (fix ? TI_FIX : 0u)};
    ((u32x4*)p)[1] = (u32x4){s.crc_last, s.P_last, 0u, 0u};
}

// Per-lane chains (structure of arrays over all lanes of the call, nl = 64 * ntiles):
//   lanes[0*nl + i] mode | term << 8 | cnt << 16,  [1] E,  [2] x,  [3] last,  [4] last_crc
#define LANE_WORDS 5
__device__ __forceinline__ void lane_store(uint32_t* lanes, uint64_t nl, uint64_t i, const LaneChain& L) {
    lanes[i] = (uint32_t)(L.mode & 0xff) | ((uint32_t)(L.term & 0xff) << 8) | (L.cnt << 16);
    lanes[nl + i] = L.E;
    lanes[2 * nl + i] = L.x;
    lanes[3 * nl + i] = L.last;
    lanes[4 * nl + i] = L.last_crc;
}
__device__ __forceinline__ LaneChain lane_load(const uint32_t* __restrict__ lanes, uint64_t nl, uint64_t i) {
    LaneChain L;
    const uint32_t m = lanes[i];
    L.mode = (int)(m & 0xff);
    L.term = (int)(int8_t)((m >> 8) & 0xff);
    L.cnt = m >> 16;
    L.E = lanes[nl + i];
    L.x = lanes[2 * nl + i];
    L.last = lanes[3 * nl + i];
    L.last_crc = lanes[4 * nl + i];
    L.prev_crc = 0;
    L.minsz = 0xFFFFFFFFu;
    L.pk[0] = L.pk[1] = L.pk[2] = L.pk[3] = 0;       // not stored: callers re-walk for record starts
    return L;
}

// The tile's LOCAL (its chain under its own entry): flags | records << 32,
// G | X << 32, crc_last | P_last << 32, tend.  Written by k_spec / k_refix.
__device__ __forceinline__ void local_store(TileLocal* d, const LaneChain& L, uint32_t G, bool fof, uint32_t tt,
                                            uint64_t flen, int lane, bool ovf) {
    const u64 bc = __ballot(L.mode == LM_CHAIN), br = __ballot(L.mode == LM_CHAIN && L.cnt > 0);
    const uint32_t c = L.mode == LM_CHAIN ? L.cnt : 0u;
    const uint32_t tile_cnt = shfl_u32(scan_add_incl(c, lane), 63);
    const int lc = bc ? 63 - __clzll((long long)bc) : 0, lr = br ? 63 - __clzll((long long)br) : 0;
    const uint32_t X = shfl_u32(L.x, lc);
    const int term = __shfl(L.term, lc, 64);
    const uint32_t crc = shfl_u32(L.last_crc, lr), Pl = shfl_u32(L.last, lr);
    const u64 bg = __ballot(L.mode == LM_CHAIN);
    const uint32_t Gl = bg ? shfl_u32(L.E, __ffsll((long long)bg) - 1) : NONE32;
    (void)G;
    if (lane == 0) {
        const uint64_t tstart = (uint64_t)tt * CLY_TILE;
        const uint32_t tend = tstart + CLY_TILE >= flen ? (uint32_t)(flen + 1) : (uint32_t)(tstart + CLY_TILE);
        u64 f0 = (u64)tile_cnt << 32;
        if (bc && term != TERM_NONE) f0 |= DF_TERM;
        if (!bc) f0 |= DF_NONE;
        if (fof) f0 |= DF_FOF;
        if (br) f0 |= DF_REC;
        if (ovf) f0 |= DF_OVF;
        d->l[0] = f0;
        d->l[1] = (u64)Gl | ((u64)X << 32);
        d->l[2] = (u64)crc | ((u64)Pl << 32);
        d->l[3] = (u64)tend;
    }
}

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
// ---------------------------------------------------------------------------
// Phase C (k_crc), uniform path.  The lane streams its chunk through the CRC
// register raw, in 128-B bursts: the loop body is the plain slicing-by-4 step.
// Each record start P changes the stream by one combined patch delta' on one
// word w of the chunk (patch_part); XORing delta' into word w changes the
// register at the chunk end by A^(4 (NW - w)) delta', which the walker adds to
// `pacc` (two nibble-table products, shift_words), so the stream itself never
// sees the records.  The walker decodes the lane's records one gather ahead
// and writes their tuples, before the stream.
__device__ __forceinline__ uint32_t mat_mul(const CLY_LDS uint32_t* t, uint32_t v) {
    uint32_t p = 0;
    #pragma unroll
    for (int n = 0; n < 8; n++) p ^= t[n * 16 + ((v >> (4 * n)) & 15u)];
    return p;
}
// A^m v (m bytes), 1 <= m <= 65536: one nibble-table product per hex digit of m
__device__ __forceinline__ uint32_t shift_bytes(const CLY_LDS uint8_t* smem, uint32_t m, uint32_t v) {
    const CLY_LDS uint32_t* t = (const CLY_LDS uint32_t*)(smem + LDS_SH);
    v = mat_mul(t + (m & 15u) * 128, v);
    v = mat_mul(t + (16u + ((m >> 4) & 15u)) * 128, v);
    v = mat_mul(t + (32u + ((m >> 8) & 15u)) * 128, v);
    v = mat_mul(t + (48u + ((m >> 12) & 15u)) * 128, v);
    if (m >> 16) v = mat_mul(t + 64u * 128, v);
    return v;
}
// The record start P (stored CRC c, the record before it stored cq) in the
// file's byte stream, as the CRC register sees it: its stored CRC bytes zeroed
// (XOR c into bytes [P, P+4)), the register checked against the previous
// record's CRC (XOR ~cq into the register before byte P; not at P = 0) and the
// record's own CRC started (XOR 0xFFFFFFFF into the register before byte P+4,
// = XOR K4 = A^-4 0xFFFFFFFF before byte P).  All three are one register XOR
// before byte P, whose effect at the tile end TE is A^(TE-P) applied to it;
// bytes of the patch past TE belong to the next tile, and A^(TE-P) accounts
// for them there exactly (the file fold shifts tile t by one tile more than
// tile t+1).
__device__ __forceinline__ uint32_t rec_patch(const CLY_LDS uint8_t* smem, uint32_t TE, uint32_t P, uint32_t c,
                                              uint32_t cq, uint32_t K4) {
    return shift_bytes(smem, TE - P, c ^ K4 ^ (P != 0 ? ~cq : 0u));
}
__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
    #pragma unroll
    for (int o = 32; o; o >>= 1) v ^= (uint32_t)__shfl_xor((int)v, o, 64);
    return v;
}

struct Walker {
    uint32_t p, cq, i;
    Gath gt;
};
__device__ __forceinline__ void walker_step(const Chunk& K, Walker& W, uint32_t nrec, uint64_t base, uint32_t fid,
                                            gtuples out, uint64_t out_cap, const CLY_LDS uint8_t* smem,
                                            uint32_t K4, uint32_t& pacc, Globals* g) {
    const Hdr h = hdr_at(K.base, W.p, K.len, W.gt);
    put_tuple(out, base + W.i, out_cap, K, W.p, h, fid, g);
    pacc ^= rec_patch(smem, K.tb + (uint32_t)CLY_TILE, W.p, h.crc, W.cq, K4);
    W.cq = h.crc;
    W.p += (uint32_t)h.size;
    W.i++;
    if (W.i < nrec && gath_ok(W.p, K.len)) gath_issue(K.base, W.p, W.gt);
}

// The raw CRC register of the lane's chunk (no patches), 128-B bursts; with
// `walk` (tiles whose record starts were not stored) the lane first walks its
// own records: tuples, and their patches into pacc.
__device__ __forceinline__ uint32_t phase_c_fast(const Chunk& K, const LaneChain& L, const LaneIn& I, bool active,
                                                 bool walk, uint32_t slim, uint32_t fid, gtuples out, uint64_t out_cap,
                                                 const CLY_LDS uint8_t* smem, const CrcLane& cl, uint32_t K4,
                                                 uint32_t& pacc, Globals* g) {
    if (walk) {
        Walker W;
        W.p = L.E; W.cq = I.crc_in; W.i = 0;
        const uint32_t nrec = (active && L.mode == LM_CHAIN) ? L.cnt : 0u;
        if (nrec && gath_ok(W.p, K.len)) gath_issue(K.base, W.p, W.gt);
        for (;;) {
            const bool need = W.i < nrec;
            if (!__ballot(need)) break;
            if (need) walker_step(K, W, nrec, I.base, fid, out, out_cap, smem, K4, pacc, g);
        }
    }
    uint32_t s = 0;
    const CLY_GL u32x4* src = (const CLY_GL u32x4*)(K.base + K.cb);
    // the stream stops at slim (the terminal lane: T) or the file's end
    Chunk Ks = K;
    if ((uint64_t)slim < Ks.len) Ks.len = slim;
    const bool full = (uint64_t)K.cb + CLY_CH <= Ks.len;
    #pragma unroll 1
    for (int b = 0; b < CLY_NB; b++) {
        u32x4 v[CLY_BW / 4];
        if (active && full) {
            #pragma unroll
            for (int k = 0; k < CLY_BW / 4; k++) v[k] = src[b * (CLY_BW / 4) + k];
        } else if (active) {
            #pragma unroll
            for (int k = 0; k < CLY_BW / 4; k++) v[k] = piece(Ks, (uint32_t)(b * CLY_BW * 4 + 16 * k));
        } else {
            #pragma unroll
            for (int k = 0; k < CLY_BW / 4; k++) v[k] = (u32x4){0u, 0u, 0u, 0u};
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
// Boundaries of exact_lane.  A record start P patches bytes [P, P+8) and a
// record is at least 6 bytes (headerSize >= 6 for a decoded record), so at
// most two record starts touch one word: two named slots (the older one drops
// out when a third is pushed) plus one for the terminal; no array, so no
// dynamic indexing and no scratch memory.
__device__ __forceinline__ uint32_t bnd_patch(const Bnd& b, uint32_t A, uint32_t d) {
    uint32_t patch = 0;
    #pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t x = A + i;
        uint32_t m = 0;
        if (!b.term && x >= b.P && x < b.P + 4) m = (d >> (8 * i)) & 0xffu;          // stored CRC zeroed
        if (!b.term && x >= b.P + 4 && x < b.P + 8) m ^= 0xffu;                     // init 0xFF
        patch ^= m << (8 * i);
    }
    if ((b.P >> 2) == (A >> 2)) patch ^= b.q;
    return patch;
}
__device__ __forceinline__ bool bnd_fails(const Bnd& b, uint32_t A, uint32_t s) {
    return (b.P >> 2) == (A >> 2) && b.P != 0 && b.start != NONE32 && s != 0;
}
__device__ __forceinline__ uint32_t exact_lane(const Chunk& K, const LaneChain& L, const LaneIn& I, uint32_t s0, bool emit,
                               bool observe, uint32_t fid, gtuples out, uint64_t out_cap,
                               const CLY_LDS uint8_t* smem, const CrcLane& cl, Globals* g, uint32_t& fail_P,
                               uint64_t& fail_i, uint32_t& expect, const CLY_LDS uint32_t* wl = nullptr) {
    uint32_t s = s0;
    fail_P = NONE32; fail_i = 0; expect = 0;
    Bnd rA, rB, tT;
    bool vA = false, vB = false, vT = false;
    rA.P = rB.P = tT.P = 0; rA.c = rB.c = tT.c = 0; rA.q = rB.q = tT.q = 0; rA.term = rB.term = 0; tT.term = 1;
    rA.start = rB.start = tT.start = NONE32; rA.idx = rB.idx = tT.idx = 0;
    if (I.spill) { rB.P = I.P_in; rB.c = I.crc_in; rB.q = 0; rB.start = NONE32; rB.idx = 0; vB = true; }
    const uint32_t T = (L.mode == LM_CHAIN && L.term != TERM_NONE) ? L.x : NONE32;
    uint32_t wp = L.E, cq = I.crc_in, wi = 0, start = I.P_in;
    uint64_t sidx = I.base - 1;
    const uint32_t nrec = L.mode == LM_CHAIN ? L.cnt : 0u;
    bool tpushed = T == NONE32;
    for (uint32_t w = 0; w < CLY_NW; w++) {
        const uint32_t A = K.cb + 4 * w;
        // the boundaries whose first patch word is this one
        for (;;) {
            if (wi < nrec && (wp >> 2) == (A >> 2)) {
                const Hdr h = hdr_load(K.base, wp, K.len);
                if (emit) put_tuple(out, I.base + wi, out_cap, K, wp, h, fid, g);
                rA = rB; vA = vB;
                rB.P = wp; rB.c = h.crc; rB.q = wp != 0 ? q_of(smem, cq, wp & 3, cl.r4) : 0u;
                rB.start = start; rB.idx = sidx; vB = true;
                start = wp; sidx = I.base + wi;
                cq = h.crc; wp += (uint32_t)h.size; wi++;
                continue;
            }
            if (!tpushed && wi >= nrec && (T >> 2) == (A >> 2)) {
                tT.P = T; tT.q = T != 0 ? q_of(smem, cq, T & 3, cl.r4) : 0u;
                tT.start = start; tT.idx = sidx; vT = true;
                tpushed = true;
                continue;
            }
            break;
        }
        uint32_t d = 0;
        if ((uint64_t)A < K.len) {
            d = wl ? wl[w] : *(const CLY_GL uint32_t*)(K.base + A);
            const uint64_t n = K.len - A;
            if (n < 4) d &= (1u << (8 * n)) - 1u;
        }
        if (T != NONE32 && A + 4 > T) d = A >= T ? 0u : (d & ((1u << (8 * (T - A))) - 1u));
        uint32_t patch = 0;
        if (vA) patch ^= bnd_patch(rA, A, d);
        if (vB) patch ^= bnd_patch(rB, A, d);
        if (vT) patch ^= bnd_patch(tT, A, d);
        s = crc_word(smem, s ^ d ^ patch, cl);
        if (observe && fail_P == NONE32) {
            if (vA && bnd_fails(rA, A, s)) { fail_P = rA.start; fail_i = rA.idx; }
            if (vB && bnd_fails(rB, A, s)) { fail_P = rB.start; fail_i = rB.idx; }
            if (vT && bnd_fails(tT, A, s)) { fail_P = tT.start; fail_i = tT.idx; }
        }
        if (vT && (tT.P >> 2) <= (A >> 2)) vT = false;
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
// ---------------------------------------------------------------------------
// Kernels of one call: k_spec (every tile on its own), k_link + k_fbase (the
// chain state entering every tile), k_refix (tiles whose own entry was wrong;
// then k_link again), k_crc (CRC stream + tuples), k_fin, k_locate.
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
    K.tb = (uint32_t)((uint64_t)tt * CLY_TILE);
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

// The record starts of a lane's final chain into the tile's list (exact walk).
__device__ __forceinline__ void emit_positions(const Chunk& K, const LaneChain& L, uint16_t* pos) {
    if (L.mode != LM_CHAIN) return;
    uint32_t p = L.E;
    for (uint32_t i = 0; i < L.cnt; i++) {
        pos[i] = (uint16_t)(p - K.tb);
        const Hdr h = hdr_load(K.base, p, K.len);
        p += (uint32_t)h.size;
    }
}
// Record starts of the tile, in chain order, into pos[t * POS_CAP ...] (from
// the chain's own packed starts; a lane with more than PK_N records re-walks
// its chain, whose headers are in L2 by now).  Returns
// the overflow flag (more than POS_CAP records in the tile).
__device__ __forceinline__ bool store_positions(const Chunk& K, const LaneChain& L, int lane, uint16_t* tpos,
                                                bool have_pk) {
    const uint32_t c = L.mode == LM_CHAIN ? L.cnt : 0u;
    const uint32_t incl = scan_add_incl(c, lane);
    const uint32_t tot = shfl_u32(incl, 63);
    if (tot > POS_CAP) return true;
    uint16_t* dst = tpos + (incl - c);
    if (have_pk && c <= PK_N) {
        #pragma unroll
        for (uint32_t i = 0; i < PK_N; i++)
            if (i < c) dst[i] = (uint16_t)(L.pk[i >> 1] >> (16 * (i & 1)));
    } else {
        emit_positions(K, L, dst);
    }
    return false;
}

// k_spec: one wave per tile.  Phase A (each lane's chain under its own guess),
// the lanes made to agree under the tile's guess G (0 for a file's first
// tile), the lane chains and the tile's LOCAL written out.
#define SPEC_WAVES 4
__global__ void __launch_bounds__(64 * SPEC_WAVES, 6)   // 6 waves/SIMD (80 VGPRs): C3 k_spec -6 %
k_spec(const DevFile* __restrict__ files, int nfiles, const uint32_t* __restrict__ tprefix, uint32_t ntiles,
       TileLocal* loc, uint32_t* lanes, uint16_t* pos, Globals* g) {
    const uint32_t t = blockIdx.x * SPEC_WAVES + (threadIdx.x >> 6);
    if (t >= ntiles) return;
    const int lane = threadIdx.x & 63;
    const int f = find_file(tprefix, nfiles, t);
    const DevFile F = files[f];
    const uint32_t tt = t - F.first_tile;
    const Chunk K = make_chunk(F, tt, lane);
    const bool fof = tt == 0;
    const LaneChain L0 = phase_a(K);
    LaneChain L = L0;
    // The tile's guess: the first lane's chain, resolved over the tile; if it
    // does not pass through the entry of the first lane whose own chain another
    // lane confirms (its exit is the start of the chain of the lane it lands
    // in, or it ends at the file's end), that entry instead.
    uint32_t G = NONE32, Gc = NONE32;
    {
        const bool isC = L.mode == LM_CHAIN;
        const uint32_t tb = (uint32_t)((uint64_t)tt * CLY_TILE);
        int m = -1;
        if (isC && L.term == TERM_NONE && L.x >= tb && (uint64_t)(L.x - tb) < (uint64_t)CLY_TILE) m = (int)((L.x - tb) / CLY_CH);
        const uint32_t Em = shfl_u32(L.E, m < 0 ? 0 : m);
        const int mm = __shfl(L.mode, m < 0 ? 0 : m, 64);
        const bool conf = isC && (L.term != TERM_NONE || (m > lane && mm == LM_CHAIN && Em == L.x));
        const u64 bc = __ballot(conf), bm = __ballot(isC);
        if (bc) Gc = shfl_u32(L.E, __ffsll((long long)bc) - 1);
        if (bm) G = shfl_u32(L.E, __ffsll((long long)bm) - 1);
    }
    L = resolve(K, L, lane, fof ? 0u : G, false, g);
    if (!fof && Gc != NONE32 && Gc != G) {
        const int m = (int)((Gc - (uint32_t)((uint64_t)tt * CLY_TILE)) / CLY_CH);
        const bool merged = __shfl(L.mode, m, 64) == LM_CHAIN && shfl_u32(L.E, m) == Gc;
        if (!merged) { G = Gc; L = resolve(K, L0, lane, G, false, g); }
    }
    const uint64_t nl = (uint64_t)ntiles * 64;
    lane_store(lanes, nl, (uint64_t)t * 64 + lane, L);
    const bool ovf = store_positions(K, L, lane, pos + (uint64_t)t * POS_CAP, true);
    local_store(&loc[t], L, G, fof, tt, F.len, lane, ovf);
}

// k_link: one workgroup per file: the chain state entering every tile.  A
// tile's LOCAL, trusted, is a function of the state entering it: the first
// tile of a file sets the state whatever it was (FOF); a tile without
// boundaries passes the state on (ID); any other tile, entered live, sets
// position, ended-ness and the last record and adds its records, and leaves a
// dead state dead (CONST).  Each thread composes its run of tiles, a
// Kogge-Stone scan over the threads' functions gives every run its entering
// state, and each thread re-applies its run from there, writing TileIn and
// checking the LOCALs against it: a chain tile entered live at X != G, or a
// tile without boundaries entered live at X < its end, is contradicted; the
// first contradicted tile of the file (the only one whose entry is certain)
// is listed for k_refix.  Round r > 0 runs only if round r-1 listed tiles.
#define LINK_NT 1024
#define RF_ID 0
#define RF_CONST 1
#define RF_FOF 2
struct RunF { uint32_t kind, X, crc, P, dead, rec; uint64_t cnt; };
__device__ __forceinline__ RunF rf_tile(u64 l0, u64 l1, u64 l2) {
    RunF f;
    f.kind = (l0 & DF_FOF) ? RF_FOF : (l0 & DF_NONE) ? RF_ID : RF_CONST;
    f.X = (uint32_t)(l1 >> 32);
    f.dead = (l0 & DF_TERM) != 0;
    f.cnt = l0 >> 32;
    f.rec = (l0 & DF_REC) || (l0 & DF_FOF);
    f.crc = (l0 & DF_REC) ? (uint32_t)l2 : 0u;
    f.P = (l0 & DF_REC) ? (uint32_t)(l2 >> 32) : NONE32;
    return f;
}
// g after f
__device__ __forceinline__ RunF rf_then(const RunF& f, const RunF& g) {
    if (g.kind == RF_FOF || f.kind == RF_ID) return g;
    if (g.kind == RF_ID || f.dead) return f;
    RunF h = f;
    h.X = g.X; h.dead = g.dead; h.cnt = f.cnt + g.cnt;
    if (g.rec) { h.crc = g.crc; h.P = g.P; h.rec = 1; }
    return h;
}
__device__ __forceinline__ LBState rf_apply(const RunF& f, LBState s) {
    if (f.kind == RF_ID || (f.kind == RF_CONST && s.dead)) return s;
    s.count = (f.kind == RF_FOF ? 0 : s.count) + f.cnt;
    s.X = f.X; s.dead = f.dead;
    if (f.rec) { s.crc_last = f.crc; s.P_last = f.P; }
    return s;
}
#define LINK_PER 4               // tiles per thread held in registers (more: re-read)
__global__ void __launch_bounds__(LINK_NT)
k_link(const DevFile* __restrict__ files, const TileLocal* __restrict__ loc, TileIn* tin, uint64_t* ftotal,
       uint32_t* fixlist, Globals* g, int round) {
    if (round > 0 && g->nfix[round - 1] == 0) return;      // nothing changed since the last round
    __shared__ RunF rf[2][LINK_NT];
    __shared__ uint32_t first_bad;
    const int f = blockIdx.x, tid = threadIdx.x;
    const DevFile F = files[f];
    const uint32_t nt = F.ntile, per = (nt + LINK_NT - 1) / LINK_NT;
    const uint32_t lo = tid * per < nt ? tid * per : nt, hi = lo + per < nt ? lo + per : nt;
    const TileLocal* L0 = loc + F.first_tile;
    u64 c0[LINK_PER], c1[LINK_PER], c2[LINK_PER], c3[LINK_PER];
    #pragma unroll
    for (int k = 0; k < LINK_PER; k++) {
        c0[k] = c1[k] = c2[k] = c3[k] = 0;
        if (lo + k < hi) { c0[k] = L0[lo + k].l[0]; c1[k] = L0[lo + k].l[1]; c2[k] = L0[lo + k].l[2]; c3[k] = L0[lo + k].l[3]; }
    }
    RunF my;
    my.kind = RF_ID; my.X = 0; my.crc = 0; my.P = NONE32; my.dead = 0; my.rec = 0; my.cnt = 0;
    #pragma unroll
    for (int k = 0; k < LINK_PER; k++)
        if (lo + k < hi) my = rf_then(my, rf_tile(c0[k], c1[k], c2[k]));
    for (uint32_t u = lo + LINK_PER; u < hi; u++) my = rf_then(my, rf_tile(L0[u].l[0], L0[u].l[1], L0[u].l[2]));
    // inclusive Kogge-Stone scan of the run functions
    int cur = 0;
    rf[0][tid] = my;
    if (tid == 0) first_bad = NONE32;
    __syncthreads();
    for (int d = 1; d < LINK_NT; d <<= 1) {
        RunF v = rf[cur][tid];
        if (tid >= d) v = rf_then(rf[cur][tid - d], v);
        rf[cur ^ 1][tid] = v;
        cur ^= 1;
        __syncthreads();
    }
    LBState s;
    s.count = 0; s.X = 0; s.crc_last = 0; s.P_last = NONE32; s.dead = 0;
    if (tid > 0) s = rf_apply(rf[cur][tid - 1], s);
    if (tid == LINK_NT - 1) {
        LBState s0;
        s0.count = 0; s0.X = 0; s0.crc_last = 0; s0.P_last = NONE32; s0.dead = 0;
        ftotal[f] = rf_apply(rf[cur][tid], s0).count;
    }
    bool stop = false;
    auto visit = [&](uint32_t u, u64 l0, u64 l1, u64 l2, u64 l3) {
        bool bad = false;
        if (l0 & DF_FOF) { s.count = 0; s.X = 0; s.dead = 0; s.crc_last = 0; s.P_last = NONE32; }
        else if (!s.dead) {
            if (l0 & DF_NONE) bad = s.X < (uint32_t)l3;
            else bad = s.X != (uint32_t)l1;
        }
        ti_store(&tin[F.first_tile + u], s, false);
        if (bad) { atomicMin(&first_bad, F.first_tile + u); stop = true; return; }   // the state after it is not known
        s = rf_apply(rf_tile(l0, l1, l2), s);
    };
    #pragma unroll
    for (int k = 0; k < LINK_PER; k++)
        if (!stop && lo + k < hi) visit(lo + k, c0[k], c1[k], c2[k], c3[k]);
    for (uint32_t u = lo + LINK_PER; u < hi && !stop; u++) visit(u, L0[u].l[0], L0[u].l[1], L0[u].l[2], L0[u].l[3]);
    __syncthreads();
    if (tid == 0 && first_bad != NONE32) {
        const uint32_t k = atomicAdd(&g->nfix[round], 1u);
        fixlist[k] = first_bad;
    }
}

// k_fbase: tuple index of every file's first record (exclusive prefix over
// the file totals) and the call's total.
#define FB_NT 1024
__global__ void __launch_bounds__(FB_NT)
k_fbase(int nfiles, const uint64_t* __restrict__ ftotal, FileInfo* finfo, Globals* g, int round) {
    if (round > 0 && g->nfix[round - 1] == 0) return;
    __shared__ uint64_t part[FB_NT];
    __shared__ uint64_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int b = 0; b < nfiles; b += FB_NT) {
        const int i = b + threadIdx.x;
        const uint64_t v = i < nfiles ? ftotal[i] : 0;
        part[threadIdx.x] = v;
        __syncthreads();
        for (int d = 1; d < FB_NT; d <<= 1) {
            const uint64_t o = threadIdx.x >= d ? part[threadIdx.x - d] : 0;
            __syncthreads();
            part[threadIdx.x] += o;
            __syncthreads();
        }
        if (i < nfiles) finfo[i].first_index = carry + part[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == 0) carry += part[FB_NT - 1];
        __syncthreads();
    }
    if (threadIdx.x == 0) g->total = carry;
}

// k_refix: one wave per listed tile: its lanes re-resolved from the entering
// state k_link gave it; new lane chains and LOCAL.  Walks on into the next
// tile of the file while that one's LOCAL disagrees with the new exit (and no
// other wave has it listed).
__global__ void __launch_bounds__(64 * SPEC_WAVES)
k_refix(const DevFile* __restrict__ files, int nfiles, const uint32_t* __restrict__ tprefix, uint32_t ntiles,
        TileLocal* loc, const TileIn* __restrict__ tin, uint32_t* lanes, uint16_t* pos,
        const uint32_t* __restrict__ fixlist, Globals* g, int round) {
    const uint32_t k = blockIdx.x * SPEC_WAVES + (threadIdx.x >> 6);
    if (k >= g->nfix[round - 1]) return;
    const int lane = threadIdx.x & 63;
    uint32_t t = fixlist[k];
    const int f = find_file(tprefix, nfiles, t);
    const DevFile F = files[f];
    LBState S = ti_load(&tin[t]);
    const uint64_t nl = (uint64_t)ntiles * 64;
    for (;;) {
        const uint32_t tt = t - F.first_tile;
        const Chunk K = make_chunk(F, tt, lane);
        LaneChain L = lane_load(lanes, nl, (uint64_t)t * 64 + lane);
        L = resolve(K, L, lane, S.dead ? 0u : S.X, S.dead != 0, g);
        lane_store(lanes, nl, (uint64_t)t * 64 + lane, L);
        // (lanes loaded from the lane arrays carry no packed starts: all re-walked)
        const bool ovf = store_positions(K, L, lane, pos + (uint64_t)t * POS_CAP, false);
        local_store(&loc[t], L, NONE32, tt == 0, tt, F.len, lane, ovf);
        // state after the tile
        const u64 bc = __ballot(L.mode == LM_CHAIN);
        if (bc) {
            const int lc = 63 - __clzll((long long)bc);
            S.X = shfl_u32(L.x, lc);
            S.dead = __shfl(L.term, lc, 64) != TERM_NONE;
        }
        if (S.dead || t + 1 >= F.first_tile + F.ntile) break;
        // the next tile: consistent with the new exit?  else it is re-resolved too
        const u64 n0 = loc[t + 1].l[0], n1 = loc[t + 1].l[1], n3 = loc[t + 1].l[3];
        const bool ok = (n0 & DF_NONE) ? S.X >= (uint32_t)n3 : S.X == (uint32_t)n1;
        if (ok) break;
        t++;
    }
}

// One record round of k_crc: record r = 64 k + lane of the tile (its start
// from the tile's list), header decoded from its gather, tuple written, patch
// added to pacc; cq chains the stored CRCs across lanes and rounds.
__device__ __forceinline__ void round_finish(const Chunk& K, bool act, uint32_t P, const Gath& gt, uint64_t idx,
                                             uint32_t TE, uint32_t fid, gtuples out, uint64_t out_cap,
                                             const CLY_LDS uint8_t* smem, uint32_t K4, uint32_t last, uint32_t& prev,
                                             uint32_t& pacc, Globals* g, int lane) {
    uint32_t c = 0;
    if (act) {
        const Hdr h = hdr_at(K.base, P, K.len, gt);
        put_tuple(out, idx, out_cap, K, P, h, fid, g);
        c = h.crc;
    }
    const uint32_t up = shfl_u32(c, lane > 0 ? lane - 1 : 0);
    const uint32_t cq = lane > 0 ? up : prev;
    if (act) pacc ^= rec_patch(smem, TE, P, c, cq, K4);
    prev = shfl_u32(c, (int)last);
}
// k_crc's tile body: the lane's raw CRC stream (128-B bursts) with the tile's
// record rounds interleaved, one round after every RSTEP-th burst: the round's
// header gathers are issued right after the burst's loads (so waiting for the
// burst never waits for them) and used after the burst's CRC steps, which hide
// their latency; all loads are issued unconditionally (a lane without a record
// reads a zero block) so that the gathers' wait counts stay static.
#define RSTEP (CLY_NB >= 4 ? CLY_NB / 4 : 1)
#define NR_IN (CLY_NB / RSTEP)                     // rounds inside the burst loop
__device__ __forceinline__ uint32_t tile_fused(const Chunk& K, const LaneChain& L, const LaneIn& I, const LBState& S,
                                               bool active, uint32_t slim, const uint16_t* __restrict__ tp,
                                               uint32_t n, uint32_t TE, uint32_t fid, gtuples out, uint64_t out_cap,
                                               const CLY_LDS uint8_t* smem, const CrcLane& cl, uint32_t K4,
                                               uint32_t& pacc, gbytes zero32, Globals* g) {
    const int lane = threadIdx.x & 63;
    const uint32_t nround = (n + 63) / 64;
    uint32_t pr[NR_IN];
    #pragma unroll
    for (int k = 0; k < NR_IN; k++) {
        const uint32_t r = 64u * k + lane;
        pr[k] = tp[r < n ? r : 0];
    }
    uint32_t prev = S.crc_last;
    uint32_t s = 0;
    const CLY_GL u32x4* src = (const CLY_GL u32x4*)(K.base + K.cb);
    Chunk Ks = K;
    if ((uint64_t)slim < Ks.len) Ks.len = slim;
    const bool full = (uint64_t)K.cb + CLY_CH <= Ks.len;
    #pragma unroll
    for (int b = 0; b < CLY_NB; b++) {
        u32x4 v[CLY_BW / 4];
        if (active && full) {
            #pragma unroll
            for (int k = 0; k < CLY_BW / 4; k++) v[k] = src[b * (CLY_BW / 4) + k];
        } else if (active) {
            #pragma unroll
            for (int k = 0; k < CLY_BW / 4; k++) v[k] = piece(Ks, (uint32_t)(b * CLY_BW * 4 + 16 * k));
        } else {
            #pragma unroll
            for (int k = 0; k < CLY_BW / 4; k++) v[k] = (u32x4){0u, 0u, 0u, 0u};
        }
        const int kr = b / RSTEP;
        const bool rb = (b % RSTEP) == 0 && (uint32_t)kr < nround;
        Gath gt;
        uint32_t P = 0;
        bool act = false;
        if (rb) {
            const uint32_t r = 64u * kr + lane;
            act = r < n;
            P = K.tb + pr[kr];
            // every lane loads (a lane without a record, or too close to the file's
            // end for a 32-B gather, reads the context's zero block)
            gath_issue_at(act && gath_ok(P, K.len) ? K.base + (P & ~3u) : zero32, gt);
        }
        #pragma unroll
        for (int k = 0; k < CLY_BW / 4; k++) {
            s = crc_word(smem, s ^ v[k].x, cl);
            s = crc_word(smem, s ^ v[k].y, cl);
            s = crc_word(smem, s ^ v[k].z, cl);
            s = crc_word(smem, s ^ v[k].w, cl);
        }
        if (rb) {
            const uint32_t last = n - 64u * kr - 1 < 63u ? n - 64u * kr - 1 : 63u;
            round_finish(K, act, P, gt, S.count + 64u * kr + lane, TE, fid, out, out_cap, smem, K4, last, prev, pacc,
                         g, lane);
        }
    }
    // rounds past the burst loop
    for (uint32_t kr = NR_IN; kr < nround; kr++) {
        const uint32_t r = 64u * kr + lane;
        const bool act = r < n;
        const uint32_t P = K.tb + tp[act ? r : 0];
        Gath gt;
        gath_issue_at(act && gath_ok(P, K.len) ? K.base + (P & ~3u) : zero32, gt);
        const uint32_t last = n - 64u * kr - 1 < 63u ? n - 64u * kr - 1 : 63u;
        round_finish(K, act, P, gt, S.count + r, TE, fid, out, out_cap, smem, K4, last, prev, pacc, g, lane);
    }
    (void)L; (void)I;
    return s;
}

// k_crc's tile stream, coalesced.  The tile is read in blocks of COAL_BLK =
// 4 KiB: in block m, load k (k < 4) of lane i + 16 q (i < 16, q < 4) reads the
// 16 B at 4096 m + 1024 k + 64 i + 16 q, so that each load instruction reads
// 1 KiB of consecutive bytes (whole cache lines); a 4 x 4 transpose of 16-B
// elements over the lane quarters (v_permlane32_swap, v_permlane16_swap) then
// leaves lane L with the 64 consecutive bytes at 4096 m + 64 L.  Lane L's
// register runs over its 16 segments, stepped by A^(4096 - 64) between them
// (Horner), so A^(4096 - 64 (L + 1)) R_L is its share of the tile's raw
// register at the tile end; bytes at or past `slim` (the chain's terminal T,
// or the file end) read as zero.  Block m+1's loads are issued before block
// m's CRC steps.  The record rounds are interleaved as in tile_fused.
#define COAL_NB ((int)(CLY_TILE / COAL_BLK))
#define COAL_RSTEP (COAL_NB >= 4 ? COAL_NB / 4 : 1)
#define COAL_NR (COAL_NB / COAL_RSTEP)

static_assert(CLY_TILE % COAL_BLK == 0, "tiles of whole 4-KiB blocks");
__device__ __forceinline__ void swap32(uint32_t& a, uint32_t& b) {
    const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    a = r[0]; b = r[1];
}
__device__ __forceinline__ void swap16(uint32_t& a, uint32_t& b) {
    const auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    a = r[0]; b = r[1];
}
// e[k] of lane quarter q -> e[j] of quarter q = what quarter j held in e[q]
__device__ __forceinline__ void quad_transpose(u32x4* e) {
    #pragma unroll
    for (int c = 0; c < 4; c++) {
        uint32_t a0 = e[0][c], a1 = e[1][c], a2 = e[2][c], a3 = e[3][c];
        swap32(a0, a2); swap32(a1, a3);
        swap16(a0, a1); swap16(a2, a3);
        e[0][c] = a0; e[1][c] = a1; e[2][c] = a2; e[3][c] = a3;
    }
}
__device__ __forceinline__ uint32_t tile_coal(const Chunk& K, const LBState& S, uint32_t slim,
                                              const uint16_t* __restrict__ tp, uint32_t n, uint32_t TE, uint32_t fid,
                                              gtuples out, uint64_t out_cap, const CLY_LDS uint8_t* smem,
                                              const CrcLane& cl, uint32_t K4, uint32_t& pacc, gbytes zero32,
                                              Globals* g) {
    const int lane = threadIdx.x & 63;
    const uint32_t nround = (n + 63) / 64;
    uint32_t pr[COAL_NR];
    #pragma unroll
    for (int k = 0; k < COAL_NR; k++) {
        const uint32_t r = 64u * k + lane;
        pr[k] = tp[r < n ? r : 0];
    }
    uint32_t prev = S.crc_last;
    Chunk Kt = K;                                    // the tile as one chunk: piece() offsets are tile-relative
    Kt.cb = K.tb;
    if ((uint64_t)slim < Kt.len) Kt.len = slim;
    const bool full = (uint64_t)K.tb + CLY_TILE <= Kt.len;
    const uint32_t lo = 64u * (uint32_t)(lane & 15) + 16u * (uint32_t)(lane >> 4);
    const CLY_GL u32x4* src = (const CLY_GL u32x4*)(K.base + K.tb + lo);
    const CLY_LDS uint32_t* tblk = (const CLY_LDS uint32_t*)(smem + LDS_SH) + (NSH - 1) * 128;
    uint32_t R = 0;
    u32x4 eb[2][4];
    auto blk_load = [&](u32x4* e, int m) {
        if (full) {
            #pragma unroll
            for (int k = 0; k < 4; k++) e[k] = src[(COAL_BLK * m + 1024 * k) / 16];
        } else {
            #pragma unroll
            for (int k = 0; k < 4; k++) e[k] = piece(Kt, (uint32_t)(COAL_BLK * m + 1024 * k) + lo);
        }
    };
    blk_load(eb[0], 0);
    #pragma unroll
    for (int m = 0; m < COAL_NB; m++) {
        u32x4* e = eb[m & 1];
        const int kr = m / COAL_RSTEP;
        const bool rb = (m % COAL_RSTEP) == 0 && (uint32_t)kr < nround;
        Gath gt;
        uint32_t P = 0;
        bool act = false;
        if (rb) {
            const uint32_t r = 64u * kr + lane;
            act = r < n;
            P = K.tb + pr[kr];
            gath_issue_at(act && gath_ok(P, K.len) ? K.base + (P & ~3u) : zero32, gt);
        }
        if (m + 1 < COAL_NB) blk_load(eb[(m + 1) & 1], m + 1);
        quad_transpose(e);
        if (m) R = mat_mul(tblk, R);
        #pragma unroll
        for (int k = 0; k < 4; k++) {
            R = crc_word(smem, R ^ e[k].x, cl);
            R = crc_word(smem, R ^ e[k].y, cl);
            R = crc_word(smem, R ^ e[k].z, cl);
            R = crc_word(smem, R ^ e[k].w, cl);
        }
        if (rb) {
            const uint32_t last = n - 64u * kr - 1 < 63u ? n - 64u * kr - 1 : 63u;
            round_finish(K, act, P, gt, S.count + 64u * kr + lane, TE, fid, out, out_cap, smem, K4, last, prev, pacc,
                         g, lane);
        }
    }
    for (uint32_t kr = COAL_NR; kr < nround; kr++) {
        const uint32_t r = 64u * kr + lane;
        const bool act = r < n;
        const uint32_t P = K.tb + tp[act ? r : 0];
        Gath gt;
        gath_issue_at(act && gath_ok(P, K.len) ? K.base + (P & ~3u) : zero32, gt);
        const uint32_t last = n - 64u * kr - 1 < 63u ? n - 64u * kr - 1 : 63u;
        round_finish(K, act, P, gt, S.count + r, TE, fid, out, out_cap, smem, K4, last, prev, pacc, g, lane);
    }
    return shift_bytes(smem, COAL_BLK - 64u * (uint32_t)(lane + 1), R);
}

// k_crc: the CRC stream and the tuples, tiles in grid-stride order.
#define CRC_WAVES 16
__global__ void __launch_bounds__(64 * CRC_WAVES)
k_crc(const DevFile* __restrict__ files, int nfiles, const uint32_t* __restrict__ tprefix, uint32_t ntiles,
      const TileIn* __restrict__ tin, const TileLocal* __restrict__ loc, const uint32_t* __restrict__ lanes,
      const uint16_t* __restrict__ pos, uint32_t* treg, FileInfo* finfo, const uint32_t* __restrict__ tabs,
      cly_tuple* out_, uint64_t out_cap, Globals* g, int round, const uint8_t* __restrict__ zero32) {
    if (g->nfix[round]) return;             // the chain is not final yet (k_refix first)
    gtuples out = (gtuples)out_;
    __shared__ __attribute__((aligned(16))) unsigned char smem_raw[SCAN_LDS];
    CLY_LDS uint8_t* smem = (CLY_LDS uint8_t*)smem_raw;
    init_tables(smem, tabs);
    const int lane = threadIdx.x & 63;
    const CrcLane cl = crc_lane(lane);
    uint32_t K4 = 0xFFFFFFFFu;              // A^-4 0xFFFFFFFF
    for (int k = 0; k < 4; k++) K4 = crc_unbyte(smem, K4, cl.r4);
    const uint64_t nl = (uint64_t)ntiles * 64;
    for (uint32_t t = blockIdx.x * CRC_WAVES + (threadIdx.x >> 6); t < ntiles; t += gridDim.x * CRC_WAVES) {
        const int f = find_file(tprefix, nfiles, t);
        const DevFile F = files[f];
        LBState S = ti_load(&tin[t]);
        if (S.dead) { if (lane == 0) treg[t] = 0; continue; }
        S.count += finfo[f].first_index;
        const uint32_t tt = t - F.first_tile;
        const Chunk K = make_chunk(F, tt, lane);
        const LaneChain L = lane_load(lanes, nl, (uint64_t)t * 64 + lane);
        const bool ovf = (loc[t].l[0] & DF_OVF) != 0;
        uint32_t tile_cnt;
        const LaneIn I = lane_inputs(K, L, S, lane, tile_cnt);
        const bool term_lane = L.mode == LM_CHAIN && L.term != TERM_NONE;
        const bool live = L.mode == LM_CHAIN || L.mode == LM_NONE;
        const uint32_t TE = K.tb + (uint32_t)CLY_TILE;
        uint32_t pacc = 0;
        if (term_lane) {
            // the chain's terminal T: the last record is checked there (XOR ~its CRC
            // into the register before byte T; none when no record precedes T), and
            // the stream stops at T (the bytes from T on are zeroed)
            const uint32_t cT = L.cnt ? L.last_crc : I.crc_in;
            if (L.cnt || I.P_in != NONE32) pacc = shift_bytes(smem, TE - L.x, ~cT);
        }
        uint32_t r;
        if (!ovf) {
            // the tile's stream stops at the chain's terminal (if in this tile)
            const uint64_t tm = __ballot(term_lane);
            const uint32_t slim = tm ? (uint32_t)__shfl((int)L.x, __builtin_ctzll(tm), 64) : 0xFFFFFFFFu;
            r = tile_coal(K, S, slim, pos + (uint64_t)t * POS_CAP, tile_cnt, TE, F.fid, out, out_cap, smem, cl, K4,
                          pacc, (gbytes)zero32, g);
        } else r = phase_c_fast(K, L, I, live, true, term_lane ? L.x : 0xFFFFFFFFu, F.fid, out, out_cap, smem, cl, K4,
                                pacc, g);
        if (term_lane) {
            FileInfo* fo = &finfo[f];
            fo->term_pos = L.x; fo->term_status = L.term; fo->term_tile = t; fo->term_lane = (uint32_t)lane;
            fo->end_index = I.base + L.cnt; fo->has_term = 1; fo->expect = 0;
        }
        if (!ovf) r = wave_xor(r ^ pacc);               // lane shares already shifted to the tile end
        else {
            if (!live) r = 0;
            r = tile_fold(smem, r, lane) ^ wave_xor(pacc);
        }
        if (lane == 0) treg[t] = r;
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
      const uint32_t* __restrict__ nib, const uint32_t* __restrict__ pw, Globals* g, int round) {
    __shared__ uint32_t tab[NIB_LEVELS * 128];
    __shared__ uint32_t part[FIN_NT];
    __shared__ uint32_t plen[FIN_NT];
    if (g->nfix[round]) return;             // k_crc did not run (link repair first)
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
// ---------------------------------------------------------------------------
// k_locate (only after a failed fold): every tile of a failing file up to its
// terminal takes its final lane chains, the register entering each chunk, and
// walks its records' checks from there; the first failing record of the file
// wins (atomicMin on offset << 32 | index).
__global__ void __launch_bounds__(512, 2)
k_locate(const DevFile* __restrict__ files, int nfiles, const uint32_t* __restrict__ tprefix, uint32_t ntiles,
         const TileIn* __restrict__ tin, const uint32_t* __restrict__ lanes, const uint32_t* __restrict__ treg,
         FileInfo* finfo, const uint32_t* __restrict__ tabs, Globals* g) {
    __shared__ __attribute__((aligned(16))) unsigned char smem_raw[SCAN_LDS];
    CLY_LDS uint8_t* smem = (CLY_LDS uint8_t*)smem_raw;
    init_tables(smem, tabs);
    const int lane = threadIdx.x & 63;
    const CrcLane cl = crc_lane(lane);
    const uint64_t nl = (uint64_t)ntiles * 64;
    for (uint32_t t = blockIdx.x * 8 + (threadIdx.x >> 6); t < ntiles; t += gridDim.x * 8) {
        const int f = find_file(tprefix, nfiles, t);
        const DevFile F = files[f];
        FileInfo* fo = &finfo[f];
        if (fo->ok || t > fo->term_tile) continue;
        LBState S = ti_load(&tin[t]);
        if (S.dead) continue;
        S.count += fo->first_index;
        const uint32_t tt = t - F.first_tile;
        const Chunk K = make_chunk(F, tt, lane);
        const LaneChain L = lane_load(lanes, nl, (uint64_t)t * 64 + lane);
        uint32_t tile_cnt;
        LaneIn I = lane_inputs(K, L, S, lane, tile_cnt);
        if (lane == 0) I.spill = false;     // a record of the previous tile: in treg[t - 1] (rec_patch)
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
    hipEvent_t ev[8];
    DevFile* d_files; uint32_t* d_tprefix; FileInfo* d_finfo; uint64_t* d_ftotal; int cap_files;
    DevFile* h_files; uint32_t* h_tprefix; FileInfo* h_finfo;
    TileLocal* d_loc; TileIn* d_tin; uint32_t* d_treg; uint32_t* d_fix; uint32_t* d_lanes; uint16_t* d_pos;
    int64_t cap_tiles;
    Globals* d_g; Globals* h_g;
    uint32_t* d_tabs;            // nibble tables: A^(CLY_CH 2^k), k < NIB_LEVELS; A^(4 m), m < 16; A^(64 m)
    uint32_t* d_pw;              // x^(8 CLY_TILE 2^k) mod P, k < 40
    uint8_t* d_zero;             // CLY_CH (>= 256) zero bytes: streams and gathers of lanes without data
    int crc_grid, loc_grid;
    float kms[6];                // last call: k_spec, link rounds (k_link/k_fbase/k_refix), k_crc, k_fin, k_locate, all
    uint8_t* d_bytes; uint64_t cap_bytes;          // host-path staging
    cly_tuple* d_tuples; uint64_t cap_tuples;
    void* merge_scratch;         // clymerge.hip's buffers (grow-only)
    int64_t now_ns;              // loadIndex's time.Now() for the TTL sweep (0: the wall clock per call)
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
    for (int i = 0; i < 8; i++) HIPCK(hipEventCreate(&c->ev[i]));
    HIPCK(hipMalloc(&c->d_g, sizeof(Globals)));
    HIPCK(hipHostMalloc(&c->h_g, sizeof(Globals), hipHostMallocDefault));
    HIPCK(hipMalloc(&c->d_zero, CLY_CH < 256 ? 256 : CLY_CH));
    HIPCK(hipMemset(c->d_zero, 0, CLY_CH < 256 ? 256 : CLY_CH));
    {
        static uint32_t hn[NTAB];
        for (int lvl = 0; lvl < NIB_LEVELS + NSH; lvl++) {
            uint64_t nbytes;
            if (lvl < NIB_LEVELS) nbytes = (uint64_t)CLY_CH << lvl;                  // A^(CLY_CH 2^lvl)
            else if (lvl < NIB_LEVELS + 64) {                                        // A^(v 16^d)
                const int k = lvl - NIB_LEVELS;
                nbytes = (uint64_t)(k & 15) << (4 * (k >> 4));
            } else if (lvl == NIB_LEVELS + 64) nbytes = 65536;                      // A^65536
            else nbytes = COAL_BLK - 64;                                             // k_crc's block step
            const uint32_t xm = cly_x8n(nbytes);
            for (int nb = 0; nb < 8; nb++)
                for (uint32_t v = 0; v < 16; v++) hn[lvl * 128 + nb * 16 + v] = cly_multmodp(xm, v << (4 * nb));
        }
        HIPCK(hipMalloc(&c->d_tabs, sizeof(hn)));
        HIPCK(hipMemcpy(c->d_tabs, hn, sizeof(hn), hipMemcpyHostToDevice));
        uint32_t hp[40];
        hp[0] = cly_x8n((uint64_t)CLY_TILE);
        for (int k = 1; k < 40; k++) hp[k] = cly_multmodp(hp[k - 1], hp[k - 1]);
        HIPCK(hipMalloc(&c->d_pw, sizeof(hp)));
        HIPCK(hipMemcpy(c->d_pw, hp, sizeof(hp), hipMemcpyHostToDevice));
    }
    {
        int ncu = 0;
        HIPCK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device));
        int per_cu = 0;
        HIPCK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_crc, 64 * CRC_WAVES, 0));
        if (per_cu < 1) per_cu = 1;
        c->crc_grid = per_cu * ncu;
        c->loc_grid = ncu * 2;
    }
    *out = c;
    return CLY_OK;
}

extern "C" void cly_ctx_destroy(cly_ctx* c) {
    if (!c) return;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    hipFree(c->d_files); hipFree(c->d_tprefix); hipFree(c->d_finfo); hipFree(c->d_ftotal);
    hipFree(c->d_loc); hipFree(c->d_tin); hipFree(c->d_treg); hipFree(c->d_fix); hipFree(c->d_lanes);
    hipFree(c->d_pos); hipFree(c->d_g); hipFree(c->d_zero); hipFree(c->d_tabs); hipFree(c->d_pw); hipFree(c->d_bytes); hipFree(c->d_tuples);
    hipHostFree(c->h_files); hipHostFree(c->h_tprefix); hipHostFree(c->h_finfo); hipHostFree(c->h_g);
    cly_merge_scratch_free(c->merge_scratch);
    for (int i = 0; i < 8; i++) hipEventDestroy(c->ev[i]);
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
    hipFree(c->d_files); hipFree(c->d_tprefix); hipFree(c->d_finfo); hipFree(c->d_ftotal);
    hipHostFree(c->h_files); hipHostFree(c->h_tprefix); hipHostFree(c->h_finfo);
    c->d_files = nullptr; c->d_tprefix = nullptr; c->d_finfo = nullptr; c->d_ftotal = nullptr;
    c->h_files = nullptr; c->h_tprefix = nullptr; c->h_finfo = nullptr;
    c->cap_files = 0;
    const int cap = nfiles < 64 ? 64 : nfiles;
    HIPCK(hipMalloc(&c->d_files, sizeof(DevFile) * cap));
    HIPCK(hipMalloc(&c->d_tprefix, sizeof(uint32_t) * (cap + 1)));
    HIPCK(hipMalloc(&c->d_finfo, sizeof(FileInfo) * cap));
    HIPCK(hipMalloc(&c->d_ftotal, sizeof(uint64_t) * cap));
    HIPCK(hipHostMalloc(&c->h_files, sizeof(DevFile) * cap, hipHostMallocDefault));
    HIPCK(hipHostMalloc(&c->h_tprefix, sizeof(uint32_t) * (cap + 1), hipHostMallocDefault));
    HIPCK(hipHostMalloc(&c->h_finfo, sizeof(FileInfo) * cap, hipHostMallocDefault));
    c->cap_files = cap;
    return CLY_OK;
}

static int ensure_tiles(cly_ctx* c, int64_t ntiles) {
    if (ntiles <= c->cap_tiles) return CLY_OK;
    hipFree(c->d_loc); hipFree(c->d_tin); hipFree(c->d_treg); hipFree(c->d_fix); hipFree(c->d_lanes); hipFree(c->d_pos);
    c->d_loc = nullptr; c->d_tin = nullptr; c->d_treg = nullptr; c->d_fix = nullptr; c->d_lanes = nullptr;
    c->d_pos = nullptr;
    c->cap_tiles = 0;
    const int64_t cap = ntiles < 1024 ? 1024 : ntiles;
    HIPCK(hipMalloc(&c->d_loc, sizeof(TileLocal) * cap));
    HIPCK(hipMalloc(&c->d_tin, sizeof(TileIn) * cap));
    HIPCK(hipMalloc(&c->d_treg, sizeof(uint32_t) * cap));
    HIPCK(hipMalloc(&c->d_fix, sizeof(uint32_t) * cap));
    HIPCK(hipMalloc(&c->d_lanes, sizeof(uint32_t) * LANE_WORDS * 64 * cap));
    HIPCK(hipMalloc(&c->d_pos, sizeof(uint16_t) * POS_CAP * cap));
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
    HIPCK(hipMemsetAsync(c->d_finfo, 0, sizeof(FileInfo) * nfiles, st));
    HIPCK(hipMemsetAsync(c->d_g, 0, sizeof(Globals), st));
    const uint32_t nt32 = (uint32_t)ntiles;
    const int spec_grid = (int)((ntiles + SPEC_WAVES - 1) / SPEC_WAVES);
    HIPCK(hipEventRecord(c->ev[0], st));
    hipLaunchKernelGGL(k_spec, dim3(spec_grid), dim3(64 * SPEC_WAVES), 0, st, c->d_files, nfiles, c->d_tprefix, nt32,
                       c->d_loc, c->d_lanes, c->d_pos, c->d_g);
    HIPCK(hipGetLastError());
    HIPCK(hipEventRecord(c->ev[1], st));
    // LINK_ROUNDS link rounds (round r > 0: k_refix of round r-1's listed tiles,
    // then k_link; both return at once when round r-1 listed none), then the
    // CRC kernels, which return at once if the last round still listed tiles;
    // no host wait in between.  Files that need more rounds continue on a host
    // loop (one wait per round).
    const int RL = LINK_ROUNDS - 1;
    const int fix_grid = (nfiles + SPEC_WAVES - 1) / SPEC_WAVES;   // at most one listed tile per file and round
    for (int r = 0; r < LINK_ROUNDS; r++) {
        if (r > 0)
            hipLaunchKernelGGL(k_refix, dim3(fix_grid), dim3(64 * SPEC_WAVES), 0, st, c->d_files, nfiles, c->d_tprefix, nt32,
                               c->d_loc, c->d_tin, c->d_lanes, c->d_pos, c->d_fix, c->d_g, r);
        hipLaunchKernelGGL(k_link, dim3(nfiles), dim3(LINK_NT), 0, st, c->d_files, c->d_loc, c->d_tin, c->d_ftotal,
                           c->d_fix, c->d_g, r);
        hipLaunchKernelGGL(k_fbase, dim3(1), dim3(FB_NT), 0, st, nfiles, c->d_ftotal, c->d_finfo, c->d_g, r);
    }
    HIPCK(hipGetLastError());
    HIPCK(hipEventRecord(c->ev[2], st));
    auto launch_crc = [&]() -> int {
        int grid = c->crc_grid;
        if ((int64_t)grid * CRC_WAVES > ntiles) grid = (int)((ntiles + CRC_WAVES - 1) / CRC_WAVES);
        hipLaunchKernelGGL(k_crc, dim3(grid), dim3(64 * CRC_WAVES), 0, st, c->d_files, nfiles, c->d_tprefix, nt32,
                           c->d_tin, c->d_loc, c->d_lanes, c->d_pos, c->d_treg, c->d_finfo, c->d_tabs, d_out, out_cap,
                           c->d_g, RL, c->d_zero);
        HIPCK(hipGetLastError());
        HIPCK(hipEventRecord(c->ev[3], st));
        hipLaunchKernelGGL(k_fin, dim3(nfiles), dim3(FIN_NT), 0, st, c->d_files, c->d_finfo, c->d_treg, c->d_tabs,
                           c->d_pw, c->d_g, RL);
        HIPCK(hipGetLastError());
        HIPCK(hipEventRecord(c->ev[4], st));
        HIPCK(hipMemcpyAsync(c->h_g, c->d_g, sizeof(Globals), hipMemcpyDeviceToHost, st));
        HIPCK(hipStreamSynchronize(st));
        return CLY_OK;
    };
    int rc2 = launch_crc();
    if (rc2) return rc2;
    float ms_fix = 0;
    uint32_t rounds = 1, refixed = 0;
    for (int r = 0; r < LINK_ROUNDS; r++) if (c->h_g->nfix[r]) { rounds++; refixed += c->h_g->nfix[r]; }
    if (c->h_g->nfix[RL]) {
        // more repair rounds on the host: round RL's list, k_link again into slot RL
        HIPCK(hipEventRecord(c->ev[5], st));
        while (c->h_g->nfix[RL]) {
            if (c->h_g->fail) break;
            if (rounds > 4096) { fprintf(stderr, "clyscan: chain repair did not converge\n"); return CLY_ERR_NOREPAIR; }
            // k_refix reads slot RL - 1: move the count there, clear slot RL
            const uint32_t nfix = c->h_g->nfix[RL];
            refixed += nfix;
            HIPCK(hipMemcpyAsync(&c->d_g->nfix[RL - 1], &c->d_g->nfix[RL], sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
            HIPCK(hipMemsetAsync(&c->d_g->nfix[RL], 0, sizeof(uint32_t), st));
            hipLaunchKernelGGL(k_refix, dim3(fix_grid), dim3(64 * SPEC_WAVES), 0, st, c->d_files, nfiles, c->d_tprefix, nt32,
                               c->d_loc, c->d_tin, c->d_lanes, c->d_pos, c->d_fix, c->d_g, RL);
            hipLaunchKernelGGL(k_link, dim3(nfiles), dim3(LINK_NT), 0, st, c->d_files, c->d_loc, c->d_tin, c->d_ftotal,
                               c->d_fix, c->d_g, RL);
            hipLaunchKernelGGL(k_fbase, dim3(1), dim3(FB_NT), 0, st, nfiles, c->d_ftotal, c->d_finfo, c->d_g, RL);
            HIPCK(hipGetLastError());
            HIPCK(hipMemcpyAsync(c->h_g, c->d_g, sizeof(Globals), hipMemcpyDeviceToHost, st));
            HIPCK(hipStreamSynchronize(st));
            rounds++;
        }
        HIPCK(hipEventRecord(c->ev[6], st));
        HIPCK(hipEventSynchronize(c->ev[6]));
        HIPCK(hipEventElapsedTime(&ms_fix, c->ev[5], c->ev[6]));
        if (!c->h_g->fail) {
            HIPCK(hipEventRecord(c->ev[2], st));
            rc2 = launch_crc();
            if (rc2) return rc2;
        }
    }
    bool located = false;
    if (c->h_g->any_fail && !c->h_g->fail) {
        HIPCK(hipMemcpyAsync(c->h_finfo, c->d_finfo, sizeof(FileInfo) * nfiles, hipMemcpyDeviceToHost, st));
        HIPCK(hipStreamSynchronize(st));
        hipLaunchKernelGGL(k_locate, dim3(c->loc_grid), dim3(512), 0, st, c->d_files, nfiles, c->d_tprefix, nt32,
                           c->d_tin, c->d_lanes, c->d_treg, c->d_finfo, c->d_tabs, c->d_g);
        HIPCK(hipGetLastError());
        located = true;
    }
    HIPCK(hipEventRecord(c->ev[7], st));
    HIPCK(hipMemcpyAsync(c->h_finfo, c->d_finfo, sizeof(FileInfo) * nfiles, hipMemcpyDeviceToHost, st));
    HIPCK(hipMemcpyAsync(c->h_g, c->d_g, sizeof(Globals), hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    float ms_spec = 0, ms_link = 0, ms_crc = 0, ms_fin = 0, ms_loc = 0;
    HIPCK(hipEventElapsedTime(&ms_spec, c->ev[0], c->ev[1]));
    HIPCK(hipEventElapsedTime(&ms_link, c->ev[1], c->ev[2]));
    HIPCK(hipEventElapsedTime(&ms_crc, c->ev[2], c->ev[3]));
    HIPCK(hipEventElapsedTime(&ms_fin, c->ev[3], c->ev[4]));
    HIPCK(hipEventElapsedTime(&ms_loc, c->ev[4], c->ev[7]));
    if (ms_fix > 0) ms_link = 0;   // ev[2] was re-recorded after the host repair loop
    c->h_g->refix = refixed;
    c->kms[0] = ms_spec; c->kms[1] = ms_link + ms_fix; c->kms[2] = ms_crc; c->kms[3] = ms_fin; c->kms[4] = ms_loc;
    c->kms[5] = ms_spec + ms_link + ms_fix + ms_crc + ms_fin + ms_loc;
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
        stats->scan_ms = ms_spec + ms_crc; stats->resolve_ms = ms_link + ms_fix + ms_fin + ms_loc;
        stats->total_ms = c->kms[5];
        stats->passes = rounds + (located ? 1 : 0);
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
        cly_tuple* gout = c->d_tuples + tbase;
        cly_tuple* big = nullptr;            // a group of exotic (< 9 B) records: its own buffer
        int r = cly_scan_device(c, df + f0, nf, gout, gcap, file_first + f0, res + f0, &slots, &sg, nullptr);
        if (r == CLY_ERR_CAPACITY && slots > gcap) {
            if (hipStreamSynchronize(c->stream) != hipSuccess || hipMalloc(&big, sizeof(cly_tuple) * (slots + 16)) != hipSuccess) {
                rc = CLY_ERR_DEVICE; break;
            }
            gout = big;
            r = cly_scan_device(c, df + f0, nf, gout, slots + 16, file_first + f0, res + f0, &slots, &sg, nullptr);
        }
        if (r != CLY_OK) { hipFree(big); rc = r; break; }
        st_acc.scan_ms += sg.scan_ms; st_acc.resolve_ms += sg.resolve_ms; st_acc.total_ms += sg.total_ms;
        st_acc.passes = st_acc.passes > sg.passes ? st_acc.passes : sg.passes;
        st_acc.n_chunks += sg.n_chunks; st_acc.bytes += sg.bytes; st_acc.records += sg.records;
        // tuples of the group's files back to host memory (per file: the slots may hold
        // tuples past an ErrInvalidCRC), while the next group is still coming in
        for (int i = f0; i < f0 + nf; i++) {
            need += res[i].n_records;
            if (over || need > out_cap) { over = true; rc = CLY_ERR_CAPACITY; continue; }
            if (res[i].n_records &&
                hipMemcpyAsync(out + o, gout + file_first[i], sizeof(cly_tuple) * res[i].n_records,
                               hipMemcpyDeviceToHost, c->stream) != hipSuccess) { rc = CLY_ERR_DEVICE; break; }
            file_first[i] = o;
            o += res[i].n_records;
        }
        if (big) { if (hipStreamSynchronize(c->stream) != hipSuccess) rc = CLY_ERR_DEVICE; hipFree(big); }
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
extern "C" int64_t cly_ctx_now_internal(cly_ctx* c) {
    if (c->now_ns) return c->now_ns;
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    return (int64_t)ts.tv_sec * 1000000000ll + ts.tv_nsec;
}
extern "C" void cly_ctx_set_clock(cly_ctx* c, int64_t now_ns) { if (c) c->now_ns = now_ns; }
extern "C" int cly_ctx_device_internal(cly_ctx* c) { return c->device; }
extern "C" void** cly_ctx_merge_slot_internal(cly_ctx* c) { return &c->merge_scratch; }

// Per-kernel times of the last cly_scan_device call (ms): k_spec, link rounds
// (k_link + k_fbase + repair), k_crc, k_fin, k_locate, all.  Not in the public header.
extern "C" int cly_dbg_kernel_ms(cly_ctx* c, double* out6) {
    for (int i = 0; i < 6; i++) out6[i] = c->kms[i];
    return 6;
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
    snprintf(buf, sizeof(buf), "clyscan gfx950 spec/link/crc CH=%d TILE=%lld LDS=%d src=%s", CLY_CH, (long long)CLY_TILE,
             (int)SCAN_LDS, CLY_SRC_HASH);
    return buf;
}
