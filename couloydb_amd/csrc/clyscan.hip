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
// Layout: a file is cut into tiles of CLY_NBLK blocks of
// 4 KiB; one wave streams a tile block by block; in a block, lane L owns the
// 64-B segment at 64 L.
//
// One call, all on one stream, no inter-workgroup waiting inside a kernel:
//   k_scan   per tile, ONE read of its bytes: each block arrives by four
//            coalesced 1-KiB loads (transposed over the lane quarters); the
//            lanes find the record starts of their segments (SWAR candidate
//            filter, header gathers from the wave's LDS copy of the block, an
//            in-wave agreement pass), XOR each record's CRC patch into the
//            copy, and run their 64-B segments through a slicing-by-4 CRC
//            register from zero.  Out go: a 16-B compact entry per record, the
//            segment registers (4 B per 64 B), and per record the register of
//            its segment before the word that holds its patch (its snapshot),
//            plus the tile's chain summary (LOCAL).  The first tile of a file
//            starts at offset 0; any other tile guesses its entry;
//   k_link   per file: the chain state entering every tile from the LOCALs;
//            tiles whose guess the state contradicts are listed;
//   k_refix  (only for listed tiles) re-runs the tile body from the true entry,
//            then k_link again;
//   k_emit   per tile: the 48-B tuples from the compact entries (a tile of
//            more than CAP_T records keeps the rest in spill chunks taken
//            from a per-call pool); a scan of the segment registers gives
//            the stream register at every segment start, from which every
//            record that ends inside the tile is checked against its own
//            stored CRC (data/dataFile.go:105-109);
//   k_fin    per file: a segmented scan of the tiles' exit registers gives the
//            register entering every tile; the record that crosses into a
//            tile is checked there.
// Every record is checked on its own, so a file fails exactly at the first
// record whose CRC differs, as ReadLogRecord's loop does.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
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
// Buffer resources (SGPRs) for the block loads and the compact-entry stores:
// 32-bit offsets only, no 64-bit addresses held in VGPRs across a block
typedef __amdgpu_buffer_rsrc_t rsrc_t;
__device__ __forceinline__ rsrc_t mk_rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
#define NONE32 0xFFFFFFFFu       // no position
#define TERM_NONE 127            // the chain leaves the segment (no terminal inside)
#define LM_NONE 0                // no record starts in the segment (the chain passes through it)
#define LM_CHAIN 1               // the chain enters the segment at E (a record start or its terminal)
#define LM_DEAD 2                // the file's chain ended before the segment
#define LM_OFF 3                 // segment beyond the end of the file
#define CAP_T ((uint32_t)(CLY_TILE / 128))   // compact entries in a tile's own area (more: spill chunks)
#define CAP_SHIFT (__builtin_ctz(CAP_T))
// k_scan walks runs of consecutive tiles of a file: a run's first tile
// guesses its entry, the others take the exit of the tile before them.  The
// run length (Globals::run_tiles) is chosen per call: RUN_TILES when the runs
// still fill the scan's wave slots, else 2 or 1 (small inputs: C1's 1024
// tiles as 256 runs left 15 of 16 wave slots idle, each run walking 64 blocks
// in a row).  The 8-KiB-tile test build keeps RUN_TILES, so that its small
// fixtures walk runs of several tiles.
#define RUN_TILES 4
#ifndef CLY_RUN_ADAPT
#define CLY_RUN_ADAPT (CLY_NBLK == 16)
#endif
// Spill: records CAP_T.. of a tile go to chunks of CAP_T entries (and their
// snapshots) taken from a per-call pool; a tile's chunk table holds up to
// NCH_MAX chunk ids and, in word CH_NWORD, how many it took.  Chain density:
// a record whose three varints end normally has headerSize >= 9.  The only
// shorter records (4 <= headerSize <= 6, step_hdr) have an expiration varint
// that overflows at its 10th byte: 9 continuation bytes, then a byte in 2..127.
// The next record's key-size varint starts inside those 9 bytes unless the
// record is >= 9 bytes long, so its first byte below 0x80 is that 10th byte,
// reached at index 9 or 10 by the key-size or value-size varint (an overflow:
// a negative index, ERR_VARINT) or only by its expiration varint, which needs
// the key and value varints to fit in front of it: impossible after <= 8 bytes.
// So a chain holds at most one record under 9 bytes before it ends, plus the
// short-buffer records of a file's last 26 bytes (at most 5): a tile holds at
// most CLY_TILE / 9 + 7 <= (NCH_MAX + 1) CAP_T records.  The bound is checked
// anyway: a chunk index past NCH_MAX stores nothing and fails the call
// (CLY_ERR_DEVICE, "internal error 0x80") instead of indexing past the table.
#define NCH_MAX 14
#define CH_WORDS 16
#define CH_NWORD 15
static_assert((NCH_MAX + 1) * (CLY_TILE / 128) >= CLY_TILE / 9 + 7, "spill chunks per tile");
static_assert((CAP_T & (CAP_T - 1)) == 0 && CAP_T >= 64, "CAP_T: a power of two, >= a round of 64 records");

struct DevFile {                 // 32 B
    const uint8_t* base;         // device pointer to the file's first byte (16-B aligned)
    uint64_t len;
    uint32_t fid;
    uint32_t first_tile;         // global index of the file's first tile
    uint32_t ntile;              // tiles of the file (>= 1)
    uint32_t _pad;
};
// Files of any length (Options.DataFileSize is an int64, options.go:10,70-71)
// are walked in parts of PART_TILES tiles: inside a part every position is a
// u32 offset from the part's first byte x0 (the tile body, TileLocal, the
// compact entries), and the part's view of the file is its bytes and up to
// VIEW_MAX past x0 (a record that crosses the part's end is read whole: records
// are below VIEW_MAX - PART_BYTES, 2 GiB - 128 KiB).  The chain state between tiles (k_link, TileIn), the
// terminal and failure positions and every tuple offset are u64 file offsets.
// A file below PART_BYTES is one part (x0 = 0).
#define PART_TILES 32768u
#define PART_BYTES ((uint64_t)PART_TILES * CLY_TILE)
#define VIEW_MAX (0xFFFFFFFFull - 2 * (uint64_t)CLY_TILE)
#define P_NONE 0xFFFFFFFFFFFFull  // no record start (u64 positions; files are below 2^48 B)
static_assert(PART_TILES % RUN_TILES == 0, "a run of tiles stays in one part (run lengths 1, 2, RUN_TILES)");
static_assert(PART_BYTES < VIEW_MAX, "a part's view: its bytes and a record that crosses its end");
__device__ __forceinline__ uint64_t part_x0(uint32_t tt) { return (uint64_t)(tt / PART_TILES) * PART_BYTES; }
// file F as tile tt's part sees it (base at x0, u32 length), and tt's index in the part
__device__ __forceinline__ DevFile part_view(const DevFile& F, uint32_t tt, uint32_t& ptt) {
    const uint64_t x0 = part_x0(tt);
    ptt = tt % PART_TILES;
    DevFile V = F;
    V.base = F.base + x0;
    V.len = F.len - x0 < VIEW_MAX ? F.len - x0 : VIEW_MAX;
    return V;
}

struct FileInfo {                // per file, zeroed per call (fail_off, fail_idx: all ones)
    uint64_t first_index;        // global tuple index of the file's first record
    uint64_t end_index;          // global index after the file's last record
    uint64_t term_pos;           // terminal position T of the file's chain
    // the first record whose CRC fails: its offset and its index in the file,
    // two atomicMins (records are in offset order: both minima are the same record's)
    u64      fail_off, fail_idx;
    int32_t  term_status;
    uint32_t term_tile;          // global tile index holding T
    uint32_t has_term;
    uint32_t _r0;
    uint64_t _r1;
};
__device__ __forceinline__ void fail_at(FileInfo* fo, uint64_t off, uint64_t idx) {
    atomicMin(&fo->fail_off, (u64)off);
    atomicMin(&fo->fail_idx, (u64)idx);
}

// Tile LOCAL (the tile's chain under its own entry), written by k_scan / k_refix:
// l[0]: bit1 the chain ends in the tile | bit2 no boundary in the tile | bit3
//       first tile of its file | bit4 a record starts in the tile | bit5 more
//       records than the compact list holds | records << 32
// l[1]: G (the tile's first boundary) | exit or terminal position << 32
// l[2]: crc_last | P_last << 32 (last record start in the tile and its stored CRC)
// l[3]: the smallest entry that passes the whole tile (tile end, or len + 1 for
//       the tile holding the file's end) | terminal status (s8) << 32
struct TileLocal { u64 l[4]; };
#define DF_TERM 2ull
#define DF_NONE 4ull
#define DF_FOF 8ull
#define DF_REC 16ull

struct Globals {                 // zeroed per call
    uint32_t nfix[2];            // tiles listed by a k_link round (slot r & 1) for the next k_refix
    uint32_t link_done;          // k_link workgroups finished (the last one computes the file bases)
    uint32_t overflow;           // tuples beyond out_cap were dropped
    uint32_t fail;               // internal invariant (never expected)
    uint32_t refix;              // tiles re-resolved over all rounds
    uint32_t rounds;             // link rounds
    uint32_t spill_next;         // spill chunks taken
    uint32_t spill_cap;          // spill chunks in the pool (set by the host)
    uint32_t spill_over;         // a chunk was refused (the host grows the pool and runs the call again)
    uint32_t walk_max;           // the longest k_refix walk (tiles), over all rounds
    uint64_t total;              // records over all files
    uint64_t walk_dbg;           // (length << 32 | first tile) of the longest k_refix walk
    uint32_t run_tiles;          // k_scan's run length this call (1, 2 or RUN_TILES; set by the host)
    uint32_t run_next;           // k_scan's run counter (runs past the grid's first one each)
};

// ---------------------------------------------------------------------------
// Nibble tables (the context's d_tabs, built on the host): 128 words each,
// entry n*16 + v = M (v << 4n) for a matrix M = A^bytes.
//   TAB_SH:   A^(v 16^d), v < 16, d < 4 (one hex digit of a byte shift), A^65536
//   TAB_TILE: A^CLY_TILE (k_fin)
//   TAB_EM:   k_emit's: A^(4k), k = 1..16 (a shift inside a segment; k = 16 is
//             the segment step A^64), A^1..A^3, and A^(RUN_BYTES 2^l), l < 6
//             (the lanes' runs of segments)
//   TAB_PW:   A^(CLY_TILE 2^k), k < NPW (k_fin's scan levels)
#define NIB_SH 65
#define TAB_SH 0
#define TAB_TILE (NIB_SH * 128)
#define TAB_EM (TAB_TILE + 128)
#define EM_F4 0                   // A^(4k): table k - 1
#define EM_F1 16                  // A^1, A^2, A^3: tables 16, 17, 18
#define EM_RUN 19                 // A^(RUN_BYTES 2^l): table 19 + l
#define EM_SEGP 25                // A^(64 2^l), l = 1..3: table 24 + l (k_emit's A^(64 j), j < 16)
#define NEM 28
#define TAB_PW (TAB_EM + NEM * 128)
#define NPW 32
#define NTAB_ALL (TAB_PW + NPW * 128)
// LDS of k_scan / k_refix (static: compile-time offsets)
//   [0, 65536)  CRC slicing-by-4 tables T0..T3, 16 replicas: dword (i*64 + t*16 + r)
//   LDS_INV     inverse of a zero-byte step (top byte of T0 -> index), 256 B
#define LDS_INV 65536
#define SCAN_LDS (LDS_INV + 256)

__device__ __forceinline__ void init_tables(CLY_LDS uint8_t* smem) {
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
    const uint32_t t0 = *(const CLY_LDS uint32_t*)(smem + a0), t1 = *(const CLY_LDS uint32_t*)(smem + a1);
    const uint32_t t2 = *(const CLY_LDS uint32_t*)(smem + a2 + 128), t3 = *(const CLY_LDS uint32_t*)(smem + a3 + 128);
    return __builtin_amdgcn_bitop3_b32(t0, t1, t2, 0x96) ^ t3;        // (0x96: a ^ b ^ c)
}
// one byte through the register: T0[(s ^ b) & 0xff] ^ (s >> 8)
__device__ __forceinline__ uint32_t crc_byte(const CLY_LDS uint8_t* smem, uint32_t s, uint32_t b, uint32_t r4) {
    const uint32_t i = (s ^ b) & 0xffu;
    return *(const CLY_LDS uint32_t*)(smem + ((i << 8) | r4)) ^ (s >> 8);
}
// inverse of one zero-byte step: s = A^-1 s'
__device__ __forceinline__ uint32_t crc_unbyte(const CLY_LDS uint8_t* smem, uint32_t s, uint32_t r4) {
    const uint32_t i = smem[LDS_INV + (s >> 24)];
    const uint32_t t = *(const CLY_LDS uint32_t*)(smem + ((i << 8) | r4));
    return ((s ^ t) << 8) | i;
}
// A^-j d (j < 4 zero bytes backwards)
__device__ __forceinline__ uint32_t crc_unbytes(const CLY_LDS uint8_t* smem, uint32_t d, uint32_t j, uint32_t r4) {
    for (uint32_t k = 0; k < j; k++) d = crc_unbyte(smem, d, r4);
    return d;
}
// M v by a nibble table of M
__device__ __forceinline__ uint32_t mat_mul(const CLY_LDS uint32_t* t, uint32_t v) {
    uint32_t q[8];
    #pragma unroll
    for (int n = 0; n < 8; n++) q[n] = t[n * 16 + ((v >> (4 * n)) & 15u)];
    // (v_bitop3 0x96: a three-input XOR, four of them instead of seven XORs)
    return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(q[0], q[1], q[2], 0x96),
                                       __builtin_amdgcn_bitop3_b32(q[3], q[4], q[5], 0x96), q[6] ^ q[7], 0x96);
}
// A^m v (m bytes), 1 <= m <= 65536: one nibble-table product per hex digit of m
// (sh: the TAB_SH tables)
__device__ __forceinline__ uint32_t shift_bytes(const CLY_LDS uint32_t* sh, uint32_t m, uint32_t v) {
    v = mat_mul(sh + (m & 15u) * 128, v);
    v = mat_mul(sh + (16u + ((m >> 4) & 15u)) * 128, v);
    v = mat_mul(sh + (32u + ((m >> 8) & 15u)) * 128, v);
    v = mat_mul(sh + (48u + ((m >> 12) & 15u)) * 128, v);
    if (m >> 16) v = mat_mul(sh + 64u * 128, v);
    return v;
}

// ---------------------------------------------------------------------------
// Header decode at file position p.  Fast path: 20 bytes gathered from
// [p & ~3, +20) (a 16-B and a 4-B load), varints of at most 4 bytes ending within
// header bytes 6..13 (every record the writer produces except long
// expirations); otherwise the exact byte-loop form over global memory.
struct Gath { uint32_t w[8]; };
__device__ __forceinline__ bool gath_ok(uint32_t p, uint64_t len) { return (uint64_t)(p & ~3u) + 32 <= len; }
// (only the 5 dwords hdr_fast reads: a loaded register left unread would keep
// a pending load on it, and the register's next writer would wait for it)
__device__ __forceinline__ void gath_issue(gbytes base, uint32_t p, Gath& g) {
    const CLY_GL u32x4u* q = (const CLY_GL u32x4u*)(base + (p & ~3u));
    const u32x4u a = q[0];
    g.w[0] = a.x; g.w[1] = a.y; g.w[2] = a.z; g.w[3] = a.w;
    g.w[4] = ((const CLY_GL uint32_t*)q)[4];
    g.w[5] = g.w[6] = g.w[7] = 0u;
}
__device__ __forceinline__ uint32_t alignb(uint32_t hi, uint32_t lo, uint32_t s) {
    return __builtin_amdgcn_alignbyte(hi, lo, s);
}
__device__ __forceinline__ uint32_t pack7(uint32_t s) {
    return (s & 0x7fu) | ((s >> 1) & 0x3f80u) | ((s >> 2) & 0x1fc000u) | ((s >> 3) & 0xfe00000u);
}
// header bytes 0..15 at p from a gather
__device__ __forceinline__ bool hdr_fast(const Gath& g, uint32_t p, uint64_t len, Hdr& h) {
    const uint64_t m64 = len - p;
    const int m = m64 > 26 ? 26 : (int)m64;
    if (m < 14) return false;
    const uint32_t s = p & 3;
    const uint32_t h0 = alignb(g.w[1], g.w[0], s), h1 = alignb(g.w[2], g.w[1], s), h2 = alignb(g.w[3], g.w[2], s),
                   h3 = alignb(g.w[4], g.w[3], s);
    h.crc = h0;
    h.type = h1 & 0xff;
    h.dt = (h1 >> 8) & 0xff;
    // Short forms first (the same results as the general form below): the three
    // varints in one byte each (keys and values under 64 B, no TTL: commit
    // markers, hint records, small records), or key size and expiration in one
    // byte and the value size in two (values of 64 B .. 8 KiB)
    const uint32_t b678 = (h1 >> 16) | ((h2 & 0xffu) << 16);                 // header bytes 6, 7, 8
    if ((b678 & 0x808080u) == 0u || ((b678 & 0x808080u) == 0x8000u && !(h2 & 0x8000u))) {
        const bool one = (b678 & 0x8000u) == 0u;
        const uint32_t b6 = b678 & 0xffu, b7 = (b678 >> 8) & 0xffu, b8 = b678 >> 16, b9 = (h2 >> 8) & 0xffu;
        const uint32_t uv = one ? b7 : (b7 & 0x7fu) | (b8 << 7), ue = one ? b8 : b9;
        const int32_t v1 = (int32_t)(b6 >> 1) ^ -(int32_t)(b6 & 1);
        const int32_t v2 = (int32_t)(uv >> 1) ^ -(int32_t)(uv & 1);
        h.ks = (uint32_t)v1;
        h.vs = (uint32_t)v2;
        h.exp = (int32_t)(ue >> 1) ^ -(int32_t)(ue & 1);
        h.hsz = one ? 9 : 10;
        h.key0 = one ? b9 : (h2 >> 16) & 0xffu;
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
    h.key0 = (((7 + e3) >= 12 ? h3 : h2) >> (8 * ((7 + e3) & 3))) & 0xffu;
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
// The wave's block stage in LDS: the block and the 32 bytes after it, each
// 64-B segment at an 80-B stride whose last 16 B repeat the
// next segment's first 16 B.  The stride spreads the lanes' 16-B stores and
// loads of their own segments over all banks (ds_write_b128: 8 lanes of 4
// dwords at 20 L mod 32; ds_read_b128: 16 lanes at 20 L mod 64), and the copy
// makes any 5 consecutive dwords of the logical stream 5 consecutive dwords of
// the stage.  Logical dword d (of the block) is stage dword d + 4 (d >> 4).
#define STG_STRIDE 80
#define STG_BYTES (CLY_NL * STG_STRIDE + 32)     // + the 32 B after the block (segment 64's first two chunks)
#define STG_SPAN (CLY_BLK + 32)                  // logical bytes the stage holds
__device__ __forceinline__ uint32_t stg_dw(uint32_t d) { return d + ((d >> 4) << 2); }
// byte view of the stage for step_hdr / go_varint (logical offsets)
struct StgBytes {
    const CLY_LDS uint8_t* s;
    uint32_t o;
    __device__ __forceinline__ uint32_t operator[](int64_t i) const {
        const uint32_t a = o + (uint32_t)i;
        return s[a + ((a >> 6) << 4)];
    }
    __device__ __forceinline__ StgBytes operator+(int64_t n) const { return StgBytes{s, o + (uint32_t)n}; }
};
// The header at p (bs <= p, p - bs + 26 <= STG_SPAN: every position the block
// body decodes) from the stage only: no global load inside the block body, so
// the next block's loads stay in flight (a vmcnt wait for a gather would wait
// for them too).  Fast form from 5 dwords; the byte-loop form otherwise.
__device__ __forceinline__ Hdr hdr_get(uint32_t p, uint64_t len, const CLY_LDS uint32_t* stg, uint32_t bs) {
    Hdr h;
    const uint32_t rel = p - bs;
    {
        Gath g;
        const CLY_LDS uint32_t* q = stg + stg_dw(rel >> 2);
        #pragma unroll
        for (int k = 0; k < 5; k++) g.w[k] = q[k];
        if (hdr_fast(g, p, len, h)) return h;
    }
    return step_hdr(StgBytes{(const CLY_LDS uint8_t*)stg, 0u}, (int64_t)rel, (int64_t)(len - bs), (int64_t)p);
}
__device__ __forceinline__ bool in_stage(uint32_t p, uint32_t bs) { return p >= bs && p - bs + 26 <= STG_SPAN; }
// The header at p from global memory (k_emit's long entries; guess-mode exit
// checks beyond the stage)
__device__ __forceinline__ Hdr hdr_load(gbytes base, uint32_t p, uint64_t len) {
    Hdr h;
    if (gath_ok(p, len)) {
        Gath g;
        gath_issue(base, p, g);
        if (hdr_fast(g, p, len, h)) return h;
    }
    return step_hdr(base, (int64_t)p, (int64_t)len, (int64_t)p);
}

// ---------------------------------------------------------------------------
// A lane's segment [cb, ce) of one block (file offsets; the segment holding
// the file's last byte also owns position len, where ReadLogRecord returns
// io.EOF; so does the empty file's first segment).
struct Seg {
    gbytes base;
    uint64_t len;
    const CLY_LDS uint32_t* stg; // the wave's copy of the block
    uint32_t bs;                 // the block's first byte
    uint32_t cb, ce;
    bool last;                   // owns position len
    bool on;                     // the segment exists (cb < len, or the empty file's segment 0)
};
__device__ __forceinline__ Seg make_seg(const DevFile& F, uint32_t bs, int lane, const CLY_LDS uint32_t* stg) {
    Seg K;
    K.base = (gbytes)F.base; K.len = F.len;
    K.stg = stg; K.bs = bs;
    const uint64_t cb = (uint64_t)bs + (uint64_t)lane * CLY_SEG;
    K.on = cb < F.len || cb == 0;
    K.last = K.on && cb + CLY_SEG >= F.len;
    K.cb = (uint32_t)cb;
    K.ce = (uint32_t)(cb + CLY_SEG < F.len ? cb + CLY_SEG : F.len);
    if (!K.on) { K.cb = 0xFFFFFFF0u; K.ce = 0xFFFFFFF0u; }
    return K;
}
__device__ __forceinline__ bool in_seg(const Seg& K, uint32_t x) {
    return (x >= K.cb && x < K.ce) || (K.last && (uint64_t)x == K.len);
}
struct SegChain {
    int      mode;               // LM_*
    uint32_t E;                  // first boundary (record start or terminal)
    uint32_t x;                  // exit (beyond the segment) or terminal position
    int      term;               // terminal status, TERM_NONE if the chain leaves the segment
    uint32_t cnt;                // records starting in the segment
    uint32_t last, last_crc;     // last record start and its stored CRC
    uint32_t sm0, sm1;           // the record starts: bit i = position cb + i
};
__device__ __forceinline__ void sc_set(SegChain& L, int mode) {
    L.mode = mode; L.E = NONE32; L.x = 0; L.term = TERM_NONE; L.cnt = 0; L.last = NONE32; L.last_crc = 0;
    L.sm0 = L.sm1 = 0;
}
// Walk from p: exact (ReadLogRecord semantics, every terminal) or speculative
// (every record one the writer produces; a terminal only at io.EOF at len).
// Returns false when a speculative chain is rejected.
__device__ __forceinline__ bool seg_walk(const Seg& K, uint32_t p, bool exact, SegChain& L) {
    sc_set(L, LM_CHAIN);
    L.E = p;
    for (int it = 0; it < 16; it++) {            // records are >= 6 bytes: <= 12 steps per segment
        if (!in_seg(K, p)) { L.x = p; return true; }
        const Hdr h = hdr_get(p, K.len, K.stg, K.bs);
        if (h.status != REC_OK) {
            L.x = p; L.term = h.status;
            return exact || (h.status == CLY_END_EOF && (uint64_t)p == K.len);
        }
        if (!exact && !h.good) return false;
        L.cnt++;
        L.last = p; L.last_crc = h.crc;
        {
            const uint32_t b = p - K.cb;             // (< 64: p is in the segment)
            if (b < 32) L.sm0 |= 1u << b; else L.sm1 |= 1u << (b - 32);
        }
        p += (uint32_t)h.size;
    }
    L.x = p;
    return exact;
}

// SWAR byte mask (bit 7 of each byte): byte <= 4 (type / data type).
__device__ __forceinline__ uint32_t swar_le4(uint32_t W) { return ~(((W | 0x80808080u) - 0x05050505u) | W) & 0x80808080u; }
// Candidate record starts of a segment (bit i: position cb + i has type and data
// type <= 4): its 16 words and the next 8 bytes (n0, n1).  The four candidate
// bits of a word are gathered by one multiply: bits 7, 15, 23, 31 times
// 1 + 2^7 + 2^14 + 2^21 land in bits 28..31.
__device__ __forceinline__ u64 cand_mask(const uint32_t (&w)[16], uint32_t n0, uint32_t n1) {
    uint32_t lo = 0, hi = 0;
    uint32_t L1 = swar_le4(w[1]);
    #pragma unroll
    for (int k = 0; k < 16; k++) {
        const uint32_t y2 = k + 2 < 16 ? w[k + 2 < 16 ? k + 2 : 0] : (k + 2 == 16 ? n0 : n1);
        const uint32_t L2 = swar_le4(y2);
        const uint32_t cm = L1 & __builtin_amdgcn_alignbit(L2, L1, 8);
        const uint32_t b4 = (cm * 0x204081u) >> 28;
        if (k < 8) lo |= b4 << (4 * k); else hi |= b4 << (4 * (k - 8));
        L1 = L2;
    }
    return ((u64)hi << 32) | lo;
}

// ---------------------------------------------------------------------------
// wave helpers: DPP row shifts / row broadcasts (gfx9 encodings), readlane for
// wave-uniform sources; no LDS round trips.
#define DPP_ROW_SHR(n) (0x110 + (n))
#define DPP_WF_SL1 0x130                 // lane i <- lane i+1
#define DPP_WF_SR1 0x138                 // lane i <- lane i-1
#define DPP_ROW_BCAST15 0x142
#define DPP_ROW_BCAST31 0x143
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ uint32_t dppu(uint32_t old, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, RM, 0xf, false);
}
__device__ __forceinline__ uint32_t rdl(uint32_t v, int lane) { return (uint32_t)__builtin_amdgcn_readlane((int)v, lane); }
// inclusive prefix sum over the wave
__device__ __forceinline__ uint32_t wave_add_incl(uint32_t v) {
    v += dppu<DPP_ROW_SHR(1)>(0u, v);
    v += dppu<DPP_ROW_SHR(2)>(0u, v);
    v += dppu<DPP_ROW_SHR(4)>(0u, v);
    v += dppu<DPP_ROW_SHR(8)>(0u, v);
    v += dppu<DPP_ROW_BCAST15, 0xa>(0u, v);
    v += dppu<DPP_ROW_BCAST31, 0xc>(0u, v);
    return v;
}
// inclusive "last set": v of the highest lane <= this one whose f is set (f: 0/1; f' = any such lane)
#define WL_STEP(CTRL, RM) { const uint32_t tv = dppu<CTRL, RM>(0u, v), tf = dppu<CTRL, RM>(0u, f); v = f ? v : tv; f |= tf; }
__device__ __forceinline__ void wave_last_incl(uint32_t& v, uint32_t& f) {
    WL_STEP(DPP_ROW_SHR(1), 0xf) WL_STEP(DPP_ROW_SHR(2), 0xf) WL_STEP(DPP_ROW_SHR(4), 0xf)
    WL_STEP(DPP_ROW_SHR(8), 0xf) WL_STEP(DPP_ROW_BCAST15, 0xa) WL_STEP(DPP_ROW_BCAST31, 0xc)
}
__device__ __forceinline__ uint32_t shfl_u32(uint32_t v, int src) { return (uint32_t)__shfl((int)v, src, 64); }

// The position of the k-th set bit of the 64-bit mask (m0 | m1 << 32), k < its popcount.
__device__ __forceinline__ uint32_t kth_bit(uint32_t m0, uint32_t m1, uint32_t k) {
    const uint32_t c0 = (uint32_t)__builtin_popcount(m0);
    uint32_t m = k < c0 ? m0 : m1, base = k < c0 ? 0u : 32u;
    k = k < c0 ? k : k - c0;
    #pragma unroll
    for (int w = 16; w >= 1; w >>= 1) {
        const uint32_t lc = (uint32_t)__builtin_popcount(m & ((1u << w) - 1u));
        const bool up = k >= lc;
        k = up ? k - lc : k;
        m = up ? m >> w : m;
        base += up ? (uint32_t)w : 0u;
    }
    return base;
}

// In-wave agreement: lane l's chain must start where the chain of the nearest
// segment before it leaves (the block's entry X0 for the first lanes); lanes
// after the first lane whose chain ends in a terminal are not checked (they are
// dead).  The lowest disagreeing lane is re-walked exactly, until every lane
// agrees.
__device__ __forceinline__ SegChain seg_resolve(const Seg& K, SegChain L, int lane, uint32_t X0, Globals* g) {
    for (int iter = 0;; iter++) {
        const bool isC = L.mode == LM_CHAIN;
        uint32_t v = L.x, f = isC ? 1u : 0u;
        wave_last_incl(v, f);
        const uint32_t vp = dppu<DPP_WF_SR1>(0u, v), fp = dppu<DPP_WF_SR1>(0u, f);
        const uint32_t Xin = fp ? vp : X0;
        const u64 bt = __ballot(isC && L.term != TERM_NONE);
        const int kT = bt ? __ffsll((long long)bt) - 1 : 64;
        bool bad = false;
        if (L.mode != LM_OFF && lane <= kT) bad = isC ? L.E != Xin : in_seg(K, Xin);
        const u64 bm = __ballot(bad);
        if (!bm) return L;
        if (iter > 4 * CLY_NL) { if (lane == 0) atomicOr(&g->fail, 1u); return L; }
        const int k = __ffsll((long long)bm) - 1;
        if (lane == k) {
            if (!in_seg(K, Xin)) sc_set(L, LM_NONE);
            else seg_walk(K, Xin, true, L);
        }
    }
}

// ---------------------------------------------------------------------------
// Chain state between tiles (k_link).
struct LBState {
    uint64_t count;              // records before (file-relative in TileIn)
    uint64_t X;                  // chain position (file offset)
    uint64_t P_last;             // the last record started before: its start (P_NONE: none in this file)
    uint32_t crc_last;           // ... and its stored CRC (its successor's Q)
    int      dead;               // the file's chain has ended
};
// TileIn (k_link): the true state entering a tile, 32 B:
//   w[0..1] count (file-relative), w[2] X (low word), w[3] dead | fix, w[4] crc_last,
//   w[5] P_last (low word), w[6] the tile's file (k_emit), w[7] X >> 32 | (P_last >> 32) << 16
struct TileIn { uint32_t w[8]; };
#define TI_DEAD 1u
__device__ __forceinline__ LBState ti_load(const TileIn* p) {
    const u32x4 a = ((const u32x4*)p)[0], b = ((const u32x4*)p)[1];
    LBState s;
    s.count = ((uint64_t)a.y << 32) | a.x; s.dead = (a.w & TI_DEAD) != 0; s.crc_last = b.x;
    s.X = a.z | ((uint64_t)(b.w & 0xFFFFu) << 32);
    s.P_last = b.y | ((uint64_t)(b.w >> 16) << 32);
    return s;
}
#define TI_FIX 2u                // listed for k_refix this round
__device__ __forceinline__ void ti_store(TileIn* p, const LBState& s, uint32_t f) {
    ((u32x4*)p)[0] = (u32x4){(uint32_t)s.count, (uint32_t)(s.count >> 32), (uint32_t)s.X, s.dead ? TI_DEAD : 0u};
    ((u32x4*)p)[1] = (u32x4){s.crc_last, (uint32_t)s.P_last, f,
                             ((uint32_t)(s.X >> 32) & 0xFFFFu) | ((uint32_t)(s.P_last >> 32) << 16)};
}

// ---------------------------------------------------------------------------
// Outputs of one record.  Tuple (48 B, cly_tuple layout):
__device__ __forceinline__ void tuple_words(gbytes base, uint32_t p, uint64_t x0, const Hdr& h, uint32_t fid, u32x4& a,
                                            u32x4& b, u32x4& c) {
    int tn;
    int64_t tx;
    if (h.key0 < 0x80 && h.ks >= 1) { tn = 1; tx = (int64_t)(h.key0 >> 1) ^ -(int64_t)(h.key0 & 1); }
    else {
        const int64_t klim = h.ks < 11u ? (int64_t)h.ks : 11;
        tx = go_varint(base + p + h.hsz, klim, tn);                     // parseLogRecordKey, db.go:706-710
    }
    const uint64_t off = x0 + p, ex = (uint64_t)h.exp, txv = tn < 0 ? 0ull : (uint64_t)tx;
    a = (u32x4){(uint32_t)off, (uint32_t)(off >> 32), (uint32_t)ex, (uint32_t)(ex >> 32)};
    b = (u32x4){(uint32_t)txv, (uint32_t)(txv >> 32), fid, (uint32_t)h.size};
    c = (u32x4){h.ks, h.vs,
                (h.type & 0xff) | ((h.dt & 0xff) << 8) | ((uint32_t)(h.hsz & 0xff) << 16) |
                    ((uint32_t)(tn < 0 ? 0xFF : tn) << 24),
                h.crc};
}
// Compact entry (16 B), k_scan -> k_emit.  w0 crc; w1 the record's snapshot
// (stored into the entry once the block's CRC pass has it: no snapshot stream
// of its own); short form (bit 23 of w3; every record the writer produces
// without a TTL or a txId >= 64, keys under 256 B, values under 2 MiB):
// w2 vs (21 bits) | hsz-6 << 21 | type << 26 | dt << 29, w3 rel | key0 << 16
// (the txId varint's single byte) | ks << 24.  Long form: w2 = 0, w3 = rel
// only (k_emit decodes the header again).
#define REC_SHORT (1u << 23)
#define SH_KS_LIM 256u
#define SH_VS_LIM (1u << 21)
// Where a block's compact entries and snapshots go (k_scan, k_refix): stored
// as they are made (an LDS sink flushed at the next block's top, after its
// loads, measured 1.6 % slower on C2 and 3.3 % on C4), and the file record
// checks of k_ovf's re-walk
struct RecSink {
    rsrc_t trs;                  // the tile's own entries
    CLY_GL u32x4* sp_rec;        // the spill pool's entries (chunk c at c CAP_T)
    CLY_LDS uint32_t* chk;       // the wave's copy of the tile's chunk ids
    uint32_t* ctab;              // the tile's chunk table (CH_WORDS words)
    Globals* g;
};
// The entry now (word 1 zero) and its snapshot into word 1 when the block's
// CRC pass has it: two stores of one wave to the same bytes, applied in issue
// order (one request queue per CU and L2 channel), merged in L2 into one line
// write (a chunk index past the table: nothing stored, spill_ensure failed the call)
__device__ __forceinline__ void rec_put(const RecSink& rs, uint32_t idx, const u32x4& v) {
    if (idx < CAP_T) __builtin_amdgcn_raw_buffer_store_b128(v, rs.trs, (int)(idx * 16u), 0, 0);
    else {
        const uint32_t ci = (idx >> CAP_SHIFT) - 1u;
        const uint32_t c = ci < NCH_MAX ? rs.chk[ci] : NONE32;
        if (c != NONE32) rs.sp_rec[(uint64_t)c * CAP_T + (idx & (CAP_T - 1u))] = v;
    }
}
__device__ __forceinline__ void snap_put(const RecSink& rs, uint32_t r, uint32_t v) {
    if (r < CAP_T) __builtin_amdgcn_raw_buffer_store_b32(v, rs.trs, (int)(r * 16u + 4u), 0, 0);
    else {
        const uint32_t ci = (r >> CAP_SHIFT) - 1u;
        const uint32_t c = ci < NCH_MAX ? rs.chk[ci] : NONE32;
        if (c != NONE32) ((CLY_GL uint32_t*)(rs.sp_rec + (uint64_t)c * CAP_T + (r & (CAP_T - 1u))))[1] = v;
    }
}
__device__ __forceinline__ void rec_store(const RecSink& rs, uint32_t idx, const Hdr& h, uint32_t rel) {
    const bool sh = h.exp == 0 && h.key0 < 0x80u && h.ks >= 1u && h.ks < SH_KS_LIM && h.vs < SH_VS_LIM &&
                    h.type < 8u && h.dt < 8u && h.hsz >= 6 && h.hsz < 38;
    u32x4 v = (u32x4){0u, 0u, 0u, rel};
    if (sh) v = (u32x4){h.crc, 0u, h.vs | ((uint32_t)(h.hsz - 6) << 21) | (h.type << 26) | (h.dt << 29),
                        rel | (h.key0 << 16) | REC_SHORT | (h.ks << 24)};
    rec_put(rs, idx, v);
}

// ---------------------------------------------------------------------------
// Block loads.  Load k (of 4) of lane i + 16q reads the 16 B at
// bs + 1024k + 64i + 16q, so that each load instruction reads 1 KiB of
// consecutive bytes; a 4 x 4 transpose of 16-B elements over the lane quarters
// (v_permlane32_swap, v_permlane16_swap) then leaves lane L with the 64 bytes
// at bs + 64L.  Bytes at or past the file end read as zero (a 16-B load that
// straddles it stays inside its 16-B-aligned block of the buffer).
__device__ __forceinline__ u32x4 load16z(gbytes base, uint64_t a, uint64_t len) {
    if (a + 16 <= len) return *(const CLY_GL u32x4*)(base + a);
    u32x4 v = {0u, 0u, 0u, 0u};
    if (a < len) {
        v = *(const CLY_GL u32x4*)(base + a);
        const uint32_t n = (uint32_t)(len - a);          // 1..15 valid bytes
        #pragma unroll
        for (int k = 0; k < 4; k++) {
            const int lo = 4 * k;
            const uint32_t m = (int)n >= lo + 4 ? 0xFFFFFFFFu : ((int)n <= lo ? 0u : ((1u << (8 * (n - lo))) - 1u));
            v[k] &= m;
        }
    }
    return v;
}
// The block's loads, and the 32 bytes after it (16 B by each of lanes 0, 1:
// the tail of the wave's stage, for headers that start near the block's end).
__device__ __forceinline__ void blk_issue(gbytes base, rsrc_t frs, uint64_t flen, uint32_t bs, int lane, u32x4 (&e)[4],
                                          u32x4& hl) {
    const uint32_t off = bs + 64u * (uint32_t)(lane & 15) + 16u * (uint32_t)(lane >> 4);
    if ((uint64_t)bs + CLY_BLK <= flen) {
        #pragma unroll
        for (int k = 0; k < 4; k++) e[k] = __builtin_amdgcn_raw_buffer_load_b128(frs, (int)(off + 1024u * k), 0, 0);
    } else {
        #pragma unroll
        for (int k = 0; k < 4; k++) e[k] = load16z(base, (uint64_t)(off + 1024u * k), flen);
    }
    hl = (u32x4){0u, 0u, 0u, 0u};
    if (lane < 2) hl = load16z(base, (uint64_t)bs + CLY_BLK + 16 * lane, flen);
}
// the first block of tile tt of file F (its loads are issued by the caller of
// tile_body, so that a wave's next tile streams in under its current one)
__device__ __forceinline__ void tile_issue(const DevFile& F, uint32_t tt, int lane, u32x4 (&e)[4], u32x4& hl) {
    blk_issue((gbytes)F.base, mk_rsrc(F.base, (uint32_t)F.len), F.len, (uint32_t)((uint64_t)tt * CLY_TILE), lane, e, hl);
}
__device__ __forceinline__ void swap32(uint32_t& a, uint32_t& b) {
    const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    a = r[0]; b = r[1];
}
__device__ __forceinline__ void swap16(uint32_t& a, uint32_t& b) {
    const auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    a = r[0]; b = r[1];
}
// e[k] of lane quarter q -> e[j] of quarter q = what quarter j held in e[q]
__device__ __forceinline__ void quad_transpose(u32x4 (&e)[4]) {
    #pragma unroll
    for (int c = 0; c < 4; c++) {
        uint32_t a0 = e[0][c], a1 = e[1][c], a2 = e[2][c], a3 = e[3][c];
        swap32(a0, a2); swap32(a1, a3);
        swap16(a0, a1); swap16(a2, a3);
        e[0][c] = a0; e[1][c] = a1; e[2][c] = a2; e[3][c] = a3;
    }
}
__device__ __forceinline__ void patch_word(uint32_t (&w)[16], uint32_t k, uint32_t e) {
    #pragma unroll
    for (int i = 0; i < 16; i++) w[i] ^= (k == (uint32_t)i) ? e : 0u;
}

// ---------------------------------------------------------------------------
// The tile body (k_scan, k_refix).  The wave streams the
// tile's blocks in order; the chain position X is carried from block to block.
//   BM_SPEC   k_scan: the entry of a tile other than its file's first is
//             unknown; the first block with a plausible record start sets the
//             tile's guess G (a candidate whose speculative walk holds and
//             leaves at a candidate, or at a plausible header beyond the block);
//   BM_EXACT  k_refix: the entry is the true state from k_link.
// CRC: GetLogRecordCRC of the record at P is the CRC-32 of
// F[P+4 : P+size] (data/logRecord.go:136-146).  In the CRC register's terms
// the stream from P on, started from the register c ^ K4 (c = the stored CRC
// at P, K4 = A^-4 0xFFFFFFFF), holds 0xFFFFFFFF after the 4 stored bytes and
// ~crc at the record's end; the record matches iff that register is ~c there.
// Each lane runs its 64-B segment's raw words from a zero register (the
// segment register S) and keeps, at every record start's patch word W (P's
// own word when P is word-aligned, else the next one), the register entering W
// (the snapshot).  From these alone (linearity) k_emit gets the register
// entering the next record's patch word as it is when the walk restarts at
// P with the known register exp_post(P) entering W (the reset), and compares
// it with the value a matching record leaves (exp_pre).  The chain's terminal
// T is closed in the data instead: ~cq of the record before it is XORed in
// before byte T and every byte from T on reads as zero, so the last record
// matches iff the register is zero after T (the tile's first boundary XORs
// 0xFFFFFFFF there when the record before it is in an earlier tile; k_fin
// completes it).
#define BM_SPEC 0
#define BM_EXACT 1
#define PW_ROUNDS 1              // pred_walk rounds per block before the general pass (C3: 1 round 12.7 ms, 2 13.6, 4 15.4)
#ifndef GP_TRIES
#define GP_TRIES 2               // candidates a general-pass lane walks for its first chain (small records: 1 try 4.90 ms, 2: 4.59, 5: 4.39 per GiB; C3: 5 tries +0.2 ms)
#endif
// Per-tile CRC outputs of the tile body: the segment registers (one per 64-B
// segment of the tile, stream order) and the records' snapshots (indexed like
// the compact entries; boundary CAP_T is the last one kept)
#define NSEG (CLY_NBLK * CLY_NL)         // segments per tile
struct TileRes { uint32_t X; bool dead; };
// The chain state a wave carries through its tile (wave-uniform).
struct TState {
    uint32_t X;                  // chain position (next boundary); NONE32: entry unknown (guess mode)
    bool dead;                   // the chain has ended (terminal found)
    bool cq_known;               // cq is the stored CRC before X (else: the tile's first boundary, deferred)
    uint32_t cq;
    uint32_t G, tcnt, last_crc, P_last;
    int term;
    uint32_t s_last, s_prev;     // sizes of the last two records (0: none yet)
    uint32_t Tb;                 // terminal position in the current block (NONE32: none)
    uint32_t tpatch;             // its patch word (XORed after the bytes from Tb on are zeroed)
    uint32_t carry_next;         // register XOR due at the next block's first byte (a patch word past the block)
    bool cmark_next;             // ... and it is a record start's patch (its snapshot is the next block's word 0)
    // stride reference (stride_round): header bytes 4..15 of the last record
    // (ref1..3) under the masks of its bytes 4..hsz, and the uniform words of
    // its compact entry; valid while ref_ok
    uint32_t nch;                // spill chunks the records so far need
    uint32_t nch_have;           // chunks the tile holds (k_refix reuses k_scan's)
    bool ref_ok;
    uint32_t ref_s;              // the reference record's size (the stride)
    uint32_t ref1, ref2, ref3, msk1, msk2, msk3, rw2, rw3;
};
// The block's outputs for record k of a round (lane k): its compact entry.
// Returns the record's patch word as an index in the block: the word whose
// entering register its CRC check reads (P's own word when P is word-aligned,
// else the word after it; PW_CARRY: the next block's first word).
__device__ __forceinline__ uint32_t rec_out(uint32_t p, const Hdr& h, uint32_t idx, uint32_t tb, uint32_t bs,
                                            const RecSink& rs) {
    rec_store(rs, idx, h, p - tb);
    return ((p - bs) >> 2) + ((p & 3u) ? 1u : 0u);
}
#define PW_CARRY (CLY_BLK / 4)
// The block's patch-word mask (per wave, in LDS: bit k of word L = word k of
// segment L holds a record start's patch), built by the lanes that place the
// patches; the segment lanes read it to know where to keep snapshots.
__device__ __forceinline__ void mark_pw(CLY_LDS uint32_t* mk, uint32_t pw) {
    __atomic_fetch_or(mk + (pw >> 4), 1u << (pw & 15u), __ATOMIC_RELAXED);
}
// The terminal T (found by lane src): the bytes from T on read as zero, and
// ~cq of the record before it (dT) is XORed in before byte T (into the word
// holding T, after the zeroing), or at the next block's first byte when T is
// the block's end.
template <int BM>
__device__ __forceinline__ void term_patch(TState& S, uint32_t T, uint32_t dT, uint32_t bs, const CLY_LDS uint8_t* smem,
                                           const CrcLane& cl, int src) {
    S.Tb = T;
    if (T < bs + CLY_BLK) S.tpatch = rdl(crc_unbytes(smem, dT, T & 3u, cl.r4), src);
    else S.carry_next ^= rdl(dT, src);
}

// The spill chunks for record indices < hi (wave-uniform): a chunk the tile
// does not hold yet comes from the pool (lane 0); a refused one (pool full)
// is NONE32 and the call is run again with a larger pool.
__device__ __forceinline__ void spill_ensure(TState& S, uint32_t hi, const RecSink& rs, int lane) {
    if (hi <= (S.nch + 1u) * CAP_T) return;
    while (hi > (S.nch + 1u) * CAP_T) {
        if (S.nch >= S.nch_have) {
            if (lane == 0) {
                uint32_t id = NONE32;
                if (S.nch < NCH_MAX) {
                    id = atomicAdd(&rs.g->spill_next, 1u);
                    if (id >= rs.g->spill_cap) { atomicOr(&rs.g->spill_over, 1u); id = NONE32; }
                } else atomicOr(&rs.g->fail, 128u);                  // (chain density: never)
                if (S.nch < NCH_MAX) { rs.chk[S.nch] = id; rs.ctab[S.nch] = id; }
            }
            S.nch_have = S.nch < NCH_MAX ? S.nch + 1u : NCH_MAX;
        }
        S.nch++;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Exact predictive walk (entry X known and in this block): lane k decodes the
// header at the position the last two record sizes predict for the k-th record
// from X (sizes alternating b, a, b, ... with a = the last size, b = the one
// before).  Lanes 0 .. kb-1 whose sizes match the prediction are records of the
// chain, and so is lane kb (the first mismatch) when its header is a record:
// its true size gives the next X; a terminal at kb ends the chain.  Every round
// is exact and advances by at least one record.  Returns false when the round
// budget runs out with X still in the block (the caller's general pass goes on).
template <int BM>
__device__ __forceinline__ bool pred_walk(const DevFile& F, TState& S, uint32_t tb, uint32_t bs, CLY_LDS uint32_t* stg,
                                          const CLY_LDS uint8_t* smem, const CrcLane& cl, uint32_t K4, const RecSink& rs,
                                          int lane, CLY_LDS uint32_t* mk) {
    const uint64_t flen = F.len, bend = (uint64_t)bs + CLY_BLK;
    for (int round = 0; round < PW_ROUNDS; round++) {
        const uint64_t X = S.X;
        const bool owned = X < bend || (X == flen && flen == bend);
        if (S.dead || !owned) return true;
        uint32_t a = S.s_last, b = S.s_prev ? S.s_prev : S.s_last;
        if (!a) {                                  // no size yet: the record at X sets the stride
            const Hdr h0 = hdr_get((uint32_t)X, flen, stg, bs);
            a = b = h0.status == REC_OK ? (uint32_t)h0.size : 64u;
        }
        const uint32_t k = (uint32_t)lane;
        const uint64_t P = X + (uint64_t)((k + 1) >> 1) * b + (uint64_t)(k >> 1) * a;
        const bool act = P < bend || (P == flen && flen == bend);
        Hdr h;
        h.status = CLY_END_EOF; h.size = 0; h.crc = 0;
        if (act) h = hdr_get((uint32_t)P, flen, stg, bs);
        const uint32_t expect = (k & 1) ? a : b;
        const bool rec = act && h.status == REC_OK;
        const u64 brk = __ballot(!(rec && (uint64_t)h.size == expect));
        const int kb = brk ? __ffsll((long long)brk) - 1 : 64;
        const bool acc = (int)k < kb || ((int)k == kb && rec);
        const u64 ba = __ballot(acc);
        const int n = __popcll(ba);
        // the stored CRC of each record's predecessor
        const uint32_t up = dppu<DPP_WF_SR1>(0u, h.crc);
        const uint32_t dq = k == 0 ? (S.cq_known ? ~S.cq : 0xFFFFFFFFu) : ~up;
        uint32_t pw = 0;
        spill_ensure(S, S.tcnt + (uint32_t)n, rs, lane);
        if (acc) {
            pw = rec_out((uint32_t)P, h, S.tcnt + k, tb, bs, rs);
            if (pw < PW_CARRY) mark_pw(mk, pw);
        }
        if (__ballot(acc && pw == PW_CARRY)) S.cmark_next = true;
        if (S.G == NONE32) S.G = (uint32_t)X;
        if (n) {
            const int kl = n - 1;
            S.last_crc = rdl(h.crc, kl);
            S.P_last = rdl((uint32_t)P, kl);
            const uint32_t sl = rdl((uint32_t)h.size, kl);
            S.s_prev = kl ? rdl((uint32_t)h.size, kl - 1) : S.s_last;
            S.s_last = sl;
            S.cq = S.last_crc; S.cq_known = true;
            S.X = S.P_last + sl;
            S.tcnt += (uint32_t)n;
        }
        if (kb < 64 && !((ba >> kb) & 1ull) && ((__ballot(act) >> kb) & 1ull)) {
            // lane kb is the chain's terminal (its header is not a record)
            const int st = (int)rdl((uint32_t)h.status, kb);
            {
                const uint32_t T = rdl((uint32_t)P, kb);
                const uint32_t dT = T == 0 ? 0u : rdl(dq, kb);
                term_patch<BM>(S, T, dT, bs, smem, cl, kb);
                S.X = T; S.dead = true; S.term = st;
                return true;
            }
        }
    }
    const uint64_t X = S.X;
    return S.dead || !(X < bend || (X == flen && flen == bend));
}

// Stride round (regular data: the last two records had the same size; s =
// the reference record's size): lane k takes X + k s; a record there whose
// header bytes 4..hsz equal the reference's (type, data type, the three
// varints and the first key byte) is a record of size s with the same fields,
// so no decode is needed, only its stored CRC.  Lanes up to the first one that differs (or leaves the block, or
// would pass the file's end) are records; the rest of the block goes to
// pred_walk from there.
template <int BM>
__device__ __forceinline__ void stride_round(const DevFile& F, TState& S, uint32_t tb, uint32_t bs,
                                             CLY_LDS uint32_t* stg, const CLY_LDS uint8_t* smem, const CrcLane& cl,
                                             uint32_t K4, const RecSink& rs, int lane, CLY_LDS uint32_t* mk) {
    const uint32_t X = S.X, s = S.ref_s, k = (uint32_t)lane;
    const uint64_t bend = (uint64_t)bs + CLY_BLK;
    if (S.dead || (uint64_t)X >= bend) return;
    const uint64_t P64 = (uint64_t)X + (uint64_t)k * s;
    const bool act = P64 < bend && P64 + s <= F.len;
    const uint32_t P = act ? (uint32_t)P64 : X;
    const CLY_LDS uint32_t* q = stg + stg_dw((P - bs) >> 2);
    const uint32_t w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3], w4 = q[4], sh = P & 3u;
    const uint32_t crc = alignb(w1, w0, sh), h1 = alignb(w2, w1, sh), h2 = alignb(w3, w2, sh), h3 = alignb(w4, w3, sh);
    const bool match = act && (((h1 ^ S.ref1) & S.msk1) | ((h2 ^ S.ref2) & S.msk2) | ((h3 ^ S.ref3) & S.msk3)) == 0u;
    const u64 bm = __ballot(!match);
    const uint32_t kb = bm ? (uint32_t)__ffsll((long long)bm) - 1 : 64u;
    if (kb == 0) return;
    uint32_t pw = 0;
    spill_ensure(S, S.tcnt + kb, rs, lane);
    if (k < kb) {
        rec_put(rs, S.tcnt + k, (u32x4){crc, 0u, S.rw2, (P - tb) | S.rw3});
        pw = ((P - bs) >> 2) + ((P & 3u) ? 1u : 0u);
        if (pw < PW_CARRY) mark_pw(mk, pw);
    }
    if (__ballot(k < kb && pw == PW_CARRY)) S.cmark_next = true;
    if (S.G == NONE32) S.G = X;
    S.last_crc = rdl(crc, (int)kb - 1);
    S.P_last = X + (kb - 1) * s;
    S.cq = S.last_crc; S.cq_known = true;
    S.X = S.P_last + s;
    S.tcnt += kb;
    S.s_prev = kb >= 2 ? s : S.s_last;
    S.s_last = s;
}
// The stride reference from the last record (after pred_walk accepted
// records): taken when the last two sizes are equal and the last record is in
// the stage and has a short compact entry with its header in bytes 0..15.
__device__ __forceinline__ void stride_ref(const DevFile& F, TState& S, uint32_t bs, const CLY_LDS uint32_t* stg) {
    S.ref_ok = false;
    if (S.dead || !S.s_last || S.s_last != S.s_prev || S.P_last == NONE32 || S.P_last < bs) return;
    const uint32_t P = S.P_last;
    const Hdr h = hdr_get(P, F.len, stg, bs);
    const bool sh = h.status == REC_OK && h.exp == 0 && h.key0 < 0x80u && h.ks >= 1u && h.ks < SH_KS_LIM &&
                    h.vs < SH_VS_LIM && h.type < 8u && h.dt < 8u && h.hsz >= 6 && h.hsz <= 15 &&
                    (uint32_t)h.size == S.s_last;
    if (!sh) return;
    const CLY_LDS uint32_t* q = stg + stg_dw((P - bs) >> 2);
    const uint32_t w1 = q[1], w2 = q[2], w3 = q[3], w4 = q[4], a = P & 3u;
    S.ref1 = __builtin_amdgcn_readfirstlane(alignb(w2, w1, a));
    S.ref2 = __builtin_amdgcn_readfirstlane(alignb(w3, w2, a));
    S.ref3 = __builtin_amdgcn_readfirstlane(alignb(w4, w3, a));
    const uint32_t hz = (uint32_t)h.hsz;                       // bytes 4..hz compared
    auto msk = [&](uint32_t b0) {                              // bytes b0..b0+3
        uint32_t m = 0;
        for (uint32_t b = 0; b < 4; b++) if (b0 + b <= hz) m |= 0xFFu << (8 * b);
        return m;
    };
    S.msk1 = msk(4); S.msk2 = msk(8); S.msk3 = msk(12);
    S.rw2 = h.vs | ((uint32_t)(h.hsz - 6) << 21) | (h.type << 26) | (h.dt << 29);
    S.rw3 = (h.key0 << 16) | REC_SHORT | (h.ks << 24);
    S.ref_s = (uint32_t)h.size;
    S.ref_ok = true;
}

// Guess mode (a tile other than its file's first, entry unknown): every
// lane's first candidate record start in its 64-B segment whose speculative
// walk holds, validated at the walk's exit (a candidate of the block, or a
// plausible header beyond it).  The tile's guessed entry G is the first such
// start whose exit was confirmed inside the block, else the first such start;
// NONE32 when the block holds none.  k_link checks the guess.
// a header a chain may continue at: a record the writer produces, a zero
// header, or the end of the file
__device__ __forceinline__ bool hdr_plausible(const Hdr& h, uint32_t x, uint64_t flen) {
    return (h.status == REC_OK && h.good) || h.status == CLY_END_ZERO || (h.status == CLY_END_EOF && (uint64_t)x == flen);
}
__device__ __forceinline__ uint32_t guess_entry(const DevFile& F, uint32_t bs, CLY_LDS uint32_t* stg, const u32x4& hc,
                                                int lane) {
    const CLY_LDS u32x4* sv = (const CLY_LDS u32x4*)stg;
    const uint64_t flen = F.len;
    const Seg K = make_seg(F, bs, lane, stg);
    uint32_t wv[16];
    #pragma unroll
    for (int k = 0; k < 4; k++) {
        const u32x4 v = sv[5 * lane + k];
        wv[4 * k] = v.x; wv[4 * k + 1] = v.y; wv[4 * k + 2] = v.z; wv[4 * k + 3] = v.w;
    }
    const uint32_t n0 = dppu<DPP_WF_SL1>(rdl(hc.x, 0), wv[0]), n1 = dppu<DPP_WF_SL1>(rdl(hc.y, 0), wv[1]);
    u64 cm = 0;
    if (K.on) {
        cm = cand_mask(wv, n0, n1);
        const uint32_t nv = K.ce - K.cb;                    // valid positions
        if (nv < 64) cm &= (1ull << nv) - 1ull;
        // a record that starts in the last 4 bytes before the block leaves a
        // false candidate 4 bytes after its start, in the block's first 4
        // bytes: its "CRC" is that record's type, data type and size varints,
        // so its first two bytes are <= 4 (a stored CRC's, 1 in 2600); its walk
        // over keys of '0'..'9' digits often holds (small records: most of the
        // wrong run-start guesses).  Not a guess, then.
        if (lane == 0) {
            const uint32_t le = swar_le4(wv[0]), le4 = swar_le4(wv[1]) & 0x80u;
            uint32_t pm = 0;
            #pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t a = (le >> (8 * k + 7)) & 1u;
                const uint32_t b = k < 3 ? (le >> (8 * (k + 1) + 7)) & 1u : le4 >> 7;
                pm |= (a & b) << k;
            }
            cm &= ~(u64)pm;
        }
    }
    uint32_t E = NONE32, ex_x = 0, ex_sz = 0;       // (an unconfirmed start: its exit and the record there)
    bool conf_in = false;
    u64 mm = cm;
    bool settled = !K.on || !mm;
    for (int tr = 0; tr < 4; tr++) {
        const bool act = !settled;
        if (!__ballot(act)) break;
        SegChain T;
        sc_set(T, LM_NONE);
        bool ok = false;
        if (act) {
            const uint32_t q = K.cb + (uint32_t)__builtin_ctzll(mm);
            mm &= mm - 1;
            ok = seg_walk(K, q, false, T);
        }
        const bool chk_in = act && ok && T.term == TERM_NONE && T.x < bs + CLY_BLK;
        const uint32_t off = chk_in ? T.x - bs : 0u;
        const int tl = (int)(off >> 6);
        const uint32_t clo = shfl_u32((uint32_t)cm, tl), chi = shfl_u32((uint32_t)(cm >> 32), tl);
        bool in = act && ok && T.term != TERM_NONE;          // walk ended at io.EOF at len
        if (act && ok && T.term == TERM_NONE) {
            if (chk_in) {
                const uint32_t bb = off & 63u;
                ok = (((bb < 32 ? clo >> bb : chi >> (bb - 32))) & 1u) != 0;
                if (ok) {
                    // two more hops from the stage: the exit's header, and the
                    // header after that record when it is in the stage too (a
                    // false start rarely passes three headers)
                    const Hdr h1 = hdr_get(T.x, flen, stg, bs);
                    ok = hdr_plausible(h1, T.x, flen);
                    if (ok && h1.status == REC_OK) {
                        const uint64_t x2 = (uint64_t)T.x + (uint64_t)h1.size;
                        if (x2 < 0xFFFFFFFFull && in_stage((uint32_t)x2, bs))
                            ok = hdr_plausible(hdr_get((uint32_t)x2, flen, stg, bs), (uint32_t)x2, flen);
                    }
                }
                in = ok;
            } else {
                // the exit's header from the stage, or (beyond it) from global
                // memory: the one global read of the block body, in guess blocks
                // only (its wait also waits for the next block's loads)
                Hdr eh;
                if (in_stage(T.x, bs)) eh = hdr_get(T.x, flen, stg, bs);
                else {
                    eh = hdr_load((gbytes)F.base, T.x, flen);
                    __builtin_amdgcn_s_waitcnt(0);          // every load of this path done here, not at a join
                }
                ok = hdr_plausible(eh, T.x, flen);
                if (ok && eh.status == REC_OK) { ex_x = T.x; ex_sz = (uint32_t)eh.size; }
            }
        }
        if (act && ok) { E = T.E; conf_in = in; settled = true; }
        if (act && !ok && !mm) settled = true;
    }
    const u64 bin = __ballot(E != NONE32 && conf_in);
    if (!bin) {
        // no start confirmed inside the block (a long record's value bytes: C3):
        // the header after the exit's record must be plausible too -- a false
        // start passes one plausible header now and then, two almost never
        // (C3: the first link round's contradicted runs)
        bool drop = false;
        if (E != NONE32 && ex_sz) {
            const uint64_t x2 = (uint64_t)ex_x + ex_sz;
            if (x2 < 0xFFFFFFFFull) {
                Hdr e2;
                if (in_stage((uint32_t)x2, bs)) e2 = hdr_get((uint32_t)x2, flen, stg, bs);
                else {
                    e2 = hdr_load((gbytes)F.base, (uint32_t)x2, flen);
                    __builtin_amdgcn_s_waitcnt(0);
                }
                drop = !hdr_plausible(e2, (uint32_t)x2, flen);
            }
        }
        if (drop) E = NONE32;
    }
    const u64 ball = __ballot(E != NONE32);
    if (!ball) return NONE32;
    return rdl(E, __ffsll((long long)(bin ? bin : ball)) - 1);
}

template <int BM>
__device__ __forceinline__ TileRes tile_body(const DevFile& F, uint32_t t, uint32_t tt, bool first, uint32_t X_in,
                                             bool dead_in,
                                             const CLY_LDS uint8_t* smem, CLY_LDS uint32_t* stg, CLY_LDS uint32_t* mk,
                                             const CrcLane& cl, uint32_t K4, TileLocal* loc,
                                             uint32_t* rec, uint32_t* seg, uint32_t* treg,
                                             CLY_LDS uint32_t* chk, uint32_t* chunks, u32x4* sp_rec,
                                             Globals* g, u32x4 (&e)[4], u32x4& hl, const uint8_t* nbase, uint32_t nlen,
                                             uint32_t ntb) {
    const int lane = threadIdx.x & 63;
    const uint32_t tb = (uint32_t)((uint64_t)tt * CLY_TILE);
    const uint64_t flen = F.len;
    const gbytes base = (gbytes)F.base;
    // (BM_SPEC: X_in is NONE32 for a guessed entry, else the exit of the run's previous tile)
    const bool known0 = BM != BM_SPEC || first || X_in != NONE32;
    TState S;
    S.X = first ? 0u : (known0 ? X_in : NONE32);
    S.dead = !first && known0 && dead_in;
    S.cq_known = first;          // the file's first tile: no record before offset 0
    S.cq = 0; S.G = NONE32; S.tcnt = 0; S.last_crc = 0; S.P_last = NONE32; S.term = TERM_NONE;
    S.s_last = 0; S.s_prev = 0; S.Tb = NONE32; S.tpatch = 0; S.carry_next = 0; S.cmark_next = false;
    S.ref_ok = false; S.ref_s = 0; S.ref1 = S.ref2 = S.ref3 = S.msk1 = S.msk2 = S.msk3 = S.rw2 = S.rw3 = 0;
    uint32_t* ctab = chunks + (uint64_t)t * CH_WORDS;
    S.nch = 0;
    // k_scan starts the tile's chunk list; k_refix reuses the chunks k_scan took
    S.nch_have = BM == BM_SPEC ? 0u : __builtin_amdgcn_readfirstlane(ctab[CH_NWORD]);
    if (BM != BM_SPEC) {
        if ((uint32_t)lane < S.nch_have && lane < NCH_MAX) chk[lane] = ctab[lane];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    uint32_t carry = 0;          // register XOR due at this block's first byte
    bool cmark = false;          // ... a record start's patch (marked as word 0 of the block)
    uint32_t nb = 0;             // snapshots taken so far (= records whose patch word was passed)
    const rsrc_t trs = mk_rsrc(rec + (uint64_t)t * CAP_T * 4, CAP_T * 16u);      // the tile's compact entries
    const rsrc_t frs = mk_rsrc(F.base, (uint32_t)flen);
    const rsrc_t srs = mk_rsrc(seg + (uint64_t)t * NSEG, NSEG * 4u);           // segment registers
    RecSink rs;
    rs.trs = trs; rs.sp_rec = (CLY_GL u32x4*)sp_rec;
    rs.chk = chk; rs.ctab = ctab; rs.g = g;
    uint32_t Rp = 0;             // the previous block's segment register (stored at the next block's top)
    CLY_LDS u32x4* sv = (CLY_LDS u32x4*)stg;
    #pragma unroll 1
    for (int m = 0; m < CLY_NBLK; m++) {
        const uint32_t bs = tb + (uint32_t)m * CLY_BLK;
        const uint64_t bend = (uint64_t)bs + CLY_BLK;
        quad_transpose(e);
        uint32_t w[16];
        #pragma unroll
        for (int k = 0; k < 4; k++) { w[4 * k] = e[k].x; w[4 * k + 1] = e[k].y; w[4 * k + 2] = e[k].z; w[4 * k + 3] = e[k].w; }
        const u32x4 hc = hl;
        // the previous block's outputs, now that this block's loads are in
        if (m > 0)
            __builtin_amdgcn_raw_buffer_store_b32(Rp, srs, (int)(((uint32_t)(m - 1) * CLY_NL + (uint32_t)lane) * 4u), 0, 0);
        if (m + 1 < CLY_NBLK) blk_issue(base, frs, flen, bs + CLY_BLK, lane, e, hl);
        else if (m + 1 == CLY_NBLK && nbase) {                                 // the wave's next tile
            uint32_t nl = nlen, nt = ntb;
            asm volatile("" : "+s"(nl), "+s"(nt));     // (keeps its tail masks from being hoisted out of the loop)
            blk_issue((gbytes)nbase, mk_rsrc(nbase, nl), nl, nt, lane, e, hl);
        }
        mk[lane] = (lane == 0 && cmark) ? 1u : 0u;       // the block's patch words (carried: word 0)
        S.Tb = NONE32;
        const bool owned = S.X != NONE32 && ((uint64_t)S.X < bend || ((uint64_t)S.X == flen && flen == bend));
        if (S.dead) {
            #pragma unroll
            for (int k = 0; k < 16; k++) w[k] = 0;
        } else if (S.X == NONE32 || owned) {
            // ---- record starts of the block; headers are read from the wave's
            // LDS copy of it (the stage), patches XORed into the stage
            {
                // segment L, then its copy of the next segment's first 16 B (lane 63:
                // the 32 B after the block, held by lanes 0 and 1, copied and stored)
                const uint32_t t0x = rdl(hc.x, 0), t0y = rdl(hc.y, 0), t0z = rdl(hc.z, 0), t0w = rdl(hc.w, 0);
                #pragma unroll
                for (int k = 0; k < 4; k++) sv[5 * lane + k] = (u32x4){w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]};
                const u32x4 nx = (u32x4){dppu<DPP_WF_SL1>(t0x, w[0]), dppu<DPP_WF_SL1>(t0y, w[1]),
                                         dppu<DPP_WF_SL1>(t0z, w[2]), dppu<DPP_WF_SL1>(t0w, w[3])};
                sv[5 * lane + 4] = nx;
                if (lane == CLY_NL - 1) {
                    sv[5 * lane + 5] = nx;
                    sv[5 * lane + 6] = (u32x4){rdl(hc.x, 1), rdl(hc.y, 1), rdl(hc.z, 1), rdl(hc.w, 1)};
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (S.X == NONE32) S.X = guess_entry(F, bs, stg, hc, lane);    // the tile's guessed entry
            bool done = true;
            if (S.X != NONE32) {
                if (S.ref_ok) stride_round<BM>(F, S, tb, bs, stg, smem, cl, K4, rs, lane, mk);
                const uint32_t c0 = S.tcnt;
                done = pred_walk<BM>(F, S, tb, bs, stg, smem, cl, K4, rs, lane, mk);
                if (S.tcnt != c0) stride_ref(F, S, bs, stg);
            }
            if (!done) {
                // ---- general pass (the predictive walk's round budget ran out):
                // every lane's first candidate record start in its 64-B segment
                // after X, then agreement
                const Seg K = make_seg(F, bs, lane, stg);
                uint32_t wv[16];
                #pragma unroll
                for (int k = 0; k < 4; k++) {
                    const u32x4 v = sv[5 * lane + k];
                    wv[4 * k] = v.x; wv[4 * k + 1] = v.y; wv[4 * k + 2] = v.z; wv[4 * k + 3] = v.w;
                }
                const uint32_t n0 = dppu<DPP_WF_SL1>(rdl(hc.x, 0), wv[0]), n1 = dppu<DPP_WF_SL1>(rdl(hc.y, 0), wv[1]);
                u64 cm = 0;
                if (K.on) {
                    cm = cand_mask(wv, n0, n1);
                    const uint32_t nv = K.ce - K.cb;                    // valid positions
                    if (nv < 64) cm &= (1ull << nv) - 1ull;
                }
                SegChain L;
                const uint32_t X = S.X;
                if (!K.on) sc_set(L, LM_OFF);
                else if (in_seg(K, X)) seg_walk(K, X, true, L);
                else sc_set(L, LM_NONE);
                {
                    // a segment after X: the chain of its first candidate whose
                    // speculative walk holds and leaves at a candidate of the
                    // block (or beyond it), else of the first whose walk holds.
                    // A false start's walk (dense records: the bytes of a
                    // record's expiration and key read as a header) rarely
                    // leaves at a candidate; each lane it picks would cost
                    // seg_resolve a serial exact re-walk.
                    u64 mm = (K.on && X < K.cb) ? cm : 0ull;
                    bool fb = false;                               // L holds a fallback chain
                    for (int tr = 0; tr < GP_TRIES; tr++) {
                        const bool act = mm != 0ull;
                        if (!__ballot(act)) break;
                        SegChain T;
                        sc_set(T, LM_NONE);
                        bool ok = false;
                        if (act) {
                            const uint32_t q = K.cb + (uint32_t)__builtin_ctzll(mm);
                            mm &= mm - 1;
                            ok = seg_walk(K, q, false, T);
                        }
                        const bool chk = ok && T.term == TERM_NONE && T.x < bs + CLY_BLK;
                        const uint32_t off = chk ? T.x - bs : 0u;
                        const int tl = (int)(off >> 6);
                        const uint32_t clo = shfl_u32((uint32_t)cm, tl), chi = shfl_u32((uint32_t)(cm >> 32), tl);
                        bool conf = ok;
                        if (chk) {
                            const uint32_t bb = off & 63u;
                            conf = ((bb < 32 ? clo >> bb : chi >> (bb - 32)) & 1u) != 0;
                        }
                        if (conf) { L = T; mm = 0; }
                        else if (ok && !fb) { L = T; fb = true; }
                    }
                }
                {
                    L = seg_resolve(K, L, lane, X, g);
                    // the first terminal ends the chain: the lanes after it are dead
                    const u64 bt = __ballot(L.mode == LM_CHAIN && L.term != TERM_NONE);
                    const int kT = bt ? __ffsll((long long)bt) - 1 : 64;
                    if (lane > kT && L.mode != LM_OFF) sc_set(L, LM_DEAD);
                    const bool isC = L.mode == LM_CHAIN;
                    const uint32_t c = isC ? L.cnt : 0u;
                    const uint32_t incl = wave_add_incl(c);
                    const uint32_t bcnt = rdl(incl, 63), lex = incl - c;
                    // the stored CRC of the record before the lane's first one
                    uint32_t lv = L.last_crc, lf = c > 0 ? 1u : 0u;
                    wave_last_incl(lv, lf);
                    const uint32_t lvp = dppu<DPP_WF_SR1>(0u, lv), lfp = dppu<DPP_WF_SR1>(0u, lf);
                    // (the stored CRC before the terminal: the lane's last record's, or inherited)
                    const uint32_t pcq = c > 0 ? L.last_crc : (lfp ? lvp : S.cq);
                    const bool pk = c > 0 || lfp || S.cq_known;
                    // the block's records, record-parallel: record r (in chain order) by
                    // lane r % 64 of round r / 64: its segment is the lane whose records
                    // [lex, incl) hold r, its start that lane's (r - lex)-th start bit;
                    // outputs, patch-word marks (headers from the stage), entries
                    // stored as consecutive 16-B slots.  The owners of a round without
                    // a search over the lanes: each lane with records in the round
                    // sets the bit of its first one (distinct bits, so a wave sum
                    // is their OR); record r's owner is the lane of the last set bit
                    // at or before r, the j-th lane with records in the round.
                    bool cf = false;
                    uint32_t sz_last = 0, sz_prev = 0;
                    spill_ensure(S, S.tcnt + bcnt, rs, lane);
                    for (uint32_t r0 = 0; r0 < bcnt; r0 += 64) {
                        const uint32_t r = r0 + (uint32_t)lane;
                        const bool isec = c > 0 && incl > r0 && lex < r0 + 64u;
                        const uint32_t sb = lex > r0 ? lex - r0 : 0u;
                        const uint32_t blo = wave_add_incl(isec && sb < 32u ? 1u << sb : 0u);
                        const uint32_t bhi = wave_add_incl(isec && sb >= 32u ? 1u << (sb - 32u) : 0u);
                        const u64 B = ((u64)rdl(bhi, 63) << 32) | rdl(blo, 63);
                        const u64 mi = __ballot(isec);
                        const u64 Bm = B & ((2ull << lane) - 1ull);              // (lane 63: every bit)
                        const uint32_t j = (uint32_t)__popcll(Bm), hb = 63u - (uint32_t)__clzll((long long)Bm);
                        uint32_t own = kth_bit((uint32_t)mi, (uint32_t)(mi >> 32), j - 1u);
                        own = own > 63u ? 63u : own;
                        // the round's first record may continue a lane's records of the round before
                        const uint32_t d0 = rdl(r0 > lex ? r0 - lex : 0u, __ffsll((long long)mi) - 1);
                        const uint32_t k = (uint32_t)lane - hb + (hb == 0u ? d0 : 0u);
                        const uint32_t m0 = shfl_u32(L.sm0, (int)own), m1 = shfl_u32(L.sm1, (int)own);
                        uint32_t sz = 0;
                        if (r < bcnt) {
                            const uint32_t p = bs + 64u * own + kth_bit(m0, m1, k);
                            const Hdr h = hdr_get(p, flen, stg, bs);
                            const uint32_t pw = rec_out(p, h, S.tcnt + r, tb, bs, rs);
                            if (pw == PW_CARRY) cf = true; else mark_pw(mk, pw);
                            sz = (uint32_t)h.size;
                        }
                        if (bcnt - 1u - r0 < 64u) sz_last = rdl(sz, (int)(bcnt - 1u - r0));
                        if (bcnt >= 2u && bcnt - 2u - r0 < 64u) sz_prev = rdl(sz, (int)(bcnt - 2u - r0));
                    }
                    if (__ballot(cf)) S.cmark_next = true;
                    if (kT < 64) {
                        const uint32_t T = rdl(L.x, kT);
                        const uint32_t dT = T == 0 ? 0u : (pk ? ~pcq : 0xFFFFFFFFu);
                        term_patch<BM>(S, T, dT, bs, smem, cl, kT);
                    }
                    // the chain after the block
                    if (bcnt) {
                        const u64 br = __ballot(c > 0);
                        const int lr = 63 - __clzll((long long)br);
                        S.last_crc = rdl(L.last_crc, lr);
                        S.P_last = rdl(L.last, lr);
                        S.cq = S.last_crc; S.cq_known = true;
                        // sizes of the last two records (0 for the one before when it is in an earlier lane)
                        const uint32_t cl_ = rdl(c, lr);
                        S.s_last = sz_last;
                        S.s_prev = cl_ >= 2 ? sz_prev : (bcnt >= 2 ? 0u : S.s_last);
                    }
                    S.tcnt += bcnt;
                    const u64 bcc = __ballot(isC);
                    if (bcc) {
                        if (S.G == NONE32) S.G = rdl(L.E, __ffsll((long long)bcc) - 1);
                        S.X = rdl(L.x, 63 - __clzll((long long)bcc));
                        if (bt) { S.dead = true; S.term = (int)rdl((uint32_t)L.term, kT); }
                    }
                }
            }
        }
        {
            // bytes from the terminal on read as zero
            if (S.Tb != NONE32) {
                const uint32_t cb = bs + 64u * (uint32_t)lane, T = S.Tb;
                #pragma unroll
                for (int k = 0; k < 16; k++) {
                    const uint32_t a = cb + 4u * k;
                    if (a >= T) w[k] = 0;
                    else if (a + 4 > T) w[k] &= (1u << (8 * (T - a))) - 1u;
                }
                if ((uint64_t)T < bend) {
                    const uint32_t wi = ((T & ~3u) - bs) >> 2;
                    if ((uint32_t)lane == (wi >> 4)) patch_word(w, wi & 15u, S.tpatch);
                }
            }
            if (lane == 0) w[0] ^= carry;
            // the segment's register from zero; w[k] becomes the register entering word k
            uint32_t R = 0;
            #pragma unroll
            for (int k = 0; k < 16; k++) { const uint32_t x = R; R = crc_word(smem, R ^ w[k], cl); w[k] = x; }
            Rp = R;
            // snapshots: the registers entering the marked words, in position
            // order = record order (one patch word per record start), through
            // the stage (the block's bytes there are no longer needed)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint32_t mm = mk[lane];
            if (__ballot(mm != 0u)) {
                #pragma unroll
                for (int k = 0; k < 4; k++) sv[5 * lane + k] = (u32x4){w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]};
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const uint32_t c = (uint32_t)__builtin_popcount(mm), incl = wave_add_incl(c);
                uint32_t r = nb + incl - c, q = mm;
                nb += rdl(incl, 63);
                while (__ballot(q != 0u)) {
                    if (q) {
                        const uint32_t k = (uint32_t)__builtin_ctz(q);
                        q &= q - 1u;
                        snap_put(rs, r, stg[20u * (uint32_t)lane + k]);
                        r++;
                    }
                }
            }
            carry = S.carry_next; cmark = S.cmark_next;
            S.carry_next = 0; S.cmark_next = false;
        }
    }
    TileRes res;
    res.X = S.X; res.dead = S.dead;
    __builtin_amdgcn_raw_buffer_store_b32(Rp, srs, (int)(((uint32_t)(CLY_NBLK - 1) * CLY_NL + (uint32_t)lane) * 4u), 0, 0);
    // a record start whose patch word is the tile's end: its snapshot is
    // the (empty) segment after the tile's, zero; the patch itself is the
    // register XOR due at the tile end
    if (cmark && lane == 0) snap_put(rs, nb, 0u);
    if (lane == 0) {
        ctab[CH_NWORD] = S.nch_have;
        treg[2 * t] = carry;
        if (nb + (cmark ? 1u : 0u) != S.tcnt) atomicOr(&g->fail, 64u);      // one snapshot per record
        const uint64_t tstart = tb;
        const uint32_t tend = tstart + CLY_TILE >= flen ? (uint32_t)(flen + 1) : (uint32_t)(tstart + CLY_TILE);
        u64 f0 = (u64)S.tcnt << 32;
        if (S.term != TERM_NONE) f0 |= DF_TERM;
        if (S.G == NONE32) f0 |= DF_NONE;
        if (first) f0 |= DF_FOF;
        if (S.P_last != NONE32) f0 |= DF_REC;
        TileLocal* d = &loc[t];
        d->l[0] = f0;
        d->l[1] = (u64)S.G | ((u64)S.X << 32);
        d->l[2] = (u64)S.last_crc | ((u64)S.P_last << 32);
        d->l[3] = (u64)tend | ((u64)(uint8_t)(int8_t)S.term << 32);
    }
    return res;
}

// ---------------------------------------------------------------------------
// Kernels of one call.
// the wave's index in its workgroup, as a wave-uniform (SGPR) value: tile
// indices, file descriptors and buffer resources derived from it stay scalar
__device__ __forceinline__ uint32_t wave_id() { return (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }
__device__ __forceinline__ int find_file(const uint32_t* __restrict__ tprefix, int nfiles, uint32_t t) {
    int lo = 0, hi = nfiles - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (tprefix[mid] <= t) lo = mid; else hi = mid - 1;
    }
    return lo;
}
#define CLY_K4 0x9226F562u        // A^-4 0xFFFFFFFF (k4_const)
__device__ __forceinline__ uint32_t k4_const(const CLY_LDS uint8_t* smem, uint32_t r4) {
    uint32_t K4 = 0xFFFFFFFFu;              // A^-4 0xFFFFFFFF
    for (int k = 0; k < 4; k++) K4 = crc_unbyte(smem, K4, r4);
    return K4;
}

// k_scan: one wave per run of run_tiles tiles, every byte of every file read
// once.  Three quarters of the runs are grid-strided, the last quarter claimed
// one at a time from a call-wide counter (runs of dense small records cost
// several times the others: with a fixed stride throughout, C3's slowest waves
// ended 15-20 % after the mean; claiming every run cost C2 1-3 %).
#define SCAN_WAVES 16
#define MK_BYTES (CLY_NL * 4)                                 // a wave's patch-word mask
#define CHK_BYTES (CH_WORDS * 4)                              // a wave's copy of its tile's spill chunk ids
#define SCAN_LDS_ALL (SCAN_LDS + SCAN_WAVES * (STG_BYTES + MK_BYTES + CHK_BYTES))   // tables + per wave a stage, a mask, chunk ids
static_assert(SCAN_LDS_ALL <= 160 * 1024, "k_scan's LDS");
__device__ __forceinline__ CLY_LDS uint32_t* wave_stage(CLY_LDS uint8_t* smem) {
    return (CLY_LDS uint32_t*)(smem + SCAN_LDS + wave_id() * STG_BYTES);
}
__device__ __forceinline__ CLY_LDS uint32_t* wave_mask(CLY_LDS uint8_t* smem) {
    return (CLY_LDS uint32_t*)(smem + SCAN_LDS + SCAN_WAVES * STG_BYTES + wave_id() * MK_BYTES);
}
__device__ __forceinline__ CLY_LDS uint32_t* wave_chk(CLY_LDS uint8_t* smem) {
    return (CLY_LDS uint32_t*)(smem + SCAN_LDS + SCAN_WAVES * (STG_BYTES + MK_BYTES) + wave_id() * CHK_BYTES);
}
__global__ void __launch_bounds__(64 * SCAN_WAVES)
k_scan(const DevFile* __restrict__ files, int nfiles, const uint32_t* __restrict__ rprefix, uint32_t nruns,
       TileLocal* loc, uint32_t* rec, uint32_t* seg, uint32_t* treg, uint32_t* chunks, u32x4* sp_rec, Globals* g) {
    __shared__ __attribute__((aligned(16))) unsigned char smem_raw[SCAN_LDS_ALL];
    CLY_LDS uint8_t* smem = (CLY_LDS uint8_t*)smem_raw;
    init_tables(smem);
    CLY_LDS uint32_t* stg = wave_stage(smem);
    CLY_LDS uint32_t* mk = wave_mask(smem);
    CLY_LDS uint32_t* chk = wave_chk(smem);
    const int lane = threadIdx.x & 63;
    const CrcLane cl = crc_lane(lane);
    const uint32_t K4 = k4_const(smem, cl.r4);
    const uint32_t slots = gridDim.x * SCAN_WAVES;
    // runs of run_tiles consecutive tiles of a file; a run's first tile (not
    // its file's first) guesses its entry, the others take the exit of the
    // tile before them.  Runs [0, nstat) are grid-strided (three quarters of
    // them, whole rounds of the grid); the rest are claimed one at a time: a
    // wave whose next run is a claimed one issues the claim (rq) as its
    // current run starts and reads it when that run's last tile starts
    uint32_t r = blockIdx.x * SCAN_WAVES + wave_id();
    if (r >= nruns) return;
    const uint32_t nstat = max(slots, (nruns - nruns / 4) / slots * slots);   // (the first round is always static)
    uint32_t rq = 0;
    if (r + slots >= nstat && lane == 0) rq = atomicAdd(&g->run_next, 1u);
    const uint32_t rt = __builtin_amdgcn_readfirstlane(g->run_tiles);
    int f = find_file(rprefix, nfiles, r);
    uint32_t t = files[f].first_tile + (r - rprefix[f]) * rt;
    u32x4 e[4], hl;
    {
        uint32_t ptt;
        const DevFile V = part_view(files[f], t - files[f].first_tile, ptt);
        tile_issue(V, ptt, lane, e, hl);
    }
    uint32_t Xc = NONE32;        // the entry carried from the run's previous tile (NONE32: guess)
    bool bad_run = false;
    for (;;) {
        const DevFile F = files[f];
        const uint32_t rend = min(F.first_tile + (r - rprefix[f] + 1u) * rt, F.first_tile + F.ntile);
        // the wave's next tile: the next of this run, else the first of its next run
        uint32_t tn = t + 1u, rn = r;
        int fn = f;
        if (tn >= rend) {
            rn = r + slots < nstat ? r + slots : nstat + (uint32_t)__builtin_amdgcn_readfirstlane((int)rq);
            if (rn <= r) { bad_run = true; rn = nruns; }   // (runs only increase: never; fails the call)
            fn = rn < nruns ? find_file(rprefix, nfiles, rn) : -1;
            if (fn >= 0) tn = files[fn].first_tile + (rn - rprefix[fn]) * rt;
        }
        const uint8_t* nbase = nullptr;
        uint32_t nlen = 0, ntb = 0;
        if (fn >= 0) {
            uint32_t pn;
            const DevFile Vn = part_view(files[fn], tn - files[fn].first_tile, pn);
            nbase = Vn.base; nlen = (uint32_t)Vn.len;
            ntb = pn * (uint32_t)CLY_TILE;
        }
        uint32_t ptt;
        const DevFile V = part_view(F, t - F.first_tile, ptt);
        const TileRes res = tile_body<BM_SPEC>(V, t, ptt, t == F.first_tile, Xc, false, smem, stg, mk, cl, K4, loc, rec,
                                               seg, treg, chk, chunks, sp_rec, g, e, hl, nbase, nlen, ntb);
        if (fn < 0) break;
        // a chain that ended in this tile is not carried: past the file's true
        // end nothing reads the tiles, and a false chain's terminal must not
        // zero the next tile's bytes for the CRC (k_link need not contradict a
        // tile the true chain only passes through), so the next tile guesses
        if (rn == r && !res.dead) Xc = res.X;
        else Xc = NONE32;
        if (rn != r) {
            r = (uint32_t)__builtin_amdgcn_readfirstlane((int)rn);
            if (r + slots >= nstat && lane == 0) rq = atomicAdd(&g->run_next, 1u);
        }
        t = tn; f = fn;
    }
    if (bad_run && lane == 0) atomicOr(&g->fail, 256u);
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
// tile without boundaries entered live at X < its end, is contradicted.  A
// contradicted tile whose predecessor is not contradicted is listed for
// k_refix (its entry X is the predecessor's own exit; a wrong guess rarely
// spoils more than its own tile).  The workgroup that finishes last also
// computes every file's first tuple index (exclusive prefix over the files'
// record totals) and the call's total.
#define LINK_NT 1024
#define LINK_MAXT 131072         // tiles per file whose contradiction / anchor bitmasks fit LDS (8-GiB files);
                                 // a longer file's are in global memory (lmask, words first_tile / 32 + f on)
#define RF_ID 0
#define RF_CONST 1
#define RF_FOF 2
#define RF_DEAD 4u
#define RF_REC 8u
// a run of tiles as a function of the state entering it; positions are file
// offsets (a tile's LOCAL positions are its part's: x0 added)
struct RunF { uint64_t X, P, cnt; uint32_t crc, fl; };   // fl: kind | RF_DEAD | RF_REC
__device__ __forceinline__ RunF rf_tile(u64 l0, u64 l1, u64 l2, uint64_t x0) {
    RunF f;
    const uint32_t kind = (l0 & DF_FOF) ? RF_FOF : (l0 & DF_NONE) ? RF_ID : RF_CONST;
    f.X = x0 + (l1 >> 32);
    f.cnt = l0 >> 32;
    f.fl = kind | ((l0 & DF_TERM) ? RF_DEAD : 0u) | (((l0 & DF_REC) || (l0 & DF_FOF)) ? RF_REC : 0u);
    f.crc = (l0 & DF_REC) ? (uint32_t)l2 : 0u;
    f.P = (l0 & DF_REC) ? x0 + (l2 >> 32) : P_NONE;
    return f;
}
// g after f
__device__ __forceinline__ RunF rf_then(const RunF& f, const RunF& g) {
    const uint32_t fk = f.fl & 3u, gk = g.fl & 3u;
    if (gk == RF_FOF || fk == RF_ID) return g;
    if (gk == RF_ID || (f.fl & RF_DEAD)) return f;
    RunF h = f;
    h.X = g.X; h.cnt = f.cnt + g.cnt;
    h.fl = (f.fl & ~RF_DEAD) | (g.fl & RF_DEAD);
    if (g.fl & RF_REC) { h.crc = g.crc; h.P = g.P; h.fl |= RF_REC; }
    return h;
}
__device__ __forceinline__ LBState rf_apply(const RunF& f, LBState s) {
    const uint32_t fk = f.fl & 3u;
    if (fk == RF_ID || (fk == RF_CONST && s.dead)) return s;
    s.count = (fk == RF_FOF ? 0 : s.count) + f.cnt;
    s.X = f.X; s.dead = (f.fl & RF_DEAD) != 0;
    if (f.fl & RF_REC) { s.crc_last = f.crc; s.P_last = f.P; }
    return s;
}
#define LINK_PER 4               // tiles per thread held in registers (more: re-read)
__global__ void __launch_bounds__(LINK_NT)
k_link(const DevFile* __restrict__ files, int nfiles, const TileLocal* __restrict__ loc, TileIn* tin,
       uint64_t* ftotal, FileInfo* finfo, uint32_t* fixlist, uint32_t* lmask, uint64_t lmask_words, Globals* g,
       int slot, int guard) {
    if (guard >= 0 && g->nfix[guard] == 0) return;  // (device round: nothing was re-resolved)
    __shared__ RunF rf[2][LINK_NT];
    __shared__ uint32_t badm_l[LINK_MAXT / 32];
    __shared__ uint32_t ancm_l[LINK_MAXT / 32];  // anchors: a run's first tile with a boundary, not contradicted
    __shared__ uint64_t part[LINK_NT];
    __shared__ uint64_t carry;
    __shared__ int last;
    const int f = blockIdx.x, tid = threadIdx.x;
    const DevFile F = files[f];
    const uint32_t rt = g->run_tiles;        // k_scan's run length (a run's first tile guessed its entry)
    const uint32_t nt = F.ntile, per = (nt + LINK_NT - 1) / LINK_NT;
    const uint32_t lo = tid * per < nt ? tid * per : nt, hi = lo + per < nt ? lo + per : nt;
    const TileLocal* L0 = loc + F.first_tile;
    // the bitmasks: LDS, or for a file of more than LINK_MAXT tiles its words of
    // lmask (generic pointers either way; reads of lmask bypass the L1)
    const uint32_t nw = (nt + 31) / 32;
    const bool far = nt > LINK_MAXT;
    uint32_t* badm = far ? lmask + F.first_tile / 32 + (uint32_t)f : (uint32_t*)badm_l;
    uint32_t* ancm = far ? lmask + lmask_words + F.first_tile / 32 + (uint32_t)f : (uint32_t*)ancm_l;
    auto bit = [](const uint32_t* m, uint32_t u) {
        return (__hip_atomic_load(m + (u >> 5), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> (u & 31)) & 1u;
    };
    u64 c0[LINK_PER], c1[LINK_PER], c2[LINK_PER], c3[LINK_PER];
    #pragma unroll
    for (int k = 0; k < LINK_PER; k++) {
        c0[k] = c1[k] = c2[k] = c3[k] = 0;
        if (lo + k < hi) { c0[k] = L0[lo + k].l[0]; c1[k] = L0[lo + k].l[1]; c2[k] = L0[lo + k].l[2]; c3[k] = L0[lo + k].l[3]; }
    }
    RunF my;
    my.fl = RF_ID; my.X = 0; my.crc = 0; my.P = P_NONE; my.cnt = 0;
    #pragma unroll
    for (int k = 0; k < LINK_PER; k++)
        if (lo + k < hi) my = rf_then(my, rf_tile(c0[k], c1[k], c2[k], part_x0(lo + k)));
    for (uint32_t u = lo + LINK_PER; u < hi; u++) my = rf_then(my, rf_tile(L0[u].l[0], L0[u].l[1], L0[u].l[2], part_x0(u)));
    // inclusive Kogge-Stone scan of the run functions
    int cur = 0;
    rf[0][tid] = my;
    for (uint32_t i = tid; i < (far ? nw : (uint32_t)(LINK_MAXT / 32)); i += LINK_NT) {
        __hip_atomic_store(badm + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ancm + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (far) __threadfence();
    __syncthreads();
    for (int d = 1; d < LINK_NT; d <<= 1) {
        RunF v = rf[cur][tid];
        if (tid >= d) v = rf_then(rf[cur][tid - d], v);
        rf[cur ^ 1][tid] = v;
        cur ^= 1;
        __syncthreads();
    }
    LBState s;
    s.count = 0; s.X = 0; s.crc_last = 0; s.P_last = P_NONE; s.dead = 0;
    if (tid > 0) s = rf_apply(rf[cur][tid - 1], s);
    if (tid == LINK_NT - 1) {
        LBState s0;
        s0.count = 0; s0.X = 0; s0.crc_last = 0; s0.P_last = P_NONE; s0.dead = 0;
        ftotal[f] = rf_apply(rf[cur][tid], s0).count;
    }
    auto visit = [&](uint32_t u, u64 l0, u64 l1, u64 l2, u64 l3) {
        bool bad = false;
        const uint64_t x0 = part_x0(u);
        if (l0 & DF_FOF) { s.count = 0; s.X = 0; s.dead = 0; s.crc_last = 0; s.P_last = P_NONE; }
        else if (!s.dead) {
            if (l0 & DF_NONE) bad = s.X < x0 + (uint32_t)l3;
            else bad = s.X != x0 + (uint32_t)l1;
        }
        ti_store(&tin[F.first_tile + u], s, (uint32_t)f);
        if (bad) atomicOr(&badm[u >> 5], 1u << (u & 31));
        else if (u == 0 || (u % rt == 0 && !(l0 & DF_NONE))) atomicOr(&ancm[u >> 5], 1u << (u & 31));
        s = rf_apply(rf_tile(l0, l1, l2, x0), s);
    };
    #pragma unroll
    for (int k = 0; k < LINK_PER; k++)
        if (lo + k < hi) visit(lo + k, c0[k], c1[k], c2[k], c3[k]);
    for (uint32_t u = lo + LINK_PER; u < hi; u++) visit(u, L0[u].l[0], L0[u].l[1], L0[u].l[2], L0[u].l[3]);
    if (far) __threadfence();
    __syncthreads();
    // list a contradicted tile only when no contradicted tile lies between it
    // and the anchor before it (the state entering it then comes from tiles
    // whose chains are right; a tile that carried a wrong exit, or passed one
    // through without a boundary, would enter it with a false state and send
    // its walk down a false chain)
    for (uint32_t u = lo; u < hi; u++) {
        const bool bu = bit(badm, u);
        bool bp = false;
        if (bu && u > 0) {
            for (uint32_t v = u - 1;; v--) {
                if (bit(badm, v)) { bp = true; break; }
                if (v == 0 || bit(ancm, v)) break;
            }
        }
        if (bu && !bp) {
            const uint32_t k = atomicAdd(&g->nfix[slot], 1u);
            fixlist[k] = F.first_tile + u;
            tin[F.first_tile + u].w[3] |= TI_FIX;
        }
    }
    // the workgroup that finishes last: the file bases (its acquire sees every
    // workgroup's ftotal: each released it before its arrival)
    __syncthreads();
    if (tid == LINK_NT - 1) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last = atomicAdd(&g->link_done, 1u) == (uint32_t)gridDim.x - 1;
        if (last) { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent"); asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
        carry = 0;
    }
    __syncthreads();
    if (!last) return;
    for (int b = 0; b < nfiles; b += LINK_NT) {
        const int i = b + tid;
        const uint64_t v = i < nfiles ? __hip_atomic_load(&ftotal[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
        part[tid] = v;
        __syncthreads();
        for (int d = 1; d < LINK_NT; d <<= 1) {
            const uint64_t o = tid >= d ? part[tid - d] : 0;
            __syncthreads();
            part[tid] += o;
            __syncthreads();
        }
        if (i < nfiles) finfo[i].first_index = carry + part[tid] - v;
        __syncthreads();
        if (tid == 0) carry += part[LINK_NT - 1];
        __syncthreads();
    }
    if (tid == 0) { g->total = carry; g->link_done = 0; }
}

#define REFIX_GRID 64             // workgroups of the device repair round (16 listed tiles each)
// k_refix: one wave per listed tile: the tile body again from the entering
// state k_link gave it (new LOCAL, compact entries, register).  Walks on into
// the next tile of the file while that one's LOCAL disagrees with the new exit
// (and is not listed itself).
__global__ void __launch_bounds__(64 * SCAN_WAVES)
k_refix(const DevFile* __restrict__ files, int nfiles, const uint32_t* __restrict__ tprefix, TileLocal* loc,
        const TileIn* __restrict__ tin, uint32_t* rec, uint32_t* seg, uint32_t* treg,
        uint32_t* chunks, u32x4* sp_rec, const uint32_t* __restrict__ fixlist, Globals* g, int slot) {
    if (g->nfix[slot] == 0) return;                        // (uniform: before the LDS setup's barrier)
    __shared__ __attribute__((aligned(16))) unsigned char smem_raw[SCAN_LDS_ALL];
    CLY_LDS uint8_t* smem = (CLY_LDS uint8_t*)smem_raw;
    init_tables(smem);
    CLY_LDS uint32_t* stg = wave_stage(smem);
    CLY_LDS uint32_t* mk = wave_mask(smem);
    CLY_LDS uint32_t* chk = wave_chk(smem);
    const uint32_t k = blockIdx.x * SCAN_WAVES + wave_id();
    if (k >= g->nfix[slot]) return;
    const int lane = threadIdx.x & 63;
    const CrcLane cl = crc_lane(lane);
    const uint32_t K4 = k4_const(smem, cl.r4);
    uint32_t t = fixlist[k];
    const int f = find_file(tprefix, nfiles, t);
    const DevFile F = files[f];
    // a run of listed tiles is walked by the wave of its first one: the
    // entry of a later one is the walk's exit, not its stale TileIn
    if (t > F.first_tile && (tin[t - 1].w[3] & TI_FIX)) return;
    const LBState S0 = ti_load(&tin[t]);
    bool dead = S0.dead != 0;
    // X: the chain position in the current tile's part
    uint32_t X = dead ? 0u : (uint32_t)(S0.X - part_x0(t - F.first_tile));
    const uint32_t t_start = t;
    for (;;) {
        // Suffix: the true entry is the start of the guessed chain's record j
        // (a false start that runs into the true chain).  The chain from there
        // on is the tile's own: drop the first j records (count, entry; k_emit
        // skips their compact entries and snapshots) instead of walking the
        // tile again; its exit stays.
        const u64 l0 = loc[t].l[0], l1 = loc[t].l[1];
        uint32_t ptt;
        const DevFile V = part_view(F, t - F.first_tile, ptt);
        const uint32_t n = (uint32_t)(l0 >> 32), tb = ptt * (uint32_t)CLY_TILE;
        bool shortcut = false;
        if (!dead && !(l0 & (DF_NONE | DF_FOF)) && n > 1 && ((loc[t].l[3] >> 40) & 0xFFFFu) == 0) {
            const uint32_t nn = n < 64u ? n : 64u;
            const uint32_t rel = (uint32_t)lane < nn ? (rec[((uint64_t)t * CAP_T + lane) * 4 + 3] & 0xFFFFu) : 0u;
            const u64 bm = __ballot(lane >= 1 && (uint32_t)lane < nn && tb + rel == X);
            if (bm) {
                const uint32_t j = (uint32_t)__ffsll((long long)bm) - 1;
                if (lane == 0) {
                    loc[t].l[0] = (l0 & 0xFFFFFFFFull) | ((u64)(n - j) << 32);
                    loc[t].l[1] = (u64)X | (l1 & 0xFFFFFFFF00000000ull);
                    loc[t].l[3] |= (u64)j << 40;
                }
                X = (uint32_t)(l1 >> 32);
                dead = (l0 & DF_TERM) != 0;
                shortcut = true;
            }
        }
        if (!shortcut) {
            u32x4 e[4], hl;
            tile_issue(V, ptt, lane, e, hl);
            const TileRes r = tile_body<BM_EXACT>(V, t, ptt, t == F.first_tile, X, dead, smem, stg, mk, cl, K4, loc,
                                                  rec, seg, treg, chk, chunks, sp_rec, g, e, hl,
                                                  nullptr, 0u, 0u);
            X = r.X; dead = r.dead;
        }
        if (dead || t + 1 >= F.first_tile + F.ntile) break;
        // a listed next tile whose predecessor is not listed has a wave of its
        // own (it starts a run); any other next tile: consistent with the new
        // exit?  else it is re-resolved here too
        if ((tin[t + 1].w[3] & TI_FIX) && !(tin[t].w[3] & TI_FIX)) break;
        if (ptt + 1 == PART_TILES) X -= (uint32_t)PART_BYTES;           // into the next part
        const u64 n0 = loc[t + 1].l[0], n1 = loc[t + 1].l[1], n3 = loc[t + 1].l[3];
        const bool ok = (n0 & DF_NONE) ? X >= (uint32_t)n3 : X == (uint32_t)n1;
        if (ok) break;
        t++;
    }
    if (lane == 0) {
        atomicMax(&g->walk_max, t - t_start + 1u);
        atomicMax((unsigned long long*)&g->walk_dbg, ((u64)(t - t_start + 1u) << 32) | t_start);
    }
}

// k_emit: per tile (one wave, grid-stride), after the chain is final: the
// tuples from the compact entries (64 per round: coalesced 16-B reads, the 48-B
// tuples assembled in the wave's LDS and written as whole 1-KiB runs), and the
// tile's CRC verdicts from its segment registers (loaded into LDS) and the
// records' snapshots.
//   The reset at a record start P (patch word W, stored CRC c): the register
//   entering W as the walk restarts at P is exp_post(P) (c ^ K4 at P, then the
//   4 - j bytes of c up to W), so XORing v = snapshot ^ exp_post into the
//   segment's own register at W gives the stream's register from there on.
//   Record r is checked from its own segments alone: the reset exit of the
//   segment holding W_r, Horner steps x -> A^64 x ^ S over the segments up to
//   the one holding W_{r+1}, then A^(W_{r+1} - segment start) x ^ snapshot
//   must equal exp_pre(P_{r+1}) = the register a matching record leaves there
//   (~c_r at P_{r+1}, then the 4 - j bytes of c_{r+1}; data/dataFile.go:
//   105-109).  The record that ends at the chain's terminal matches iff the
//   register is zero at the end of the terminal's segment (k_scan closed it
//   there).  The record that crosses into the tile is k_fin's, which knows the
//   register entering the tile: the tile gives it its own register entering
//   its first patch word (dev, with exp_pre folded in).
//   Tiles of long records (one spanning more than SHORT_KMAX segments) or
//   without a record start take the tile-wide scan instead: every segment whose last boundary is a record
//   start gets its reset exit (a constant), lane L owns the run of RUN
//   consecutive segments at L RUN_BYTES; a Horner pass gives each run as a
//   function of the register entering it, a Kogge-Stone scan over the lanes
//   composes them, a second Horner pass gives the register entering every
//   segment (gin), and every record is checked from gin.
//   Outputs per tile for k_fin: the register at the tile's end (a tile with a
//   record start: past its last reset; a tile without one: its own, from
//   zero) and dev.
#define RUN (CLY_NBLK)                          // segments per lane in k_emit's scan
#define RUN_BYTES (RUN * CLY_SEG)
#define EMIT_WAVES 8
#define SHORT_KMAX 32                           // segments one record may span there
#define GIN_WORDS (NSEG + 4)                    // segment registers / the scan (+ the tile's end)
#define FLG_BYTES (NSEG / 8)                    // segments that hold a reset (tile-wide scan)
#define TUP_BYTES (64 * 48)                     // a round's tuples (stored as contiguous 1-KiB runs)
#define EW_BYTES ((GIN_WORDS * 4 + FLG_BYTES + TUP_BYTES + 15) & ~15)
#define EMIT_KJ (NEM * 128)                    // kj[4] after the tables (words)
#define EMIT_LDS (NEM * 128 * 4 + 16 + 4096 + EMIT_WAVES * EW_BYTES)
static_assert(CLY_NL * RUN == NSEG, "one run of segments per lane");
static_assert(RUN <= 16, "gin_true's A^(64 j) from A^64 .. A^512");
// LDS word of segment sg: plain (the per-record path: neighbouring records'
// segments in different banks) or lane-transposed (the tile-wide scan: lane
// L's run of RUN segments in one bank column)
__device__ __forceinline__ uint32_t gin_at(uint32_t sg, bool plain) {
    return sg < NSEG ? (plain ? sg : (sg % RUN) * 64u + sg / RUN) : NSEG;
}
// A^(4k) v, 0 <= k <= 16 (k = 16: the segment step A^64)
__device__ __forceinline__ uint32_t em_f4(const CLY_LDS uint32_t* emt, uint32_t k, uint32_t v) {
    return k ? mat_mul(emt + (EM_F4 + k - 1u) * 128u, v) : v;
}
__device__ __forceinline__ uint32_t em_a64(const CLY_LDS uint32_t* emt, uint32_t v) {
    return mat_mul(emt + (EM_F4 + 15) * 128, v);
}
// A^64 v by byte tables (4 lookups; k_emit keeps them after the nibble tables)
#define EMIT_A64B (NEM * 128 + 4)                       // words: after the nibble tables and kj
__device__ __forceinline__ uint32_t em_a64b(const CLY_LDS uint32_t* emt, uint32_t v) {
    const CLY_LDS uint32_t* bt = emt + EMIT_A64B;
    return __builtin_amdgcn_bitop3_b32(bt[v & 255u], bt[256 + ((v >> 8) & 255u)], bt[512 + ((v >> 16) & 255u)], 0x96) ^
           bt[768 + (v >> 24)];
}
// A^(4-j) v, 1 <= j <= 3
__device__ __forceinline__ uint32_t em_fj(const CLY_LDS uint32_t* emt, uint32_t j, uint32_t v) {
    return mat_mul(emt + (EM_F1 + 3u - j) * 128u, v);
}
// The register entering the patch word of a record start P (j = P & 3) when
// the record before it (stored CRC cq) matches: ~cq at P, then for j != 0 the
// 4 - j first bytes of the new record's stored CRC c in the same word.
__device__ __forceinline__ uint32_t exp_pre(const CLY_LDS uint32_t* emt, uint32_t j, uint32_t cq, uint32_t c) {
    return j ? em_fj(emt, j, ~cq ^ (c & ((1u << (8u * (4u - j))) - 1u))) : ~cq;
}
// The register entering the patch word of a record start P (stored CRC c) as
// the walk restarts at P: c ^ K4 at P; for j != 0 the 4 - j bytes of c up to
// the word boundary, A^(4-j) (c ^ K4 ^ (c's low bytes)) = (c >> 8 (4-j)) ^
// A^(4-j) K4 (kj[j], in LDS: a lane-indexed register array would live in scratch).
__device__ __forceinline__ uint32_t exp_post(uint32_t j, uint32_t c, const CLY_LDS uint32_t* kj) {
    return (j ? c >> (8u * (4u - j)) : c) ^ kj[j];
}
__device__ __forceinline__ uint32_t entry_crc(gbytes base, uint64_t len, uint32_t tb, const u32x4& v) {
    return (v.w & REC_SHORT) ? v.x : hdr_load(base, tb + (v.w & 0xFFFFu), len).crc;
}
__device__ __forceinline__ uint32_t patch_word_of(uint32_t P) { return (P & 3u) ? (P & ~3u) + 4u : P; }
// A tile's compact entries and snapshots as k_emit reads them: index i (after
// k_refix's suffix skip) in the tile's own area below CAP_T, else in its spill
// chunks
struct EntSrc {
    const u32x4* tile;
    const u32x4* sp_rec; const uint32_t* ctab;
    uint32_t skip;
    __device__ __forceinline__ u32x4 ent(uint32_t i) const {
        const uint32_t a = i + skip;
        if (a < CAP_T) return tile[a];
        return sp_rec[(uint64_t)ctab[(a >> CAP_SHIFT) - 1u] * CAP_T + (a & (CAP_T - 1u))];
    }
    __device__ __forceinline__ uint32_t snap(uint32_t i) const {        // (word 1 of the entry)
        const uint32_t a = i + skip;
        if (a < CAP_T) return ((const uint32_t*)(tile + a))[1];
        return ((const uint32_t*)(sp_rec + (uint64_t)ctab[(a >> CAP_SHIFT) - 1u] * CAP_T + (a & (CAP_T - 1u))))[1];
    }
};
// the fields of record i's check (per-record path): its start's patch word
// Wr in segment sa with reset value inj; its end W2 in segment sb (kind 1: a
// record start, expected register expn, snapshot s2; kind 2: the terminal's
// segment end, expected zero; kind 3: the tile's end)
struct RecChk { uint32_t sa, sb, Wr, W2, inj, s2, expn, kind; };
__device__ __forceinline__ uint32_t chk_eval(const CLY_LDS uint32_t* emt, const CLY_LDS uint32_t* gin,
                                             const RecChk& q, uint32_t tb) {
    // the register entering W2 (kind 1), or at the end of segment sb - 1 (kinds 2, 3)
    // (gin in the plain layout)
    if (q.sb == q.sa) return q.s2 ^ em_f4(emt, (q.W2 - q.Wr) >> 2, q.inj);
    uint32_t x = gin[q.sa] ^ em_f4(emt, (64u * (q.sa + 1u) - (q.Wr - tb)) >> 2, q.inj);
    const uint32_t steps = q.sb - q.sa - 1u;
    for (uint32_t k = 0; __ballot(k < steps); k++)
        if (k < steps) x = em_a64b(emt, x) ^ gin[q.sa + 1u + k];
    return em_f4(emt, (q.W2 - tb - 64u * q.sb) >> 2, x) ^ q.s2;
}
__global__ void __launch_bounds__(64 * EMIT_WAVES)
k_emit(const DevFile* __restrict__ files, int nfiles, const uint32_t* __restrict__ tprefix, uint32_t ntiles,
       const TileIn* __restrict__ tin, const TileLocal* __restrict__ loc, const uint32_t* __restrict__ rec,
       const uint32_t* __restrict__ seg, uint32_t* treg, FileInfo* finfo,
       const uint32_t* __restrict__ tabs, cly_tuple* out_, uint64_t out_cap, const uint32_t* __restrict__ chunks,
       const u32x4* __restrict__ sp_rec, Globals* g, int slot) {
    if (g->nfix[slot] || g->spill_over || g->fail) return;   // the chain is not final yet (k_refix first) / run again / failed
    gtuples out = (gtuples)out_;
    __shared__ __attribute__((aligned(16))) unsigned char smem_raw[EMIT_LDS];
    CLY_LDS uint32_t* emt = (CLY_LDS uint32_t*)smem_raw;
    for (int i = threadIdx.x; i < NEM * 128; i += blockDim.x) emt[i] = tabs[TAB_EM + i];
    __syncthreads();
    CLY_LDS uint32_t* kj = emt + EMIT_KJ;
    if (threadIdx.x < 4) kj[threadIdx.x] = threadIdx.x ? em_fj(emt, threadIdx.x, CLY_K4) : CLY_K4;
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) {       // A^64 by bytes from its nibble table
        const CLY_LDS uint32_t* a = emt + (EM_F4 + 15) * 128;
        const int b = i >> 8, x = i & 255;
        emt[EMIT_A64B + i] = a[(2 * b) * 16 + (x & 15)] ^ a[(2 * b + 1) * 16 + (x >> 4)];
    }
    __syncthreads();
    CLY_LDS uint8_t* wreg = (CLY_LDS uint8_t*)smem_raw + NEM * 128 * 4 + 16 + 4096 + wave_id() * EW_BYTES;
    CLY_LDS uint32_t* gin = (CLY_LDS uint32_t*)wreg;                  // segment registers, then the scan
    CLY_LDS uint32_t* flg = (CLY_LDS uint32_t*)(wreg + GIN_WORDS * 4);   // reset segments (bitmap)
    CLY_LDS u32x4* sv = (CLY_LDS u32x4*)(wreg + ((GIN_WORDS * 4 + FLG_BYTES + 15) & ~15));   // a round's tuples
    const int lane = threadIdx.x & 63;
    for (uint32_t t = blockIdx.x * EMIT_WAVES + wave_id(); t < ntiles; t += gridDim.x * EMIT_WAVES) {
        const LBState S = ti_load(&tin[t]);
        if (S.dead) continue;
        const int f = (int)__builtin_amdgcn_readfirstlane(((const uint32_t*)&tin[t])[6]);
        const uint32_t tt = t - files[f].first_tile;
        uint32_t ptt;
        const DevFile F = part_view(files[f], tt, ptt);                    // positions below: the part's
        const uint64_t x0 = part_x0(tt);
        FileInfo* fo = &finfo[f];
        const uint64_t gb = S.count + fo->first_index;
        const u64 l0 = loc[t].l[0], l1 = loc[t].l[1], l3 = loc[t].l[3];
        const uint32_t tb = ptt * (uint32_t)CLY_TILE, TE = tb + (uint32_t)CLY_TILE;
        const uint32_t n = (uint32_t)(l0 >> 32);
        const uint32_t skip = (uint32_t)(l3 >> 40) & 0xFFFFu;              // k_refix's suffix (records dropped)
        const gbytes base = (gbytes)F.base;
        const bool none = (l0 & DF_NONE) != 0, term = (l0 & DF_TERM) != 0;
        const bool gterm = !none && term && n == 0;                         // the first boundary is the terminal
        const bool grec = !none && !gterm;                                  // ... a record start
        const uint32_t T = (uint32_t)(l1 >> 32);                            // the terminal (term)
        EntSrc E;
        E.tile = (const u32x4*)(rec + (uint64_t)t * CAP_T * 4);
        E.sp_rec = sp_rec; E.ctab = chunks + (uint64_t)t * CH_WORDS; E.skip = skip;
        const uint32_t cout = treg[2 * t];                                  // the register XOR due at the tile's end
        // the tile's segment registers into LDS (lane-transposed: lane L's run)
        uint32_t sr[RUN];
        {
            const uint32_t* sp = seg + (uint64_t)t * NSEG + (uint32_t)lane * RUN;
            if (RUN % 4 == 0) {
                #pragma unroll
                for (int k = 0; k < RUN; k += 4) {
                    const u32x4 q = *(const u32x4*)(sp + k);
                    sr[k] = q.x; sr[k + 1 < RUN ? k + 1 : 0] = q.y;
                    sr[k + 2 < RUN ? k + 2 : 0] = q.z; sr[k + 3 < RUN ? k + 3 : 0] = q.w;
                }
            } else {
                #pragma unroll
                for (int k = 0; k < RUN; k++) sr[k] = sp[k];
            }
        }
        // ---- G (a record start): its patch word WG, its snapshot, and the
        // register entering WG when the record ending at G matches (expG)
        const uint32_t G = (uint32_t)l1;
        uint32_t WG = 0, sigG = NSEG + 1, expG = 0, sG = 0;
        if (grec) {
            WG = patch_word_of(G);
            sigG = (WG - tb) >> 6;
            sG = E.snap(0);
            if (tt > 0) expG = exp_pre(emt, G & 3u, S.crc_last, entry_crc(base, F.len, tb, E.ent(0)));
        }
        bool full = !grec || sigG >= NSEG || (tt > 0 && sigG > SHORT_KMAX);
        // the segment registers into LDS: plain for the per-record path,
        // lane-transposed for the tile-wide scan
        bool plain = !full;
        if (plain) {
            if (RUN % 4 == 0) {
                #pragma unroll
                for (int k = 0; k < RUN; k += 4)
                    *(CLY_LDS u32x4*)(gin + (uint32_t)lane * RUN + k) =
                        (u32x4){sr[k], sr[k + 1 < RUN ? k + 1 : 0], sr[k + 2 < RUN ? k + 2 : 0], sr[k + 3 < RUN ? k + 3 : 0]};
            } else {
                #pragma unroll
                for (int k = 0; k < RUN; k++) gin[(uint32_t)lane * RUN + k] = sr[k];
            }
        } else {
            #pragma unroll
            for (int k = 0; k < RUN; k++) gin[k * 64 + lane] = sr[k];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint32_t ex = 0, dev = 0;
        if (!full && tt > 0) {
            // the tile's own register entering WG (from zero at the tile's start)
            uint32_t x = 0;
            for (uint32_t k = 0; k < sigG; k++) x = em_a64b(emt, x) ^ gin[k];
            dev = em_f4(emt, (WG - tb - 64u * sigG) >> 2, x) ^ sG ^ expG;
        }
        // ---- tuples, and on the per-record path the records' checks
        {
            // a round's compact entries and snapshots, loaded one round ahead;
            // the next record's come from lane + 1 (lane 63 loads its own)
            const u32x4 z4 = (u32x4){0u, 0u, 0u, 0u};
            auto ld = [&](uint32_t j0, u32x4& v, uint32_t& sv, u32x4& vx, uint32_t& sx) {
                const uint32_t j = j0 + (uint32_t)lane;
                v = j < n ? E.ent(j) : z4;
                sv = v.y;
                vx = z4; sx = 0u;
                if (lane == 63 && j + 1 < n) { vx = E.ent(j + 1); sx = vx.y; }
            };
            u32x4 vc, vx;
            uint32_t sc, sx;
            ld(0u, vc, sc, vx, sx);
            for (uint32_t i0 = 0; i0 < n; i0 += 64) {
                u32x4 vN = z4, vxN = z4;
                uint32_t sN = 0, sxN = 0;
                if (i0 + 64 < n) ld(i0 + 64, vN, sN, vxN, sxN);
                const uint32_t i = i0 + lane;
                const u32x4 v2n = (u32x4){dppu<DPP_WF_SL1>(vx.x, vc.x), dppu<DPP_WF_SL1>(vx.y, vc.y),
                                          dppu<DPP_WF_SL1>(vx.z, vc.z), dppu<DPP_WF_SL1>(vx.w, vc.w)};
                const uint32_t s2n = dppu<DPP_WF_SL1>(sx, sc);
                RecChk q = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
                uint32_t p = 0;
                if (i < n) {
                    const u32x4 v = vc;
                    const uint32_t rel = v.w & 0xFFFFu;
                    p = tb + rel;
                    u32x4 a, b, c;
                    if (v.w & REC_SHORT) {
                        const uint32_t vs = v.z & (SH_VS_LIM - 1u), hsz = 6u + ((v.z >> 21) & 31u);
                        const uint32_t type = (v.z >> 26) & 7u, dt = v.z >> 29;
                        const uint32_t ks = v.w >> 24, key0 = (v.w >> 16) & 0x7Fu;
                        const uint64_t tx = (uint64_t)((int64_t)(key0 >> 1) ^ -(int64_t)(key0 & 1u));
                        a = (u32x4){(uint32_t)(x0 + p), (uint32_t)((x0 + p) >> 32), 0u, 0u};
                        b = (u32x4){(uint32_t)tx, (uint32_t)(tx >> 32), F.fid, hsz + ks + vs};
                        c = (u32x4){ks, vs, type | (dt << 8) | (hsz << 16) | (1u << 24), v.x};
                    } else {
                        const Hdr h = hdr_load(base, p, F.len);
                        tuple_words(base, p, x0, h, F.fid, a, b, c);
                    }
                    sv[3 * lane] = a; sv[3 * lane + 1] = b; sv[3 * lane + 2] = c;
                    if (!full) {
                        const uint32_t cr = c.w;                            // this record's stored CRC
                        q.Wr = patch_word_of(p);
                        q.sa = (q.Wr - tb) >> 6;
                        q.inj = sc ^ exp_post(p & 3u, cr, kj);
                        if (i + 1 < n) {                                    // ends at the next record's patch word
                            const u32x4 v2 = v2n;
                            const uint32_t P2 = tb + (v2.w & 0xFFFFu);
                            q.W2 = patch_word_of(P2);
                            q.sb = (q.W2 - tb) >> 6;
                            q.s2 = s2n;
                            q.expn = exp_pre(emt, P2 & 3u, cr, entry_crc(base, F.len, tb, v2));
                            q.kind = 1;
                        } else if (term && T < TE) {                        // at the terminal's segment end
                            q.sb = (((T & ~3u) - tb) >> 6) + 1u;
                            q.W2 = tb + 64u * q.sb;
                            q.kind = 2;
                        } else {                                            // at the tile's end
                            q.sb = NSEG;
                            q.W2 = TE;
                            q.kind = 3;
                        }
                    }
                }
                if (!full) {
                    if (__ballot(q.kind != 0 && q.sb > q.sa + SHORT_KMAX + 1u)) full = true;     // (uniform)
                    else {
                        const uint32_t val = q.kind ? chk_eval(emt, gin, q, tb) : 0u;
                        if ((q.kind == 1 && val != q.expn) || (q.kind == 2 && val != 0u) ||
                            (q.kind == 3 && term && (val ^ cout) != 0u))
                            fail_at(fo, x0 + p, S.count + i);
                        const u64 bl = __ballot(q.kind == 3);
                        if (bl) ex = rdl(val, __ffsll((long long)bl) - 1) ^ cout;
                    }
                }
                // the round's tuples are 48 (n - i0) contiguous bytes: 16-B pieces q = lane + 64 k
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                {
                    const uint32_t nr = n - i0 < 64 ? n - i0 : 64;
                    CLY_GL u32x4* dst = (CLY_GL u32x4*)(out + gb + i0);
                    #pragma unroll
                    for (int k = 0; k < 3; k++) {
                        const uint32_t qq = (uint32_t)lane + 64u * k;
                        if (qq < 3 * nr) {
                            if (gb + i0 + qq / 3 < out_cap) dst[qq] = sv[qq];
                            else atomicOr(&g->overflow, 1u);
                        }
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                vc = vN; sc = sN; vx = vxN; sx = sxN;
            }
        }
        if (full) {
            if (plain) {
                // (a record spanning too many segments turned the tile over to the scan)
                #pragma unroll
                for (int k = 0; k < RUN; k++) gin[k * 64 + lane] = sr[k];
                plain = false;
            }
            // ---- the tile-wide scan: the segments whose last boundary is a
            // record start get their reset exit (flagged: a constant in the scan)
            if (lane < NSEG / 32) flg[lane] = 0u;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            uint32_t wlast = 0, clast = 0, plast = 0;                       // (the tile's last record start)
            if (grec) {
                for (uint32_t i0 = 0; i0 < n; i0 += 64) {
                    const uint32_t i = i0 + (uint32_t)lane;
                    if (i < n) {
                        const u32x4 v = E.ent(i);
                        const uint32_t P = tb + (v.w & 0xFFFFu), W = patch_word_of(P), sg = (W - tb) >> 6;
                        bool lastin = true;
                        if (i + 1 < n) lastin = ((patch_word_of(tb + (E.ent(i + 1).w & 0xFFFFu)) - tb) >> 6) != sg;
                        if (sg < NSEG && lastin) {
                            const uint32_t inj = E.snap(i) ^ exp_post(P & 3u, entry_crc(base, F.len, tb, v), kj);
                            gin[gin_at(sg, false)] ^= em_f4(emt, (64u * (sg + 1u) - (W - tb)) >> 2, inj);
                            __atomic_fetch_or(flg + (sg >> 5), 1u << (sg & 31u), __ATOMIC_RELAXED);
                        }
                    }
                }
                const u32x4 vl = E.ent(n - 1);
                plast = tb + (vl.w & 0xFFFFu);
                wlast = patch_word_of(plast);
                clast = entry_crc(base, F.len, tb, vl);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            // one Horner pass over the lane's run of segments from zero (resets
            // applied): gin keeps the register entering each of them relative to
            // the run's start (h); the register entering segment j of lane L's
            // run is h, or, with no reset before it in the run, A^(64 j) y_L ^ h
            // (y_L: the scan's register entering the run; gin_true)
            uint32_t x = 0, rc = 0, fl = 0;
            #pragma unroll
            for (int k = 0; k < RUN; k++) {
                const uint32_t sg = (uint32_t)lane * RUN + k;
                const uint32_t sk = gin[k * 64 + lane];
                const uint32_t fk = (flg[sg >> 5] >> (sg & 31u)) & 1u;
                fl |= fk << k;
                gin[k * 64 + lane] = x;
                x = fk ? sk : em_a64b(emt, x) ^ sk;
                rc |= fk;
            }
            #pragma unroll
            for (int l = 0; l < 6; l++) {
                const int d = 1 << l;
                const uint32_t px = (uint32_t)__shfl_up((int)x, d, 64), pc = (uint32_t)__shfl_up((int)rc, d, 64);
                if (lane >= d && !rc) { x = mat_mul(emt + (EM_RUN + l) * 128, px) ^ x; rc = pc; }
            }
            uint32_t y = (uint32_t)__shfl_up((int)x, 1, 64);
            if (lane == 0) y = 0;
            const uint32_t gte = rdl(x, 63);                                // the register at the tile's end
            // the lanes' entering registers and reset masks, for gin_true (in the
            // round's tuple stage: the tuples are out)
            CLY_LDS uint32_t* yarr = (CLY_LDS uint32_t*)sv;
            yarr[lane] = y;
            yarr[64 + lane] = fl;
            if (lane == 0) gin[NSEG] = gte;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            auto gin_true = [&](uint32_t sg) -> uint32_t {
                if (sg >= NSEG) return gte;
                const uint32_t L = sg / RUN, j = sg % RUN;
                uint32_t h = gin[j * 64u + L];
                if ((yarr[64 + L] & ((1u << j) - 1u)) == 0u) {
                    uint32_t v = yarr[L];
                    if (j & 1u) v = em_a64b(emt, v);
                    if (j & 2u) v = mat_mul(emt + (EM_SEGP + 0) * 128, v);
                    if (j & 4u) v = mat_mul(emt + (EM_SEGP + 1) * 128, v);
                    if (j & 8u) v = mat_mul(emt + (EM_SEGP + 2) * 128, v);
                    h ^= v;
                }
                return h;
            };
            ex = gte;
            if (gterm) { ex = 0; dev = gte ^ cout; }
            else if (grec) {
                // the tile's own register entering WG (no reset before G)
                dev = (sigG < NSEG ? em_f4(emt, (WG - tb - 64u * sigG) >> 2, gin_true(sigG)) : gte) ^ sG ^ expG;
                {
                    // past the last record start: its reset at the tile's end
                    // when its patch word is there, else the scan's register
                    ex = wlast == TE ? exp_post(plast & 3u, clast, kj) : gte ^ cout;
                    if (term && ex != 0u && lane == 0)                      // the record ending at the terminal
                        fail_at(fo, x0 + (uint32_t)(loc[t].l[2] >> 32), S.count + n - 1);
                    // every record that ends at a record start inside the tile
                    for (uint32_t i = lane; i + 1 < n; i += 64) {
                        const u32x4 v = E.ent(i), v2 = E.ent(i + 1);
                        const uint32_t p = tb + (v.w & 0xFFFFu), P2 = tb + (v2.w & 0xFFFFu);
                        const uint32_t W = patch_word_of(p), W2 = patch_word_of(P2), sg = (W - tb) >> 6, sg2 = (W2 - tb) >> 6;
                        const uint32_t c1 = entry_crc(base, F.len, tb, v), c2 = entry_crc(base, F.len, tb, v2);
                        const uint32_t s1 = E.snap(i), s2 = E.snap(i + 1);
                        const uint32_t pre = sg2 == sg ? s2 ^ em_f4(emt, (W2 - W) >> 2, s1 ^ exp_post(p & 3u, c1, kj))
                                                       : em_f4(emt, (W2 - tb - 64u * sg2) >> 2, gin_true(sg2)) ^ s2;
                        if (pre != exp_pre(emt, P2 & 3u, c1, c2))
                            fail_at(fo, x0 + p, S.count + i);
                    }
                }
            }
        }
        if (lane == 0) {
            treg[2 * t] = ex;
            treg[2 * t + 1] = dev;
            if (term) {
                fo->term_pos = x0 + T;
                fo->term_status = (int32_t)(int8_t)(uint8_t)(l3 >> 32);
                fo->term_tile = t;
                fo->end_index = gb + n;
                fo->has_term = 1;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// k_fin: per file (FIN_NT threads), after k_emit: the register entering every
// tile up to the terminal's, as a segmented scan over the tiles (a tile with a
// boundary fixes the register at its end to its exit value; a tile without one
// passes it on as A^CLY_TILE r ^ its own register), and in every tile after the first that has a boundary, the check of the
// record that crosses into it (its start: the last record before the tile,
// TileIn): A^CLY_TILE (the register entering the tile) must equal the tile's
// dev shifted to its end.
#define FIN_NT 1024
#define FIN_LEV 10                      // log2(FIN_NT): the scan's levels
#define FIN_B 4                         // tiles a thread loads at once
__device__ __forceinline__ uint32_t shift_b(const CLY_LDS uint32_t* sh, uint32_t m, uint32_t v) {
    return m ? shift_bytes(sh, m, v) : v;
}
__global__ void __launch_bounds__(FIN_NT)
k_fin(const DevFile* __restrict__ files, FileInfo* finfo, const uint32_t* __restrict__ treg,
      const TileLocal* __restrict__ loc, const TileIn* __restrict__ tin, const uint32_t* __restrict__ tabs,
      Globals* g, int slot) {
    __shared__ uint32_t tabl[NIB_SH * 128 + 128];           // TAB_SH, TAB_TILE
    __shared__ uint32_t levt[FIN_LEV * 128];                // A^(CLY_TILE per 2^l): level l of the scan
    __shared__ uint32_t px[FIN_NT], pc[FIN_NT];
    if (g->nfix[slot] || g->spill_over || g->fail) return;   // k_emit did not run
    const int f = blockIdx.x, tid = threadIdx.x;
    const DevFile F = files[f];
    FileInfo* fo = &finfo[f];
    if (!fo->has_term) {
        if (tid == 0) atomicOr(&g->fail, 32u);
        return;
    }
    // a thread's tiles: a power of two (per = 2^e), so that level l's shift is
    // the host-built table A^(CLY_TILE 2^(e + l))
    const uint32_t ft = F.first_tile, nt = fo->term_tile - ft + 1;
    const uint32_t per0 = (nt + FIN_NT - 1) / FIN_NT;
    const uint32_t e = per0 <= 1u ? 0u : 32u - (uint32_t)__clz((int)(per0 - 1u)), per = 1u << e;
    const uint32_t lo = tid * per < nt ? tid * per : nt, hi = lo + per < nt ? lo + per : nt;
    for (int i = tid; i < NIB_SH * 128 + 128; i += FIN_NT) tabl[i] = tabs[TAB_SH + i];
    for (int i = tid; i < FIN_LEV * 128; i += FIN_NT) levt[i] = tabs[TAB_PW + e * 128 + i];
    const CLY_LDS uint32_t* sht = (const CLY_LDS uint32_t*)tabl;
    const CLY_LDS uint32_t* tilet = sht + NIB_SH * 128;
    uint64_t a0[FIN_B];
    uint32_t av[FIN_B];
    auto fetch = [&](uint32_t u0) {
        #pragma unroll
        for (int q = 0; q < FIN_B; q++)
            if (u0 + q < hi) { a0[q] = loc[ft + u0 + q].l[0]; av[q] = treg[2 * (ft + u0 + q)]; }
    };
    uint32_t x = 0, c = 0;
    fetch(lo);
    __syncthreads();                                        // (the tables)
    for (uint32_t u0 = lo; u0 < hi; u0 += FIN_B) {
        if (u0 != lo) fetch(u0);
        #pragma unroll
        for (int q = 0; q < FIN_B; q++) {
            if (u0 + q >= hi) break;
            if (!(a0[q] & DF_NONE)) { x = av[q]; c = 1; }
            else x = mat_mul(tilet, x) ^ av[q];
        }
    }
    px[tid] = x; pc[tid] = c;
    __syncthreads();
    for (int l = 0; l < FIN_LEV; l++) {
        const int d = 1 << l;
        uint32_t ox = 0, oc = 0;
        if (tid >= d) { ox = px[tid - d]; oc = pc[tid - d]; }
        __syncthreads();
        if (tid >= d && !c) { x = mat_mul((const CLY_LDS uint32_t*)levt + l * 128, ox) ^ x; c = oc; }
        px[tid] = x; pc[tid] = c;
        __syncthreads();
    }
    uint32_t y = tid ? px[tid - 1] : 0u;
    for (uint32_t u0 = lo; u0 < hi; u0 += FIN_B) {
        fetch(u0);
        #pragma unroll
        for (int q = 0; q < FIN_B; q++) {
            const uint32_t u = u0 + q;
            if (u >= hi) break;
            const uint32_t t = ft + u;
            const u64 l0 = a0[q];
            const uint32_t v = av[q];
            if (l0 & DF_NONE) { y = mat_mul(tilet, y) ^ v; continue; }
            if (u > 0) {
                const LBState S = ti_load(&tin[t]);
                const uint32_t n = (uint32_t)(l0 >> 32), G = (uint32_t)loc[t].l[1];
                const uint32_t tb = (u % PART_TILES) * (uint32_t)CLY_TILE, TE = tb + (uint32_t)CLY_TILE;   // (the part's)
                uint32_t dev = treg[2 * t + 1];
                if ((l0 & DF_TERM) && n == 0) dev ^= shift_b(sht, TE - G, S.crc_last);     // G is the terminal
                else dev = shift_b(sht, TE - patch_word_of(G), dev);
                if (mat_mul(tilet, y) != dev)
                    fail_at(fo, S.P_last, S.count - 1);
            }
            y = v;
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
    uint8_t* d_call; uint8_t* h_call; size_t call_bytes;     // the per-call block (ensure_files)
    DevFile* d_files; uint32_t* d_tprefix; FileInfo* d_finfo; uint64_t* d_ftotal; int cap_files;
    DevFile* h_files; uint32_t* h_tprefix; FileInfo* h_finfo;
    uint32_t* d_rprefix; uint32_t* h_rprefix;        // per file its first run of tiles (k_scan)
    TileLocal* d_loc; TileIn* d_tin; uint32_t* d_treg; uint32_t* d_fix; uint32_t* d_rec;
    uint32_t* d_seg;             // segment registers
    uint32_t* d_chunks;          // per tile CH_WORDS words: spill chunk ids and their count
    uint32_t* d_lmask;           // k_link's bitmasks of files past LINK_MAXT tiles (2 x lmask_words)
    uint64_t lmask_words;
    int64_t cap_tiles;
    u32x4* d_sp_rec; uint32_t cap_spill;   // the spill pool (chunks of CAP_T entries)
    Globals* d_g; Globals* h_g;
    uint32_t* d_tabs;            // nibble tables (TAB_SH, TAB_TILE, TAB_EM)
    int scan_grid, emit_grid, loc_grid;
    float kms[6];                // last call: k_scan, link rounds (k_link/k_refix), k_emit, k_fin, discarded attempts, all
    uint8_t* d_bytes; uint64_t cap_bytes;          // host-path staging
    cly_tuple* d_tuples; uint64_t cap_tuples;
    void* merge_scratch;         // clymerge.hip's buffers (grow-only)
    int64_t now_ns;              // loadIndex's time.Now() for the TTL sweep (0: the wall clock per call)
    int dbg;                     // cly_dbg_set: bit 0 = keep k_scan's LOCALs (before any repair) in d_dbg,
                                 // bit 1 = print the repair rounds, bit 2 = per-kernel timing markers
    TileLocal* d_dbg; int64_t cap_dbg;
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
    // timing-only markers: no system-scope fence (its L2 writeback and
    // invalidate left a 6-us gap after every marked kernel); the results come
    // back by copies and stream waits
    for (int i = 0; i < 8; i++) HIPCK(hipEventCreateWithFlags(&c->ev[i], hipEventDisableSystemFence));
    {
        static uint32_t hn[NTAB_ALL];
        for (int k = 0; k < NTAB_ALL / 128; k++) {
            uint64_t nbytes;
            if (k < 64) nbytes = (uint64_t)(k & 15) << (4 * (k >> 4));               // A^(v 16^d)
            else if (k == 64) nbytes = 65536;                                        // A^65536
            else if (k == 65) nbytes = (uint64_t)CLY_TILE;                           // k_fin's tile step
            else if (k >= TAB_PW / 128) nbytes = (uint64_t)CLY_TILE << (k - TAB_PW / 128);   // k_fin's levels
            else {
                const int e = k - 66;                                                // TAB_EM
                if (e < EM_F1) nbytes = 4ull * (uint64_t)(e + 1);                    // A^(4k), k = 1..16
                else if (e < EM_RUN) nbytes = (uint64_t)(e - EM_F1 + 1);             // A^1..A^3
                else if (e < EM_SEGP) nbytes = (uint64_t)RUN_BYTES << (e - EM_RUN);  // A^(RUN_BYTES 2^l)
                else nbytes = 64ull << (e - EM_SEGP + 1);                            // A^128, A^256, A^512
            }
            const uint32_t xm = cly_x8n(nbytes);
            for (int nb = 0; nb < 8; nb++)
                for (uint32_t v = 0; v < 16; v++) hn[k * 128 + nb * 16 + v] = cly_multmodp(xm, v << (4 * nb));
        }
        HIPCK(hipMalloc(&c->d_tabs, sizeof(hn)));
        HIPCK(hipMemcpy(c->d_tabs, hn, sizeof(hn), hipMemcpyHostToDevice));
    }
    {
        int ncu = 0;
        HIPCK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device));
        int per_cu = 0;
        HIPCK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_scan, 64 * SCAN_WAVES, 0));
        if (per_cu < 1) per_cu = 1;
        c->scan_grid = per_cu * ncu;
        per_cu = 0;
        HIPCK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_emit, 64 * EMIT_WAVES, 0));
        if (per_cu < 1) per_cu = 1;
        c->emit_grid = per_cu * ncu;
        c->loc_grid = ncu;
    }
    *out = c;
    return CLY_OK;
}

extern "C" void cly_ctx_destroy(cly_ctx* c) {
    if (!c) return;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    hipFree(c->d_call); hipFree(c->d_ftotal);
    hipFree(c->d_loc); hipFree(c->d_tin); hipFree(c->d_treg); hipFree(c->d_fix); hipFree(c->d_rec);
    hipFree(c->d_seg); hipFree(c->d_chunks); hipFree(c->d_lmask); hipFree(c->d_sp_rec);
    hipFree(c->d_tabs); hipFree(c->d_bytes); hipFree(c->d_tuples); hipFree(c->d_dbg);
    hipHostFree(c->h_call);
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

// The per-call block, one device allocation and its page-locked mirror:
// [Globals | FileInfo x cap | DevFile x cap | tprefix x (cap + 1) | rprefix x (cap + 1)], so that a
// call moves its inputs (and zeroes the outputs) with one copy in and reads
// the results back with one copy out.
static inline size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }
static int ensure_files(cly_ctx* c, int nfiles) {
    if (nfiles <= c->cap_files) return CLY_OK;
    hipFree(c->d_call); hipFree(c->d_ftotal); hipHostFree(c->h_call);
    c->d_call = nullptr; c->h_call = nullptr; c->d_ftotal = nullptr;
    c->cap_files = 0;
    const int cap = nfiles < 64 ? 64 : nfiles;
    const size_t o_fi = al16(sizeof(Globals)), o_f = o_fi + al16(sizeof(FileInfo) * cap);
    const size_t o_tp = o_f + al16(sizeof(DevFile) * cap), o_rp = o_tp + al16(sizeof(uint32_t) * (cap + 1));
    const size_t tot = o_rp + al16(sizeof(uint32_t) * (cap + 1));
    HIPCK(hipMalloc(&c->d_call, tot));
    HIPCK(hipMalloc(&c->d_ftotal, sizeof(uint64_t) * cap));
    HIPCK(hipHostMalloc(&c->h_call, tot, hipHostMallocDefault));
    c->d_g = (Globals*)c->d_call; c->h_g = (Globals*)c->h_call;
    c->d_finfo = (FileInfo*)(c->d_call + o_fi); c->h_finfo = (FileInfo*)(c->h_call + o_fi);
    c->d_files = (DevFile*)(c->d_call + o_f); c->h_files = (DevFile*)(c->h_call + o_f);
    c->d_tprefix = (uint32_t*)(c->d_call + o_tp); c->h_tprefix = (uint32_t*)(c->h_call + o_tp);
    c->d_rprefix = (uint32_t*)(c->d_call + o_rp); c->h_rprefix = (uint32_t*)(c->h_call + o_rp);
    c->call_bytes = tot;
    c->cap_files = cap;
    return CLY_OK;
}

static int ensure_tiles(cly_ctx* c, int64_t ntiles) {
    if (ntiles <= c->cap_tiles) return CLY_OK;
    hipFree(c->d_loc); hipFree(c->d_tin); hipFree(c->d_treg); hipFree(c->d_fix); hipFree(c->d_rec);
    hipFree(c->d_seg); hipFree(c->d_chunks); hipFree(c->d_lmask);
    c->d_lmask = nullptr; c->lmask_words = 0;
    c->d_loc = nullptr; c->d_tin = nullptr; c->d_treg = nullptr; c->d_fix = nullptr; c->d_rec = nullptr;
    c->d_seg = nullptr; c->d_chunks = nullptr;
    c->cap_tiles = 0;
    const int64_t cap = ntiles < 1024 ? 1024 : ntiles;
    HIPCK(hipMalloc(&c->d_loc, sizeof(TileLocal) * cap));
    HIPCK(hipMalloc(&c->d_tin, sizeof(TileIn) * cap));
    HIPCK(hipMalloc(&c->d_treg, sizeof(uint32_t) * 2 * cap));
    HIPCK(hipMalloc(&c->d_seg, sizeof(uint32_t) * NSEG * (uint64_t)cap));
    HIPCK(hipMalloc(&c->d_chunks, sizeof(uint32_t) * CH_WORDS * (uint64_t)cap));
    HIPCK(hipMalloc(&c->d_fix, sizeof(uint32_t) * cap));
    HIPCK(hipMalloc(&c->d_rec, sizeof(uint32_t) * 4 * (uint64_t)CAP_T * cap));
    c->cap_tiles = cap;
    return CLY_OK;
}
// k_link's global bitmasks (files of more than LINK_MAXT tiles): file f's words
// start at first_tile / 32 + f, so no two files share one
static int ensure_lmask(cly_ctx* c, int64_t ntiles, int nfiles) {
    const uint64_t words = (uint64_t)ntiles / 32 + (uint64_t)nfiles + 2;
    if (words <= c->lmask_words) return CLY_OK;
    hipFree(c->d_lmask);
    c->d_lmask = nullptr; c->lmask_words = 0;
    HIPCK(hipMalloc(&c->d_lmask, sizeof(uint32_t) * 2 * words));
    c->lmask_words = words;
    return CLY_OK;
}

// The spill pool: at least `chunks` chunks (grow-only; the first call of a
// context sizes it for one chunk per 8 tiles)
static int ensure_spill(cly_ctx* c, uint64_t chunks) {
    if (chunks <= c->cap_spill) return CLY_OK;
    if (chunks > 0xFFFFFFF0ull) return CLY_ERR_ARG;
    hipFree(c->d_sp_rec);
    c->d_sp_rec = nullptr; c->cap_spill = 0;
    HIPCK(hipMalloc(&c->d_sp_rec, sizeof(u32x4) * CAP_T * chunks));
    c->cap_spill = (uint32_t)chunks;
    return CLY_OK;
}

// the largest file length: u64 chain positions in TileIn keep 48 bits (P_NONE above them)
#define MAX_FILE_LEN ((1ull << 47) - 1)

// alloc != nullptr: the output is allocated here (hipMalloc, the caller frees
// it) once the link knows the exact record count, so that it holds exactly
// needed + 16 tuples (d_out and out_cap are ignored).
static int scan_attempt(cly_ctx* c, const cly_file* files, int nfiles, cly_tuple* d_out, uint64_t out_cap,
                        uint64_t* file_first, cly_file_result* res, uint64_t* needed, cly_stats* stats, void* stream_v,
                        cly_tuple** alloc, uint64_t* alloc_cap) {
    if (!c || (!files && nfiles) || nfiles < 0 || !res || !file_first) return CLY_ERR_ARG;
    if (alloc) { *alloc = nullptr; d_out = nullptr; out_cap = 0; }
    if (nfiles == 0) { if (needed) *needed = 0; return CLY_OK; }
    HIPCK(hipSetDevice(c->device));
    hipStream_t st = stream_v ? (hipStream_t)stream_v : c->stream;
    int rc = ensure_files(c, nfiles);
    if (rc) return rc;
    int64_t ntiles = 0, nruns = 0;
    uint64_t bytes = 0;
    // the run length: the longest (up to RUN_TILES) whose runs fill the wave slots
    uint32_t rt = RUN_TILES;
    if (CLY_RUN_ADAPT) {
        const int64_t slots = (int64_t)c->scan_grid * SCAN_WAVES;
        for (; rt > 1; rt >>= 1) {
            int64_t nr = 0;
            for (int i = 0; i < nfiles; i++) {
                const uint64_t nt = files[i].len ? (files[i].len + CLY_TILE - 1) / CLY_TILE : 1;
                nr += (int64_t)((nt + rt - 1) / rt);
            }
            if (nr >= slots) break;
        }
    }
    for (int i = 0; i < nfiles; i++) {
        if (files[i].len > MAX_FILE_LEN) return CLY_ERR_ARG;
        if (files[i].len && (((uintptr_t)files[i].base) & 15)) return CLY_ERR_ARG;
        const uint64_t nt = files[i].len ? (files[i].len + CLY_TILE - 1) / CLY_TILE : 1;
        c->h_files[i].base = files[i].base;
        c->h_files[i].len = files[i].len;
        c->h_files[i].fid = files[i].fid;
        c->h_files[i].first_tile = (uint32_t)ntiles;
        c->h_files[i].ntile = (uint32_t)nt;
        c->h_files[i]._pad = 0;
        c->h_tprefix[i] = (uint32_t)ntiles;
        c->h_rprefix[i] = (uint32_t)nruns;
        ntiles += (int64_t)nt;
        nruns += (int64_t)((nt + rt - 1) / rt);
        bytes += files[i].len;
    }
    if (ntiles >= (1LL << 31)) return CLY_ERR_ARG;
    c->h_tprefix[nfiles] = (uint32_t)ntiles;
    c->h_rprefix[nfiles] = (uint32_t)nruns;
    rc = ensure_tiles(c, ntiles);
    if (rc) return rc;
    {
        bool far = false;
        for (int i = 0; i < nfiles; i++) far |= c->h_files[i].ntile > LINK_MAXT;
        if (far && (rc = ensure_lmask(c, ntiles, nfiles))) return rc;
    }
    rc = ensure_spill(c, (uint64_t)ntiles / 8 + 64);
    if (rc) return rc;
    memset(c->h_g, 0, sizeof(Globals));
    c->h_g->spill_cap = c->cap_spill;
    c->h_g->run_tiles = rt;
    memset(c->h_finfo, 0, sizeof(FileInfo) * nfiles);
    for (int i = 0; i < nfiles; i++) c->h_finfo[i].fail_off = c->h_finfo[i].fail_idx = ~0ull;
    HIPCK(hipMemcpyAsync(c->d_call, c->h_call, c->call_bytes, hipMemcpyHostToDevice, st));
    const uint32_t nt32 = (uint32_t)ntiles;
    int grid = c->scan_grid;
    if ((int64_t)grid * SCAN_WAVES > nruns) grid = (int)((nruns + SCAN_WAVES - 1) / SCAN_WAVES);
    HIPCK(hipEventRecord(c->ev[0], st));
    hipLaunchKernelGGL(k_scan, dim3(grid), dim3(64 * SCAN_WAVES), 0, st, c->d_files, nfiles, c->d_rprefix, (uint32_t)nruns,
                       c->d_loc, c->d_rec, c->d_seg, c->d_treg, c->d_chunks, c->d_sp_rec, c->d_g);
    HIPCK(hipGetLastError());
    HIPCK(hipEventRecord(c->ev[1], st));
    if (c->dbg & 1) {
        if (c->cap_dbg < ntiles) {
            hipFree(c->d_dbg); c->d_dbg = nullptr; c->cap_dbg = 0;
            HIPCK(hipMalloc(&c->d_dbg, sizeof(TileLocal) * ntiles));
            c->cap_dbg = ntiles;
        }
        HIPCK(hipMemcpyAsync(c->d_dbg, c->d_loc, sizeof(TileLocal) * ntiles, hipMemcpyDeviceToDevice, st));
    }
    // the link (k_link: chain states, contradicted tiles, file bases), then
    // k_emit/k_fin, which return at once if the link listed tiles; only then
    // the host waits.  Repair rounds (k_refix + k_link) follow on the host loop.
    hipLaunchKernelGGL(k_link, dim3(nfiles), dim3(LINK_NT), 0, st, c->d_files, nfiles, c->d_loc, c->d_tin, c->d_ftotal,
                       c->d_finfo, c->d_fix, c->d_lmask, c->lmask_words, c->d_g, 0, -1);
    // one repair round on the device, without a host wait: k_refix and
    // k_link return at once when the first link listed no tile
    hipLaunchKernelGGL(k_refix, dim3(REFIX_GRID), dim3(64 * SCAN_WAVES), 0, st, c->d_files, nfiles, c->d_tprefix,
                       c->d_loc, c->d_tin, c->d_rec, c->d_seg, c->d_treg, c->d_chunks, c->d_sp_rec,
                       c->d_fix, c->d_g, 0);
    hipLaunchKernelGGL(k_link, dim3(nfiles), dim3(LINK_NT), 0, st, c->d_files, nfiles, c->d_loc, c->d_tin, c->d_ftotal,
                       c->d_finfo, c->d_fix, c->d_lmask, c->lmask_words, c->d_g, 1, 0);
    HIPCK(hipGetLastError());
    // per-kernel markers between the link and k_emit and between k_emit and
    // k_fin only on request (cly_dbg_set bit 2: each marker costs a gap of
    // ~5 us); otherwise link + k_emit + k_fin are timed as one span
    const bool detail = (c->dbg & 4) != 0;
    if (detail) HIPCK(hipEventRecord(c->ev[2], st));
    int slot = 1;
    auto launch_emit = [&]() -> int {
        int eg = c->emit_grid;
        if ((int64_t)eg * EMIT_WAVES > ntiles) eg = (int)((ntiles + EMIT_WAVES - 1) / EMIT_WAVES);
        hipLaunchKernelGGL(k_emit, dim3(eg), dim3(64 * EMIT_WAVES), 0, st, c->d_files, nfiles, c->d_tprefix, nt32,
                           c->d_tin, c->d_loc, c->d_rec, c->d_seg, c->d_treg, c->d_finfo, c->d_tabs, d_out,
                           out_cap, c->d_chunks, c->d_sp_rec, c->d_g, slot);
        HIPCK(hipGetLastError());
        if (detail) HIPCK(hipEventRecord(c->ev[3], st));
        hipLaunchKernelGGL(k_fin, dim3(nfiles), dim3(FIN_NT), 0, st, c->d_files, c->d_finfo, c->d_treg, c->d_loc,
                           c->d_tin, c->d_tabs, c->d_g, slot);
        HIPCK(hipGetLastError());
        HIPCK(hipEventRecord(c->ev[4], st));
        // one read-back and one wait for the whole call when no repair round is needed
        HIPCK(hipMemcpyAsync(c->h_call, c->d_call, (uint8_t*)(c->h_finfo + nfiles) - c->h_call, hipMemcpyDeviceToHost, st));
        HIPCK(hipStreamSynchronize(st));
        return CLY_OK;
    };
    // (alloc: the output once the count is final, after any repair rounds)
    auto emit_alloc = [&]() -> int {
        out_cap = c->h_g->total + 16;
        HIPCK(hipMalloc((void**)alloc, sizeof(cly_tuple) * out_cap));
        d_out = *alloc;
        if (alloc_cap) *alloc_cap = out_cap;
        return launch_emit();
    };
    int rc2 = CLY_OK;
    if (!alloc) rc2 = launch_emit();
    else {
        HIPCK(hipMemcpyAsync(c->h_g, c->d_g, sizeof(Globals), hipMemcpyDeviceToHost, st));
        HIPCK(hipStreamSynchronize(st));
        if (!c->h_g->nfix[slot] && !c->h_g->fail && !c->h_g->spill_over) rc2 = emit_alloc();
    }
    if (rc2) return rc2;
    float ms_fix = 0;
    uint32_t rounds = 1, refixed = 0;
    if (c->h_g->nfix[0]) { rounds++; refixed += c->h_g->nfix[0]; }          // the device round
    if ((c->dbg & 2) && c->h_g->nfix[0])
        fprintf(stderr, "clyscan: device repair round: %u tiles listed, longest walk %u from tile %u\n", c->h_g->nfix[0],
                c->h_g->walk_max, (uint32_t)c->h_g->walk_dbg);
    if (c->h_g->nfix[slot]) {
        HIPCK(hipEventRecord(c->ev[5], st));
        while (c->h_g->nfix[slot]) {
            if (c->h_g->fail) break;
            if (rounds > 4096) { fprintf(stderr, "clyscan: chain repair did not converge\n"); return CLY_ERR_NOREPAIR; }
            const uint32_t nfix = c->h_g->nfix[slot];
            refixed += nfix;
            if (c->dbg & 2) fprintf(stderr, "clyscan: repair round %u: %u tiles listed, longest walk so far %u from tile %u\n",
                                    rounds, nfix, c->h_g->walk_max, (uint32_t)c->h_g->walk_dbg);
            const int ns = slot ^ 1;
            HIPCK(hipMemsetAsync(&c->d_g->nfix[ns], 0, sizeof(uint32_t), st));
            hipLaunchKernelGGL(k_refix, dim3((nfix + SCAN_WAVES - 1) / SCAN_WAVES), dim3(64 * SCAN_WAVES), 0, st,
                               c->d_files, nfiles, c->d_tprefix, c->d_loc, c->d_tin, c->d_rec, c->d_seg,
                               c->d_treg, c->d_chunks, c->d_sp_rec, c->d_fix, c->d_g, slot);
            hipLaunchKernelGGL(k_link, dim3(nfiles), dim3(LINK_NT), 0, st, c->d_files, nfiles, c->d_loc, c->d_tin,
                               c->d_ftotal, c->d_finfo, c->d_fix, c->d_lmask, c->lmask_words, c->d_g, ns, -1);
            HIPCK(hipGetLastError());
            HIPCK(hipMemcpyAsync(c->h_g, c->d_g, sizeof(Globals), hipMemcpyDeviceToHost, st));
            HIPCK(hipStreamSynchronize(st));
            slot = ns;
            rounds++;
        }
        HIPCK(hipEventRecord(c->ev[6], st));
        HIPCK(hipEventSynchronize(c->ev[6]));
        HIPCK(hipEventElapsedTime(&ms_fix, c->ev[5], c->ev[6]));
        if (!c->h_g->fail && !c->h_g->spill_over) {
            HIPCK(hipEventRecord(c->ev[2], st));
            rc2 = alloc ? emit_alloc() : launch_emit();
            if (rc2) return rc2;
        }
    }
    float ms_scan = 0, ms_link = 0, ms_emit = 0, ms_fin = 0;
    if (c->h_g->spill_over) {                    // (k_emit / k_fin did not run: the caller runs the call again)
        HIPCK(hipStreamSynchronize(st));
        HIPCK(hipEventElapsedTime(&ms_scan, c->ev[0], c->ev[1]));
        c->kms[5] = ms_scan + ms_fix;
        return CLY_OK;
    }
    HIPCK(hipEventElapsedTime(&ms_scan, c->ev[0], c->ev[1]));
    if (detail) {
        HIPCK(hipEventElapsedTime(&ms_link, c->ev[1], c->ev[2]));
        HIPCK(hipEventElapsedTime(&ms_emit, c->ev[2], c->ev[3]));
        HIPCK(hipEventElapsedTime(&ms_fin, c->ev[3], c->ev[4]));
        if (ms_fix > 0) ms_link = 0;   // ev[2] was re-recorded after the host repair loop
    } else {
        // one span: the link and k_emit + k_fin (after a host repair loop, ev[2]
        // marks the relaunched k_emit)
        HIPCK(hipEventElapsedTime(&ms_emit, ms_fix > 0 ? c->ev[2] : c->ev[1], c->ev[4]));
    }
    c->h_g->refix = refixed;
    c->kms[0] = ms_scan; c->kms[1] = ms_link + ms_fix; c->kms[2] = ms_emit; c->kms[3] = ms_fin; c->kms[4] = 0;
    c->kms[5] = ms_scan + ms_link + ms_fix + ms_emit + ms_fin;
    if (c->h_g->fail) {
        fprintf(stderr, "clyscan: internal error (code %#x)\n", c->h_g->fail);
        return CLY_ERR_DEVICE;
    }
    uint64_t total = 0;
    for (int i = 0; i < nfiles; i++) {
        const FileInfo& fi = c->h_finfo[i];
        file_first[i] = fi.first_index;
        if (fi.fail_idx == ~0ull) {              // every record matches its CRC
            res[i].n_records = fi.end_index - fi.first_index;
            res[i].end_offset = (int64_t)fi.term_pos;
            res[i].status = fi.term_status;
        } else {                                 // the first record whose CRC fails
            res[i].n_records = fi.fail_idx;
            res[i].end_offset = (int64_t)fi.fail_off;
            res[i].status = CLY_ERR_CRC;
        }
        res[i]._pad = 0;
        total += res[i].n_records;
        // A part's view ends VIEW_MAX past its first byte: a record of 2+ GiB that
        // starts there and passes the view's end reads as torn although the file
        // holds it whole.  Such a terminal is decoded again against the whole
        // file: a record there is beyond this library's limit (CLY_ERR_ARG), not
        // the io.EOF ReadLogRecord would not return.
        if (res[i].status == CLY_END_TORN) {
            const uint64_t T = (uint64_t)res[i].end_offset, x0 = (T / PART_BYTES) * PART_BYTES;
            if (files[i].len - x0 > VIEW_MAX) {
                uint8_t hb[26] = {0};
                const uint64_t nh = files[i].len - T < 26 ? files[i].len - T : 26;
                HIPCK(hipMemcpy(hb, files[i].base + T, nh, hipMemcpyDeviceToHost));
                const Hdr h = step_hdr((const uint8_t*)hb, 0, (int64_t)(files[i].len - T), (int64_t)T);
                if (h.status == REC_OK) {
                    fprintf(stderr, "clyscan: file %d: a record of %lld B at %llu crosses a part's 4-GiB view\n", i,
                            (long long)h.size, (unsigned long long)T);
                    return CLY_ERR_ARG;
                }
            }
        }
    }
    if (needed) *needed = c->h_g->total;
    if (stats) {
        stats->scan_ms = ms_scan + ms_emit; stats->resolve_ms = ms_link + ms_fix + ms_fin;
        stats->total_ms = c->kms[5];
        stats->passes = rounds;
        stats->n_chunks = (uint32_t)(ntiles * CLY_NBLK * CLY_NL); stats->bytes = bytes; stats->records = total;
    }
    if (c->h_g->overflow || c->h_g->total > out_cap) return CLY_ERR_CAPACITY;
    return CLY_OK;
}
// One call: an attempt whose tiles needed more spill chunks than the pool
// held (small records, CAP_T+ per tile) is run again with a pool of the size
// it asked for; the context keeps the pool for later calls.
static int scan_device(cly_ctx* c, const cly_file* files, int nfiles, cly_tuple* d_out, uint64_t out_cap,
                       uint64_t* file_first, cly_file_result* res, uint64_t* needed, cly_stats* stats, void* stream_v,
                       cly_tuple** alloc, uint64_t* alloc_cap) {
    float discarded = 0;
    for (int attempt = 0;; attempt++) {
        const int rc = scan_attempt(c, files, nfiles, d_out, out_cap, file_first, res, needed, stats, stream_v, alloc,
                                    alloc_cap);
        if (nfiles == 0 || !c->h_g->spill_over || (rc != CLY_OK && rc != CLY_ERR_CAPACITY)) {
            c->kms[4] = discarded;
            c->kms[5] += discarded;
            return rc;
        }
        discarded += c->kms[5];
        if (alloc && *alloc) { hipFree(*alloc); *alloc = nullptr; }
        if (attempt >= 3) return CLY_ERR_DEVICE;
        const uint64_t want = (uint64_t)c->h_g->spill_next;
        const int r2 = ensure_spill(c, std::max<uint64_t>(2ull * c->cap_spill, want + want / 4 + 64));
        if (r2) return r2;
    }
}
extern "C" int cly_scan_device(cly_ctx* c, const cly_file* files, int nfiles, cly_tuple* d_out, uint64_t out_cap,
                               uint64_t* file_first, cly_file_result* res, uint64_t* needed, cly_stats* stats,
                               void* stream_v) {
    return scan_device(c, files, nfiles, d_out, out_cap, file_first, res, needed, stats, stream_v, nullptr, nullptr);
}
// The open's scan (clyload.hip; not in the public header): the tuple buffer
// sized by the exact record count (*d_out, *cap slots; the caller frees it).
extern "C" int cly_scan_device_alloc_internal(cly_ctx* c, const cly_file* files, int nfiles, cly_tuple** d_out,
                                              uint64_t* cap, uint64_t* file_first, cly_file_result* res,
                                              uint64_t* needed) {
    if (!d_out) return CLY_ERR_ARG;
    const int rc = scan_device(c, files, nfiles, nullptr, 0, file_first, res, needed, nullptr, nullptr, d_out, cap);
    if (rc != CLY_OK && *d_out) { hipFree(*d_out); *d_out = nullptr; }
    return rc;
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
        if (files[i].len > MAX_FILE_LEN) return CLY_ERR_ARG;
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

// Per-kernel times of the last cly_scan_device call (ms): k_scan, link rounds
// (k_link + repair), k_emit, k_fin, k_ovf, all.  Not in the public header.
// Debug (not in the public header): flags (bit 0: snapshot k_scan's tile
// LOCALs); cly_dbg_tiles copies the snapshot (32 B per tile) and the final
// TileIns (32 B per tile) of the last call to host memory.
extern "C" void cly_dbg_set(cly_ctx* c, int flags) { c->dbg = flags; }
extern "C" int cly_dbg_tiles(cly_ctx* c, void* loc_out, void* tin_out, int64_t ntiles) {
    HIPCK(hipSetDevice(c->device));
    if (loc_out && c->d_dbg && ntiles <= c->cap_dbg)
        HIPCK(hipMemcpy(loc_out, c->d_dbg, sizeof(TileLocal) * ntiles, hipMemcpyDeviceToHost));
    if (tin_out && ntiles <= c->cap_tiles) HIPCK(hipMemcpy(tin_out, c->d_tin, sizeof(TileIn) * ntiles, hipMemcpyDeviceToHost));
    return CLY_OK;
}
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
        case -14: return "the data dir maybe contaminated or damaged";            // CLY_ERR_DIR (clyload.h)
        case -15: return "merge-finished: no readable record / value not an integer";   // CLY_ERR_MERGE_FIN
        case -16: return "the key can not be empty";                              // CLY_ERR_KEY_EMPTY (clyload.h)
        default: return "unknown status";
    }
}

#ifndef CLY_SRC_HASH
#define CLY_SRC_HASH "unknown"
#endif
extern "C" const char* cly_build_info(void) {
    static char buf[200];
    snprintf(buf, sizeof(buf), "clyscan gfx950 scan/link/emit SEG=%d TILE=%lld CAP_T=%u LDS=%d src=%s", CLY_SEG,
             (long long)CLY_TILE, (unsigned)CAP_T, (int)SCAN_LDS, CLY_SRC_HASH);
    return buf;
}
