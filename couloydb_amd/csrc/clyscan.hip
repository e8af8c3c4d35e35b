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
// Launches per call (one HIP stream):
//   k_scan  persistent, one workgroup per CU: CLY_NDW data waves + 1 coordinator
//           wave.  Units (CLY_NDW sub-tiles of 64 stripes) are taken in ticket
//           order; each data wave stages one sub-tile in LDS, speculates and
//           resolves its record chain, checks every CRC and emits tuples; the
//           coordinator composes the unit, runs the decoupled look-back over
//           unit descriptors and hands out exact entries and output slots.
//   k_fin   one workgroup per file: CRC of records that straddle sub-tiles, and
//           the file's first event (ErrInvalidCRC / io.EOF variants / panics).
// Design and data layout: DESIGN.md.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <thread>

#include "scan_core.h"

#ifndef CLY_EXP                 // timing experiments only (tools/exp_time.py): phases skipped, results wrong
#define CLY_EXP 0
#endif
#define CLY_KS_LEVELS 6                          // Kogge-Stone levels over 64 lanes
#define MODE_EMPTY 0                             // sub-tile beyond the end of its file
#define MODE_NORMAL 1                            // the chain enters (or ends) inside the sub-tile
#define MODE_PASS 2                              // one record covers the whole sub-tile
#define MODE_DEAD 3                              // the file's chain ended in an earlier sub-tile

struct DevFile {                 // 32 B
    const uint8_t* base;         // device pointer to the file's first byte (16-B aligned)
    uint64_t len;
    uint32_t fid;
    uint32_t first_sub;          // global index of the file's first sub-tile
    uint32_t nsub;               // sub-tiles of the file (>= 1)
    uint32_t _pad;
};

struct Globals {                 // zeroed per call
    uint32_t ticket;
    uint32_t overflow;           // tuples beyond out_cap were dropped
    uint32_t lb_timeout;         // a look-back / mailbox spin hit its bound (never expected)
    uint32_t fail;               // an internal invariant was violated (never expected)
    uint64_t total;              // tuple slots used (records + any past an ErrInvalidCRC)
    uint32_t nfix;               // fix list length (this round)
    uint32_t fix_total;          // statistics: all fixes of the call
    uint32_t ncand;              // sub-tiles whose chain disagrees with the link (this round)
    uint32_t novf;               // sub-tiles with more tuples than their staging slot
    uint64_t prof[24];           // profiling build (-DCLY_PROF): summed cycles per phase
};

#ifdef CLY_PROF
#define PROF_INIT() uint64_t prof_t = __builtin_amdgcn_s_memtime(); uint64_t prof_acc[12] = {0,0,0,0,0,0,0,0,0,0,0,0}
#define PROF(i) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); prof_acc[i] += t_ - prof_t; prof_t = t_; } while (0)
#define PROF_FLUSH(base) do { if (lane == 0) for (int i_ = 0; i_ < 6; i_++) atomicAdd((unsigned long long*)&g->prof[(base) + i_], (unsigned long long)prof_acc[i_]); } while (0)
#else
#define PROF_INIT()
#define PROF(i)
#define PROF_FLUSH(base)
#endif

struct SubDbg {                  // debug trace of one sub-tile (cly_dbg_enable)
    int32_t mode, E, cnt, term, tst, last, lterm, eof_exit, k0, guess, bad, bpos;
    int64_t tpos, xrel;
};

struct FileOut {
    uint64_t n_records;
    int64_t  end_offset;
    int32_t  status;
    int32_t  ok;
    uint64_t first_index;
};

// ---------------------------------------------------------------------------
// LDS layout of k_scan / k_fix (dynamic shared memory, byte offsets)
//   [0, 65536)        CRC slicing-by-4 tables T0..T3, 16 replicas: dword
//                     (i*64 + t*16 + r) = T_t[i] (replica r); lane l reads replica
//                     l & 15, so one lookup instruction touches 16 banks x 2 lanes
//   [65536, +256)     inverse of a zero-byte step (top byte of T0 -> index)
//   [LDS_WIN + k*WIN) window of wave k (sub-tile + halo, zero past the file end)
//   [LDS_POOL ...)    per-wave check-point pools
//   [LDS_KSNIB ...)   nibble tables of the Kogge-Stone shifts A^(SUB*2^k): 8 x 16 words each
//   then nibble tables of A^(4b), b < 6, and A^(24a), a < HS_A: A^(4w) = A^(4b) A^(24a), w = 6a + b
#define LDS_TAB 0
#define LDS_INV 65536
#define LDS_WIN (LDS_INV + 256)
#define LDS_POOL (LDS_WIN + CLY_NDW * CLY_WIN)
#define LDS_KSNIB (LDS_POOL + CLY_NDW * 192 * 8)
#define HS_A ((CLY_NWD + 5) / 6)
#define NIB_HSB (CLY_KS_LEVELS * 128)                             // word offsets from LDS_KSNIB
#define NIB_HSA (NIB_HSB + 6 * 128)
#define CLY_COLS (NIB_HSA + HS_A * 128)                           // words of the shift tables
#define CLY_SCAN_LDS (LDS_KSNIB + CLY_COLS * 4)

// Per-sub-tile result of k_scan / k_fix, read by the link scan (16 B).
struct SubDesc {
    int64_t  x;                  // global chain position after the sub-tile (MODE_NORMAL, not terminated)
    uint32_t cnt;                // records of the sub-tile under its chain
    int16_t  entry;              // sub-tile-relative entry of the chain (MODE_NORMAL)
    uint8_t  mode;               // MODE_NORMAL / MODE_PASS / MODE_DEAD
    uint8_t  flags;              // SD_*
};
#define SD_TERM 1                // the chain ends inside the sub-tile (incl. at the end of the file)
#define SD_FOF 2                 // first sub-tile of its file
#define SD_OVF 4                 // more tuples than the staging slot holds: k_place emits them from the data
#define CLY_CAP 64               // tuples per sub-tile staging slot

// Link-scan element: what a run of sub-tiles does to the chain state, for
// each state it can be entered in (br[0]: chain live, br[1]: chain already
// ended in this file).  A guessed chain counts only when entered live; the
// first sub-tile of a file resets the state whatever it was.
struct LinkBr {
    int64_t  x;                  // chain position after the run (set)
    uint64_t cnt;                // records the run adds
    int32_t  set;                // the run fixes the state (else: passes it through)
    int32_t  term;               // ... to ended
};
struct LinkAgg { LinkBr br[2]; };
struct Fix {                     // a sub-tile whose chain disagrees with the state the link gives it
    uint32_t s;
    int32_t  mode, entry;        // the chain that state implies (mode < 0: not determined yet)
    uint32_t file;
    int64_t  x_in;               // chain position entering the sub-tile
    uint32_t certain;            // the state is certain (no wrong chain before it in the file)
    uint32_t _pad;
};
#define LISTED_U 0x80000000u     // listed[s] = stamp: certain fix or walked; stamp | LISTED_U: uncertain fix
static_assert(CLY_SCAN_LDS <= 163840, "LDS budget");

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// ---------------------------------------------------------------------------
// small helpers
__device__ __forceinline__ uint64_t ld_agent(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(unsigned long long* p, uint64_t v) {
    __hip_atomic_store(p, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int lds_ld_acq(const CLY_LDS int32_t* p) {
    const int v = *(const volatile CLY_LDS int32_t*)p;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    return v;
}
__device__ __forceinline__ void lds_st_rel(CLY_LDS int32_t* p, int v) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    *(volatile CLY_LDS int32_t*)p = v;
}
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ int wave_min(int v) {
    #pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ int wave_max(int v) {
    #pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ int scan_max_incl(int v, int lane) {
    #pragma unroll
    for (int o = 1; o < 64; o <<= 1) { const int u = __shfl_up(v, o, 64); if (lane >= o) v = max(v, u); }
    return v;
}
__device__ __forceinline__ uint32_t scan_add_incl(uint32_t v, int lane) {
    #pragma unroll
    for (int o = 1; o < 64; o <<= 1) { const uint32_t u = __shfl_up(v, o, 64); if (lane >= o) v += u; }
    return v;
}
__device__ __forceinline__ uint32_t alignb(uint32_t hi, uint32_t lo, uint32_t s) {
    return __builtin_amdgcn_alignbyte(hi, lo, s);
}
// 4 bytes at LDS byte position p (any alignment)
__device__ __forceinline__ uint32_t lds_le32(const CLY_LDS uint32_t* w32, int p) {
    return alignb(w32[(p >> 2) + 1], w32[p >> 2], p & 3);
}
// struct copies to / from LDS (word by word: no generic-pointer flat access)
template <class T> __device__ __forceinline__ T lds_get(const CLY_LDS T* p) {
    static_assert(sizeof(T) % 4 == 0, "word-sized");
    T v;
    uint32_t* d = (uint32_t*)&v;
    const CLY_LDS uint32_t* q = (const CLY_LDS uint32_t*)p;
    #pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); i++) d[i] = q[i];
    return v;
}
template <class T> __device__ __forceinline__ void lds_put(CLY_LDS T* p, const T& v) {
    const uint32_t* d = (const uint32_t*)&v;
    CLY_LDS uint32_t* q = (CLY_LDS uint32_t*)p;
    #pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); i++) q[i] = d[i];
}
#define LDS_SPIN_MAX (1u << 26)
#define LB_SPIN_MAX (1u << 24)

// Wait until *p >= v (LDS mailbox), bounded.
__device__ __forceinline__ bool lds_wait_ge(const CLY_LDS int32_t* p, int v, Globals* g) {
    uint32_t n = 0;
    while (lds_ld_acq(p) < v) {
        __builtin_amdgcn_s_sleep(1);
        if (++n > LDS_SPIN_MAX) { atomicOr(&g->lb_timeout, 2u); return false; }
    }
    return true;
}

// ---------------------------------------------------------------------------
// CRC-32 table step on a 4-byte word: s' = T3[x0]^T2[x1]^T1[x2]^T0[x3] where
// x = s ^ data.  Lookup address = (byte << 8) | lane_off via one v_perm;
// the table number goes into the ds_read offset field.
__device__ __forceinline__ uint32_t tab_addr(uint32_t x, uint32_t lane_off, uint32_t k) {
    return __builtin_amdgcn_perm(x, lane_off, 0x0c0c0000u | ((4u + k) << 8));
}
__device__ __forceinline__ uint32_t crc_word(const CLY_LDS uint8_t* smem, uint32_t x, uint32_t lane_off) {
    const uint32_t a0 = tab_addr(x, lane_off, 0), a1 = tab_addr(x, lane_off, 1);
    const uint32_t a2 = tab_addr(x, lane_off, 2), a3 = tab_addr(x, lane_off, 3);
    const uint32_t t3 = *(const CLY_LDS uint32_t*)(smem + a0 + 3 * 64);
    const uint32_t t2 = *(const CLY_LDS uint32_t*)(smem + a1 + 2 * 64);
    const uint32_t t1 = *(const CLY_LDS uint32_t*)(smem + a2 + 1 * 64);
    const uint32_t t0 = *(const CLY_LDS uint32_t*)(smem + a3 + 0 * 64);
    return t3 ^ t2 ^ t1 ^ t0;
}
// Bank-conflict-free form of crc_word for the main loop.  Table slot k of
// byte row v sits at v*256 + k*64 + replica*4 (replica = lane & 15), so for
// ds_read_b32 (banks (a/4) mod 32 per 32-lane group) lanes l and l+16 hit the
// same bank whenever they read the same slot.  Here lookup i of lanes with
// bit 4 set reads slot i^1 instead of slot i (with the byte that slot takes):
// the two half-groups always read slots 16 banks apart.
#ifndef CLY_CRC_XB
#define CLY_CRC_XB 1
#endif
struct CrcLane { uint32_t oe, oo, s0, s1, s2, s3; };
__device__ __forceinline__ CrcLane crc_lane(int lane) {
    const uint32_t r4 = (uint32_t)(lane & 15) * 4, h = (uint32_t)(lane >> 4) & 1u;
    CrcLane c;
    c.oe = r4 + 64 * h;                      // even lookups: offset field i*64
    c.oo = r4 + 64 * (1 - h);                // odd lookups: offset field (i-1)*64
    // lookup i reads slot i^h, which takes byte 3 - (i^h) of x
    c.s0 = 0x0c0c0000u | ((4u + (3u - (0u ^ h))) << 8);
    c.s1 = 0x0c0c0000u | ((4u + (3u - (1u ^ h))) << 8);
    c.s2 = 0x0c0c0000u | ((4u + (3u - (2u ^ h))) << 8);
    c.s3 = 0x0c0c0000u | ((4u + (3u - (3u ^ h))) << 8);
    return c;
}
__device__ __forceinline__ uint32_t crc_word_xb(const CLY_LDS uint8_t* smem, uint32_t x, const CrcLane& c) {
    const uint32_t a0 = __builtin_amdgcn_perm(x, c.oe, c.s0), a1 = __builtin_amdgcn_perm(x, c.oo, c.s1);
    const uint32_t a2 = __builtin_amdgcn_perm(x, c.oe, c.s2), a3 = __builtin_amdgcn_perm(x, c.oo, c.s3);
    const uint32_t t0 = *(const CLY_LDS uint32_t*)(smem + a0);
    const uint32_t t1 = *(const CLY_LDS uint32_t*)(smem + a1);
    const uint32_t t2 = *(const CLY_LDS uint32_t*)(smem + a2 + 128);
    const uint32_t t3 = *(const CLY_LDS uint32_t*)(smem + a3 + 128);
    return t0 ^ t1 ^ t2 ^ t3;
}
// one byte through the register (table T0, replica of lane_off)
__device__ __forceinline__ uint32_t crc_byte(const CLY_LDS uint8_t* smem, uint32_t s, uint32_t b, uint32_t lane_off) {
    const uint32_t i = (s ^ b) & 0xff;
    return *(const CLY_LDS uint32_t*)(smem + ((i << 8) | lane_off)) ^ (s >> 8);
}
// inverse of one zero-byte step: s = A^-1 s'
__device__ __forceinline__ uint32_t crc_unbyte(const CLY_LDS uint8_t* smem, uint32_t s, uint32_t lane_off) {
    const uint32_t i = smem[LDS_INV + (s >> 24)];
    const uint32_t t = *(const CLY_LDS uint32_t*)(smem + ((i << 8) | lane_off));
    return ((s ^ t) << 8) | i;
}

// M v for a linear map M given by its nibble tables (word offset `off` from
// LDS_KSNIB: 8 x 16 words, entry n*16+k = M (k << 4n)): 8 lookups
__device__ __forceinline__ uint32_t nib_mul(const CLY_LDS uint8_t* smem, int off, uint32_t v) {
    const CLY_LDS uint32_t* t = (const CLY_LDS uint32_t*)(smem + LDS_KSNIB) + off;
    uint32_t p = 0;
    #pragma unroll
    for (int n = 0; n < 8; n++) p ^= t[n * 16 + ((v >> (4 * n)) & 15u)];
    return p;
}
// A^(SUB*2^lvl) v
__device__ __forceinline__ uint32_t ks_mul(const CLY_LDS uint8_t* smem, int lvl, uint32_t v) {
    return nib_mul(smem, lvl * 128, v);
}
// A^(4w) v, w < NWD
__device__ __forceinline__ uint32_t word_shift(const CLY_LDS uint8_t* smem, int w, uint32_t v) {
    const int a = w / 6, b = w - 6 * a;
    return nib_mul(smem, NIB_HSB + b * 128, nib_mul(smem, NIB_HSA + a * 128, v));
}

// ---------------------------------------------------------------------------
// Header decode at window position p: fast path for headers whose three
// varints are at most 4 bytes each and end within bytes 6..13 (every record
// the writer produces except multi-byte expirations / huge sizes), else the
// exact byte-loop form step_hdr.
__device__ __noinline__ void hdr_slow(const CLY_LDS uint8_t* w8, int64_t p, int64_t nrel, int64_t p_abs, Hdr& h) {
    h = step_hdr(w8, p, nrel, p_abs);
}
__device__ __forceinline__ uint32_t pack7(uint32_t s) {
    return (s & 0x7fu) | ((s >> 1) & 0x3f80u) | ((s >> 2) & 0x1fc000u) | ((s >> 3) & 0xfe00000u);
}
__device__ __forceinline__ Hdr hdr_at(const CLY_LDS uint32_t* w32, int p, int64_t nrel, int64_t p_abs) {
    int64_t m = nrel - p;
    if (m > 26) m = 26;
    if (m >= 14) {
        const int wi = p >> 2;
        const uint32_t s = p & 3;
        const uint32_t a0 = w32[wi], a1 = w32[wi + 1], a2 = w32[wi + 2], a3 = w32[wi + 3], a4 = w32[wi + 4];
        const uint32_t h0 = alignb(a1, a0, s), h1 = alignb(a2, a1, s), h2 = alignb(a3, a2, s), h3 = alignb(a4, a3, s);
        const uint32_t lo = alignb(h2, h1, 2), hi = alignb(h3, h2, 2);       // bytes 6..9, 10..13
        const uint64_t W = ((uint64_t)hi << 32) | lo;
        const uint64_t T = ~W & 0x8080808080808080ull;
        const uint64_t T2 = T & (T - 1), T3 = T2 & (T2 - 1);
        const int e1 = __builtin_ctzll(T | (1ull << 63)) >> 3;
        const int e2 = __builtin_ctzll(T2 | (1ull << 63)) >> 3;
        const int e3 = __builtin_ctzll(T3 | (1ull << 63)) >> 3;
        const int n1 = e1 + 1, n2 = e2 - e1, n3 = e3 - e2;
        if (T3 != 0 && n1 <= 4 && n2 <= 4 && n3 <= 4 && 6 + e3 < m) {
            const uint32_t u1 = pack7((uint32_t)W) & ((1u << (7 * n1)) - 1);
            const uint32_t u2 = pack7((uint32_t)(W >> (8 * n1))) & ((1u << (7 * n2)) - 1);
            const uint32_t u3 = pack7((uint32_t)(W >> (8 * (e2 + 1)))) & ((1u << (7 * n3)) - 1);
            const int32_t v1 = (int32_t)(u1 >> 1) ^ -(int32_t)(u1 & 1);
            const int32_t v2 = (int32_t)(u2 >> 1) ^ -(int32_t)(u2 & 1);
            const int32_t v3 = (int32_t)(u3 >> 1) ^ -(int32_t)(u3 & 1);
            Hdr h;
            h.crc = h0;
            h.type = h1 & 0xff;
            h.dt = (h1 >> 8) & 0xff;
            h.ks = (uint32_t)v1;
            h.vs = (uint32_t)v2;
            h.exp = v3;
            h.hsz = 7 + e3;
            h.size = 0;
            h.good = false;
            if (h.crc == 0 && h.ks == 0 && h.vs == 0) { h.status = CLY_END_ZERO; return h; }
            const int64_t kv = (int64_t)h.ks + (int64_t)h.vs;
            if (kv > 0 && nrel - (p + h.hsz) < kv) { h.status = CLY_END_TORN; return h; }
            h.status = REC_OK;
            h.size = h.hsz + kv;
            h.good = h.type <= 4 && h.dt <= 4 && v1 >= 1 && v2 >= 0;
            return h;
        }
    }
    Hdr h;
    hdr_slow((const CLY_LDS uint8_t*)w32, p, nrel, p_abs, h);
    return h;
}

// Header at a position beyond the staged window (exit check of a long record):
// read from global memory.
__device__ __noinline__ void hdr_global(const uint8_t* gfile, int64_t cbase, int64_t x, int64_t nrel, Hdr& h) {
    // bytes [x, x+26) from the dwords covering them (never past the file's last dword)
    uint32_t wv[8];
    const int64_t a = cbase + x, a0 = a & ~3ll;
    const int64_t flen = cbase + nrel;
    const uint32_t* gw = (const uint32_t*)(gfile + a0);
    #pragma unroll
    for (int k = 0; k < 8; k++) wv[k] = (a0 + 4 * k < flen) ? gw[k] : 0u;
    uint8_t hb[28];
    const int sh = (int)(a - a0);
    const int64_t need = nrel - x < 26 ? nrel - x : 26;
    #pragma unroll
    for (int k = 0; k < 26; k++) {
        const int q = k + sh;
        hb[k] = k < need ? (uint8_t)(wv[q >> 2] >> (8 * (q & 3))) : 0;
    }
    h = step_hdr(hb, 0, nrel - x, cbase + x);
}

// SWAR byte masks (bit 7 of each byte): byte <= 4 (type/dtype), and
// byte nonzero and even (first byte of the key-size varint of a record with ks >= 1).
__device__ __forceinline__ uint32_t swar_le4(uint32_t W) { return ~(((W | 0x80808080u) - 0x05050505u) | W) & 0x80808080u; }
__device__ __forceinline__ uint32_t swar_ks(uint32_t W) {
    const uint32_t nz = ((W & 0x7f7f7f7fu) + 0x7f7f7f7fu) | W;
    return nz & ~(W << 7) & 0x80808080u;
}
// ---------------------------------------------------------------------------
// Sub-tile context (wave-uniform, registers)
struct Sub {
    const uint8_t* gfile;        // the file's bytes (HBM)
    const CLY_LDS uint32_t* w32; // window
    int64_t cbase;               // file offset of the sub-tile
    int64_t nrel;                // bytes from the sub-tile start to the end of the file
    int     dlen;                // data bytes in the sub-tile (<= TS)
    int     win_len;             // bytes staged in the window
    int     fof, lof;            // first / last sub-tile of its file
    int64_t chunk;               // global sub-tile index (ChunkSum slot)
    uint32_t fid;
};

// Per-lane chain state of a resolved sub-tile
struct Lane {
    int      ws;                 // first chain record starting in the stripe (-1 none)
    int      wc;                 // chain records starting in the stripe
    int      wl;                 // last of them
    int64_t  wx;                 // exit of the stripe's chain part, or terminal position
    int      wterm, wtst;        // terminal inside the stripe
    int      pk;                 // last lane <= this one holding a chain record (-1 none)
    uint32_t base;               // chain records before the stripe
};
struct Chain {                   // wave-uniform result of resolve()
    int      mode;
    int      E;                  // entry (sub-tile-relative)
    int      k0;                 // lane of E
    uint32_t cnt;                // records in the sub-tile
    int      term, tst;          // the chain ends inside the sub-tile (incl. at the file end)
    int64_t  tpos;               // terminal position
    int64_t  xrel;               // exit when not terminated
    int      last;               // start of the last record (-1 none)
    int      lterm;              // lane of the terminal (CLY_NT none)
    int      eof_exit;           // leaves the file's last sub-tile exactly at the end of the file
};

// Speculative walk of one lane: first candidate in its stripe whose chain of
// plain records leaves the stripe at an exit that decodes as a plain record
// (or is the end of the file).
struct Spec {
    int s, last, c;
    int v;                       // the exit was checked (else: beyond the window, unchecked)
    int64_t x;
    Hdr h;                       // header of the record at s (reused for its tuple)
};

// Exact walk (ReadLogRecord semantics, any record or terminal) of the lane's
// stripe [a, b) from position e.
__device__ __forceinline__ void exact_walk(const Sub& T, int a, int b, int e, Lane& L) {
    (void)a;
    L.ws = e;
    int64_t p = e;
    int c = 0, last = -1;
    for (;;) {
        const Hdr h = hdr_at(T.w32, (int)p, T.nrel, T.cbase + p);
        if (h.status != REC_OK) { L.wc = c; L.wl = last; L.wx = p; L.wterm = 1; L.wtst = h.status; return; }
        c++;
        last = (int)p;
        const int64_t p2 = p + h.size;
        if (p2 >= b) { L.wc = c; L.wl = last; L.wx = p2; L.wterm = 0; L.wtst = 0; return; }
        p = p2;
    }
}

// Candidate bits of stripe word m (positions 4m..4m+3 of the stripe starting at
// window byte a): type and data type bytes <= 4 (bit 8j+7 for position 4m+j).
__device__ __forceinline__ uint32_t cand_bits(const CLY_LDS uint32_t* w32, int a, int m) {
    const int i = (a >> 2) + m + 1;
    const uint32_t L1 = swar_le4(w32[i]), L2 = swar_le4(w32[i + 1]);
    return L1 & __builtin_amdgcn_alignbit(L2, L1, 8);
}

// Speculative walk of one lane: the first candidate of its stripe (from the
// word mask wm) whose chain of plain records leaves the stripe at an exit that
// decodes as a plain record or is the end of the file; failing that, the first
// whose exit lies beyond the window (left unchecked: the chain check of
// resolve() and the guess's own deep check cover it).  Candidates whose
// key-size byte is odd or zero (ks < 1) are skipped before decoding.
__device__ __forceinline__ void spec_lane(const Sub& T, int lane, uint64_t wm, Spec& r) {
    r.s = -1; r.last = -1; r.c = 0; r.v = 0; r.x = 0;
    const int a = lane * CLY_SUB;
    if (a >= T.dlen) return;
    const int b = a + CLY_SUB < T.dlen ? a + CLY_SUB : T.dlen;
    const CLY_LDS uint8_t* w8 = (const CLY_LDS uint8_t*)T.w32;
    // (one flat loop over (word, bit): the nested form of this loop with the
    // early return was miscompiled by the ROCm 7.2 toolchain - R.last came out -1)
    uint32_t cm = 0;
    int m = 0;
    for (;;) {
        if (cm == 0) {
            if (wm == 0) break;
            m = __builtin_ctzll(wm);
            wm &= wm - 1;
            cm = cand_bits(T.w32, a, m);
            continue;
        }
        {
            const int q = a + 4 * m + (__builtin_ctz(cm) >> 3);
            cm &= cm - 1;
            if (q >= b) break;
            const uint32_t kb = w8[q + 6];          // key-size varint: >= 1 needs an even nonzero first byte
            if (kb == 0 || (kb & 1)) continue;
            const Hdr h = hdr_at(T.w32, q, T.nrel, T.cbase + q);
            if (!h.good) continue;
            int64_t p = q;
            int c = 1;
            int64_t x = p + h.size;
            bool ok = true;
            while (x < b) {
                const Hdr h2 = hdr_at(T.w32, (int)x, T.nrel, T.cbase + x);
                if (!h2.good) { ok = false; break; }
                p = x;
                c++;
                x = p + h2.size;
            }
            if (!ok || x > T.nrel) continue;           // a chain past the end of the file is not a guess
            if (x < T.nrel && x + 26 > T.win_len) {
                // exit beyond the window: kept unchecked as a fallback, but a
                // later candidate with a checked exit wins (a false candidate
                // must not hide the lane's true record)
                if (r.s < 0) { r.s = q; r.last = (int)p; r.c = c; r.v = 0; r.x = x; r.h = h; }
                continue;
            }
            if (x < T.nrel) {
                const Hdr e = hdr_at(T.w32, (int)x, T.nrel, T.cbase + x);
                if (!e.good) continue;
            }
            r.s = q; r.last = (int)p; r.c = c; r.v = 1; r.x = x; r.h = h;
            return;
        }
    }
}

// Second exit check of a speculative chain leaving its stripe at x: the record
// at x and the one after it must decode as plain records.
__device__ __forceinline__ int deep_check(const Sub& T, int64_t x) {
    if (x >= T.nrel) return x == T.nrel;
    Hdr e;
    if (x + 26 <= T.win_len) e = hdr_at(T.w32, (int)x, T.nrel, T.cbase + x);
    else hdr_global(T.gfile, T.cbase, x, T.nrel, e);
    if (!e.good) return 0;
    const int64_t x2 = x + e.size;
    if (x2 >= T.nrel) return x2 == T.nrel;
    Hdr f;
    if (x2 + 26 <= T.win_len) f = hdr_at(T.w32, (int)x2, T.nrel, T.cbase + x2);
    else hdr_global(T.gfile, T.cbase, x2, T.nrel, f);
    return f.good ? 1 : 0;
}

// Speculation over the staged window: per lane the candidate word mask of its
// stripe (register SWAR filter), then the candidate walks; the sub-tile guess.
__device__ __forceinline__ void sub_spec(const Sub& T, int lane, Spec& sp, int& guess) {
    const CLY_LDS uint32_t* w32 = T.w32;
    uint64_t wm = 0;
    const int a = lane * CLY_SUB;
    if (a < T.dlen) {
        uint32_t dw[CLY_NWD + 2];
        const CLY_LDS u32x4* s4 = (const CLY_LDS u32x4*)(w32 + lane * CLY_NWD);
        #pragma unroll
        for (int i = 0; i < CLY_NWD / 4; i++) {
            const u32x4 v = s4[i];
            dw[4 * i] = v.x; dw[4 * i + 1] = v.y; dw[4 * i + 2] = v.z; dw[4 * i + 3] = v.w;
        }
        dw[CLY_NWD] = w32[lane * CLY_NWD + CLY_NWD];
        dw[CLY_NWD + 1] = w32[lane * CLY_NWD + CLY_NWD + 1];
        uint32_t wlo = 0, whi = 0;
        uint32_t Ln = swar_le4(dw[CLY_NWD + 1]);
        #pragma unroll
        for (int m = CLY_NWD - 1; m >= 0; m--) {
            const uint32_t Lm = swar_le4(dw[m + 1]);
            const uint32_t cm = Lm & __builtin_amdgcn_alignbit(Ln, Lm, 8);
            if (m < 32) wlo |= cm ? (1u << m) : 0u;
            else whi |= cm ? (1u << (m - 32)) : 0u;
            Ln = Lm;
        }
        wm = ((uint64_t)whi << 32) | wlo;
    }
    spec_lane(T, lane, wm, sp);
    if (T.fof) { guess = 0; return; }
    // guess: the first lane whose chain also survives a second exit check
    // (a lane whose exit is where the stripe holding it starts its own chain is
    // confirmed without it)
    const bool ext = sp.s >= 0 && sp.x < T.dlen;
    const int tl = ext ? (int)(sp.x / CLY_SUB) : lane;
    const int ts = __shfl(sp.s, tl, 64), tv = __shfl(sp.v, tl, 64);
    const int conf = ext && ts == (int)sp.x && tv;      // (an unchecked spec confirms nothing)
    unsigned long long m = __ballot(sp.s >= 0);
    guess = -1;
    while (m) {
        const int k = __ffsll((long long)m) - 1;
        int ok = conf;
        if (lane == k && !ok) ok = deep_check(T, sp.x);
        if (__shfl(ok, k, 64)) { guess = __shfl(sp.s, k, 64); break; }
        m &= m - 1;
    }
}

// resolve(E): the sub-tile's record chain from entry E (sub-tile-relative).
__device__ __forceinline__ void resolve(const Sub& T, const Spec& sp, int lane, int E, Lane& L, Chain& R) {
    R.mode = MODE_NORMAL; R.E = E; R.eof_exit = 0;
    if (E >= T.dlen) {
        // only in the file's last sub-tile: E is the end of the file (ReadLogRecord there: io.EOF)
        L.ws = -1; L.wc = 0; L.wl = -1; L.wx = 0; L.wterm = 0; L.wtst = 0; L.pk = -1; L.base = 0;
        const Hdr h = hdr_at(T.w32, E, T.nrel, T.cbase + E);
        R.k0 = CLY_NT; R.cnt = 0; R.last = -1; R.lterm = CLY_NT; R.xrel = E; R.tpos = E;
        R.term = h.status != REC_OK;
        R.tst = h.status != REC_OK ? h.status : 0;
        return;
    }
    const int k0 = E / CLY_SUB;
    const int a = lane * CLY_SUB;
    const int b = a + CLY_SUB < T.dlen ? a + CLY_SUB : T.dlen;
    const bool in = a < T.dlen;
    if (lane < k0 || !in) { L.ws = -1; L.wc = 0; }
    else { L.ws = sp.s; L.wc = sp.c; }
    L.wl = sp.last; L.wx = sp.x; L.wterm = 0; L.wtst = 0;
    if (lane == k0 && L.ws != E) exact_walk(T, a, b, E, L);
    int kill = __shfl(L.wterm, k0, 64) ? k0 : CLY_NT;
    if (lane > kill) L.ws = -1;
    for (int iter = 0;; iter++) {
        L.pk = scan_max_incl(L.ws >= 0 ? lane : -1, lane);
        const int j = __shfl_up(L.pk, 1, 64);
        const int64_t Xj = __shfl(L.wx, j < 0 ? 0 : j, 64);
        const int wtj = __shfl(L.wterm, j < 0 ? 0 : j, 64);
        bool bad = false;
        if (lane > k0 && in && j >= 0 && !wtj) {
            if (L.ws >= 0) bad = Xj != (int64_t)L.ws;
            else bad = Xj < (int64_t)b;
        }
        const unsigned long long bm = __ballot(bad);
        if (!bm) break;
        if (iter > CLY_NT + 1) break;                   // cannot happen: every fix advances
        const int kstar = __ffsll((long long)bm) - 1;
        const int jj = __shfl(L.pk, kstar - 1, 64);
        const int64_t X = __shfl(L.wx, jj, 64);
        const int K = X < T.dlen ? (int)(X / CLY_SUB) : CLY_NT;
        if (lane > jj && lane < K) L.ws = -1;
        if (K < CLY_NT) {
            const int wsK = __shfl(L.ws, K, 64);
            if (wsK != (int)X) {
                if (lane == K) exact_walk(T, a, b, (int)X, L);
                if (__shfl(L.wterm, K, 64) && lane > K) L.ws = -1;
            }
        }
    }
    const uint32_t cnt = L.ws >= 0 ? (uint32_t)L.wc : 0u;
    const uint32_t incl = scan_add_incl(cnt, lane);
    L.base = incl - cnt;
    const int Ll = __shfl(L.pk, CLY_NT - 1, 64);
    R.k0 = k0;
    R.cnt = __shfl(incl, CLY_NT - 1, 64);
    R.term = __shfl(L.wterm, Ll, 64);
    R.tst = __shfl(L.wtst, Ll, 64);
    R.lterm = R.term ? Ll : CLY_NT;
    R.tpos = __shfl(L.wx, Ll, 64);
    R.xrel = R.tpos;
    R.last = __shfl(L.wl, Ll, 64);
    if (!R.term && T.lof && R.xrel == T.nrel) {
        // the chain leaves the file's last sub-tile exactly at the end of the
        // file: the next ReadLogRecord there returns io.EOF
        R.term = 1; R.tst = CLY_END_EOF; R.tpos = R.xrel; R.eof_exit = 1;
        // the lane holding the end of the file owns that check point
        const int lt = R.xrel < CLY_TS ? (int)(R.xrel / CLY_SUB) : CLY_NT;
        R.lterm = lt;
        if (lane == lt) { L.wterm = 1; L.wx = R.xrel; L.wtst = CLY_END_EOF; }
    }
}

__device__ __forceinline__ void chain_none(Lane& L, Chain& R, int mode) {
    L.ws = -1; L.wc = 0; L.wl = -1; L.wx = 0; L.wterm = 0; L.wtst = 0; L.pk = -1; L.base = 0;
    R.mode = mode; R.E = CLY_TS; R.k0 = CLY_NT; R.cnt = 0; R.term = mode == MODE_DEAD; R.tst = 0; R.tpos = 0;
    R.xrel = 0; R.last = -1; R.lterm = CLY_NT; R.eof_exit = 0;
}

// ---------------------------------------------------------------------------
// CRC of every record of the resolved chain.
//
// Check points: every chain record start P (its predecessor's region ends at
// P) and the terminal position.  XOR patches on the LDS window make one
// uniform word loop verify all of them:
//   W_a = word of P:     stored-CRC bytes (>= P) zeroed, and, when the record
//                        ending at P started inside the sub-tile, Q = A^-j ~crc
//                        XORed in, so that the register after W_a is zero iff
//                        that record's CRC matches;
//   W_b = W_a + 1:       rest of the stored CRC zeroed, 0xFF init on region bytes;
//   W_c = W_a + 2:       0xFF init on the rest of the first 4 region bytes.
// Each lane runs its stripe from register 0; the first check point whose W_b
// lies in the stripe is a hard reset (the register before it is kept as
// `obs`), later ones are observed directly (`chk` words).  A segmented
// Kogge-Stone scan over lanes gives the register entering each stripe; the
// reset check is obs ^ A^(4*rs) S_in.  All patches are XORs, so applying them
// a second time restores the window.
struct CrcOut {
    uint32_t first4, open_crc, open_tail;   // pristine window values for the summary
    int      bad;                // some check failed (localised by crc_locate)
    uint32_t head_raw, head_z;   // Z_z(raw [4, E)) for k_fin
    uint32_t end_state;          // register at the end of the sub-tile (lane 63's inclusive scan)
};

// Check points are collected (positions + the 4 bytes stored there) from the
// pristine window into a per-wave pool before any patch is applied, in chain
// order; patches, marks and the restore pass all read the pool.
#define CP_POOL 192
#define CP_REAL 0x10000u

// Patch words of pool entry m (pos P, stored bytes c; cprev = previous entry's
// stored bytes, or none for the sub-tile's first check point).
__device__ __forceinline__ void crc_apply(CLY_LDS uint8_t* smem, CLY_LDS uint32_t* w32, uint32_t lane_off, uint32_t ent,
                                          uint32_t c, bool has_prev, uint32_t cprev) {
    const int P = (int)(ent & 0xffff);
    const bool real = (ent & CP_REAL) != 0;
    const int j = P & 3, wa = P >> 2;
    const uint32_t lom = j ? (1u << (8 * j)) - 1 : 0u, him = ~lom;
    uint32_t pa = j ? (c << (8 * j)) : c;
    uint32_t pb = j ? (c >> (32 - 8 * j)) : 0u;
    uint32_t pc = 0;
    if (real) { pb ^= him; pc = lom; }
    if (has_prev) {
        uint32_t q = ~cprev;
        for (int k = 0; k < j; k++) q = crc_unbyte(smem, q, lane_off);
        pa ^= q;
    }
    __hip_atomic_fetch_xor(&w32[wa], pa, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    if (pb) __hip_atomic_fetch_xor(&w32[wa + 1], pb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    if (pc) __hip_atomic_fetch_xor(&w32[wa + 2], pc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

__device__ __forceinline__ void crc_patch_all(CLY_LDS uint8_t* smem, CLY_LDS uint32_t* w32, const CLY_LDS u32x2* pool,
                                              int off, int n, uint32_t lane_off) {
    for (int i = off; i < off + n; i++) {
        const u32x2 e = pool[i];
        const bool has_prev = i > 0;
        const uint32_t cprev = has_prev ? pool[i - 1].y : 0u;
        crc_apply(smem, w32, lane_off, e.x, e.y, has_prev, cprev);
    }
}

// Register of one lane over its stripe words d[] (patched), with the reset.
template <bool OBSERVE>
__device__ __forceinline__ void crc_loop(const CLY_LDS uint8_t* smem, const uint32_t* d, int rs, uint64_t chk,
                                         uint32_t lane_off, uint32_t& s_out, uint32_t& obs_out, uint32_t& err_out) {
    uint32_t s = 0, obs = 0, err = 0;
    const uint32_t chk_lo = (uint32_t)chk, chk_hi = (uint32_t)(chk >> 32);
#if CLY_CRC_XB
    const CrcLane cl = crc_lane((int)__lane_id());
#endif
    #pragma unroll
    for (int i = 0; i < CLY_NWD; i++) {
        const bool r = i == rs;
        obs = r ? s : obs;
        const uint32_t x = (r ? 0u : s) ^ d[i];
#if CLY_CRC_XB
        s = crc_word_xb(smem, x, cl);
#else
        s = crc_word(smem, x, lane_off);
#endif
        if (OBSERVE) {
            // all-ones when word i holds a check point: one v_bfe_i32 (and the
            // AND-OR below fuses) instead of and + cmp + cndmask per word
            const uint32_t cw = i < 32 ? chk_lo : chk_hi;
            const uint32_t m = (uint32_t)__builtin_amdgcn_sbfe((int32_t)cw, (uint32_t)(i & 31), 1u);
            err |= s & m;
        }
    }
    s_out = s; obs_out = obs; err_out = err;
}

// The same register without observations, as two independent chains over the
// stripe's halves (twice the lookups in flight): the second half runs from 0
// and the halves are joined by linearity, s = A^(4 H) s1 ^ s2 when the reset
// (if any) is in the first half; with the reset in the second half the
// register before it is A^(4 (rs - H)) s1 ^ ob, and s = s2.
// (measured on C2: no gain over the single chain, 3.31 vs 3.25-3.29 ms; kept off)
#ifndef CLY_CRC_SPLIT
#define CLY_CRC_SPLIT 0
#endif
#define CRC_H (CLY_NWD / 2)
__device__ __forceinline__ uint32_t word_shift(const CLY_LDS uint8_t* smem, int w, uint32_t v);
__device__ __forceinline__ uint32_t nib_mul(const CLY_LDS uint8_t* smem, int off, uint32_t v);
__device__ __forceinline__ void crc_loop_split(const CLY_LDS uint8_t* smem, const uint32_t* d, int rs, uint32_t lane_off,
                                               uint32_t& s_out, uint32_t& obs_out) {
    uint32_t sa = 0, sb = 0, oa = 0, ob = 0;
#if CLY_CRC_XB
    const CrcLane cl = crc_lane((int)__lane_id());
#endif
    #pragma unroll
    for (int i = 0; i < CRC_H; i++) {
        const bool ra = i == rs, rb = i + CRC_H == rs;
        oa = ra ? sa : oa;
        ob = rb ? sb : ob;
        const uint32_t xa = (ra ? 0u : sa) ^ d[i];
        const uint32_t xb = (rb ? 0u : sb) ^ d[i + CRC_H];
#if CLY_CRC_XB
        sa = crc_word_xb(smem, xa, cl);
        sb = crc_word_xb(smem, xb, cl);
#else
        sa = crc_word(smem, xa, lane_off);
        sb = crc_word(smem, xb, lane_off);
#endif
    }
    if (rs >= CRC_H) {
        obs_out = ob ^ word_shift(smem, rs - CRC_H, sa);
        s_out = sb;
    } else {
        obs_out = oa;
#if CRC_H % 6 == 0
        s_out = nib_mul(smem, NIB_HSA + (CRC_H / 6) * 128, sa) ^ sb;     // A^(24 a) table, a = H/6
#else
        s_out = word_shift(smem, CRC_H, sa) ^ sb;
#endif
    }
}

__device__ __noinline__ void crc_slow(const CLY_LDS uint32_t* w32, int64_t nrel, int64_t cbase, int E, uint32_t cnt,
                                      CLY_LDS uint8_t* smem, CrcOut& out);

__device__ __forceinline__ void crc_phase(const Sub& T, const Lane& L, const Chain& R, int lane, CLY_LDS uint8_t* smem,
                                       CLY_LDS uint32_t* w32, CLY_LDS u32x2* pool, CrcOut& out) {
    const uint32_t lane_off = (uint32_t)(lane & 15) * 4;
    out.bad = 0; out.head_raw = 0; out.head_z = 0; out.end_state = 0;
    const bool normal = R.mode == MODE_NORMAL;
    out.first4 = w32[0];
    out.open_crc = 0; out.open_tail = 0xFFFFFFFFu;
    if (normal && R.last >= 0) {
        out.open_crc = lds_le32(w32, R.last);
        const int ocs = R.last + 4;
        if (ocs < CLY_TS && ocs + 4 > CLY_TS) {
            const CLY_LDS uint8_t* w8 = (const CLY_LDS uint8_t*)w32;
            uint32_t st = 0xFFFFFFFFu;
            for (int q = ocs; q < CLY_TS; q++) st = crc_byte(smem, st, w8[q], lane_off);
            out.open_tail = st;
        }
    }
    // ---- check points of this lane: chain records, then its terminal
    const bool tcp = normal && L.wterm && L.wx < CLY_TS;
    const int n = normal ? ((L.ws >= 0 ? L.wc : 0) + (tcp ? 1 : 0)) : 0;
    const uint32_t incl = scan_add_incl((uint32_t)n, lane);
    const int off = (int)(incl - (uint32_t)n);
    const int total = (int)__shfl(incl, CLY_NT - 1, 64);
    if (total > CP_POOL) {
        if (lane == 0) {
            CrcOut t;                               // (own object: `out` stays in registers)
            crc_slow(w32, T.nrel, T.cbase, R.E, R.cnt, smem, t);
            out.bad = t.bad; out.head_raw = t.head_raw; out.head_z = t.head_z; out.end_state = t.end_state;
        }
        out.bad = __shfl(out.bad, 0, 64); out.head_raw = __shfl(out.head_raw, 0, 64);
        out.head_z = __shfl(out.head_z, 0, 64); out.end_state = __shfl(out.end_state, 0, 64);
        return;
    }
    if (n && !(CLY_EXP & 64)) {
        int i = off;
        if (L.ws >= 0) {
            int p = L.ws;
            for (int r = 0; r < L.wc; r++, i++) {
                pool[i] = (u32x2){(uint32_t)p | CP_REAL, lds_le32(w32, p)};
                if (r + 1 < L.wc) {
                    const Hdr h = hdr_at(w32, p, T.nrel, T.cbase + p);
                    p += (int)h.size;
                }
            }
        }
        if (tcp) pool[i] = (u32x2){(uint32_t)L.wx, lds_le32(w32, (int)L.wx)};
    }
    wave_sync();
    if (!(CLY_EXP & 64)) crc_patch_all(smem, w32, pool, off, n, lane_off);
    wave_sync();
    // ---- reset word and check mask (lane-local word indices)
    const int w0 = lane * CLY_NWD;
    int rs = -1, rs_first = 0;
    uint64_t chk = 0;
    if (off > 0) {
        const int P = (int)(pool[off - 1].x & 0xffff);
        if ((P >> 2) + 1 == w0) { rs = 0; rs_first = P == R.E; }
    }
    for (int i = off; i < off + n; i++) {
        const int P = (int)(pool[i].x & 0xffff);
        const int wa = (P >> 2) - w0;
        if (rs < 0) {
            if (wa + 1 < CLY_NWD) { rs = wa + 1; rs_first = P == R.E; }
        } else {
            chk |= 1ull << wa;
        }
    }
    // ---- stripe words
    uint32_t d[CLY_NWD];
    {
        const CLY_LDS u32x4* s4 = (const CLY_LDS u32x4*)(w32 + lane * CLY_NWD);
        #pragma unroll
        for (int i = 0; i < CLY_NWD / 4; i++) {
            const u32x4 v = s4[i];
            d[4 * i] = v.x; d[4 * i + 1] = v.y; d[4 * i + 2] = v.z; d[4 * i + 3] = v.w;
        }
        if (lane == 0) d[0] = 0;                // head raw register counts from byte 4
    }
    uint32_t s, obs, err;
    // (no lane with a second check point: the loop without observations)
    if (CLY_EXP & 32) { s = d[0] ^ d[CLY_NWD - 1]; obs = d[1]; err = 0; }   // experiment: no CRC loop
    else if (__ballot(chk != 0)) crc_loop<true>(smem, d, rs, chk, lane_off, s, obs, err);
#if CLY_CRC_SPLIT
    else { crc_loop_split(smem, d, rs, lane_off, s, obs); err = 0; }
#else
    else crc_loop<false>(smem, d, rs, chk, lane_off, s, obs, err);
#endif
    // ---- segmented scan: element (c, v), S -> c ? v : A^SUB S ^ v
    int c = rs >= 0;
    uint32_t v = s;
    #pragma unroll
    for (int lvl = 0; lvl < CLY_KS_LEVELS; lvl++) {
        const int dd = 1 << lvl;
        const bool fin_lane = c || lane < dd;
        if (__ballot(!fin_lane) == 0ull) break;
        const int pc = __shfl_up(c, dd, 64);
        const uint32_t pv = __shfl_up(v, dd, 64);
        if (!fin_lane) { v ^= ks_mul(smem, lvl, pv); c = pc; }
    }
    uint32_t s_in = __shfl_up(v, 1, 64);
    if (lane == 0) s_in = 0;
    out.end_state = __shfl(v, CLY_NT - 1, 64);
    // ---- reset checks: T = obs ^ A^(4 rs) S_in
    const uint32_t y = word_shift(smem, rs > 0 ? rs : 0, s_in);
    const uint32_t Tv = obs ^ y;
    bool bad = err != 0;
    if (rs >= 0 && !rs_first) bad |= Tv != 0;
    const unsigned long long hm = __ballot(rs >= 0 && rs_first);
    if (hm) {
        out.head_raw = __shfl(Tv, __ffsll((long long)hm) - 1, 64);
        out.head_z = 4 - (R.E & 3);
    } else if (normal && R.E < T.dlen) {
        // the check point at E is in the sub-tile's last word (its reset word
        // is outside): the register at the end is Z_z(raw [4, E))
        out.head_raw = out.end_state;
        out.head_z = 4 - (R.E & 3);
    } else {
        out.head_raw = out.end_state;     // no boundary: the whole sub-tile is head
        out.head_z = (uint32_t)(CLY_TS - T.dlen);
    }
    // a later check point in the last word: observed at the end of the sub-tile
    if (normal && total > 0) {
        const int Pl = (int)(pool[total - 1].x & 0xffff);
        if ((Pl >> 2) + 1 == CLY_NT * CLY_NWD && Pl != R.E && out.end_state != 0) bad = true;
    }
    out.bad = __ballot(bad && normal) != 0ull;
    if (CLY_EXP & 96) out.bad = 0;                  // experiments: checks meaningless
    // ---- restore the window for crc_locate (XOR patches are involutions);
    // nothing else reads it after this phase
    if (out.bad) {
        crc_patch_all(smem, w32, pool, off, n, lane_off);
        wave_sync();
    }
}

// Slow path (more check points than the pool holds: sub-tiles of tiny
// records): one lane recomputes everything byte-serially from the window.
// (scalar arguments only: a struct passed by reference to a non-inlined
// function is kept in scratch memory on every sub-tile)
__device__ __noinline__ void crc_slow(const CLY_LDS uint32_t* w32, int64_t nrel, int64_t cbase, int E, uint32_t cnt,
                                      CLY_LDS uint8_t* smem, CrcOut& out) {
    const CLY_LDS uint8_t* w8 = (const CLY_LDS uint8_t*)w32;
    out.bad = 0;
    // head: Z_z(raw [4, E))
    uint32_t s = 0;
    for (int q = 4; q < E; q++) s = crc_byte(smem, s, w8[q], 0);
    const uint32_t z = 4 - (E & 3);
    for (uint32_t k = 0; k < z; k++) s = crc_byte(smem, s, 0, 0);
    out.head_raw = s;
    out.head_z = z;
    // records
    int64_t p = E;
    uint32_t last_state = 0xFFFFFFFFu;
    for (uint32_t i = 0; i < cnt; i++) {
        const Hdr h = hdr_at(w32, (int)p, nrel, cbase + p);
        const int64_t e = p + h.size;
        uint32_t r = 0xFFFFFFFFu;
        const int64_t hi = e < CLY_TS ? e : CLY_TS;
        for (int64_t q = p + 4; q < hi; q++) r = crc_byte(smem, r, w8[q], 0);
        if (e < CLY_TS) { if (~r != h.crc) out.bad = 1; }
        else last_state = r;
        p = e;
    }
    out.end_state = last_state;
}

// Rare path: locate the first failing in-sub-tile record by a serial exact
// walk (one lane) over the restored window.  Returns its position and local
// index via (pos, idx); pos = -1 if none (cannot happen after a failed check).
__device__ __noinline__ void crc_locate(const CLY_LDS uint32_t* w32, int64_t nrel, int64_t cbase, int E, uint32_t cnt,
                                        CLY_LDS uint8_t* smem, int& pos, uint32_t& idx) {
    pos = -1; idx = 0;
    const CLY_LDS uint8_t* w8 = (const CLY_LDS uint8_t*)w32;
    int64_t p = E;
    uint32_t i = 0;
    while (p < CLY_TS && i < cnt) {
        const Hdr h = hdr_at(w32, (int)p, nrel, cbase + p);
        const int64_t e = p + h.size;
        if (e >= CLY_TS) break;                        // no in-tile check point: k_fin
        uint32_t s = 0xFFFFFFFFu;
        for (int64_t q = p + 4; q < e; q++) s = crc_byte(smem, s, w8[q], 0);
        if (~s != h.crc) { pos = (int)p; idx = i; return; }
        p = e;
        i++;
    }
}

// ---------------------------------------------------------------------------
// Staging: the sub-tile bytes (+halo) into the window.  Whole windows go by
// LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave instruction); a window cut
// by the file end is staged through registers with a zero-filled tail.
// Returns true when the window was issued by LDS-DMA and still has to be
// waited for (stage_wait); the register path completes before returning.
__device__ __forceinline__ bool stage(const Sub& T, int lane, CLY_LDS uint32_t* w32) {
    const int wl = T.win_len;
    const uint8_t* src = T.gfile + T.cbase;
    if (wl == CLY_WIN) {
        #pragma unroll
        for (int k = 0; k < (CLY_WIN / 16 + 63) / 64; k++) {
            const int slot0 = k * 64;
            if (slot0 + lane < CLY_WIN / 16)
                __builtin_amdgcn_global_load_lds((const void*)(src + (size_t)(slot0 + lane) * 16),
                                                 (CLY_LDS void*)((CLY_LDS char*)w32 + slot0 * 16), 16, 0, 0);
        }
        return true;
    }
    CLY_LDS u32x4* w4 = (CLY_LDS u32x4*)w32;
    const int nvec = wl > 0 ? (wl >> 4) : 0;
    const u32x4* s4 = reinterpret_cast<const u32x4*>(src);
    for (int i = lane; i < CLY_WIN / 16; i += 64) w4[i] = i < nvec ? s4[i] : (u32x4){0u, 0u, 0u, 0u};
    wave_sync();
    if (lane == 0 && wl > 0 && (wl & 15)) {
        uint32_t v4[4] = {0, 0, 0, 0};
        const uint8_t* b = src + (nvec << 4);
        for (int k = 0; k < (wl & 15); k++) v4[k >> 2] |= (uint32_t)b[k] << (8 * (k & 3));
        w4[nvec] = (u32x4){v4[0], v4[1], v4[2], v4[3]};
    }
    wave_sync();
    return false;
}
__device__ __forceinline__ void stage_wait() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
}

// ---------------------------------------------------------------------------
// Data-wave pieces.
// Geometry of global sub-tile sidx (file F).
__device__ __forceinline__ void sub_setup(Sub& T, int64_t sidx, const DevFile& F, CLY_LDS uint32_t* w32) {
    T.gfile = F.base;
    T.w32 = w32;
    T.cbase = (sidx - (int64_t)F.first_sub) * CLY_TS;
    T.nrel = (int64_t)F.len - T.cbase;
    T.dlen = (int)(T.nrel < CLY_TS ? (T.nrel > 0 ? T.nrel : 0) : CLY_TS);
    T.win_len = (int)(T.nrel < CLY_WIN ? (T.nrel > 0 ? T.nrel : 0) : CLY_WIN);
    T.fof = T.cbase == 0;
    T.lof = T.cbase + CLY_TS >= (int64_t)F.len;
    T.chunk = sidx;
    T.fid = F.fid;
}

// Chain for the given final mode / entry.
__device__ __forceinline__ void sub_chain(const Sub& T, const Spec& sp, int lane, int mode, int entry, Lane& L,
                                          Chain& R) {
    if (mode == MODE_NORMAL) resolve(T, sp, lane, entry, L, R);
    else chain_none(L, R, mode);
}

// Per-sub-tile summary for k_fin (lane 0), with unit-relative record counts.
__device__ __forceinline__ void sub_summary(const Sub& T, const Chain& R, const CrcOut& co, CLY_LDS uint8_t* smem,
                                            uint32_t base, int bpos, uint32_t bidx, ChunkSum* sums, Globals* g) {
    ChunkSum cs;
    cs.evt_off = EVT_NONE; cs.evt_gidx = 0; cs.evt_status = 0; cs.cnt = 0;
    cs.open_pos = -1; cs.open_state = 0; cs.open_crc = 0;
    cs.first4 = co.first4;
    cs.head_raw = 0; cs.head_len = 0; cs.head_shift = 0; cs.head_z = 0; cs.flags = 0;
    if (R.mode == MODE_DEAD) {
        cs.flags = SUM_DEAD;
    } else if (R.mode == MODE_PASS) {
        cs.head_len = (uint32_t)T.dlen;
        cs.head_raw = co.end_state;
        cs.head_z = (uint32_t)(CLY_TS - T.dlen);
        if (T.lof) {
            cs.flags |= SUM_CLOSES;
            cs.evt_off = T.cbase + T.dlen;
            cs.evt_gidx = base;
            cs.evt_status = CLY_END_EOF;
        }
    } else {
        cs.cnt = R.cnt;
        cs.flags |= SUM_CLOSES;
        cs.head_len = (uint32_t)(R.E < T.dlen ? R.E : T.dlen);
        cs.head_raw = co.head_raw;
        cs.head_z = co.head_z;
        if (bpos >= 0) {
            cs.evt_off = T.cbase + bpos;
            cs.evt_gidx = base + bidx;
            cs.evt_status = CLY_ERR_CRC;
        } else if (co.bad) {
            atomicMax(&g->fail, 5u);
        }
        if (R.term && bpos < 0) {
            cs.evt_off = T.cbase + R.tpos;
            cs.evt_gidx = base + R.cnt;
            cs.evt_status = R.tst;
        }
        // the last record is open at the end of the sub-tile unless a check
        // point follows it inside the sub-tile
        if (R.cnt > 0 && R.last >= 0 && (!R.term || (R.eof_exit && R.tpos >= CLY_TS))) {
            cs.flags |= SUM_OPEN;
            cs.open_pos = T.cbase + R.last;
            cs.open_crc = co.open_crc;
            const int ocs = R.last + 4;
            if (ocs >= CLY_TS) {
                cs.open_state = 0xFFFFFFFFu;
            } else if (ocs + 4 > CLY_TS) {
                cs.open_state = co.open_tail;
            } else {
                cs.open_state = co.end_state;
            }
        }
    }
    cs.head_shift = cs.head_len > 4 ? cs.head_len - 4 + cs.head_z : 0;   // exponent; k_fin maps it
    sums[T.chunk] = cs;
}

// CRC + first failure + summary of a resolved sub-tile.
__device__ __forceinline__ void sub_crc(const Sub& T, const Lane& L, const Chain& R, int lane, CLY_LDS uint8_t* smem,
                                        CLY_LDS u32x2* pool, uint32_t base, ChunkSum* sums, Globals* g) {
    CrcOut co;
    crc_phase(T, L, R, lane, smem, (CLY_LDS uint32_t*)T.w32, pool, co);
    int bpos = -1;
    uint32_t bidx = 0;
    if (lane == 0) {
        if (co.bad) {
            int tp;
            uint32_t ti;
            crc_locate(T.w32, T.nrel, T.cbase, R.E, R.cnt, smem, tp, ti);
            bpos = tp; bidx = ti;
        }
        sub_summary(T, R, co, smem, base, bpos, bidx, sums, g);
    }
}

// Tuple words of one record at window position p (index independent).
__device__ __forceinline__ void tuple_words_h(const Sub& T, int p, const Hdr& h, u32x4& q0, u32x4& q1, u32x4& q2,
                                              int64_t& size) {
    const CLY_LDS uint8_t* w8 = (const CLY_LDS uint8_t*)T.w32;
    int tn;
    const int64_t klim = h.ks < 11u ? (int64_t)h.ks : 11;
    const int64_t tx = go_varint(w8 + p + h.hsz, klim, tn);      // parseLogRecordKey, db.go:706-710
    const uint64_t off = (uint64_t)(T.cbase + p);
    const uint64_t ex = (uint64_t)h.exp;
    const uint64_t txv = tn < 0 ? 0ull : (uint64_t)tx;
    q0 = (u32x4){(uint32_t)off, (uint32_t)(off >> 32), (uint32_t)ex, (uint32_t)(ex >> 32)};
    q1 = (u32x4){(uint32_t)txv, (uint32_t)(txv >> 32), T.fid, (uint32_t)h.size};
    q2 = (u32x4){h.ks, h.vs,
                 (h.type & 0xff) | ((h.dt & 0xff) << 8) | ((uint32_t)(h.hsz & 0xff) << 16) |
                     ((uint32_t)(tn < 0 ? 0xFF : tn) << 24),
                 h.crc};
    size = h.size;
}
__device__ __forceinline__ void tuple_words(const Sub& T, int p, u32x4& q0, u32x4& q1, u32x4& q2, int64_t& size) {
    const Hdr h = hdr_at(T.w32, p, T.nrel, T.cbase + p);
    tuple_words_h(T, p, h, q0, q1, q2, size);
}

__device__ __forceinline__ void put_tuple(cly_tuple* out, uint64_t idx, uint64_t out_cap, const u32x4& q0,
                                          const u32x4& q1, const u32x4& q2, bool& of) {
    if (idx < out_cap) {
        u32x4* dst = (u32x4*)(out + idx);
        dst[0] = q0; dst[1] = q1; dst[2] = q2;
    } else {
        of = true;
    }
}

// Tuples of this lane's records, written directly (output slot known).
__device__ __forceinline__ void emit_direct(const Sub& T, const Lane& L, uint64_t idx0, cly_tuple* out, uint64_t out_cap,
                                            Globals* g) {
    bool of = false;
    if (L.ws >= 0) {
        int p = L.ws;
        for (int i = 0; i < L.wc; i++) {
            u32x4 q0, q1, q2;
            int64_t size;
            tuple_words(T, p, q0, q1, q2, size);
            put_tuple(out, idx0 + i, out_cap, q0, q1, q2, of);
            p += (int)size;
        }
    }
    if (of && g) atomicOr(&g->overflow, 1u);
}

// ---------------------------------------------------------------------------
// Kernels.
//   k_scan   every sub-tile independently: speculate, resolve the chain under
//            its own guess, CRC, tuples into the sub-tile's staging slot
//   k_link1/2/3   scan over sub-tile results: each guess is checked against the
//            chain entering its sub-tile; output slot of every sub-tile
//   k_fix    the (rare) sub-tiles whose guess was wrong, from their true entry
//   k_place  staged tuples to their output slots
//   k_fin    per file: straddling CRCs and the first event
__device__ __forceinline__ int find_file(const uint32_t* __restrict__ sub_prefix, int nfiles, int64_t s) {
    int lo = 0, hi = nfiles - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if ((int64_t)sub_prefix[mid] <= s) lo = mid; else hi = mid - 1;
    }
    return lo;
}

__device__ __forceinline__ void init_tables(CLY_LDS uint8_t* smem, const uint32_t* __restrict__ cols) {
    // tables: entry i of T_t replicated 16x, dword (i*64 + t*16 + r)
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
    for (int i = threadIdx.x; i < CLY_COLS; i += blockDim.x) ((CLY_LDS uint32_t*)(smem + LDS_KSNIB))[i] = cols[i];
    __syncthreads();
}

// Tuples of this lane's records into the sub-tile's staging slot (when they
// fit).  The slot is three planes of CLY_CAP 16-B pieces (piece k of tuple i
// at plane k, row i), so with one record per lane each store instruction
// writes one contiguous run; k_copy interleaves the planes back.
__device__ __forceinline__ void stage_tuples(const Sub& T, const Spec& sp, const Lane& L, const Chain& R,
                                             cly_tuple* staging) {
    if (R.mode != MODE_NORMAL || R.cnt > CLY_CAP) return;
    if (L.ws < 0) return;
    u32x4* slot = (u32x4*)staging + (uint64_t)T.chunk * (3 * CLY_CAP);
    int p = L.ws;
    for (int i = 0; i < L.wc; i++) {
        u32x4 q0, q1, q2;
        int64_t size;
        if (i == 0 && p == sp.s) tuple_words_h(T, p, sp.h, q0, q1, q2, size);   // decoded by the speculation
        else tuple_words(T, p, q0, q1, q2, size);
        const int r = (int)L.base + i;
        slot[r] = q0;
        slot[CLY_CAP + r] = q1;
        slot[2 * CLY_CAP + r] = q2;
        p += (int)size;
    }
}

__device__ __forceinline__ SubDesc make_desc(const Sub& T, const Chain& R) {
    SubDesc d;
    d.mode = (uint8_t)R.mode;
    d.cnt = R.mode == MODE_NORMAL ? R.cnt : 0;
    d.entry = (int16_t)(R.mode == MODE_NORMAL ? R.E : -1);
    d.x = (R.mode == MODE_NORMAL && !R.term) ? T.chunk * (int64_t)CLY_TS + R.xrel : 0;
    d.flags = (uint8_t)(((R.mode == MODE_NORMAL && R.term) ? SD_TERM : 0) | (T.fof ? SD_FOF : 0) |
                        (d.cnt > CLY_CAP ? SD_OVF : 0));
    return d;
}

// One sub-tile, start to end, for a chain given by (mode, entry) or, mode < 0,
// by its own guess (mode -2: test mode, odd sub-tiles take a wrong guess).
#ifndef CLY_SCHED
#define CLY_SCHED "default"
#endif
#ifndef CLY_SRC_HASH
#define CLY_SRC_HASH "unknown"
#endif
#define PF_N ((CLY_WIN / 16 + 63) / 64)       // 16-B pieces per lane of a prefetched window
__device__ __forceinline__ void prefetch_issue(const uint8_t* src, int lane, u32x4 (&pf)[PF_N]) {
    const u32x4* s4 = reinterpret_cast<const u32x4*>(src);
    #pragma unroll
    for (int k = 0; k < PF_N; k++) {
        const int slot = k * 64 + lane;
        if (slot < CLY_WIN / 16) pf[k] = __builtin_nontemporal_load(s4 + slot);
    }
}
__device__ __forceinline__ void prefetch_commit(CLY_LDS uint32_t* w32, int lane, const u32x4 (&pf)[PF_N]) {
    CLY_LDS u32x4* w4 = (CLY_LDS u32x4*)w32;
    #pragma unroll
    for (int k = 0; k < PF_N; k++) {
        const int slot = k * 64 + lane;
        if (slot < CLY_WIN / 16) w4[slot] = pf[k];
    }
    wave_sync();
}

// One sub-tile: window (already in LDS when `ready`), speculation, chain,
// tuples, CRC, descriptor.  When pf_src is set, the window of the wave's next
// sub-tile is loaded into pf[] on the way (after the phases that read HBM).
__device__ __forceinline__ bool process_sub(int64_t sidx, int mode, int entry, const DevFile& F, int lane,
                                            CLY_LDS uint8_t* smem, CLY_LDS uint32_t* w32, CLY_LDS u32x2* pool,
                                            SubDesc* descs, ChunkSum* sums, cly_tuple* staging, Globals* g,
                                            int prof_base, SubDesc& d, bool ready, const uint8_t* pf_src,
                                            u32x4 (&pf)[PF_N], bool tentative = false) {
    PROF_INIT();
    Sub T;
    sub_setup(T, sidx, F, w32);
    if (!ready && stage(T, lane, w32)) stage_wait();
    PROF(0);
    Spec sp;
    int guess = -1;
    if (CLY_EXP & 4) {          // experiment: no speculation
        sp.s = -1; sp.last = -1; sp.c = 0; sp.v = 0; sp.x = 0; guess = T.fof ? 0 : -1;
    } else {
        sub_spec(T, lane, sp, guess);
    }
    if (pf_src) prefetch_issue(pf_src, lane, pf);
    PROF(1);
    Lane L;
    Chain R;
    if (mode < 0) {
        const bool force = mode == -2 && !T.fof && (sidx & 1);     // test mode: wrong guesses
        mode = guess >= 0 ? MODE_NORMAL : MODE_PASS;
        entry = guess;
        if (force) mode = (sidx & 2) ? MODE_DEAD : MODE_PASS;
    }
    if ((CLY_EXP & 8) && !T.fof) mode = MODE_PASS;    // experiment: no chain
    sub_chain(T, sp, lane, mode, entry, L, R);
    PROF(2);
    if (tentative && R.mode == MODE_NORMAL && R.term && !T.lof) {
        // an uncertain fix whose chain ends inside the file: most likely a
        // false entry; leave the sub-tile as it is (its state gets certain later)
        d = descs[T.chunk];
        return false;
    }
    if (!(CLY_EXP & 1)) stage_tuples(T, sp, L, R, staging);     // before the CRC phase patches the window
    PROF(3);
    if (!(CLY_EXP & 2)) sub_crc(T, L, R, lane, smem, pool, 0, sums, g);
    PROF(4);
    d = make_desc(T, R);
    if (lane == 0) {
        descs[T.chunk] = d;
        if (d.flags & SD_OVF) atomicAdd(&g->novf, 1u);
    }
    PROF(5);
    PROF_FLUSH(prof_base);
    return true;
}

__global__ void __launch_bounds__(64 * CLY_NDW)
k_scan(const DevFile* __restrict__ files, int nfiles, const uint32_t* __restrict__ sub_prefix, int64_t nsub,
       SubDesc* descs, ChunkSum* sums, const uint32_t* __restrict__ cols, cly_tuple* staging, Globals* g, int gmode) {
    // static LDS: its offsets are known when compiling, so table and window
    // addresses need no base add (a dynamic extern array costs one v_add per lookup)
    __shared__ __attribute__((aligned(16))) unsigned char smem_raw[CLY_SCAN_LDS];
    CLY_LDS uint8_t* smem = (CLY_LDS uint8_t*)smem_raw;
    init_tables(smem, cols);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    CLY_LDS uint32_t* w32 = (CLY_LDS uint32_t*)(smem + LDS_WIN + wave * CLY_WIN);
    CLY_LDS u32x2* pool = (CLY_LDS u32x2*)(smem + LDS_POOL + wave * CP_POOL * 8);
    const int64_t stride = (int64_t)gridDim.x * CLY_NDW;
    int64_t s = (int64_t)blockIdx.x * CLY_NDW + wave;
    if (s >= nsub) return;
    int f = find_file(sub_prefix, nfiles, s);
    DevFile F = files[f];
    u32x4 pf[PF_N];
    bool ready = false;
    for (;;) {
        if (ready) prefetch_commit(w32, lane, pf);
        // the wave's next sub-tile (files in order: walk forward from f)
        const int64_t s2 = s + stride;
        int f2 = f;
        DevFile F2 = F;
        const uint8_t* src2 = nullptr;
        if (s2 < nsub) {
            while (s2 >= (int64_t)F2.first_sub + F2.nsub) F2 = files[++f2];
            const int64_t cb2 = (s2 - (int64_t)F2.first_sub) * CLY_TS;
            if ((int64_t)F2.len - cb2 >= CLY_WIN) src2 = F2.base + cb2;
        }
        SubDesc d;
        process_sub(s, gmode, 0, F, lane, smem, w32, pool, descs, sums, staging, g, 0, d, ready, src2, pf);
        if (s2 >= nsub) break;
        s = s2; f = f2; F = F2;
        ready = src2 != nullptr;
    }
}

// Re-process the sub-tiles of the fix list from the chain the link gives them,
// then walk on through the following sub-tiles of the file while the chain
// stays live and disagrees with what they hold (stopping at a sub-tile listed
// or walked this round).  Pass 0 takes the certain fixes, pass 1 the uncertain
// ones that no pass-0 walk went through.
__global__ void __launch_bounds__(64 * CLY_NDW)
k_fix(const DevFile* __restrict__ files, const Fix* fixes, uint32_t nfix, uint32_t* listed, uint32_t stamp, int pass,
      SubDesc* descs, ChunkSum* sums, const uint32_t* __restrict__ cols, cly_tuple* staging, Globals* g) {
    if (nfix == ~0u) nfix = __hip_atomic_load(&g->nfix, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // (launched ahead)
    if (blockIdx.x * CLY_NDW >= nfix) return;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    CLY_LDS uint8_t* smem = (CLY_LDS uint8_t*)smem_raw;
    init_tables(smem, cols);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    CLY_LDS uint32_t* w32 = (CLY_LDS uint32_t*)(smem + LDS_WIN + wave * CLY_WIN);
    CLY_LDS u32x2* pool = (CLY_LDS u32x2*)(smem + LDS_POOL + wave * CP_POOL * 8);
    for (uint32_t i = blockIdx.x * CLY_NDW + wave; i < nfix; i += gridDim.x * CLY_NDW) {
        const Fix fx = fixes[i];
        if ((int)fx.certain != (pass == 0)) continue;
        // an uncertain fix gives way to a walk of the first pass that went through it
        if (pass == 1 && __builtin_nontemporal_load(&listed[fx.s]) != (stamp | LISTED_U)) continue;
        const DevFile F = files[fx.file];
        const int64_t s_end = (int64_t)F.first_sub + F.nsub;
        int64_t s = fx.s, x = fx.x_in;
        int mode = fx.mode, entry = fx.entry;
        for (;;) {
            SubDesc d;
            u32x4 pf[PF_N];
            if (!process_sub(s, mode, entry, F, lane, smem, w32, pool, descs, sums, staging, g, 8, d, false, nullptr, pf,
                             pass == 1 && s == (int64_t)fx.s)) break;
            if (d.mode == MODE_DEAD || (d.mode == MODE_NORMAL && (d.flags & SD_TERM))) break;
            if (d.mode == MODE_NORMAL) x = d.x;
            if (++s >= s_end) break;
            const uint32_t ls = __builtin_nontemporal_load(&listed[s]);
            // certain-listed or walked this round: its own wave has it (pass 0
            // walks through uncertain fixes, which then give way)
            if (ls == stamp || (pass == 1 && ls == (stamp | LISTED_U))) break;
            const int64_t rel = x - s * (int64_t)CLY_TS;
            if (rel < 0) { if (lane == 0) atomicOr(&g->fail, 8u); break; }      // cannot happen
            mode = rel >= CLY_TS ? MODE_PASS : MODE_NORMAL;
            entry = rel >= CLY_TS ? 0 : (int)rel;
            const SubDesc n = descs[s];
            // walked (or already right for the walked chain): claimed for this round,
            // so an uncertain fix listed there gives way
            if (lane == 0) listed[s] = stamp;
            if (n.mode == mode && (mode != MODE_NORMAL || n.entry == entry)) break;
        }
    }
}

// ---- link scan over sub-tiles (three passes of LINK_NT threads x LINK_IT items)
#define LINK_NT 256
#define LINK_IT 8
#define LINK_BLK (LINK_NT * LINK_IT)
__device__ __forceinline__ LinkAgg link_op(const LinkAgg& a, const LinkAgg& b) {
    LinkAgg r;
    #pragma unroll
    for (int t = 0; t < 2; t++) {
        const LinkBr& ra = a.br[t];
        const LinkBr& rb = b.br[ra.set ? ra.term : t];
        r.br[t].set = ra.set | rb.set;
        r.br[t].x = rb.set ? rb.x : ra.x;
        r.br[t].term = rb.set ? rb.term : ra.term;
        r.br[t].cnt = ra.cnt + rb.cnt;
    }
    return r;
}
__device__ __forceinline__ LinkAgg link_ident() {
    LinkAgg e;
    #pragma unroll
    for (int t = 0; t < 2; t++) { e.br[t].x = 0; e.br[t].cnt = 0; e.br[t].set = 0; e.br[t].term = 0; }
    return e;
}
__device__ __forceinline__ LinkAgg link_elem(const SubDesc& d) {
    LinkAgg e = link_ident();
    if (d.mode == MODE_NORMAL) {
        const int32_t term = (d.flags & SD_TERM) != 0;
        e.br[0].set = 1; e.br[0].x = d.x; e.br[0].term = term; e.br[0].cnt = d.cnt;
        if (d.flags & SD_FOF) e.br[1] = e.br[0];
    }
    return e;
}
// Exclusive block scan of the threads' aggregates; returns the block total.
__device__ __forceinline__ LinkAgg link_block_scan(LinkAgg v, LinkAgg& excl) {
    __shared__ LinkAgg sh[LINK_NT];
    const int t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
    for (int o = 1; o < LINK_NT; o <<= 1) {
        LinkAgg u = link_ident();
        if (t >= o) u = sh[t - o];
        __syncthreads();
        if (t >= o) sh[t] = link_op(u, sh[t]);
        __syncthreads();
    }
    excl = t > 0 ? sh[t - 1] : link_ident();
    const LinkAgg tot = sh[LINK_NT - 1];
    __syncthreads();
    return tot;
}

__global__ void __launch_bounds__(LINK_NT)
k_link1(const SubDesc* __restrict__ descs, int64_t nsub, LinkAgg* blk) {
    const int64_t b0 = (int64_t)blockIdx.x * LINK_BLK + (int64_t)threadIdx.x * LINK_IT;
    LinkAgg v = link_ident();
    for (int i = 0; i < LINK_IT; i++) if (b0 + i < nsub) v = link_op(v, link_elem(descs[b0 + i]));
    LinkAgg ex;
    const LinkAgg tot = link_block_scan(v, ex);
    if (threadIdx.x == 0) blk[blockIdx.x] = tot;
}

// One block: exclusive scan of the block aggregates (in place).
__global__ void __launch_bounds__(LINK_NT)
k_link2(LinkAgg* blk, int64_t nblk) {
    const int64_t per = (nblk + LINK_NT - 1) / LINK_NT;
    const int64_t b0 = (int64_t)threadIdx.x * per;
    LinkAgg v = link_ident();
    for (int64_t i = 0; i < per; i++) if (b0 + i < nblk) v = link_op(v, blk[b0 + i]);
    LinkAgg ex;
    link_block_scan(v, ex);
    LinkAgg run = ex;
    for (int64_t i = 0; i < per; i++) {
        if (b0 + i < nblk) { const LinkAgg a = blk[b0 + i]; blk[b0 + i] = run; run = link_op(run, a); }
    }
}

// Per sub-tile: output slot, and whether its chain is the one the link state
// implies; if not, a candidate (with the implied chain).  A wrong chain entered
// live is "harmful" (it misleads the state of what follows): the first harmful
// sub-tile of each file goes to fh[file].
__global__ void __launch_bounds__(LINK_NT)
k_link3(const DevFile* __restrict__ files, int nfiles, const uint32_t* __restrict__ sub_prefix,
        const SubDesc* __restrict__ descs, int64_t nsub, const LinkAgg* __restrict__ blk, uint64_t* sub_P, Fix* cand,
        uint32_t cand_cap, int32_t* fh, unsigned long long* fck, uint32_t* cflag, uint32_t stamp, Globals* g) {
    const int64_t b0 = (int64_t)blockIdx.x * LINK_BLK + (int64_t)threadIdx.x * LINK_IT;
    LinkAgg v = link_ident();
    SubDesc d[LINK_IT];
    for (int i = 0; i < LINK_IT; i++) {
        if (b0 + i < nsub) { d[i] = descs[b0 + i]; v = link_op(v, link_elem(d[i])); }
    }
    LinkAgg ex;
    link_block_scan(v, ex);
    LinkAgg run = link_op(blk[blockIdx.x], ex);
    for (int i = 0; i < LINK_IT; i++) {
        const int64_t s = b0 + i;
        if (s >= nsub) break;
        const LinkBr& st = run.br[1];          // state entering s (sub-tile 0 resets it)
        sub_P[s] = st.cnt;
        int mode, entry = 0;
        int64_t x_in = st.x;
        bool live = true;
        if (d[i].flags & SD_FOF) { mode = MODE_NORMAL; entry = 0; x_in = s * (int64_t)CLY_TS; }
        else if (!st.set) { mode = -1; atomicOr(&g->fail, 6u); }            // cannot happen
        else if (st.term) { mode = MODE_DEAD; live = false; }
        else {
            const int64_t rel = st.x - s * (int64_t)CLY_TS;
            if (rel >= CLY_TS) mode = MODE_PASS;
            else if (rel < 0) mode = -1;       // a sub-tile before s is wrong (and a candidate)
            else { mode = MODE_NORMAL; entry = (int)rel; }
        }
        const bool ok = mode >= 0 && d[i].mode == mode && (mode != MODE_NORMAL || d[i].entry == entry);
        if (!ok) {
            const uint32_t f = (uint32_t)find_file(sub_prefix, nfiles, s);
            // harmful: the wrong chain changes the state passed on (PASS and DEAD both pass it through)
            const bool harmful = live && mode >= 0 && (mode == MODE_NORMAL || d[i].mode == MODE_NORMAL);
            if (harmful) atomicMin(&fh[f], (int32_t)s);
            cflag[s] = 2 * stamp + (harmful ? 1u : 0u);
            const uint32_t k = atomicAdd(&g->ncand, 1u);
            if (k < cand_cap) {
                Fix c;
                c.s = (uint32_t)s; c.mode = mode; c.entry = entry; c.file = f; c.x_in = x_in;
                c.certain = 0; c._pad = 0;
                cand[k] = c;
                atomicMin(&fck[f], ((unsigned long long)s << 32) | k);      // first candidate of the file
            }
        }
        run = link_op(run, link_elem(d[i]));
        if (s == nsub - 1) g->total = run.br[1].cnt;
    }
}

// Serial resolution (after parallel rounds that did not converge): one wave per
// file walks from the file's first candidate to its end, keeping the exact
// chain state, and re-processes every sub-tile that disagrees with it.  The
// descriptors are read 64 ahead (one per lane).
__global__ void __launch_bounds__(64)
k_serial(const DevFile* __restrict__ files, const Fix* __restrict__ cand, const unsigned long long* __restrict__ fck,
         SubDesc* descs, ChunkSum* sums, const uint32_t* __restrict__ cols, cly_tuple* staging, Globals* g) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const unsigned long long key = fck[blockIdx.x];
    if (key == ~0ull) return;
    CLY_LDS uint8_t* smem = (CLY_LDS uint8_t*)smem_raw;
    init_tables(smem, cols);
    const int lane = threadIdx.x;
    CLY_LDS uint32_t* w32 = (CLY_LDS uint32_t*)(smem + LDS_WIN);
    CLY_LDS u32x2* pool = (CLY_LDS u32x2*)(smem + LDS_POOL);
    const Fix c = cand[key & 0xffffffffull];
    const DevFile F = files[blockIdx.x];
    const int64_t s_end = (int64_t)F.first_sub + F.nsub;
    if (c.mode < 0) { if (lane == 0) atomicOr(&g->fail, 9u); return; }      // cannot happen
    int64_t s = c.s, x = c.x_in;
    int mode = c.mode, entry = c.entry;
    int64_t base = -1;
    SubDesc ahead;
    for (;;) {
        if (s >= base + 64) {
            base = s;
            if (s + lane < s_end) ahead = descs[s + lane];
        }
        const int k = (int)(s - base);
        SubDesc d;
        d.x = (int64_t)__shfl((long long)ahead.x, k, 64);
        d.cnt = (uint32_t)__shfl((int)ahead.cnt, k, 64);
        d.entry = (int16_t)__shfl((int)ahead.entry, k, 64);
        d.mode = (uint8_t)__shfl((int)ahead.mode, k, 64);
        d.flags = (uint8_t)__shfl((int)ahead.flags, k, 64);
        if (!(d.mode == mode && (mode != MODE_NORMAL || d.entry == entry))) {
            u32x4 pf[PF_N];
            process_sub(s, mode, entry, F, lane, smem, w32, pool, descs, sums, staging, g, 8, d, false, nullptr, pf);
        }
        bool dead = mode == MODE_DEAD || (d.mode == MODE_NORMAL && (d.flags & SD_TERM));
        if (d.mode == MODE_NORMAL && !dead) x = d.x;
        if (++s >= s_end) break;
        if (dead) { mode = MODE_DEAD; entry = 0; continue; }
        const int64_t rel = x - s * (int64_t)CLY_TS;
        if (rel < 0) { if (lane == 0) atomicOr(&g->fail, 10u); break; }    // cannot happen
        mode = rel >= CLY_TS ? MODE_PASS : MODE_NORMAL;
        entry = rel >= CLY_TS ? 0 : (int)rel;
    }
}

// Per-round reset of the link state (one launch instead of four memsets).
__global__ void __launch_bounds__(LINK_NT)
k_round_init(int32_t* fh, unsigned long long* fck, int nfiles, Globals* g) {
    const int i = blockIdx.x * LINK_NT + threadIdx.x;
    if (i == 0) { g->nfix = 0; g->ncand = 0; }
    if (i < nfiles) { fh[i] = 0x7f7f7f7f; fck[i] = ~0ull; }
}

// Fix list of the round: every candidate up to and including the first harmful
// sub-tile of its file (its state is certain); later candidates only when they
// hold a wrong record chain (never turned into PASS / DEAD on an uncertain
// state, which would discard a good guess: a false exit far ahead makes every
// sub-tile up to it look covered).  Uncertain fixes run after the certain walks
// and are dropped when their chain ends before the file does.
__global__ void __launch_bounds__(LINK_NT)
k_link4(const DevFile* __restrict__ files, const SubDesc* __restrict__ descs, const Fix* __restrict__ cand,
        const int32_t* __restrict__ fh, const uint32_t* __restrict__ cflag, Fix* fixes, uint32_t* listed,
        uint32_t stamp, Globals* g) {
    const uint32_t n = g->ncand;
    for (uint32_t i = blockIdx.x * LINK_NT + threadIdx.x; i < n; i += gridDim.x * LINK_NT) {
        const Fix c = cand[i];
        if (c.mode < 0) continue;
        // certain: no harmful candidate since the last sub-tile that agreed with
        // its state on a record entry (its own exit then fixes the state), or
        // since the file start; past 256 sub-tiles back: since the file start
        bool certain = (int64_t)c.s <= (int64_t)fh[c.file];
        if (!certain) {
            const int64_t s_first = files[c.file].first_sub;
            int64_t t = (int64_t)c.s - 1;
            for (int k = 0; k < 256 && t >= s_first; k++, t--) {
                const uint32_t cf = cflag[t];
                if (cf == 2 * stamp + 1) break;                      // harmful candidate: uncertain
                if (cf == 2 * stamp) continue;                       // harmless candidate
                if (descs[t].mode == MODE_NORMAL) { certain = true; break; }   // agreed on an entry
            }
            if (t < s_first) certain = true;
        }
        if (!certain && c.mode != MODE_NORMAL) continue;
        listed[c.s] = certain ? stamp : (stamp | LISTED_U);
        Fix e = c;
        e.certain = certain;
        fixes[atomicAdd(&g->nfix, 1u)] = e;
        atomicAdd(&g->fix_total, 1u);
    }
}

// Staged tuples to their output slots: CP_SUBS sub-tiles per workgroup, one
// 16-B piece per thread and step, all loads of a thread issued before its stores.
#define CP_SUBS 16
#define CP_NT 256
#define CP_PER ((CP_SUBS * CLY_CAP * 3 + CP_NT - 1) / CP_NT)
__global__ void __launch_bounds__(CP_NT)
k_copy(const SubDesc* __restrict__ descs, const uint64_t* __restrict__ sub_P, const cly_tuple* __restrict__ staging,
       cly_tuple* out, uint64_t out_cap, int64_t nsub, Globals* g) {
    __shared__ uint32_t n_s[CP_SUBS];
    __shared__ uint64_t p_s[CP_SUBS];
    const int64_t s0 = (int64_t)blockIdx.x * CP_SUBS;
    const int tid = threadIdx.x;
    if (tid < CP_SUBS) {
        const int64_t s = s0 + tid;
        uint32_t n = 0;
        uint64_t P = 0;
        if (s < nsub) {
            const SubDesc d = descs[s];
            if (d.mode == MODE_NORMAL && !(d.flags & SD_OVF)) n = d.cnt * 3;
            P = sub_P[s];
        }
        n_s[tid] = n;
        p_s[tid] = P;
    }
    __syncthreads();
    const u32x4* src = (const u32x4*)(staging + (uint64_t)s0 * CLY_CAP);
    u32x4* dst = (u32x4*)out;
    const uint64_t lim = out_cap * 3;
    u32x4 v[CP_PER];
    #pragma unroll
    for (int k = 0; k < CP_PER; k++) {
        const int e = k * CP_NT + tid, j = e / (CLY_CAP * 3), q = e - j * (CLY_CAP * 3);
        const int r = q / 3, pl = q - 3 * r;                 // tuple r, piece pl (plane layout)
        if (j < CP_SUBS && (uint32_t)q < n_s[j])
            v[k] = __builtin_nontemporal_load(src + j * (CLY_CAP * 3) + pl * CLY_CAP + r);
    }
    bool of = false;
    #pragma unroll
    for (int k = 0; k < CP_PER; k++) {
        const int e = k * CP_NT + tid, j = e / (CLY_CAP * 3), q = e - j * (CLY_CAP * 3);
        if (j < CP_SUBS && (uint32_t)q < n_s[j]) {
            const uint64_t i = p_s[j] * 3 + (uint64_t)q;
            if (i < lim) dst[i] = v[k]; else of = true;
        }
    }
    if (of) atomicOr(&g->overflow, 1u);
}

// Sub-tiles whose tuples did not fit the staging slot: re-read and emitted
// (one wave per sub-tile; launched only when there are any).
__global__ void __launch_bounds__(64 * CLY_NDW)
k_place(const DevFile* __restrict__ files, int nfiles, const uint32_t* __restrict__ sub_prefix, int64_t nsub,
        const SubDesc* __restrict__ descs, const uint64_t* __restrict__ sub_P, const cly_tuple* __restrict__ staging,
        cly_tuple* out, uint64_t out_cap, Globals* g) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    CLY_LDS uint8_t* smem = (CLY_LDS uint8_t*)smem_raw;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    CLY_LDS uint32_t* w32 = (CLY_LDS uint32_t*)(smem + wave * CLY_WIN);
    const int64_t stride = (int64_t)gridDim.x * CLY_NDW;
    for (int64_t s = (int64_t)blockIdx.x * CLY_NDW + wave; s < nsub; s += stride) {
        const SubDesc d = descs[s];
        if (d.mode != MODE_NORMAL || d.cnt == 0) continue;
        const uint64_t P = sub_P[s];
        if (d.flags & SD_OVF) {
            const DevFile F = files[find_file(sub_prefix, nfiles, s)];
            Sub T;
            sub_setup(T, s, F, w32);
            if (stage(T, lane, w32)) stage_wait();
            Spec sp;
            int guess = -1;
            sub_spec(T, lane, sp, guess);
            Lane L;
            Chain R;
            sub_chain(T, sp, lane, MODE_NORMAL, d.entry, L, R);
            emit_direct(T, L, P + L.base, out, out_cap, g);
        }
    }
}

// First event of every file: one thread per sub-tile (its in-tile event, or
// the CRC failure of its open record), min-reduced per file on the key
// (offset << 32 | sub-tile of the file); then one thread per file.
#define FIN_NT 256
__global__ void __launch_bounds__(FIN_NT)
k_fin1(const DevFile* __restrict__ files, int nfiles, const uint32_t* __restrict__ sub_prefix, int64_t nsub,
       const ChunkSum* __restrict__ sums, const uint64_t* __restrict__ sub_P, const uint32_t* __restrict__ x8n,
       unsigned long long* fkey) {
    const int64_t s = (int64_t)blockIdx.x * FIN_NT + threadIdx.x;
    if (s >= nsub) return;
    const int f = find_file(sub_prefix, nfiles, s);
    const DevFile F = files[f];
    uint64_t gi = 0;
    int32_t st = 0;
    const int64_t i = s - (int64_t)F.first_sub;
    const int64_t o = fin_chunk_event(sums, sub_P, x8n, F.first_sub, F.nsub, i, &gi, &st);
    if (o != EVT_NONE) atomicMin(&fkey[f], ((unsigned long long)o << 32) | (unsigned long long)i);
}
__global__ void __launch_bounds__(FIN_NT)
k_fin2(const DevFile* __restrict__ files, int nfiles, const ChunkSum* __restrict__ sums,
       const uint64_t* __restrict__ sub_P, const uint32_t* __restrict__ x8n, const unsigned long long* fkey,
       FileOut* __restrict__ fout) {
    const int f = blockIdx.x * FIN_NT + threadIdx.x;
    if (f >= nfiles) return;
    const DevFile F = files[f];
    const unsigned long long key = fkey[f];
    FileOut fo;
    fo.first_index = sub_P[F.first_sub];
    fo.ok = key != ~0ull;
    fo.n_records = 0; fo.end_offset = EVT_NONE; fo.status = 0;
    if (fo.ok) {
        uint64_t gi = 0;
        int32_t st = 0;
        const int64_t i = (int64_t)(key & 0xffffffffull);
        fo.end_offset = fin_chunk_event(sums, sub_P, x8n, F.first_sub, F.nsub, i, &gi, &st);
        fo.n_records = gi - fo.first_index;
        fo.status = st;
    }
    fout[f] = fo;
}

// ---------------------------------------------------------------------------
// Host side
#define HIPCK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "clyscan: %s failed: %s\n", #x, hipGetErrorString(e_)); return CLY_ERR_DEVICE; } } while (0)

struct cly_ctx {
    int device;
    hipStream_t stream;
    hipEvent_t ev[4];
    DevFile* d_files; int cap_files;
    uint32_t* d_prefix;
    FileOut* d_fout;
    int64_t cap_subs;
    SubDesc* d_desc;
    ChunkSum* d_sums;
    uint64_t* d_subP;
    cly_tuple* d_staging;
    LinkAgg* d_blk;
    Fix* d_fix;                  // fix list of a round
    Fix* d_cand;                 // candidates of a round
    uint32_t* d_listed;          // per sub-tile: stamp of the last round that listed it
    uint32_t* d_cflag;           // per sub-tile: 2 stamp + harmful, for the candidates of a round
    int32_t* d_fh;               // per file: first harmful sub-tile of a round
    unsigned long long* d_fkey;  // per file: first event key (k_fin1)
    unsigned long long* d_fck;   // per file: first candidate key of a round
    uint32_t stamp;
    Globals* d_g;
    uint32_t* d_cols;            // columns of A^(SUB*2^k) (Kogge-Stone) and A^(4w) (head shifts)
    uint32_t* d_x8n;
    DevFile* h_files;
    uint32_t* h_prefix;
    FileOut* h_fout;
    Globals* h_g;
    int scan_grid;
    uint8_t* d_bytes; uint64_t cap_bytes;          // host-path staging
    cly_tuple* d_tuples; uint64_t cap_tuples;
    int dbg_flags;
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
    c->device = device;
    HIPCK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    for (int i = 0; i < 4; i++) HIPCK(hipEventCreate(&c->ev[i]));
    HIPCK(hipMalloc(&c->d_g, sizeof(Globals)));
    HIPCK(hipHostMalloc(&c->h_g, sizeof(Globals), hipHostMallocDefault));
    {
        uint32_t* hc = (uint32_t*)calloc(CLY_COLS, sizeof(uint32_t));
        for (int lvl = 0; lvl < CLY_KS_LEVELS; lvl++) {
            const uint32_t xm = cly_x8n((uint64_t)CLY_SUB << lvl);
            for (int nb = 0; nb < 8; nb++)
                for (uint32_t v = 0; v < 16; v++) hc[lvl * 128 + nb * 16 + v] = cly_multmodp(xm, v << (4 * nb));
        }
        for (int w = 0; w < 6 + HS_A; w++) {          // A^(4b), b < 6, then A^(24a), a < HS_A
            const uint32_t xm = cly_x8n(w < 6 ? (uint64_t)4 * w : (uint64_t)24 * (w - 6));
            for (int nb = 0; nb < 8; nb++)
                for (uint32_t v = 0; v < 16; v++) hc[NIB_HSB + w * 128 + nb * 16 + v] = cly_multmodp(xm, v << (4 * nb));
        }
        HIPCK(hipMalloc(&c->d_cols, sizeof(uint32_t) * CLY_COLS));
        HIPCK(hipMemcpy(c->d_cols, hc, sizeof(uint32_t) * CLY_COLS, hipMemcpyHostToDevice));
        free(hc);
    }
    const size_t x8_bytes = sizeof(uint32_t) * (CLY_TS + 8);
    HIPCK(hipMalloc(&c->d_x8n, x8_bytes));
    uint32_t* hx = (uint32_t*)malloc(x8_bytes);
    hx[0] = 1u << 31;
    const uint32_t x8 = cly_x8n(1);
    for (int n = 1; n < CLY_TS + 8; n++) hx[n] = cly_multmodp(x8, hx[n - 1]);
    HIPCK(hipMemcpy(c->d_x8n, hx, x8_bytes, hipMemcpyHostToDevice));
    free(hx);
    HIPCK(hipFuncSetAttribute((const void*)k_fix, hipFuncAttributeMaxDynamicSharedMemorySize, (int)CLY_SCAN_LDS));
    HIPCK(hipFuncSetAttribute((const void*)k_serial, hipFuncAttributeMaxDynamicSharedMemorySize, (int)CLY_SCAN_LDS));
    HIPCK(hipFuncSetAttribute((const void*)k_place, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)(CLY_NDW * CLY_WIN)));
    {
        int per_cu = 0, ncu = 0;
        HIPCK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_scan, 64 * CLY_NDW, 0));
        HIPCK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device));
        if (per_cu < 1) per_cu = 1;
        c->scan_grid = per_cu * ncu;
    }
    *out = c;
    return CLY_OK;
}

extern "C" void cly_ctx_destroy(cly_ctx* c) {
    if (!c) return;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    hipFree(c->d_files); hipFree(c->d_prefix); hipFree(c->d_fout); hipFree(c->d_desc); hipFree(c->d_sums);
    hipFree(c->d_subP); hipFree(c->d_staging); hipFree(c->d_blk); hipFree(c->d_fix); hipFree(c->d_cand);
    hipFree(c->d_listed); hipFree(c->d_cflag); hipFree(c->d_fh); hipFree(c->d_fkey); hipFree(c->d_fck); hipFree(c->d_g); hipFree(c->d_cols); hipFree(c->d_x8n); hipFree(c->d_bytes); hipFree(c->d_tuples);
    hipHostFree(c->h_files); hipHostFree(c->h_prefix); hipHostFree(c->h_fout); hipHostFree(c->h_g);
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
    hipFree(c->d_files); hipFree(c->d_prefix); hipFree(c->d_fout); hipFree(c->d_fh); hipFree(c->d_fkey); hipFree(c->d_fck);
    hipHostFree(c->h_files); hipHostFree(c->h_prefix); hipHostFree(c->h_fout);
    const int cap = nfiles < 64 ? 64 : nfiles;
    HIPCK(hipMalloc(&c->d_fh, sizeof(int32_t) * cap));
    HIPCK(hipMalloc(&c->d_fkey, sizeof(unsigned long long) * cap));
    HIPCK(hipMalloc(&c->d_fck, sizeof(unsigned long long) * cap));
    HIPCK(hipMalloc(&c->d_files, sizeof(DevFile) * cap));
    HIPCK(hipMalloc(&c->d_prefix, sizeof(uint32_t) * (cap + 1)));
    HIPCK(hipMalloc(&c->d_fout, sizeof(FileOut) * cap));
    HIPCK(hipHostMalloc(&c->h_files, sizeof(DevFile) * cap, hipHostMallocDefault));
    HIPCK(hipHostMalloc(&c->h_prefix, sizeof(uint32_t) * (cap + 1), hipHostMallocDefault));
    HIPCK(hipHostMalloc(&c->h_fout, sizeof(FileOut) * cap, hipHostMallocDefault));
    c->cap_files = cap;
    return CLY_OK;
}

static int ensure_subs(cly_ctx* c, int64_t nsub) {
    if (nsub <= c->cap_subs) return CLY_OK;
    hipFree(c->d_desc); hipFree(c->d_sums); hipFree(c->d_subP); hipFree(c->d_staging); hipFree(c->d_blk);
    hipFree(c->d_fix); hipFree(c->d_cand); hipFree(c->d_listed); hipFree(c->d_cflag);
    const int64_t cap = nsub < 1024 ? 1024 : nsub;
    HIPCK(hipMalloc(&c->d_desc, sizeof(SubDesc) * cap));
    HIPCK(hipMalloc(&c->d_sums, sizeof(ChunkSum) * cap));
    HIPCK(hipMalloc(&c->d_subP, sizeof(uint64_t) * cap));
    HIPCK(hipMalloc(&c->d_staging, sizeof(cly_tuple) * CLY_CAP * cap));
    HIPCK(hipMalloc(&c->d_blk, sizeof(LinkAgg) * (cap / LINK_BLK + 2)));
    HIPCK(hipMalloc(&c->d_fix, sizeof(Fix) * cap));
    HIPCK(hipMalloc(&c->d_cand, sizeof(Fix) * cap));
    HIPCK(hipMalloc(&c->d_listed, sizeof(uint32_t) * cap));
    HIPCK(hipMemset(c->d_listed, 0, sizeof(uint32_t) * cap));
    HIPCK(hipMalloc(&c->d_cflag, sizeof(uint32_t) * cap));
    HIPCK(hipMemset(c->d_cflag, 0, sizeof(uint32_t) * cap));
    c->stamp = 0;
    c->cap_subs = cap;
    return CLY_OK;
}

#define FIX_ROUNDS 8
#define SERIAL_AFTER 2           // parallel fix rounds before the serial walk

extern "C" int cly_scan_device(cly_ctx* c, const cly_file* files, int nfiles, cly_tuple* d_out, uint64_t out_cap,
                               uint64_t* file_first, cly_file_result* res, uint64_t* needed, cly_stats* stats,
                               void* stream_v) {
    if (!c || (!files && nfiles) || nfiles < 0 || !res || !file_first) return CLY_ERR_ARG;
    if (nfiles == 0) { if (needed) *needed = 0; return CLY_OK; }
    HIPCK(hipSetDevice(c->device));
    hipStream_t st = stream_v ? (hipStream_t)stream_v : c->stream;
    int rc = ensure_files(c, nfiles);
    if (rc) return rc;
    int64_t nsub = 0;
    uint64_t bytes = 0;
    for (int i = 0; i < nfiles; i++) {
        if (files[i].len >= (1ULL << 32)) return CLY_ERR_ARG;
        if (files[i].len && (((uintptr_t)files[i].base) & 15)) return CLY_ERR_ARG;
        const uint64_t ns = files[i].len ? (files[i].len + CLY_TS - 1) / CLY_TS : 1;
        c->h_files[i].base = files[i].base;
        c->h_files[i].len = files[i].len;
        c->h_files[i].fid = files[i].fid;
        c->h_files[i].first_sub = (uint32_t)nsub;
        c->h_files[i].nsub = (uint32_t)ns;
        c->h_files[i]._pad = 0;
        c->h_prefix[i] = (uint32_t)nsub;
        nsub += (int64_t)ns;
        bytes += files[i].len;
    }
    if (nsub >= (1LL << 31)) return CLY_ERR_ARG;
    c->h_prefix[nfiles] = (uint32_t)nsub;
    rc = ensure_subs(c, nsub);
    if (rc) return rc;
    HIPCK(hipMemcpyAsync(c->d_files, c->h_files, sizeof(DevFile) * nfiles, hipMemcpyHostToDevice, st));
    HIPCK(hipMemcpyAsync(c->d_prefix, c->h_prefix, sizeof(uint32_t) * (nfiles + 1), hipMemcpyHostToDevice, st));
    HIPCK(hipMemsetAsync(c->d_g, 0, sizeof(Globals), st));
    const int64_t nblk = (nsub + LINK_BLK - 1) / LINK_BLK;
    HIPCK(hipEventRecord(c->ev[0], st));
    int grid = c->scan_grid;
    if ((int64_t)grid * CLY_NDW > nsub) grid = (int)((nsub + CLY_NDW - 1) / CLY_NDW);
    hipLaunchKernelGGL(k_scan, dim3(grid), dim3(64 * CLY_NDW), 0, st, c->d_files, nfiles, c->d_prefix, nsub,
                       c->d_desc, c->d_sums, c->d_cols, c->d_staging, c->d_g, (c->dbg_flags & 2) ? -2 : -1);
    HIPCK(hipGetLastError());
    HIPCK(hipEventRecord(c->ev[1], st));
    // link scan, then fix rounds until every sub-tile holds the chain its state
    // implies.  The first fix round is launched without waiting for the first
    // scan (k_fix reads the fix count itself), so the common case costs one
    // host synchronisation.
    uint32_t rounds = 0;
    const int fix_grid = c->scan_grid < 64 ? c->scan_grid : 64;
    auto link_round = [&](uint32_t stamp) -> int {
        hipLaunchKernelGGL(k_round_init, dim3((nfiles + LINK_NT - 1) / LINK_NT), dim3(LINK_NT), 0, st, c->d_fh,
                           c->d_fck, nfiles, c->d_g);
        hipLaunchKernelGGL(k_link1, dim3(nblk), dim3(LINK_NT), 0, st, c->d_desc, nsub, c->d_blk);
        hipLaunchKernelGGL(k_link2, dim3(1), dim3(LINK_NT), 0, st, c->d_blk, nblk);
        hipLaunchKernelGGL(k_link3, dim3(nblk), dim3(LINK_NT), 0, st, c->d_files, nfiles, c->d_prefix, c->d_desc, nsub,
                           c->d_blk, c->d_subP, c->d_cand, (uint32_t)c->cap_subs, c->d_fh, c->d_fck, c->d_cflag, stamp,
                           c->d_g);
        hipLaunchKernelGGL(k_link4, dim3(64), dim3(LINK_NT), 0, st, c->d_files, c->d_desc, c->d_cand, c->d_fh, c->d_cflag,
                           c->d_fix, c->d_listed, stamp, c->d_g);
        HIPCK(hipGetLastError());
        return CLY_OK;
    };
    auto fix_round = [&](uint32_t stamp, uint32_t nfix) -> int {
        int fgrid = nfix == ~0u ? fix_grid : (int)((nfix + CLY_NDW - 1) / CLY_NDW);
        if (fgrid > c->scan_grid) fgrid = c->scan_grid;
        for (int pass = 0; pass < 2; pass++)
            hipLaunchKernelGGL(k_fix, dim3(fgrid), dim3(64 * CLY_NDW), CLY_SCAN_LDS, st, c->d_files, c->d_fix, nfix,
                               c->d_listed, stamp, pass, c->d_desc, c->d_sums, c->d_cols, c->d_staging, c->d_g);
        HIPCK(hipGetLastError());
        return CLY_OK;
    };
    const bool ahead = !CLY_EXP && !(c->dbg_flags & (4 | 8 | 16));
    {
        const uint32_t stamp = ++c->stamp;
        if ((rc = link_round(stamp))) return rc;
        if (ahead) {
            if ((rc = fix_round(stamp, ~0u))) return rc;
            if ((rc = link_round(++c->stamp))) return rc;
            rounds = 1;
        }
    }
    for (;;) {
        HIPCK(hipMemcpyAsync(c->h_g, c->d_g, sizeof(Globals), hipMemcpyDeviceToHost, st));
        HIPCK(hipStreamSynchronize(st));
        const uint32_t ncand = c->h_g->ncand, nfix = c->h_g->nfix;
        if (c->h_g->fail) break;
        if (ncand == 0 || CLY_EXP || (c->dbg_flags & 16)) break;   // (experiment builds / debug: no fix rounds)
        if (++rounds > FIX_ROUNDS) {
            fprintf(stderr, "clyscan: chain resolution did not converge (%u candidates, %u fixes)\n", ncand, nfix);
            return CLY_ERR_NOREPAIR;
        }
        const uint32_t stamp = c->stamp;
        if (c->dbg_flags & 4) {                          // debug trace of the fix rounds
            const uint32_t nshow = nfix < 64 ? nfix : 64;
            Fix* hf = (Fix*)malloc(sizeof(Fix) * (nshow ? nshow : 1));
            HIPCK(hipMemcpy(hf, c->d_fix, sizeof(Fix) * nshow, hipMemcpyDeviceToHost));
            fprintf(stderr, "round %u: %u candidates, %u fixes:", rounds, ncand, nfix);
            for (uint32_t k = 0; k < nshow; k++) {
                SubDesc d;
                HIPCK(hipMemcpy(&d, c->d_desc + hf[k].s, sizeof(SubDesc), hipMemcpyDeviceToHost));
                fprintf(stderr, " [s=%u%s want %d/%d have %d/%d cnt %u]", hf[k].s, hf[k].certain ? "C" : "", hf[k].mode,
                        hf[k].entry, d.mode, d.entry, d.cnt);
            }
            fprintf(stderr, "\n");
            free(hf);
        }
        if (rounds > SERIAL_AFTER || nfix == 0) {
            // the parallel rounds did not settle: one exact serial walk per file
            hipLaunchKernelGGL(k_serial, dim3(nfiles), dim3(64), CLY_SCAN_LDS, st, c->d_files, c->d_cand, c->d_fck,
                               c->d_desc, c->d_sums, c->d_cols, c->d_staging, c->d_g);
            HIPCK(hipGetLastError());
        } else {
            if ((rc = fix_round(stamp, nfix))) return rc;
        }
        if (c->dbg_flags & 8) {                          // debug: descriptors and stamps after the round
            HIPCK(hipStreamSynchronize(st));
            const int64_t nd = nsub < 64 ? nsub : 64;
            SubDesc hd[64];
            uint32_t hl[64];
            HIPCK(hipMemcpy(hd, c->d_desc, sizeof(SubDesc) * nd, hipMemcpyDeviceToHost));
            HIPCK(hipMemcpy(hl, c->d_listed, sizeof(uint32_t) * nd, hipMemcpyDeviceToHost));
            fprintf(stderr, "  after (stamp %u):", stamp);
            for (int64_t k = 0; k < nd; k++)
                fprintf(stderr, " %lld:%d/%d/%u%s", (long long)k, hd[k].mode, hd[k].entry, hd[k].cnt,
                        hl[k] == stamp ? "w" : (hl[k] == (stamp | LISTED_U) ? "u" : ""));
            fprintf(stderr, "\n");
        }
        if ((rc = link_round(++c->stamp))) return rc;
    }
    HIPCK(hipEventRecord(c->ev[2], st));
    hipLaunchKernelGGL(k_copy, dim3((unsigned)((nsub + CP_SUBS - 1) / CP_SUBS)), dim3(CP_NT), 0, st, c->d_desc,
                       c->d_subP, c->d_staging, d_out, out_cap, nsub, c->d_g);
    if (c->h_g->novf) {
        hipLaunchKernelGGL(k_place, dim3(c->scan_grid), dim3(64 * CLY_NDW), CLY_NDW * CLY_WIN, st, c->d_files,
                           nfiles, c->d_prefix, nsub, c->d_desc, c->d_subP, c->d_staging, d_out, out_cap, c->d_g);
    }
    HIPCK(hipMemsetAsync(c->d_fkey, 0xff, sizeof(unsigned long long) * nfiles, st));
    hipLaunchKernelGGL(k_fin1, dim3((unsigned)((nsub + FIN_NT - 1) / FIN_NT)), dim3(FIN_NT), 0, st, c->d_files, nfiles,
                       c->d_prefix, nsub, c->d_sums, c->d_subP, c->d_x8n, c->d_fkey);
    hipLaunchKernelGGL(k_fin2, dim3((nfiles + FIN_NT - 1) / FIN_NT), dim3(FIN_NT), 0, st, c->d_files, nfiles, c->d_sums,
                       c->d_subP, c->d_x8n, c->d_fkey, c->d_fout);
    HIPCK(hipGetLastError());
    HIPCK(hipEventRecord(c->ev[3], st));
    HIPCK(hipMemcpyAsync(c->h_g, c->d_g, sizeof(Globals), hipMemcpyDeviceToHost, st));
    HIPCK(hipMemcpyAsync(c->h_fout, c->d_fout, sizeof(FileOut) * nfiles, hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    float ms_scan = 0, ms_link = 0, ms_tail = 0;
    HIPCK(hipEventElapsedTime(&ms_scan, c->ev[0], c->ev[1]));
    HIPCK(hipEventElapsedTime(&ms_link, c->ev[1], c->ev[2]));
    HIPCK(hipEventElapsedTime(&ms_tail, c->ev[2], c->ev[3]));
    if ((c->h_g->lb_timeout || c->h_g->fail) && !CLY_EXP) {
        fprintf(stderr, "clyscan: internal error (timeout %u, invariant %u)\n", c->h_g->lb_timeout, c->h_g->fail);
        return CLY_ERR_DEVICE;
    }
    uint64_t total = 0;
    for (int i = 0; i < nfiles; i++) {
        if (!c->h_fout[i].ok && !CLY_EXP) { fprintf(stderr, "clyscan: internal error (file %d has no end event)\n", i); return CLY_ERR_DEVICE; }
        file_first[i] = c->h_fout[i].first_index;
        res[i].n_records = c->h_fout[i].n_records;
        res[i].end_offset = c->h_fout[i].end_offset;
        res[i].status = c->h_fout[i].status;
        res[i]._pad = 0;
        total += c->h_fout[i].n_records;
    }
    if (needed) *needed = c->h_g->total;

    if (stats) {
        stats->scan_ms = ms_scan; stats->resolve_ms = ms_link + ms_tail; stats->total_ms = ms_scan + ms_link + ms_tail;
        stats->passes = 1 + rounds;
        stats->n_chunks = (uint32_t)nsub; stats->bytes = bytes; stats->records = total;
    }
    if (c->h_g->overflow || c->h_g->total > out_cap) return CLY_ERR_CAPACITY;
    return CLY_OK;
}

// Host-memory entry.  Inputs of at least PIPE_MIN bytes go through a
// pipeline: the files are split into groups of >= PIPE_GROUP bytes (whole
// files); a copy thread moves group g+1 host->device while group g is scanned
// and its tuples travel device->host (PCIe is full duplex), so the H2D stream
// of the file bytes sets the pace.
#define PIPE_MIN (256ull << 20)
#define PIPE_GROUP (512ull << 20)
extern "C" int cly_scan(cly_ctx* c, const cly_file* files, int nfiles, cly_tuple* out, uint64_t out_cap,
                        uint64_t* file_first, cly_file_result* res, uint64_t* needed, cly_stats* stats) {
    if (!c || (!files && nfiles) || nfiles < 0 || !res || !file_first) return CLY_ERR_ARG;
    if (nfiles == 0) { if (needed) *needed = 0; return CLY_OK; }
    HIPCK(hipSetDevice(c->device));
    // pack the files into one device buffer, each at a 4 KiB-aligned offset
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
    const uint64_t cap = cly_scan_capacity(files, nfiles) + 16 * (uint64_t)nfiles + 16;
    if (cap > c->cap_tuples) {
        hipFree(c->d_tuples);
        c->cap_tuples = cap;
        HIPCK(hipMalloc(&c->d_tuples, sizeof(cly_tuple) * cap));
    }
    cly_file* df = (cly_file*)malloc(sizeof(cly_file) * nfiles);
    uint64_t* goff = (uint64_t*)malloc(sizeof(uint64_t) * (nfiles + 1));   // device byte offset of each file
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
    // groups of whole files
    int ng = 0;
    int* gstart = (int*)malloc(sizeof(int) * (nfiles + 1));
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
    uint64_t tbase = 0, o = 0, slots_total = 0, need = 0;
    cly_stats st_acc;
    memset(&st_acc, 0, sizeof(st_acc));
    for (int g = 0; g < ng && rc == CLY_OK; g++) {
        while (ready.load(std::memory_order_acquire) <= g) std::this_thread::yield();
        if (copy_err) { rc = CLY_ERR_DEVICE; break; }
        const int f0 = gstart[g], nf = gstart[g + 1] - gstart[g];
        const uint64_t gcap = cly_scan_capacity(files + f0, nf) + 16;
        uint64_t slots = 0;
        cly_stats sg;
        rc = cly_scan_device(c, df + f0, nf, c->d_tuples + tbase, gcap, file_first + f0, res + f0, &slots, &sg, nullptr);
        if (rc == CLY_ERR_CAPACITY) slots_total += slots;
        if (rc != CLY_OK) break;
        st_acc.scan_ms += sg.scan_ms; st_acc.resolve_ms += sg.resolve_ms; st_acc.total_ms += sg.total_ms;
        st_acc.passes = st_acc.passes > sg.passes ? st_acc.passes : sg.passes;
        st_acc.n_chunks += sg.n_chunks; st_acc.bytes += sg.bytes; st_acc.records += sg.records;
        // tuples of the group's files back to host memory (per file: the slots may hold
        // tuples past an ErrInvalidCRC), while the next group is still coming in
        for (int i = f0; i < f0 + nf; i++) {
            need += res[i].n_records;
            if (need > out_cap) { rc = CLY_ERR_CAPACITY; break; }
            if (res[i].n_records &&
                hipMemcpyAsync(out + o, c->d_tuples + tbase + file_first[i], sizeof(cly_tuple) * res[i].n_records,
                               hipMemcpyDeviceToHost, c->stream) != hipSuccess) { rc = CLY_ERR_DEVICE; break; }
            file_first[i] = o;
            o += res[i].n_records;
        }
        tbase += gcap;
    }
    if (rc != CLY_OK) ready.store(ng);            // (the copier only reads `ready`'s own stores; it finishes its groups)
    copier.join();                                // no return before this: the copier must be joined
    if (hipStreamSynchronize(c->stream) != hipSuccess && rc == CLY_OK) rc = CLY_ERR_DEVICE;
    free(df); free(goff); free(gstart);
    if (stats) *stats = st_acc;
    if (needed) {
        if (rc == CLY_ERR_CAPACITY) {
            uint64_t n_all = 0;
            for (int i = 0; i < nfiles; i++) n_all += res[i].n_records;
            *needed = slots_total > n_all ? slots_total : n_all;
        } else {
            *needed = need;
        }
    }
    return rc;
}

// Context accessors for the merge entries (clymerge.hip); not in the public header.
extern "C" hipStream_t cly_ctx_stream_internal(cly_ctx* c) { return c->stream; }
extern "C" int cly_ctx_device_internal(cly_ctx* c) { return c->device; }
extern "C" void** cly_ctx_merge_slot_internal(cly_ctx* c) { return &c->merge_scratch; }

// Debug / statistics (not part of include/clyscan.h)
extern "C" int cly_dbg_sums(cly_ctx* c, void* out, int n) {
    HIPCK(hipDeviceSynchronize());
    HIPCK(hipMemcpy(out, c->d_sums, sizeof(ChunkSum) * n, hipMemcpyDeviceToHost));
    return n;
}
extern "C" int cly_dbg_sumsize(void) { return (int)sizeof(ChunkSum); }
extern "C" int cly_dbg_descs(cly_ctx* c, void* out, int n) {
    HIPCK(hipDeviceSynchronize());
    HIPCK(hipMemcpy(out, c->d_desc, sizeof(SubDesc) * n, hipMemcpyDeviceToHost));
    return n;
}
extern "C" int cly_dbg_subp(cly_ctx* c, uint64_t* out, int n) {
    HIPCK(hipDeviceSynchronize());
    HIPCK(hipMemcpy(out, c->d_subP, sizeof(uint64_t) * n, hipMemcpyDeviceToHost));
    return n;
}
extern "C" int cly_dbg_stats(cly_ctx* c, uint32_t* out4) {
    out4[0] = c->h_g->fix_total; out4[1] = 0; out4[2] = c->scan_grid; out4[3] = CLY_SCAN_LDS;
    return 4;
}
extern "C" int cly_dbg_prof(cly_ctx* c, uint64_t* out24) {
    for (int i = 0; i < 24; i++) out24[i] = c->h_g->prof[i];
    return 24;
}
extern "C" int cly_dbg_enable(cly_ctx* c, int on) { c->dbg_flags = on; return 0; }

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

extern "C" const char* cly_build_info(void) {
    static char buf[200];
    snprintf(buf, sizeof(buf), "clyscan gfx950 SUB=%d WAVES=%d TS=%d CAP=%d LDS=%d tables=16x sched=%s src=%s", CLY_SUB,
             CLY_NDW, CLY_TS, CLY_CAP, (int)CLY_SCAN_LDS, CLY_SCHED, CLY_SRC_HASH);
    return buf;
}
