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

#include "scan_core.h"

#define CLY_KS_LEVELS 6                          // Kogge-Stone levels over 64 lanes
#define MODE_EMPTY 0                             // sub-tile beyond the end of its file
#define MODE_NORMAL 1                            // the chain enters (or ends) inside the sub-tile
#define MODE_PASS 2                              // one record covers the whole sub-tile
#define MODE_DEAD 3                              // the file's chain ended in an earlier sub-tile

struct DevFile {                 // 32 B
    const uint8_t* base;         // device pointer to the file's first byte (16-B aligned)
    uint64_t len;
    uint32_t fid;
    uint32_t first_unit;         // global index of the file's first unit
    uint32_t nsub;               // sub-tiles of the file (>= 1)
    uint32_t _pad;
};

struct Globals {                 // zeroed per call
    uint32_t ticket;
    uint32_t overflow;           // tuples beyond out_cap were dropped
    uint32_t lb_timeout;         // a look-back / mailbox spin hit its bound (never expected)
    uint32_t fail;               // an internal invariant was violated (never expected)
    uint64_t total;              // tuple slots used (records + any past an ErrInvalidCRC)
    uint32_t redo_units;         // units whose guessed entry was wrong (statistics)
    uint32_t redo_subs;          // sub-tiles re-resolved inside a unit (statistics)
    uint64_t prof[24];           // profiling build (-DCLY_PROF): summed cycles per phase
};

#ifdef CLY_PROF
#define PROF_INIT() uint64_t prof_t = __builtin_amdgcn_s_memtime(); uint64_t prof_acc[12] = {0,0,0,0,0,0,0,0,0,0,0,0}
#define PROF(i) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); prof_acc[i] += t_ - prof_t; prof_t = t_; } while (0)
#define PROF_FLUSH(base) do { if (lane == 0) for (int i_ = 0; i_ < 12; i_++) atomicAdd((unsigned long long*)&g->prof[(base) + i_], (unsigned long long)prof_acc[i_]); } while (0)
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
// LDS layout (dynamic shared memory, byte offsets)
//   [0, 65536)        CRC slicing-by-4 tables T0..T3, 16 replicas: dword
//                     (i*64 + t*16 + r) = T_t[i] (replica r); lane l reads replica
//                     l & 15, so one lookup instruction touches 16 banks x 2 lanes
//   [65536, +256)     inverse of a zero-byte step (top byte of T0 -> index)
//   [LDS_CTRL, ...)   coordinator <-> data-wave mailboxes
//   [LDS_WIN + k*WIN) window of data wave k (sub-tile + halo, zero past the file end)
#define LDS_TAB 0
#define LDS_INV 65536
#define LDS_CTRL (LDS_INV + 256)

struct SubSum {                  // data wave -> coordinator (under its own guess)
    int32_t  mode;               // MODE_EMPTY / MODE_NORMAL (guess found) / MODE_PASS (none)
    int32_t  guess;              // sub-tile-relative guessed entry
    int64_t  exit;               // sub-tile-relative exit of the guessed chain
    uint32_t cnt;
    int32_t  term;               // the guessed chain ends inside the sub-tile
};
struct SubEnt {                  // coordinator -> data wave
    int32_t  mode;
    int32_t  entry;              // sub-tile-relative entry (MODE_NORMAL)
    uint32_t base;               // records of the unit before this sub-tile
    int32_t  _pad;
};
struct Job {
    int32_t  unit;               // global unit index, -1: no more work
    int32_t  fidx;
    uint32_t uoff;               // the unit's offset in its file
    int32_t  _pad;
};
struct Cmp {                     // composer -> looker, per unit (slot = iteration & 1)
    int32_t  unit, fidx;
    uint32_t uoff;
    int32_t  fof, gvalid, dead;
    int64_t  G, X;               // unit-relative guessed entry and exit of the composed chain
    uint32_t N;                  // records of the composed chain
    int32_t  _pad;
};
struct Ctrl {
    Job      job[2];
    SubSum   sum[CLY_NDW];
    SubEnt   ent[CLY_NDW];       // under the unit's composed entry
    Cmp      cmp[2];
    SubEnt   fin[2][CLY_NDW];    // final (after the look-back), slot = iteration & 1
    uint64_t P[2];               // records before the unit (global)
    int32_t  job_seq, ent_seq, spec_seq, fin_seq;
    int32_t  sum_seq[CLY_NDW];
};
#define LDS_WIN ((LDS_CTRL + (int)sizeof(Ctrl) + 15) & ~15)
#define LDS_POOL (LDS_WIN + CLY_NDW * CLY_WIN)
#define LDS_KSCOL (LDS_POOL + CLY_NDW * 192 * 8)              // 6 x 32 columns of A^(SUB*2^k)
#define LDS_HSCOL (LDS_KSCOL + CLY_KS_LEVELS * 32 * 4)          // NWD x 32 columns of A^(4*w)
#define CLY_SCAN_LDS (LDS_HSCOL + CLY_NWD * 32 * 4)
#define CLY_COLS ((CLY_KS_LEVELS + CLY_NWD) * 32)                // words of the column table
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
// M v for a linear map M given by its 32 columns M(1 << b) in LDS
__device__ __forceinline__ uint32_t col_mul(const CLY_LDS uint8_t* smem, int col_byte_off, uint32_t v) {
    const CLY_LDS u32x4* c4 = (const CLY_LDS u32x4*)(smem + col_byte_off);
    uint32_t p = 0;
    #pragma unroll
    for (int q = 0; q < 8; q++) {
        const u32x4 c = c4[q];
        p ^= c.x & (uint32_t)__builtin_amdgcn_sbfe((int)v, 4 * q + 0, 1);
        p ^= c.y & (uint32_t)__builtin_amdgcn_sbfe((int)v, 4 * q + 1, 1);
        p ^= c.z & (uint32_t)__builtin_amdgcn_sbfe((int)v, 4 * q + 2, 1);
        p ^= c.w & (uint32_t)__builtin_amdgcn_sbfe((int)v, 4 * q + 3, 1);
    }
    return p;
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
    uint8_t hb[28];
    const int64_t need = nrel - x < 26 ? nrel - x : 26;
    const uint8_t* gp = gfile + cbase + x;
    for (int k = 0; k < need; k++) hb[k] = gp[k];
    h = step_hdr(hb, 0, nrel - x, cbase + x);
}

// SWAR byte masks (bit 7 of each byte): byte <= 4 (type/dtype), and
// byte nonzero and even (first byte of the key-size varint of a record with ks >= 1).
__device__ __forceinline__ uint32_t swar_le4(uint32_t W) { return ~(((W | 0x80808080u) - 0x05050505u) | W) & 0x80808080u; }
__device__ __forceinline__ uint32_t swar_ks(uint32_t W) {
    const uint32_t nz = ((W & 0x7f7f7f7fu) + 0x7f7f7f7fu) | W;
    return nz & ~(W << 7) & 0x80808080u;
}
// First q in [q0, b) whose bytes q+4, q+5 are <= 4 and q+6 is nonzero and
// even (word-parallel filter over the LDS window); b if none.
__device__ int next_candidate(const CLY_LDS uint32_t* w32, int q0, int b) {
    int i = (q0 + 4) >> 2;
    uint32_t Li = swar_le4(w32[i]), Ki = swar_ks(w32[i]);
    for (;;) {
        const int qbase = 4 * i - 4;
        if (qbase >= b) return b;
        const uint32_t Wn = w32[i + 1];
        const uint32_t Ln = swar_le4(Wn), Kn = swar_ks(Wn);
        uint32_t c = Li & __builtin_amdgcn_alignbit(Ln, Li, 8) & __builtin_amdgcn_alignbit(Kn, Ki, 16);
        if (qbase < q0) c &= ~0u << (8 * (q0 - qbase));
        if (c) {
            const int q = qbase + (__builtin_ctz(c) >> 3);
            return q < b ? q : b;
        }
        i++;
        Li = Ln;
        Ki = Kn;
    }
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
    int64_t x;
};

// Exact walk (ReadLogRecord semantics, any record or terminal) of the lane's
// stripe [a, b) from position e.
__device__ __noinline__ void exact_walk(const Sub& T, int a, int b, int e, Lane& L) {
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

__device__ __noinline__ void spec_lane(const Sub& T, int lane, int q0, Spec& r) {
    r.s = -1; r.last = -1; r.c = 0; r.x = 0;
    const int a = lane * CLY_SUB;
    if (a >= T.dlen) return;
    const int b = a + CLY_SUB < T.dlen ? a + CLY_SUB : T.dlen;
    for (int q = q0; q < b; q = next_candidate(T.w32, q + 1, b)) {
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
        if (!ok) continue;
        if (x < T.nrel) {
            const int64_t need = T.nrel - x < 26 ? T.nrel - x : 26;
            Hdr e;
            if (x + need <= T.win_len) e = hdr_at(T.w32, (int)x, T.nrel, T.cbase + x);
            else hdr_global(T.gfile, T.cbase, x, T.nrel, e);
            if (!e.good) continue;
        }
        r.s = q; r.last = (int)p; r.c = c; r.x = x;
        return;
    }
}

// resolve(E): the sub-tile's record chain from entry E (sub-tile-relative).
__device__ __noinline__ void resolve(const Sub& T, const Spec& sp, int lane, int E, Lane& L, Chain& R) {
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
__device__ __forceinline__ void crc_loop(const CLY_LDS uint8_t* smem, const uint32_t* d, int rs, uint64_t chk,
                                         uint32_t lane_off, uint32_t& s_out, uint32_t& obs_out, uint32_t& err_out) {
    uint32_t s = 0, obs = 0, err = 0;
    #pragma unroll
    for (int i = 0; i < CLY_NWD; i++) {
        const bool r = i == rs;
        obs = r ? s : obs;
        const uint32_t x = (r ? 0u : s) ^ d[i];
        s = crc_word(smem, x, lane_off);
        const uint32_t m = (uint32_t)(-(int32_t)((chk >> i) & 1));
        err |= s & m;
    }
    s_out = s; obs_out = obs; err_out = err;
}

__device__ __noinline__ void crc_slow(const Sub& T, const Chain& R, CLY_LDS uint8_t* smem, CrcOut& out);

__device__ __noinline__ void crc_phase(const Sub& T, const Lane& L, const Chain& R, int lane, CLY_LDS uint8_t* smem,
                                       CLY_LDS uint32_t* w32, CLY_LDS u32x2* pool, CrcOut& out) {
    const uint32_t lane_off = (uint32_t)(lane & 15) * 4;
    out.bad = 0; out.head_raw = 0; out.head_z = 0; out.end_state = 0;
    const bool normal = R.mode == MODE_NORMAL;
    // ---- check points of this lane: chain records, then its terminal
    const bool tcp = normal && L.wterm && L.wx < CLY_TS;
    const int n = normal ? ((L.ws >= 0 ? L.wc : 0) + (tcp ? 1 : 0)) : 0;
    const uint32_t incl = scan_add_incl((uint32_t)n, lane);
    const int off = (int)(incl - (uint32_t)n);
    const int total = (int)__shfl(incl, CLY_NT - 1, 64);
    if (total > CP_POOL) {
        if (lane == 0) crc_slow(T, R, smem, out);
        out.bad = __shfl(out.bad, 0, 64); out.head_raw = __shfl(out.head_raw, 0, 64);
        out.head_z = __shfl(out.head_z, 0, 64); out.end_state = __shfl(out.end_state, 0, 64);
        return;
    }
    if (n) {
        int i = off;
        if (L.ws >= 0) {
            int p = L.ws;
            for (int r = 0; r < L.wc; r++, i++) {
                pool[i] = (u32x2){(uint32_t)p | CP_REAL, lds_le32(w32, p)};
                const Hdr h = hdr_at(w32, p, T.nrel, T.cbase + p);
                p += (int)h.size;
            }
        }
        if (tcp) pool[i] = (u32x2){(uint32_t)L.wx, lds_le32(w32, (int)L.wx)};
    }
    wave_sync();
    crc_patch_all(smem, w32, pool, off, n, lane_off);
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
    crc_loop(smem, d, rs, chk, lane_off, s, obs, err);
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
        if (!fin_lane) { v ^= col_mul(smem, LDS_KSCOL + lvl * 128, pv); c = pc; }
    }
    uint32_t s_in = __shfl_up(v, 1, 64);
    if (lane == 0) s_in = 0;
    out.end_state = __shfl(v, CLY_NT - 1, 64);
    // ---- reset checks: T = obs ^ A^(4 rs) S_in
    const uint32_t y = col_mul(smem, LDS_HSCOL + (rs > 0 ? rs : 0) * 128, s_in);
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
    // ---- restore the window (XOR patches are involutions)
    crc_patch_all(smem, w32, pool, off, n, lane_off);
    wave_sync();
}

// Slow path (more check points than the pool holds: sub-tiles of tiny
// records): one lane recomputes everything byte-serially from the window.
__device__ __noinline__ void crc_slow(const Sub& T, const Chain& R, CLY_LDS uint8_t* smem, CrcOut& out) {
    const CLY_LDS uint8_t* w8 = (const CLY_LDS uint8_t*)T.w32;
    out.bad = 0;
    // head: Z_z(raw [4, E))
    uint32_t s = 0;
    for (int q = 4; q < R.E; q++) s = crc_byte(smem, s, w8[q], 0);
    const uint32_t z = 4 - (R.E & 3);
    for (uint32_t k = 0; k < z; k++) s = crc_byte(smem, s, 0, 0);
    out.head_raw = s;
    out.head_z = z;
    // records
    int64_t p = R.E;
    uint32_t last_state = 0xFFFFFFFFu;
    for (uint32_t i = 0; i < R.cnt; i++) {
        const Hdr h = hdr_at(T.w32, (int)p, T.nrel, T.cbase + p);
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
__device__ __noinline__ void crc_locate(const Sub& T, const Chain& R, CLY_LDS uint8_t* smem, int& pos, uint32_t& idx) {
    pos = -1; idx = 0;
    const CLY_LDS uint8_t* w8 = (const CLY_LDS uint8_t*)T.w32;
    int64_t p = R.E;
    uint32_t i = 0;
    while (p < CLY_TS && i < R.cnt) {
        const Hdr h = hdr_at(T.w32, (int)p, T.nrel, T.cbase + p);
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
// Coordinator pieces.
struct DevEnv {
    Desc* desc;
    Globals* g;
    uint32_t epoch;
    uint32_t spins;
    int64_t nunits;
    __device__ __forceinline__ uint64_t ld(int64_t j, int k) { return ld_agent(&desc[j].w[k]); }
    __device__ __forceinline__ bool spin() {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > LB_SPIN_MAX) { atomicOr(&g->lb_timeout, 1u); return false; }
        return true;
    }
};

// Decoupled look-back by the coordinator wave: 64 descriptors per round trip,
// then every lane folds them in order (uniform; scan_core.h lb_walk_step).
__device__ __noinline__ void lookback(DevEnv& env, int64_t c, int fof, int lane, LbState& res) {
    const uint32_t epoch = env.epoch;
    LbWalk w;
    lb_walk_init(w, c, fof);
    LbState out;
    out.E = 0; out.P = 0; out.dead = 1; out._pad = 0;
    int64_t jf = -1;
    int r = 0;
    bool ok = true;
    for (int64_t base = c - 1; r == 0 && ok; base -= 64) {
        if (base < 0) {
            r = lb_apply_full_walk(w, 0, 0, 0, out) ? 1 : 2;
            jf = -1;
            break;
        }
        const int64_t j = base - lane;
        uint64_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
        int stop;
        for (;;) {
            bool ready = true, full = false;
            if (j >= 0) {
                w1 = env.ld(j, 1); w2 = env.ld(j, 2); w3 = env.ld(j, 3);
                w0 = env.ld(j, 0);
                const uint64_t st = ds_state(w0, epoch);
                if (st == DS_SPEC) ready = ds_ok(w1, epoch);
                else if (st == DS_FULL) { ready = ds_ok(w2, epoch) && ds_ok(w3, epoch); full = ready; }
                else ready = false;
            }
            const unsigned long long endm = __ballot(full || j < 0);
            stop = endm ? __ffsll((long long)endm) - 1 : 64;
            const unsigned long long need = stop >= 63 ? ~0ull : ((2ull << stop) - 1);
            if (!(__ballot(!ready) & need)) break;
            int go = 1;
            if (lane == 0) go = env.spin() ? 1 : 0;
            if (!__shfl(go, 0, 64)) { ok = false; break; }
        }
        if (!ok) break;
        // fast path: a run of "tight" speculative descriptors from lane 0
        int i0 = 0;
        {
            const int64_t jn = j + 1;
            const uint64_t w0n = __shfl_up(w0, 1, 64);
            const bool spec = j >= 0 && ds_state(w0, epoch) == DS_SPEC && ds_gvalid(w0) && !ds_fof(w0) && !ds_term(w0);
            const int64_t xj = (int64_t)(w1 & DS_VAL_MASK);
            bool tight;
            if (lane == 0) tight = spec && lb_req_ok(w, xj);
            else tight = spec && ds_gvalid(w0n) && !ds_fof(w0n) && xj == jn * CLY_UNIT + ds_grel(w0n);
            const unsigned long long tm = __ballot(tight && lane < stop);
            const int run = (~tm) ? __ffsll((long long)~tm) - 1 : 64;
            if (run > 0) {
                uint32_t cnt = (lane < run) ? ds_cnt(w0) : 0u;
                #pragma unroll
                for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
                const uint64_t w0l = __shfl(w0, run - 1, 64);
                const uint64_t x0 = __shfl(w1, 0, 64);
                if (run >= 2) {
                    const uint64_t w0p = __shfl(w0, run - 2, 64);
                    w.prev = static_cast<const LbSum&>(w);
                    if (w.prev.res == LB_RES_IDENT) { w.prev.res = LB_RES_CONST; w.prev.rx = (int64_t)(x0 & DS_VAL_MASK); }
                    w.prev.dp += cnt - ds_cnt(w0l);
                    w.prev.req = LB_REQ_EXACT;
                    w.prev.e0 = (base - (run - 2)) * CLY_UNIT + ds_grel(w0p);
                } else {
                    w.prev = static_cast<const LbSum&>(w);
                }
                w.kreq = base - (run - 1);
                if (w.res == LB_RES_IDENT) { w.res = LB_RES_CONST; w.rx = (int64_t)(x0 & DS_VAL_MASK); }
                w.dp += cnt;
                w.req = LB_REQ_EXACT;
                w.e0 = (base - (run - 1)) * CLY_UNIT + ds_grel(w0l);
                i0 = run;
            }
        }
        const int last = stop < 64 ? stop : 63;
        for (int i = i0; i <= last && r == 0; i++) {
            const int64_t ji = base - i;
            if (ji < 0) {
                r = lb_apply_full_walk(w, 0, 0, 0, out) ? 1 : 2;
                jf = -1;
            } else {
                r = lb_walk_step(w, ji, __shfl(w0, i, 64), __shfl(w1, i, 64), __shfl(w2, i, 64),
                                 __shfl(w3, i, 64), epoch, out, jf);
            }
        }
    }
    if (ok && r == 2 && lb_recover_kreq(env, w, epoch, out)) r = 1;
    if (ok && r == 2) {
        if (jf == -3) {
            jf = -1;
            for (int64_t k = c - 1; k >= 0; k--) {
                uint64_t a0 = env.ld(k, 0);
                while (ds_state(a0, epoch) == 0 && env.spin()) a0 = env.ld(k, 0);
                if (ds_state(a0, epoch) == DS_FULL) { jf = k; break; }
            }
        }
        lb_forward(env, c, fof, jf, epoch, out);
    }
    res = out;
    res.E = __shfl(res.E, 0, 64);
    res.P = __shfl(res.P, 0, 64);
    res.dead = __shfl(res.dead, 0, 64);
}

// Serial exact walk of sub-tile k from rel (one lane): chain exit, records,
// terminated.  data/dataFile.go:64-111 per step.  From the LDS window, or
// (late recompose, the window is gone) from HBM.
__device__ __noinline__ void coord_walk(const CLY_LDS uint32_t* w32, const uint8_t* gfile, int64_t cbase, int64_t nrel,
                                        int lof, int64_t rel, int64_t& exit, uint32_t& n, int& term) {
    int64_t p = rel;
    n = 0;
    term = 0;
    while (p < CLY_TS) {
        Hdr h;
        if (w32) h = hdr_at(w32, (int)p, nrel, cbase + p);
        else hdr_global(gfile, cbase, p, nrel, h);
        if (h.status != REC_OK) { term = 1; break; }
        n++;
        p += h.size;
    }
    if (!term && lof && p == nrel) term = 1;
    exit = p;
}

// Compose the unit's sub-tile chains from unit-relative entry e (exact: a
// sub-tile whose data wave guessed differently is walked here).  Writes the
// per-sub-tile entries to `ent` (LDS) and returns the unit exit / count / dead.
__device__ __noinline__ void compose(CLY_LDS Ctrl* C, CLY_LDS SubEnt* ent, const DevFile& F, uint32_t uoff,
                                     CLY_LDS uint8_t* smem, bool from_global, int64_t e, int64_t& X, uint32_t& N,
                                     int& dead, Globals* g) {
    uint32_t count = 0;
    dead = 0;
    for (int k = 0; k < CLY_NDW; k++) {
        const SubSum s = lds_get(&C->sum[k]);
        SubEnt o;
        o.base = count; o.entry = 0; o._pad = 0;
        const int64_t ks = (int64_t)k * CLY_TS;
        if (s.mode == MODE_EMPTY) o.mode = MODE_EMPTY;
        else if (dead) o.mode = MODE_DEAD;
        else if (e - ks >= CLY_TS) o.mode = MODE_PASS;
        else {
            const int64_t rel = e - ks;
            o.mode = MODE_NORMAL;
            o.entry = (int)rel;
            if (!from_global && s.mode == MODE_NORMAL && rel == s.guess) {
                count += s.cnt;
                if (s.term) dead = 1;
                else e = ks + s.exit;
            } else {
                const int64_t cbase = (int64_t)uoff + ks;
                const int64_t nrel = (int64_t)F.len - cbase;
                const int lof = cbase + CLY_TS >= (int64_t)F.len;
                const CLY_LDS uint32_t* w32 =
                    from_global ? nullptr : (const CLY_LDS uint32_t*)(smem + LDS_WIN + k * CLY_WIN);
                int64_t x;
                uint32_t n;
                int term;
                coord_walk(w32, F.base, cbase, nrel, lof, rel, x, n, term);
                atomicAdd(&g->redo_subs, 1u);
                count += n;
                if (term) dead = 1;
                else e = ks + x;
            }
        }
        lds_put(&ent[k], o);
    }
    X = e;
    N = count;
}

// ---------------------------------------------------------------------------
// Data-wave pieces.
// Sub-tile geometry of data wave k for job jb.
__device__ __forceinline__ void sub_setup(Sub& T, const Job& jb, const DevFile& F, int k, CLY_LDS uint32_t* w32) {
    T.gfile = F.base;
    T.w32 = w32;
    T.cbase = (int64_t)jb.uoff + (int64_t)k * CLY_TS;
    T.nrel = (int64_t)F.len - T.cbase;
    T.dlen = (int)(T.nrel < CLY_TS ? (T.nrel > 0 ? T.nrel : 0) : CLY_TS);
    T.win_len = (int)(T.nrel < CLY_WIN ? (T.nrel > 0 ? T.nrel : 0) : CLY_WIN);
    T.fof = T.cbase == 0;
    T.lof = T.cbase + CLY_TS >= (int64_t)F.len;
    T.chunk = (int64_t)jb.unit * CLY_NDW + k;
    T.fid = F.fid;
}

// Speculation over the staged window: per lane the first candidate (register
// SWAR filter over its stripe), then the candidate walks; the sub-tile guess.
__device__ __noinline__ void sub_spec(const Sub& T, int lane, Spec& sp, int& guess) {
    const CLY_LDS uint32_t* w32 = T.w32;
    sp.s = -1; sp.last = -1; sp.c = 0; sp.x = 0;
    int q0 = CLY_TS;
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
        int fm = CLY_NWD;
        uint32_t Ln = swar_le4(dw[CLY_NWD + 1]), Kn = swar_ks(dw[CLY_NWD + 1]);
        #pragma unroll
        for (int m = CLY_NWD - 1; m >= 0; m--) {
            const uint32_t Lm = swar_le4(dw[m + 1]), Km = swar_ks(dw[m + 1]);
            const uint32_t cm = Lm & __builtin_amdgcn_alignbit(Ln, Lm, 8) & __builtin_amdgcn_alignbit(Kn, Km, 16);
            fm = cm ? m : fm;
            Ln = Lm; Kn = Km;
        }
        if (fm < CLY_NWD) q0 = next_candidate(w32, a + 4 * fm, a + CLY_SUB < T.dlen ? a + CLY_SUB : T.dlen);
    }
    spec_lane(T, lane, q0, sp);
    if (T.fof) { guess = 0; return; }
    const unsigned long long m = __ballot(sp.s >= 0);
    guess = m ? __shfl(sp.s, __ffsll((long long)m) - 1, 64) : -1;
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
    const CLY_LDS uint32_t* w32 = T.w32;
    ChunkSum cs;
    cs.p_excl = base;
    cs.evt_off = EVT_NONE; cs.evt_gidx = 0; cs.evt_status = 0; cs.cnt = 0;
    cs.open_pos = -1; cs.open_state = 0; cs.open_crc = 0;
    cs.first4 = w32[0];
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
            cs.open_crc = lds_le32(w32, R.last);
            const int ocs = R.last + 4;
            if (ocs >= CLY_TS) {
                cs.open_state = 0xFFFFFFFFu;
            } else if (ocs + 4 > CLY_TS) {
                uint32_t s = 0xFFFFFFFFu;
                const CLY_LDS uint8_t* w8 = (const CLY_LDS uint8_t*)w32;
                for (int q = ocs; q < CLY_TS; q++) s = crc_byte(smem, s, w8[q], 0);
                cs.open_state = s;
            } else {
                cs.open_state = co.end_state;
            }
        }
    }
    cs.head_shift = cs.head_len > 4 ? cs.head_len - 4 + cs.head_z : 0;   // exponent; k_fin maps it
    sums[T.chunk] = cs;
}

// CRC + first failure + summary of a resolved sub-tile.
__device__ __noinline__ void sub_crc(const Sub& T, const Lane& L, const Chain& R, int lane, CLY_LDS uint8_t* smem,
                                        CLY_LDS u32x2* pool, uint32_t base, ChunkSum* sums, Globals* g) {
    CrcOut co;
    crc_phase(T, L, R, lane, smem, (CLY_LDS uint32_t*)T.w32, pool, co);
    int bpos = -1;
    uint32_t bidx = 0;
    if (lane == 0) {
        if (co.bad) crc_locate(T, R, smem, bpos, bidx);
        sub_summary(T, R, co, smem, base, bpos, bidx, sums, g);
    }
}

// Tuple words of one record at window position p (index independent).
__device__ __forceinline__ void tuple_words(const Sub& T, int p, u32x4& q0, u32x4& q1, u32x4& q2, int64_t& size) {
    const CLY_LDS uint8_t* w8 = (const CLY_LDS uint8_t*)T.w32;
    const Hdr h = hdr_at(T.w32, p, T.nrel, T.cbase + p);
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
__device__ __noinline__ void emit_direct(const Sub& T, const Lane& L, uint64_t idx0, cly_tuple* out, uint64_t out_cap,
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
    if (of) atomicOr(&g->overflow, 1u);
}

// ---------------------------------------------------------------------------
// The scan kernel: CLY_NDW data waves + a composer wave + a look-back wave per
// workgroup (one workgroup per CU).  Pipeline of a data wave, iteration i on
// unit u_i:  [window staged]  speculate + resolve -> summary  | composer:
// compose u_i, SPEC |  CRC of u_i, tuples kept in registers  |  flush u_{i-1}
// (output slot from the looker's look-back of u_{i-1})  |  issue the staging
// of u_{i+1}.  The look-back of a unit thus overlaps the next unit's work.
#define WAVES_PER_WG (CLY_NDW + 2)
#define FLAG_FORCE_REDO 1

__global__ void __launch_bounds__(64 * WAVES_PER_WG)
k_scan(const DevFile* __restrict__ files, int nfiles, const uint32_t* __restrict__ file_unit_prefix, int64_t nunits,
       Desc* desc, ChunkSum* sums, uint64_t* unit_P, const uint32_t* __restrict__ cols, cly_tuple* out,
       uint64_t out_cap, Globals* g, uint32_t epoch, SubDbg* dbg, int flags) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    CLY_LDS uint8_t* smem = (CLY_LDS uint8_t*)smem_raw;
    CLY_LDS Ctrl* C = (CLY_LDS Ctrl*)(smem + LDS_CTRL);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
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
    for (int i = threadIdx.x; i < CLY_COLS; i += blockDim.x) ((CLY_LDS uint32_t*)(smem + LDS_KSCOL))[i] = cols[i];
    if (threadIdx.x == 0) {
        C->job_seq = 0; C->ent_seq = 0; C->spec_seq = 0; C->fin_seq = 0;
        for (int k = 0; k < CLY_NDW; k++) C->sum_seq[k] = 0;
    }
    __syncthreads();

    if (wave == CLY_NDW) {
        // ================= composer: tickets, unit composition, SPEC =================
        PROF_INIT();
        auto take = [&](int slot, int seq) {
            int u = 0;
            if (lane == 0) u = (int)atomicAdd(&g->ticket, 1u);
            u = __shfl(u, 0, 64);
            Job jb;
            jb.unit = -1; jb.fidx = 0; jb.uoff = 0; jb._pad = 0;
            if (u < nunits) {
                int lo = 0, hi = nfiles - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if ((int64_t)file_unit_prefix[mid] <= u) lo = mid; else hi = mid - 1;
                }
                jb.unit = u; jb.fidx = lo; jb.uoff = (uint32_t)((int64_t)(u - (int)files[lo].first_unit) * CLY_UNIT);
            }
            if (lane == 0) { lds_put(&C->job[slot], jb); lds_st_rel(&C->job_seq, seq); }
            return jb;
        };
        Job jb = take(0, 1);
        for (int it = 0;; it++) {
            Cmp cm;
            cm.unit = jb.unit; cm.fidx = jb.fidx; cm.uoff = jb.uoff; cm.fof = 0; cm.gvalid = 0; cm.dead = 0;
            cm.G = 0; cm.X = 0; cm.N = 0; cm._pad = 0;
            if (jb.unit >= 0) {
                const DevFile F = files[jb.fidx];
                const int64_t u = jb.unit;
                const int fof = jb.uoff == 0;
                // predecessor's published exit (a hint that corrects false-merge guesses)
                uint64_t pw0 = 0, pw1 = 0, pw2 = 0;
                if (!fof && lane == 0) { pw1 = ld_agent(&desc[u - 1].w[1]); pw2 = ld_agent(&desc[u - 1].w[2]); pw0 = ld_agent(&desc[u - 1].w[0]); }
                for (int k = 0; k < CLY_NDW; k++) if (!lds_wait_ge(&C->sum_seq[k], it + 1, g)) return;
                PROF(0);
                const Job next = take((it + 1) & 1, it + 2);
                PROF(1);
                int gvalid = 0;
                int64_t G = 0;
                if (fof) { gvalid = 1; G = 0; }
                else {
                    for (int k = 0; k < CLY_NDW; k++) {
                        const SubSum sk = lds_get(&C->sum[k]);
                        if (sk.mode == MODE_NORMAL) { gvalid = 1; G = (int64_t)k * CLY_TS + sk.guess; break; }
                    }
                }
                int64_t X = 0;
                uint32_t N = 0;
                int dead = 0;
                if (lane == 0) {
                    int64_t e0 = gvalid ? G : -1;
                    if (!fof) {
                        const uint64_t st = ds_state(pw0, epoch);
                        const int64_t ustart = u * CLY_UNIT;
                        int64_t hx = -1;
                        if (st == DS_FULL && ds_ok(pw2, epoch) && !ds_term(pw0)) hx = (int64_t)(pw2 & DS_VAL_MASK);
                        else if (st == DS_SPEC && ds_ok(pw1, epoch) && ds_gvalid(pw0) && !ds_term(pw0)) hx = (int64_t)(pw1 & DS_VAL_MASK);
                        if (hx >= ustart && hx < ustart + CLY_UNIT && hx - ustart != e0) {
                            e0 = hx - ustart; gvalid = 1; G = e0;
                        }
                    }
                    if (gvalid) compose(C, C->ent, F, jb.uoff, smem, false, G, X, N, dead, g);
                    else {
                        for (int k = 0; k < CLY_NDW; k++) {
                            SubEnt o;
                            o.mode = lds_get(&C->sum[k]).mode == MODE_EMPTY ? MODE_EMPTY : MODE_PASS;
                            o.entry = 0; o.base = 0; o._pad = 0;
                            lds_put(&C->ent[k], o);
                        }
                    }
                    lds_st_rel(&C->ent_seq, it + 1);
                }
                gvalid = __shfl(gvalid, 0, 64); G = __shfl(G, 0, 64);
                X = __shfl(X, 0, 64); N = __shfl(N, 0, 64); dead = __shfl(dead, 0, 64);
                cm.fof = fof; cm.gvalid = gvalid; cm.dead = dead; cm.G = G; cm.X = X; cm.N = N;
                PROF(2);
                // the looker's slot it&1 is free once it finished unit it-2
                if (it >= 2 && !lds_wait_ge(&C->fin_seq, it - 1, g)) return;
                if (lane == 0) {
                    lds_put(&C->cmp[it & 1], cm);
                    st_agent(&desc[u].w[1], ds_tag(epoch, (uint64_t)(u * CLY_UNIT + X)));
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    st_agent(&desc[u].w[0], ds_pack(epoch, DS_SPEC, fof, dead, gvalid, G, N));
                    lds_st_rel(&C->spec_seq, it + 1);
                }
                PROF(3);
                jb = next;
            } else {
                if (it >= 2 && !lds_wait_ge(&C->fin_seq, it - 1, g)) return;
                if (lane == 0) { lds_put(&C->cmp[it & 1], cm); lds_st_rel(&C->spec_seq, it + 1); }
                break;
            }
        }
        PROF_FLUSH(12);
        return;
    }

    if (wave == CLY_NDW + 1) {
        // ================= looker: look-back, final entries, FULL =================
        PROF_INIT();
        DevEnv env;
        env.desc = desc; env.g = g; env.epoch = epoch; env.spins = 0; env.nunits = nunits;
        for (int it = 0;; it++) {
            if (!lds_wait_ge(&C->spec_seq, it + 1, g)) return;
            const Cmp cm = lds_get(&C->cmp[it & 1]);
            if (cm.unit < 0) break;
            PROF(6);
            const int64_t u = cm.unit;
            const DevFile F = files[cm.fidx];
            LbState lb;
            lookback(env, u, cm.fof, lane, lb);
            PROF(7);
            if (env.spins > LB_SPIN_MAX) lb.dead = 1;
            const int64_t ustart = u * CLY_UNIT;
            CLY_LDS SubEnt* fin = C->fin[it & 1];
            int64_t Xf = cm.X;
            uint32_t Nf = cm.N;
            int deadf = cm.dead;
            if (lane == 0) {
                if (lb.dead) {
                    Nf = 0; deadf = 1; Xf = 0;
                    for (int k = 0; k < CLY_NDW; k++) {
                        SubEnt o; o.entry = 0; o.base = 0; o._pad = 0;
                        o.mode = lds_get(&C->ent[k]).mode == MODE_EMPTY ? MODE_EMPTY : MODE_DEAD;
                        lds_put(&fin[k], o);
                    }
                } else if (cm.gvalid && lb.E == ustart + cm.G) {
                    for (int k = 0; k < CLY_NDW; k++) lds_put(&fin[k], lds_get(&C->ent[k]));
                } else if (lb.E - ustart >= CLY_UNIT) {
                    Nf = 0; deadf = 0; Xf = lb.E - ustart;
                    for (int k = 0; k < CLY_NDW; k++) {
                        SubEnt o; o.entry = 0; o.base = 0; o._pad = 0;
                        o.mode = lds_get(&C->ent[k]).mode == MODE_EMPTY ? MODE_EMPTY : MODE_PASS;
                        lds_put(&fin[k], o);
                    }
                } else {
                    // wrong guess: recompose from the true entry, walking HBM (rare)
                    atomicAdd(&g->redo_units, 1u);
                    compose(C, fin, F, cm.uoff, smem, true, lb.E - ustart, Xf, Nf, deadf, g);
                }
                const uint64_t incl = lb.P + Nf;
                st_agent(&desc[u].w[2], ds_tag(epoch, (uint64_t)(ustart + Xf)));
                st_agent(&desc[u].w[3], ds_tag(epoch, incl));
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                st_agent(&desc[u].w[0], ds_pack(epoch, DS_FULL, cm.fof, deadf, 0, 0, Nf));
                if (u == nunits - 1) g->total = incl;
                unit_P[u] = lb.P;
                C->P[it & 1] = lb.P;
                lds_st_rel(&C->fin_seq, it + 1);
            }
            PROF(8);
        }
        PROF_FLUSH(12);
        return;
    }

    // ================= data wave =================
    const int k = wave;
    CLY_LDS uint32_t* w32 = (CLY_LDS uint32_t*)(smem + LDS_WIN + k * CLY_WIN);
    CLY_LDS u32x2* pool = (CLY_LDS u32x2*)(smem + LDS_POOL + k * CP_POOL * 8);
    PROF_INIT();
    bool pending_dma = false;
    for (int it = 0;; it++) {
        if (!lds_wait_ge(&C->job_seq, it + 1, g)) return;
        const Job jb = lds_get(&C->job[it & 1]);
        if (jb.unit < 0) break;
        PROF(0);
        const DevFile F = files[jb.fidx];
        Sub T;
        sub_setup(T, jb, F, k, w32);
        const bool empty = T.nrel <= 0 && !T.fof;
        Spec sp;
        sp.s = -1; sp.last = -1; sp.c = 0; sp.x = 0;
        Lane L;
        Chain R;
        chain_none(L, R, MODE_PASS);
        int guess = -1;
        if (!empty) {
            if (!pending_dma) { if (stage(T, lane, w32)) stage_wait(); }
            else stage_wait();
            PROF(1);
            sub_spec(T, lane, sp, guess);
            PROF(2);
            if (guess >= 0) resolve(T, sp, lane, guess, L, R);
            PROF(3);
        }
        pending_dma = false;
        if (lane == 0) {
            SubSum ss;
            ss.mode = empty ? MODE_EMPTY : (guess >= 0 ? MODE_NORMAL : MODE_PASS);
            ss.guess = guess;
            ss.exit = R.xrel;
            ss.cnt = R.cnt;
            ss.term = R.term;
            lds_put(&C->sum[k], ss);
            lds_st_rel(&C->sum_seq[k], it + 1);
        }
        if (!lds_wait_ge(&C->ent_seq, it + 1, g)) return;
        PROF(4);
        const SubEnt e = lds_get(&C->ent[k]);
        if (!empty) {
            if (e.mode == MODE_NORMAL ? !(guess >= 0 && e.entry == guess) : true) sub_chain(T, sp, lane, e.mode, e.entry, L, R);
            sub_crc(T, L, R, lane, smem, pool, e.base, sums, g);
        }
        PROF(5);
        if (!lds_wait_ge(&C->fin_seq, it + 1, g)) return;
        PROF(6);
        const SubEnt f = lds_get(&C->fin[it & 1][k]);
        const uint64_t P = C->P[it & 1];
        if (!empty) {
            if (f.mode != e.mode || (f.mode == MODE_NORMAL && f.entry != e.entry) || (flags & FLAG_FORCE_REDO)) {
                sub_chain(T, sp, lane, f.mode, f.entry, L, R);
                sub_crc(T, L, R, lane, smem, pool, f.base, sums, g);
            } else if (f.base != e.base && lane == 0) {
                // same chain, but the unit was recomposed: only its record base moved
                ChunkSum* cs = &sums[T.chunk];
                cs->p_excl = f.base;
                if (cs->evt_off != EVT_NONE) cs->evt_gidx += (uint64_t)f.base - (uint64_t)e.base;
            }
            PROF(7);
            if (R.mode == MODE_NORMAL) emit_direct(T, L, P + f.base + L.base, out, out_cap, g);
            PROF(8);
            if (dbg && lane == 0) {
                SubDbg d;
                d.mode = R.mode; d.E = R.E; d.cnt = (int)R.cnt; d.term = R.term; d.tst = R.tst; d.last = R.last;
                d.lterm = R.lterm; d.eof_exit = R.eof_exit; d.k0 = R.k0; d.guess = guess; d.bad = 0; d.bpos = 0;
                d.tpos = R.tpos; d.xrel = R.xrel;
                dbg[T.chunk] = d;
            }
        }
        // stage the next unit's sub-tile now (the window is free)
        if (!lds_wait_ge(&C->job_seq, it + 2, g)) return;
        const Job nj = lds_get(&C->job[(it + 1) & 1]);
        if (nj.unit >= 0) {
            const DevFile F2 = files[nj.fidx];
            Sub T2;
            sub_setup(T2, nj, F2, k, w32);
            if (T2.nrel > 0 || T2.fof) pending_dma = stage(T2, lane, w32);
        }
        PROF(9);
    }
    PROF_FLUSH(0);
}

// One workgroup per file: first event of the file.
#define FIN_NT 256
__global__ void __launch_bounds__(FIN_NT)
k_fin(const DevFile* __restrict__ files, const ChunkSum* __restrict__ sums, const uint64_t* __restrict__ unit_P,
      const uint32_t* __restrict__ x8n, FileOut* __restrict__ fout) {
    const int f = blockIdx.x, tid = threadIdx.x;
    const DevFile F = files[f];
    const int64_t c0 = (int64_t)F.first_unit * CLY_NDW, nc = F.nsub;
    __shared__ int64_t r_off[FIN_NT];
    __shared__ uint64_t r_g[FIN_NT];
    __shared__ int32_t r_st[FIN_NT];
    int64_t best = EVT_NONE;
    uint64_t bg = 0;
    int32_t bs = 0;
    for (int64_t i = tid; i < nc; i += FIN_NT) {
        uint64_t gi = 0;
        int32_t st = 0;
        const int64_t o = fin_chunk_event(sums, unit_P, x8n, c0, nc, i, &gi, &st);
        if (o < best) { best = o; bg = gi; bs = st; }
    }
    r_off[tid] = best; r_g[tid] = bg; r_st[tid] = bs;
    __syncthreads();
    for (int d = FIN_NT / 2; d > 0; d >>= 1) {
        if (tid < d && r_off[tid + d] < r_off[tid]) {
            r_off[tid] = r_off[tid + d]; r_g[tid] = r_g[tid + d]; r_st[tid] = r_st[tid + d];
        }
        __syncthreads();
    }
    if (tid == 0) {
        FileOut fo;
        const uint64_t first = unit_P[F.first_unit] + sums[c0].p_excl;
        fo.first_index = first;
        fo.ok = r_off[0] != EVT_NONE;
        fo.n_records = fo.ok ? r_g[0] - first : 0;
        fo.end_offset = r_off[0];
        fo.status = r_st[0];
        fout[f] = fo;
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
    DevFile* d_files; int cap_files;
    uint32_t* d_prefix;
    FileOut* d_fout;
    Desc* d_desc; int64_t cap_units;
    ChunkSum* d_sums;
    Globals* d_g;
    uint32_t* d_cols;            // columns of A^(SUB*2^k) (Kogge-Stone) and A^(4w) (head shifts)
    uint32_t* d_x8n;
    DevFile* h_files;
    uint32_t* h_prefix;
    FileOut* h_fout;
    Globals* h_g;
    uint32_t epoch; int desc_fresh;
    int scan_grid;
    uint8_t* d_bytes; uint64_t cap_bytes;          // host-path staging
    SubDbg* d_dbg; int dbg_on;
    uint64_t* d_unitP;
    cly_tuple* d_tuples; uint64_t cap_tuples;
};

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
            for (int b = 0; b < 32; b++) hc[lvl * 32 + b] = cly_multmodp(xm, 1u << b);
        }
        for (int w = 0; w < CLY_NWD; w++) {
            const uint32_t xm = cly_x8n((uint64_t)4 * w);
            for (int b = 0; b < 32; b++) hc[(CLY_KS_LEVELS + w) * 32 + b] = cly_multmodp(xm, 1u << b);
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
    HIPCK(hipFuncSetAttribute((const void*)k_scan, hipFuncAttributeMaxDynamicSharedMemorySize, (int)CLY_SCAN_LDS));
    {
        int per_cu = 0, ncu = 0;
        HIPCK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_scan, 64 * WAVES_PER_WG, CLY_SCAN_LDS));
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
    hipFree(c->d_files); hipFree(c->d_prefix); hipFree(c->d_fout); hipFree(c->d_desc); hipFree(c->d_sums); hipFree(c->d_dbg); hipFree(c->d_unitP);
    hipFree(c->d_g); hipFree(c->d_cols); hipFree(c->d_x8n); hipFree(c->d_bytes); hipFree(c->d_tuples);
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
    const int cap = nfiles < 64 ? 64 : nfiles;
    HIPCK(hipMalloc(&c->d_files, sizeof(DevFile) * cap));
    HIPCK(hipMalloc(&c->d_prefix, sizeof(uint32_t) * (cap + 1)));
    HIPCK(hipMalloc(&c->d_fout, sizeof(FileOut) * cap));
    HIPCK(hipHostMalloc(&c->h_files, sizeof(DevFile) * cap, hipHostMallocDefault));
    HIPCK(hipHostMalloc(&c->h_prefix, sizeof(uint32_t) * (cap + 1), hipHostMallocDefault));
    HIPCK(hipHostMalloc(&c->h_fout, sizeof(FileOut) * cap, hipHostMallocDefault));
    c->cap_files = cap;
    return CLY_OK;
}

static int ensure_units(cly_ctx* c, int64_t nunits) {
    if (nunits <= c->cap_units) return CLY_OK;
    hipFree(c->d_desc); hipFree(c->d_sums);
    const int64_t cap = nunits < 1024 ? 1024 : nunits;
    HIPCK(hipMalloc(&c->d_desc, sizeof(Desc) * cap));
    c->desc_fresh = 1;
    HIPCK(hipMalloc(&c->d_sums, sizeof(ChunkSum) * cap * CLY_NDW));
    hipFree(c->d_dbg);
    HIPCK(hipMalloc(&c->d_dbg, sizeof(SubDbg) * cap * CLY_NDW));
    hipFree(c->d_unitP);
    HIPCK(hipMalloc(&c->d_unitP, sizeof(uint64_t) * cap));
    c->cap_units = cap;
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
    int64_t nunits = 0;
    uint64_t bytes = 0, nsub_total = 0;
    for (int i = 0; i < nfiles; i++) {
        if (files[i].len >= (1ULL << 32)) return CLY_ERR_ARG;
        if (files[i].len && (((uintptr_t)files[i].base) & 15)) return CLY_ERR_ARG;
        const uint64_t nu = files[i].len ? (files[i].len + CLY_UNIT - 1) / CLY_UNIT : 1;
        const uint64_t ns = files[i].len ? (files[i].len + CLY_TS - 1) / CLY_TS : 1;
        c->h_files[i].base = files[i].base;
        c->h_files[i].len = files[i].len;
        c->h_files[i].fid = files[i].fid;
        c->h_files[i].first_unit = (uint32_t)nunits;
        c->h_files[i].nsub = (uint32_t)ns;
        c->h_files[i]._pad = 0;
        c->h_prefix[i] = (uint32_t)nunits;
        nunits += (int64_t)nu;
        nsub_total += ns;
        bytes += files[i].len;
    }
    if (nunits >= (1LL << 31) / CLY_NDW) return CLY_ERR_ARG;
    c->h_prefix[nfiles] = (uint32_t)nunits;
    rc = ensure_units(c, nunits);
    if (rc) return rc;
    HIPCK(hipMemcpyAsync(c->d_files, c->h_files, sizeof(DevFile) * nfiles, hipMemcpyHostToDevice, st));
    HIPCK(hipMemcpyAsync(c->d_prefix, c->h_prefix, sizeof(uint32_t) * (nfiles + 1), hipMemcpyHostToDevice, st));
    // descriptor words are tagged with the call epoch: zero them only when the
    // 16-bit epoch wraps (or the buffer is new)
    if (++c->epoch > 0xffff || c->desc_fresh) {
        if (c->epoch > 0xffff) c->epoch = 1;
        c->desc_fresh = 0;
        HIPCK(hipMemsetAsync(c->d_desc, 0, sizeof(Desc) * c->cap_units, st));
    }
    HIPCK(hipMemsetAsync(c->d_g, 0, sizeof(Globals), st));
    HIPCK(hipEventRecord(c->ev[0], st));
    int grid = c->scan_grid;
    if ((int64_t)grid > nunits) grid = (int)nunits;
    hipLaunchKernelGGL(k_scan, dim3(grid), dim3(64 * WAVES_PER_WG), CLY_SCAN_LDS, st, c->d_files, nfiles, c->d_prefix,
                       nunits, c->d_desc, c->d_sums, c->d_unitP, c->d_cols, d_out, out_cap, c->d_g, c->epoch,
                       c->dbg_on ? c->d_dbg : nullptr, c->dbg_on > 1 ? FLAG_FORCE_REDO : 0);
    HIPCK(hipGetLastError());
    HIPCK(hipEventRecord(c->ev[1], st));
    hipLaunchKernelGGL(k_fin, dim3(nfiles), dim3(FIN_NT), 0, st, c->d_files, c->d_sums, c->d_unitP, c->d_x8n, c->d_fout);
    HIPCK(hipGetLastError());
    HIPCK(hipEventRecord(c->ev[2], st));
    HIPCK(hipMemcpyAsync(c->h_g, c->d_g, sizeof(Globals), hipMemcpyDeviceToHost, st));
    HIPCK(hipMemcpyAsync(c->h_fout, c->d_fout, sizeof(FileOut) * nfiles, hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    float ms_scan = 0, ms_fin = 0;
    HIPCK(hipEventElapsedTime(&ms_scan, c->ev[0], c->ev[1]));
    HIPCK(hipEventElapsedTime(&ms_fin, c->ev[1], c->ev[2]));
    if (c->h_g->lb_timeout || c->h_g->fail) {
        fprintf(stderr, "clyscan: internal error (timeout %u, invariant %u)\n", c->h_g->lb_timeout, c->h_g->fail);
        return CLY_ERR_DEVICE;
    }
    uint64_t total = 0;
    for (int i = 0; i < nfiles; i++) {
        if (!c->h_fout[i].ok) { fprintf(stderr, "clyscan: internal error (file %d has no end event)\n", i); return CLY_ERR_DEVICE; }
        file_first[i] = c->h_fout[i].first_index;
        res[i].n_records = c->h_fout[i].n_records;
        res[i].end_offset = c->h_fout[i].end_offset;
        res[i].status = c->h_fout[i].status;
        res[i]._pad = 0;
        total += c->h_fout[i].n_records;
    }
    if (needed) *needed = c->h_g->total;
    if (stats) {
        stats->scan_ms = ms_scan; stats->resolve_ms = ms_fin; stats->total_ms = ms_scan + ms_fin;
        stats->passes = 1 + (c->h_g->redo_units ? 1 : 0);
        stats->n_chunks = (uint32_t)nsub_total; stats->bytes = bytes; stats->records = total;
    }
    if (c->h_g->overflow || c->h_g->total > out_cap) return CLY_ERR_CAPACITY;
    return CLY_OK;
}

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
    cly_file* df = (cly_file*)malloc(sizeof(cly_file) * nfiles);
    uint64_t off = 0;
    for (int i = 0; i < nfiles; i++) {
        df[i] = files[i];
        df[i].base = c->d_bytes + off;
        if (files[i].len)
            HIPCK(hipMemcpyAsync(c->d_bytes + off, files[i].base, files[i].len, hipMemcpyHostToDevice, c->stream));
        off += (files[i].len + 4095) & ~4095ULL;
    }
    const uint64_t cap = cly_scan_capacity(files, nfiles) + 16;
    if (cap > c->cap_tuples) {
        hipFree(c->d_tuples);
        c->cap_tuples = cap;
        HIPCK(hipMalloc(&c->d_tuples, sizeof(cly_tuple) * cap));
    }
    uint64_t slots = 0;
    int rc = cly_scan_device(c, df, nfiles, c->d_tuples, c->cap_tuples, file_first, res, &slots, stats, nullptr);
    free(df);
    uint64_t need = 0;
    for (int i = 0; i < nfiles; i++) need += res[i].n_records;
    if (needed) *needed = rc == CLY_ERR_CAPACITY ? slots : need;
    if (rc != CLY_OK) return rc;
    if (need > out_cap) return CLY_ERR_CAPACITY;
    // per-file copies: the device buffer may hold tuples past an ErrInvalidCRC
    uint64_t o = 0;
    for (int i = 0; i < nfiles; i++) {
        if (res[i].n_records)
            HIPCK(hipMemcpyAsync(out + o, c->d_tuples + file_first[i], sizeof(cly_tuple) * res[i].n_records,
                                 hipMemcpyDeviceToHost, c->stream));
        file_first[i] = o;
        o += res[i].n_records;
    }
    HIPCK(hipStreamSynchronize(c->stream));
    return CLY_OK;
}

// Debug / statistics (not part of include/clyscan.h)
extern "C" int cly_dbg_sums(cly_ctx* c, void* out, int n) {
    HIPCK(hipDeviceSynchronize());
    HIPCK(hipMemcpy(out, c->d_sums, sizeof(ChunkSum) * n, hipMemcpyDeviceToHost));
    return n;
}
extern "C" int cly_dbg_sumsize(void) { return (int)sizeof(ChunkSum); }
extern "C" int cly_dbg_enable(cly_ctx* c, int on) { c->dbg_on = on; return 0; }
extern "C" int cly_dbg_unitp(cly_ctx* c, uint64_t* out, int n) {
    HIPCK(hipDeviceSynchronize());
    HIPCK(hipMemcpy(out, c->d_unitP, sizeof(uint64_t) * n, hipMemcpyDeviceToHost));
    return n;
}
extern "C" int cly_dbg_subs(cly_ctx* c, void* out, int n) {
    HIPCK(hipDeviceSynchronize());
    HIPCK(hipMemcpy(out, c->d_dbg, sizeof(SubDbg) * n, hipMemcpyDeviceToHost));
    return n;
}
extern "C" int cly_dbg_prof(cly_ctx* c, uint64_t* out24) {
    for (int i = 0; i < 24; i++) out24[i] = c->h_g->prof[i];
    return 24;
}
extern "C" int cly_dbg_stats(cly_ctx* c, uint32_t* out4) {
    out4[0] = c->h_g->redo_units; out4[1] = c->h_g->redo_subs; out4[2] = c->scan_grid; out4[3] = CLY_SCAN_LDS;
    return 4;
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

extern "C" const char* cly_build_info(void) {
    static char buf[200];
    snprintf(buf, sizeof(buf), "clyscan gfx950 SUB=%d NDW=%d TS=%d UNIT=%d LDS=%d tables=16x", CLY_SUB, CLY_NDW, CLY_TS,
             (int)CLY_UNIT, (int)CLY_SCAN_LDS);
    return buf;
}
