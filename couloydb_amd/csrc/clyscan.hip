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
//   k_scan  one 256-lane workgroup per 32 KiB chunk, chunks taken in ticket
//           order; the per-chunk algorithm is scan_core.h (chain speculation,
//           resolution, decoupled look-back, CRC, tuple emission).
//   k_fin   one workgroup per file: CRC of records that straddle chunks, and the
//           file's first event (ErrInvalidCRC / io.EOF variants / panics).
// Design and data layout: DESIGN.md.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "scan_core.h"

#define CLY_SCAN_LEVELS_ cly_log2_(CLY_NT)
constexpr int cly_log2_(int v) { return v <= 1 ? 0 : 1 + cly_log2_(v >> 1); }

struct DevFile {                 // 32 B
    const uint8_t* base;         // device pointer to the file's first byte (16-B aligned)
    uint64_t len;
    uint32_t fid;
    uint32_t first_chunk;        // global index of the file's first chunk
    uint32_t nchunks;
    uint32_t _pad;
};

struct Globals {                 // zeroed per call
    uint32_t ticket;
    uint32_t overflow;           // tuples beyond out_cap were dropped
    uint32_t lb_timeout;         // a look-back spin hit its bound (never expected)
    uint32_t fail;               // a chunk violated an internal invariant (never expected)
    uint64_t total;              // tuple slots used (records + any past an ErrInvalidCRC)
    uint64_t phase[10];          // profiling build: summed clock cycles per chunk phase
    uint64_t lbstat[8];          // profiling build: look-back windows, spins, slow steps, fallbacks, distance
    uint32_t nfb, _pad2;
    int64_t  fb[32][6];          // profiling build: first fallbacks (c, jf, req, e0, X, state)
};

struct FileOut {
    uint64_t n_records;
    int64_t  end_offset;
    int32_t  status;
    int32_t  ok;
    uint64_t first_index;
};

// ---------------------------------------------------------------------------
// Executor: one chunk per wave, one stripe per lane.  A phase ends with a
// wave-local LDS ordering point (no workgroup barrier: the waves of a
// workgroup work on independent chunks); collectives are wave reductions.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct DevExec {
    int lane;
    template <class F> __device__ __forceinline__ void all(F f) { f(lane); wave_sync(); }
    template <class F> __device__ __forceinline__ void one(F f) { if (lane == 0) f(); wave_sync(); }
    // phase whose lanes each return a predicate; true iff it holds for all lanes
    template <class F> __device__ __forceinline__ bool all_and(F f) {
        const int v = f(lane);
        wave_sync();
        return __ballot(v != 0) == ~0ull;
    }
    template <class F> __device__ __forceinline__ int reduce_min(F f) {
        int v = f(lane);
        #pragma unroll
        for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
        return v;
    }
    template <class F> __device__ __forceinline__ void scan_max_incl(F f, int16_t* out) {
        int v = f(lane);
        #pragma unroll
        for (int o = 1; o < 64; o <<= 1) { const int u = __shfl_up(v, o, 64); if (lane >= o) v = max(v, u); }
        out[lane] = (int16_t)v;
        wave_sync();
    }
    template <class F> __device__ __forceinline__ int scan_add_excl(F f, int16_t* out) {
        const int x = f(lane);
        int v = x;
        #pragma unroll
        for (int o = 1; o < 64; o <<= 1) { const int u = __shfl_up(v, o, 64); if (lane >= o) v += u; }
        out[lane] = (int16_t)(v - x);
        wave_sync();
        return __shfl(v, 63, 64);
    }
};

// ---------------------------------------------------------------------------
// Global-memory side of a chunk.
__device__ __forceinline__ uint64_t ld_agent(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(unsigned long long* p, uint64_t v) {
    __hip_atomic_store(p, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

#define LB_SPIN_MAX (1u << 24)

struct DevEnv {
    DevFile F;
    Desc* desc;
    ChunkSum* sums;
    const uint32_t* shift;
    const uint32_t* x8n;
    cly_tuple* out;
    uint64_t out_cap;
    Globals* g;
    ChunkDbg* dbg;
    int* trace;                  // debug: host-mapped progress marks (survive a hang)
    int nchunks;
    uint32_t epoch;              // call epoch tagging every descriptor word
    uint32_t spins;

    __device__ __forceinline__ void mark(CLY_LDS ScanShared& S, int v) {
#ifdef CLY_PHASE_PROF
        S.tstamp[v] = __builtin_amdgcn_s_memtime();
        if (v == 8)
            for (int k = 1; k <= 8; k++) S.pacc[k] += S.tstamp[k] - S.tstamp[k - 1];
#endif
        if (trace) { trace[2 * (S.C.chunk & 1023)] = v; trace[2 * (S.C.chunk & 1023) + 1] = S.C.chunk; __threadfence_system(); }
    }
    __device__ __forceinline__ void report_fail(CLY_LDS ScanShared& S) { atomicMax(&g->fail, (uint32_t)S.fail); }
    int* lanes;                  // debug: per-lane trace of the first chunks
    __device__ __forceinline__ void dbg_lane(CLY_LDS ScanShared& S, int t) {
        if (lanes && S.C.chunk < 4) dbg_lane_fill(S, t, lanes + (S.C.chunk * CLY_NT + t) * 8);
    }

    __device__ __forceinline__ ChunkDbg* dbg_slot(int c) { return dbg ? dbg + c : nullptr; }
    // Chunk bytes (+halo) into LDS.  Whole windows go by LDS-DMA
    // (global_load_lds_dwordx4: 1 KiB per wave instruction, all in flight at
    // once, no register staging); the last chunk of a file (window cut by the
    // file end) is staged through registers with a zero-filled tail.
    __device__ __forceinline__ void stage_lane(CLY_LDS ScanShared& S, int t) {
        const int wl = S.C.win_len;
        if (wl == CLY_WIN) {
            const int lane = t;
            const uint8_t* src = F.base + S.C.cbase;
            #pragma unroll
            for (int k = 0; k < (CLY_WIN / 16 + CLY_NT - 1) / CLY_NT; k++) {
                const int slot0 = k * CLY_NT;
                if (slot0 + lane < CLY_WIN / 16)
                    __builtin_amdgcn_global_load_lds((const void*)(src + (size_t)(slot0 + lane) * 16),
                                                     (CLY_LDS void*)((CLY_LDS char*)S.win + slot0 * 16),
                                                     16, 0, 0);
            }
            return;
        }
        CLY_LDS uint4* w4 = (CLY_LDS uint4*)(S.win);
        const int nvec = wl >> 4;
        const uint4* src = reinterpret_cast<const uint4*>(F.base + S.C.cbase);
        uint4 v[(CLY_WIN / 16 + CLY_NT - 1) / CLY_NT];
        #pragma unroll
        for (int k = 0; k < (CLY_WIN / 16 + CLY_NT - 1) / CLY_NT; k++) {
            const int i = t + k * CLY_NT;
            v[k] = i < nvec ? src[i] : make_uint4(0, 0, 0, 0);
        }
        #pragma unroll
        for (int k = 0; k < (CLY_WIN / 16 + CLY_NT - 1) / CLY_NT; k++) {
            const int i = t + k * CLY_NT;
            if (i < CLY_WIN / 16) w4[i] = v[k];
        }
        if (t == 0 && (wl & 15)) {
            uint32_t wv4[4] = {0, 0, 0, 0};
            const uint8_t* b = F.base + S.C.cbase + (nvec << 4);
            for (int k = 0; k < (wl & 15); k++) wv4[k >> 2] |= (uint32_t)b[k] << (8 * (k & 3));
            w4[nvec] = make_uint4(wv4[0], wv4[1], wv4[2], wv4[3]);
        }
    }
    __device__ __forceinline__ void stage_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
    __device__ __forceinline__ void publish_spec(int c, uint64_t w0, uint64_t w1) {
        st_agent(&desc[c].w[1], w1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        st_agent(&desc[c].w[0], w0);
    }
    __device__ __forceinline__ void publish_full(int c, uint64_t w0, uint64_t w2, uint64_t w3, uint64_t total) {
        st_agent(&desc[c].w[2], w2);
        st_agent(&desc[c].w[3], w3);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        st_agent(&desc[c].w[0], w0);
        if (c == nchunks - 1) g->total = total;
    }
    // look-back primitives (lookback_seq in scan_core.h)
    __device__ __forceinline__ uint64_t ld(int64_t j, int k) { return ld_agent(&desc[j].w[k]); }
    __device__ __forceinline__ bool spin() {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > LB_SPIN_MAX) { atomicOr(&g->lb_timeout, 1u); return false; }
        return true;
    }
    __device__ __forceinline__ bool spin_ok() const { return spins <= LB_SPIN_MAX; }
    // Decoupled look-back by wave 0: 64 descriptors per round trip into LDS,
    // then every lane folds them in order (uniform; scan_core.h lb_walk_step).
    __device__ void lookback(CLY_LDS ScanShared& S, int t) {
        if (t >= 64) return;
        const int64_t c = S.C.chunk;
        LbWalk w;
        lb_walk_init(w, c, S.C.fof);
        LbState out;
        out.E = 0; out.P = 0; out.dead = 1; out._pad = 0;
        int64_t jf = -1;
        int r = 0;
        bool ok = true;
#ifdef CLY_PHASE_PROF
        uint32_t st_win = 0, st_spin = 0, st_slow = 0;
#define LBSTAT(v) v
#else
#define LBSTAT(v)
#endif
        for (int64_t base = c - 1; r == 0 && ok; base -= 64) {
            LBSTAT(st_win++);
            if (base < 0) {
                r = lb_apply_full_walk(w, 0, 0, 0, out) ? 1 : 2;
                jf = -1;
                break;
            }
            const int64_t j = base - t;
            uint64_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
            int stop;
            for (;;) {
                bool ready = true, full = false;
                if (j >= 0) {
                    // all four words in one round trip (w0 last: words written
                    // before it are complete when it shows their state)
                    w1 = ld(j, 1); w2 = ld(j, 2); w3 = ld(j, 3);
                    w0 = ld(j, 0);
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
                LBSTAT(st_spin++);
                if (t == 0) go = spin() ? 1 : 0;
                if (!__shfl(go, 0, 64)) { ok = false; break; }
            }
            if (!ok) break;
            // fast path: a run of "tight" speculative descriptors from lane 0
            // (guess valid, not first-of-file, not terminal, exit == the guessed
            // entry of the chunk after it) folds at once: requirement == the
            // last one's guess, counts summed by a wave reduction.
            int i0 = 0;
            {
                const int64_t jn = j + 1;                          // chunk after lane t's chunk
                const uint64_t w0n = __shfl_up(w0, 1, 64);          // its state word (lane t-1)
                const bool spec = j >= 0 && ds_state(w0, epoch) == DS_SPEC && ds_gvalid(w0) && !ds_fof(w0) &&
                                  !ds_term(w0);
                const int64_t xj = (int64_t)(w1 & DS_VAL_MASK);
                bool tight;
                if (t == 0) tight = spec && lb_req_ok(w, xj);
                else tight = spec && ds_gvalid(w0n) && !ds_fof(w0n) && xj == jn * (int64_t)CLY_CHUNK + ds_grel(w0n);
                const unsigned long long tm = __ballot(tight && t < stop);
                const int run = (~tm) ? __ffsll((long long)~tm) - 1 : 64;    // tight lanes 0..run-1
                if (run > 0) {
                    uint32_t cnt = (t < run) ? ds_cnt(w0) : 0u;
                    #pragma unroll
                    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
                    const uint64_t w0l = __shfl(w0, run - 1, 64);
                    const uint64_t x0 = __shfl(w1, 0, 64);
                    // summary just before folding the run's last chunk (recovery)
                    if (run >= 2) {
                        const uint64_t w0p = __shfl(w0, run - 2, 64);
                        w.prev = static_cast<const LbSum&>(w);
                        if (w.prev.res == LB_RES_IDENT) { w.prev.res = LB_RES_CONST; w.prev.rx = (int64_t)(x0 & DS_VAL_MASK); }
                        w.prev.dp += cnt - ds_cnt(w0l);
                        w.prev.req = LB_REQ_EXACT;
                        w.prev.e0 = (base - (run - 2)) * (int64_t)CLY_CHUNK + ds_grel(w0p);
                    } else {
                        w.prev = static_cast<const LbSum&>(w);
                    }
                    w.kreq = base - (run - 1);
                    if (w.res == LB_RES_IDENT) { w.res = LB_RES_CONST; w.rx = (int64_t)(x0 & DS_VAL_MASK); }
                    w.dp += cnt;
                    w.req = LB_REQ_EXACT;
                    w.e0 = (base - (run - 1)) * (int64_t)CLY_CHUNK + ds_grel(w0l);
                    i0 = run;
                }
            }
            const int last = stop < 64 ? stop : 63;
            LBSTAT(st_slow += (last + 1 - i0));
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
        if (t != 0) return;
#ifdef CLY_PHASE_PROF
        S.lacc[0] += st_win; S.lacc[1] += st_spin; S.lacc[2] += st_slow;
        if (ok && r == 2) S.lacc[3] += 1;
#endif
#ifdef CLY_PHASE_PROF
        if (ok && r == 2) {
            const uint32_t k = atomicAdd(&g->nfb, 1u);
            if (k < 32) {
                g->fb[k][0] = c; g->fb[k][1] = jf; g->fb[k][2] = w.req; g->fb[k][3] = w.e0;
                g->fb[k][4] = jf >= 0 ? (int64_t)(ld(jf, 2) & DS_VAL_MASK) : -1;
                g->fb[k][5] = jf >= 0 ? (int64_t)ld(jf, 0) : -1;
            }
        }
#endif
        if (ok && r == 2 && lb_recover_kreq(*this, w, epoch, out)) r = 1;
        if (ok && r == 2) {
            if (jf == -3) {
                // nearest FULL before the chunk where the walk failed
                jf = -1;
                for (int64_t k = S.C.chunk - 1; k >= 0; k--) {
                    uint64_t a0 = ld(k, 0);
                    while (ds_state(a0, epoch) == 0 && spin()) a0 = ld(k, 0);
                    if (ds_state(a0, epoch) == DS_FULL) { jf = k; break; }
                }
            }
            lb_forward(*this, c, S.C.fof, jf, epoch, out);
        }
        S.entry_g = out.E;
        S.p_excl = out.P;
        S.in_dead = out.dead;
    }
    template <class EX> __device__ __forceinline__ void crc(EX& ex, CLY_LDS ScanShared& S) { crc_phase(ex, S, shift); }
    __device__ __forceinline__ void emit_lane(CLY_LDS ScanShared& S, int t) {
        unsigned of = 0;
        ::emit_lane(S, t, out, out_cap, &of);
        if (of) atomicOr(&g->overflow, 1u);
    }
    __device__ __forceinline__ void summary(CLY_LDS ScanShared& S) { write_summary(S, sums, x8n); }
};

#ifndef CLY_WPB
#define CLY_WPB 4                // waves (= chunks in flight) per workgroup
#endif
#define CLY_SCAN_LDS (CLY_TAB_WORDS * 4 + CLY_WPB * sizeof(ScanShared))

// Persistent: every wave takes chunk tickets until none are left (tickets in
// order, so a chunk only waits on chunks already taken by running waves).
__global__ void __launch_bounds__(64 * CLY_WPB)
k_scan(const DevFile* __restrict__ files, int nfiles, const uint32_t* __restrict__ file_chunk_prefix, int nchunks,
       Desc* desc, ChunkSum* sums, const uint32_t* __restrict__ shift, const uint32_t* __restrict__ x8n,
       cly_tuple* out, uint64_t out_cap, Globals* g, ChunkDbg* dbg, int* trace, uint32_t epoch) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    CLY_LDS uint32_t* tab = (CLY_LDS uint32_t*)(smem_raw);
    for (int i = threadIdx.x; i < 256; i += blockDim.x) build_tab_lane(tab, i, 256);
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    CLY_LDS ScanShared& S = ((CLY_LDS ScanShared*)(smem_raw + CLY_TAB_WORDS * 4))[wave];
    DevExec ex{lane};
    DevEnv env;
    env.desc = desc; env.sums = sums; env.shift = shift; env.x8n = x8n;
    env.out = out; env.out_cap = out_cap; env.g = g; env.nchunks = nchunks; env.dbg = dbg; env.trace = trace;
    env.epoch = epoch;
    env.lanes = trace ? trace + 2048 : nullptr;
#ifdef CLY_PHASE_PROF
    if (lane == 0) { for (int k = 0; k < 10; k++) S.pacc[k] = 0; for (int k = 0; k < 4; k++) S.lacc[k] = 0; }
#endif
    for (;;) {
        int c = 0;
        if (lane == 0) c = (int)atomicAdd(&g->ticket, 1u);
        c = __shfl(c, 0, 64);
        if (c >= nchunks) break;
        int lo = 0, hi = nfiles - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if ((int)file_chunk_prefix[mid] <= c) lo = mid; else hi = mid - 1;
        }
        env.F = files[lo];
        env.spins = 0;
        if (lane == 0) {
#ifdef CLY_PHASE_PROF
            S.tstamp[0] = __builtin_amdgcn_s_memtime();
#endif
            const int cl = c - (int)env.F.first_chunk;
            S.C.chunk = c;
            S.C.fidx = lo;
            S.C.cbase = (int64_t)cl * CLY_CHUNK;
            S.C.nrel = (int64_t)env.F.len - S.C.cbase;
            S.C.dlen = (int)(S.C.nrel < CLY_CHUNK ? S.C.nrel : CLY_CHUNK);
            S.C.win_len = (int)(S.C.nrel < CLY_WIN ? S.C.nrel : CLY_WIN);
            S.C.fof = cl == 0;
            S.C.lof = cl == (int)env.F.nchunks - 1;
            S.C.fid = env.F.fid;
            S.C.gfile = env.F.base;
            S.tab = tab;
        }
        wave_sync();
        chunk_body(ex, S, env);
    }
#ifdef CLY_PHASE_PROF
    if (lane == 0) {
        for (int k = 0; k < 10; k++) atomicAdd((unsigned long long*)&g->phase[k], (unsigned long long)S.pacc[k]);
        for (int k = 0; k < 4; k++) atomicAdd((unsigned long long*)&g->lbstat[k], (unsigned long long)S.lacc[k]);
    }
#endif
}

// One workgroup per file: first event of the file.
#define FIN_NT 256
__global__ void __launch_bounds__(FIN_NT)
k_fin(const DevFile* __restrict__ files, const ChunkSum* __restrict__ sums, FileOut* __restrict__ fout) {
    const int f = blockIdx.x, tid = threadIdx.x;
    const DevFile F = files[f];
    const int c0 = (int)F.first_chunk, nc = (int)F.nchunks;
    __shared__ int64_t r_off[FIN_NT];
    __shared__ uint64_t r_g[FIN_NT];
    __shared__ int32_t r_st[FIN_NT];
    int64_t best = EVT_NONE;
    uint64_t bg = 0;
    int32_t bs = 0;
    for (int i = tid; i < nc; i += FIN_NT) {
        uint64_t gi = 0;
        int32_t st = 0;
        const int64_t o = fin_chunk_event(sums, c0, nc, i, &gi, &st);
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
        const uint64_t first = sums[c0].p_excl;
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
    Desc* d_desc; ChunkSum* d_sums; int cap_chunks;
    Globals* d_g;
    uint32_t* d_shift;
    uint32_t* d_x8n;
    DevFile* h_files;
    uint32_t* h_prefix;
    FileOut* h_fout;
    Globals* h_g;
    ChunkDbg* d_dbg; int dbg_on; int last_nchunks;  // debug trace (cly_dbg_chunks)
    int* h_trace; int* d_trace;
    uint32_t epoch; int desc_fresh;
    int scan_grid;
    uint8_t* d_bytes; uint64_t cap_bytes;          // host-path staging
    cly_tuple* d_tuples; uint64_t cap_tuples;
};

static void build_shift_tables(uint32_t* h) {
    for (int lvl = 0; lvl < CLY_SCAN_LEVELS_; lvl++) {
        const uint32_t xm = cly_x8n((uint64_t)CLY_SUB << lvl);
        for (int bpos = 0; bpos < 4; bpos++)
            for (uint32_t i = 0; i < 256; i++) h[lvl * 1024 + bpos * 256 + i] = cly_multmodp(xm, i << (8 * bpos));
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
    const size_t shift_bytes = sizeof(uint32_t) * 1024 * (CLY_SCAN_LEVELS_ ? CLY_SCAN_LEVELS_ : 1);
    HIPCK(hipMalloc(&c->d_shift, shift_bytes));
    uint32_t* hs = (uint32_t*)calloc(1, shift_bytes);
    build_shift_tables(hs);
    HIPCK(hipMemcpy(c->d_shift, hs, shift_bytes, hipMemcpyHostToDevice));
    free(hs);
    const size_t x8_bytes = sizeof(uint32_t) * (CLY_CHUNK + 1);
    HIPCK(hipMalloc(&c->d_x8n, x8_bytes));
    uint32_t* hx = (uint32_t*)malloc(x8_bytes);
    hx[0] = 1u << 31;
    const uint32_t x8 = cly_x8n(1);
    for (int n = 1; n <= CLY_CHUNK; n++) hx[n] = cly_multmodp(x8, hx[n - 1]);
    HIPCK(hipMemcpy(c->d_x8n, hx, x8_bytes, hipMemcpyHostToDevice));
    free(hx);
    HIPCK(hipFuncSetAttribute((const void*)k_scan, hipFuncAttributeMaxDynamicSharedMemorySize, (int)CLY_SCAN_LDS));
    // persistent grid: resident workgroups per CU x CUs
    {
        int per_cu = 0, ncu = 0;
        HIPCK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_scan, 64 * CLY_WPB, CLY_SCAN_LDS));
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
    hipFree(c->d_g); hipFree(c->d_shift); hipFree(c->d_x8n); hipFree(c->d_bytes); hipFree(c->d_tuples);
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

static int ensure_chunks(cly_ctx* c, int nchunks) {
    if (nchunks <= c->cap_chunks) return CLY_OK;
    hipFree(c->d_desc); hipFree(c->d_sums); hipFree(c->d_dbg); c->d_dbg = nullptr;
    const int cap = nchunks < 1024 ? 1024 : nchunks;
    HIPCK(hipMalloc(&c->d_desc, sizeof(Desc) * cap));
    c->desc_fresh = 1;
    HIPCK(hipMalloc(&c->d_sums, sizeof(ChunkSum) * cap));
    if (c->dbg_on) HIPCK(hipMalloc(&c->d_dbg, sizeof(ChunkDbg) * cap));
    c->cap_chunks = cap;
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
    uint64_t nchunks64 = 0, bytes = 0;
    for (int i = 0; i < nfiles; i++) {
        if (files[i].len >= (1ULL << 32)) return CLY_ERR_ARG;
        if (files[i].len && (((uintptr_t)files[i].base) & 15)) return CLY_ERR_ARG;
        const uint32_t nch = files[i].len ? (uint32_t)((files[i].len + CLY_CHUNK - 1) / CLY_CHUNK) : 1;
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
    if (c->dbg_on && !c->d_dbg) c->cap_chunks = 0;
    rc = ensure_chunks(c, nchunks);
    if (rc) return rc;
    c->last_nchunks = nchunks;
    HIPCK(hipMemcpyAsync(c->d_files, c->h_files, sizeof(DevFile) * nfiles, hipMemcpyHostToDevice, st));
    HIPCK(hipMemcpyAsync(c->d_prefix, c->h_prefix, sizeof(uint32_t) * (nfiles + 1), hipMemcpyHostToDevice, st));
    // descriptor words are tagged with the call epoch: zero them only when the
    // 16-bit epoch wraps (or the buffer is new)
    if (++c->epoch > 0xffff || c->desc_fresh) {
        if (c->epoch > 0xffff) c->epoch = 1;
        c->desc_fresh = 0;
        HIPCK(hipMemsetAsync(c->d_desc, 0, sizeof(Desc) * c->cap_chunks, st));
    }
    HIPCK(hipMemsetAsync(c->d_g, 0, sizeof(Globals), st));
    HIPCK(hipEventRecord(c->ev[0], st));
    hipLaunchKernelGGL(k_scan, dim3(c->scan_grid), dim3(64 * CLY_WPB), CLY_SCAN_LDS, st, c->d_files, nfiles, c->d_prefix,
                       nchunks, c->d_desc, c->d_sums, c->d_shift, c->d_x8n, d_out, out_cap, c->d_g,
                       c->dbg_on ? c->d_dbg : nullptr, c->dbg_on > 1 ? c->d_trace : nullptr, c->epoch);
    HIPCK(hipGetLastError());
    HIPCK(hipEventRecord(c->ev[1], st));
    hipLaunchKernelGGL(k_fin, dim3(nfiles), dim3(FIN_NT), 0, st, c->d_files, c->d_sums, c->d_fout);
    HIPCK(hipGetLastError());
    HIPCK(hipEventRecord(c->ev[2], st));
    HIPCK(hipMemcpyAsync(c->h_g, c->d_g, sizeof(Globals), hipMemcpyDeviceToHost, st));
    HIPCK(hipMemcpyAsync(c->h_fout, c->d_fout, sizeof(FileOut) * nfiles, hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    float ms_scan = 0, ms_fin = 0;
    HIPCK(hipEventElapsedTime(&ms_scan, c->ev[0], c->ev[1]));
    HIPCK(hipEventElapsedTime(&ms_fin, c->ev[1], c->ev[2]));
    if (c->h_g->lb_timeout || c->h_g->fail) {
        fprintf(stderr, "clyscan: internal error (lookback timeout %u, invariant %u)\n", c->h_g->lb_timeout,
                c->h_g->fail);
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
        stats->passes = 1; stats->n_chunks = (uint32_t)nchunks; stats->bytes = bytes; stats->records = total;
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

// Debug (not part of include/clyscan.h): enable the per-chunk trace, and copy
// the trace + chunk summaries of the last call to host memory.
extern "C" int cly_dbg_enable(cly_ctx* c, int on) {
    c->dbg_on = on; c->cap_chunks = 0;
    if (on > 1 && !c->h_trace) {
        HIPCK(hipHostMalloc(&c->h_trace, (2048 + 4 * CLY_NT * 8) * sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
        memset(c->h_trace, 0, (2048 + 4 * CLY_NT * 8) * sizeof(int));
        HIPCK(hipHostGetDevicePointer((void**)&c->d_trace, c->h_trace, 0));
    }
    return 0;
}
// progress marks of the last call (valid even after a device hang/fault)
extern "C" int cly_dbg_trace(cly_ctx* c, int* out, int n) {
    if (!c->h_trace) return 0;
    const int lim = 2048 + 4 * CLY_NT * 8;
    memcpy(out, c->h_trace, sizeof(int) * (n < lim ? n : lim));
    return n;
}
extern "C" int cly_dbg_fout(cly_ctx* c, void* out, int n) {
    memcpy(out, c->h_fout, sizeof(FileOut) * n);
    return n;
}
extern "C" int cly_dbg_chunks(cly_ctx* c, void* dbg_out, void* sums_out, int max) {
    const int n = c->last_nchunks < max ? c->last_nchunks : max;
    HIPCK(hipDeviceSynchronize());
    if (dbg_out && c->d_dbg) HIPCK(hipMemcpy(dbg_out, c->d_dbg, sizeof(ChunkDbg) * n, hipMemcpyDeviceToHost));
    if (sums_out) HIPCK(hipMemcpy(sums_out, c->d_sums, sizeof(ChunkSum) * n, hipMemcpyDeviceToHost));
    return n;
}
// profiling build: summed cycles per phase of the last call (10 counters)
extern "C" int cly_dbg_phases(cly_ctx* c, uint64_t* out) {
    for (int k = 0; k < 10; k++) out[k] = c->h_g->phase[k];
    for (int k = 0; k < 8; k++) out[10 + k] = c->h_g->lbstat[k];
    out[18] = c->h_g->nfb;
    for (int k = 0; k < 32; k++) for (int m = 0; m < 6; m++) out[19 + k * 6 + m] = (uint64_t)c->h_g->fb[k][m];
    return 19 + 32 * 6;
}
extern "C" int cly_dbg_sizes(int* out3) { out3[0] = sizeof(ChunkDbg); out3[1] = sizeof(ChunkSum); out3[2] = sizeof(ScanShared); return 0; }
extern "C" int cly_dbg_grid(cly_ctx* c) { return c->scan_grid; }

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
    static char buf[160];
    snprintf(buf, sizeof(buf), "clyscan gfx950 NT=%d SUB=%d CHUNK=%d REP=%d WPB=%d LDS=%d", CLY_NT, CLY_SUB, CLY_CHUNK,
             CLY_REP, CLY_WPB, (int)CLY_SCAN_LDS);
    return buf;
}
