// clyscan_emu.cpp — TEST INFRASTRUCTURE ONLY.
//
// A CPU emulator of the gfx950 scan pipeline: it runs the SAME per-chunk code
// (couloydb_amd/csrc/scan_core.h: speculation, chain resolution, decoupled
// look-back, CRC phases, tuple emission, k_fin's straddle checks) with one CPU
// thread per in-flight "workgroup" and a loop over the 256 lanes in place of
// the lanes themselves.  It exports the host entry points of include/clyscan.h
// so the CPU test suite can check the kernel logic against the oracle without
// a GPU.  It is never loaded by the product path (couloydb_amd.Scanner loads
// libclyscan.so, which has no CPU fallback).
//
// Scheduling stress: CLY_EMU_THREADS workers (default 8) pull chunk tickets in
// order like the GPU's dynamic ticket; CLY_EMU_JITTER=1 adds random sleeps so
// chunks see predecessors that have published only their speculative
// descriptor, exercising every look-back path.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <random>
#include <thread>
#include <vector>

#include "../../couloydb_amd/csrc/scan_core.h"

struct HostExec {
    template <class F> void all(F f) { for (int t = 0; t < CLY_NT; t++) f(t); }
    template <class F> void one(F f) { f(); }
    template <class F> bool all_and(F f) {
        bool r = true;
        for (int t = 0; t < CLY_NT; t++) r = (f(t) != 0) && r;
        return r;
    }
    template <class F> int reduce_min(F f) {
        int r = 0x7fffffff;
        for (int t = 0; t < CLY_NT; t++) { int v = f(t); if (v < r) r = v; }
        return r;
    }
    template <class F> void scan_max_incl(F f, int16_t* out) {
        int m = -1;
        for (int t = 0; t < CLY_NT; t++) { int v = f(t); if (v > m) m = v; out[t] = (int16_t)m; }
    }
    template <class F> int scan_add_excl(F f, int16_t* out) {
        int s = 0;
        for (int t = 0; t < CLY_NT; t++) { out[t] = (int16_t)s; s += f(t); }
        return s;
    }
};

struct FileRec {
    const uint8_t* base;
    uint64_t len;
    uint32_t fid;
    uint32_t first_chunk, nchunks;
};

struct EmuRun {
    std::vector<FileRec> files;
    std::vector<uint32_t> prefix;         // first chunk per file (+ total)
    std::vector<Desc> desc;
    std::vector<ChunkSum> sums;
    std::vector<uint32_t> shift;          // segmented-scan shift tables
    std::vector<uint32_t> x8n;
    std::vector<ChunkDbg> dbg;
    std::vector<int> lanes;
    cly_tuple* out;
    uint64_t out_cap;
    std::atomic<unsigned> overflow{0};
    std::atomic<unsigned> fail{0};
    std::atomic<unsigned> fallbacks{0};
    std::atomic<unsigned> recoveries{0};
    std::atomic<uint64_t> total{0};
    int nchunks;
    int jitter;
    int delay_full;
    uint32_t epoch;
};

static void jitter_sleep(int jitter, std::mt19937& rng) {
    if (!jitter) return;
    unsigned r = rng() % 8;
    if (r == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 300));
    else if (r == 1) std::this_thread::yield();
}

struct HostEnv {
    EmuRun* run;
    const FileRec* F;
    std::mt19937* rng;

    void mark(ScanShared&, int) {}
    void stage_wait() {}
    void note_fallback(int64_t c, int64_t jf) {
        run->fallbacks.fetch_add(1);
        if (getenv("CLY_EMU_VERBOSE")) fprintf(stderr, "fallback chunk %lld jf %lld\n", (long long)c, (long long)jf);
    }
    // Same windowed walk as the GPU (DevEnv::lookback): 64 descriptors per
    // round, tight-run fast path, then the exact steps; ballots are loops.
    void lookback(ScanShared& S, int t) {
        if (t != 0) return;
        if (getenv("CLY_EMU_SEQ_LB")) {
            LbState ls;
            lookback_seq(*this, S.C.chunk, S.C.fof, epoch, ls);
            S.entry_g = ls.E; S.p_excl = ls.P; S.in_dead = ls.dead;
            return;
        }
        const int64_t c = S.C.chunk;
        LbWalk w;
        lb_walk_init(w, c, S.C.fof);
        LbState out;
        out.E = 0; out.P = 0; out.dead = 1; out._pad = 0;
        int64_t jf = -1;
        int r = 0;
        for (int64_t base = c - 1; r == 0; base -= 64) {
            if (base < 0) { r = lb_apply_full_walk(w, 0, 0, 0, out) ? 1 : 2; jf = -1; break; }
            uint64_t W0[64], W1[64], W2[64], W3[64];
            bool full[64], ready[64];
            int stop;
            for (;;) {
                for (int l = 0; l < 64; l++) {
                    const int64_t j = base - l;
                    W0[l] = W1[l] = W2[l] = W3[l] = 0; ready[l] = true; full[l] = false;
                    if (j >= 0) {
                        W1[l] = ld(j, 1); W2[l] = ld(j, 2); W3[l] = ld(j, 3); W0[l] = ld(j, 0);
                        const uint64_t st = ds_state(W0[l], epoch);
                        if (st == DS_SPEC) ready[l] = ds_ok(W1[l], epoch);
                        else if (st == DS_FULL) { ready[l] = ds_ok(W2[l], epoch) && ds_ok(W3[l], epoch); full[l] = ready[l]; }
                        else ready[l] = false;
                    }
                }
                stop = 64;
                for (int l = 0; l < 64; l++) if (full[l] || base - l < 0) { stop = l; break; }
                bool wait = false;
                for (int l = 0; l <= (stop < 64 ? stop : 63); l++) if (!ready[l]) wait = true;
                if (!wait) break;
                spin();
            }
            int i0 = 0;
            {
                int run = 0;
                for (int l = 0; l < stop; l++) {
                    const int64_t j = base - l;
                    const uint64_t w0 = W0[l];
                    const bool spec = ds_state(w0, epoch) == DS_SPEC && ds_gvalid(w0) && !ds_fof(w0) && !ds_term(w0);
                    const int64_t xj = (int64_t)(W1[l] & DS_VAL_MASK);
                    bool tight;
                    if (l == 0) tight = spec && lb_req_ok(w, xj);
                    else tight = spec && ds_gvalid(W0[l - 1]) && !ds_fof(W0[l - 1]) &&
                                 xj == (j + 1) * (int64_t)CLY_CHUNK + ds_grel(W0[l - 1]);
                    if (!tight) break;
                    run++;
                }
                if (run > 0) {
                    uint32_t cnt = 0;
                    for (int l = 0; l < run; l++) cnt += ds_cnt(W0[l]);
                    const int64_t x0 = (int64_t)(W1[0] & DS_VAL_MASK);
                    w.prev = static_cast<const LbSum&>(w);
                    if (run >= 2) {
                        if (w.prev.res == LB_RES_IDENT) { w.prev.res = LB_RES_CONST; w.prev.rx = x0; }
                        w.prev.dp += cnt - ds_cnt(W0[run - 1]);
                        w.prev.req = LB_REQ_EXACT;
                        w.prev.e0 = (base - (run - 2)) * (int64_t)CLY_CHUNK + ds_grel(W0[run - 2]);
                    }
                    w.kreq = base - (run - 1);
                    if (w.res == LB_RES_IDENT) { w.res = LB_RES_CONST; w.rx = (int64_t)(W1[0] & DS_VAL_MASK); }
                    w.dp += cnt;
                    w.req = LB_REQ_EXACT;
                    w.e0 = (base - (run - 1)) * (int64_t)CLY_CHUNK + ds_grel(W0[run - 1]);
                    i0 = run;
                }
            }
            const int last = stop < 64 ? stop : 63;
            for (int i = i0; i <= last && r == 0; i++) {
                const int64_t ji = base - i;
                if (ji < 0) { r = lb_apply_full_walk(w, 0, 0, 0, out) ? 1 : 2; jf = -1; }
                else r = lb_walk_step(w, ji, W0[i], W1[i], W2[i], W3[i], epoch, out, jf);
            }
        }
        if (r == 2 && lb_recover_kreq(*this, w, epoch, out)) { r = 1; run->recoveries.fetch_add(1); }
        if (r == 2) {
            if (jf == -3) {
                jf = -1;
                for (int64_t k = c - 1; k >= 0; k--) {
                    uint64_t a0 = ld(k, 0);
                    while (ds_state(a0, epoch) == 0) { spin(); a0 = ld(k, 0); }
                    if (ds_state(a0, epoch) == DS_FULL) { jf = k; break; }
                }
            }
            note_fallback(c, jf);
            lb_forward(*this, c, S.C.fof, jf, epoch, out);
        }
        S.entry_g = out.E; S.p_excl = out.P; S.in_dead = out.dead;
    }
    void dbg_lane(ScanShared& S, int t) {
        if (!run->lanes.empty() && S.C.chunk < 4) dbg_lane_fill(S, t, &run->lanes[(S.C.chunk * CLY_NT + t) * 8]);
    }
    void report_fail(ScanShared&) { run->fail.store(1); }
    ChunkDbg* dbg_slot(int c) { return run->dbg.empty() ? nullptr : &run->dbg[c]; }
    void stage_lane(ScanShared& S, int t) {
        // lane t stages 16-B slots t, t+NT, ... of the window, zero past the file end
        uint8_t* w = reinterpret_cast<uint8_t*>(S.win);
        for (int i = t; i < CLY_WIN / 16; i += CLY_NT) {
            for (int k = 0; k < 16; k++) {
                const int64_t o = (int64_t)i * 16 + k;
                w[o] = o < S.C.win_len ? F->base[S.C.cbase + o] : 0;
            }
        }
    }
    uint32_t epoch;
    uint64_t spins = 0;
    uint64_t ld(int64_t j, int k) { return __atomic_load_n(&run->desc[j].w[k], __ATOMIC_ACQUIRE); }
    void st(unsigned long long* p, uint64_t v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }
    bool spin() { std::this_thread::yield(); return ++spins < (1ull << 40); }
    bool spin_ok() const { return true; }
    void publish_spec(int c, uint64_t w0, uint64_t w1) {
        jitter_sleep(run->jitter, *rng);
        st(&run->desc[c].w[1], w1);
        if (run->jitter && ((*rng)() % 4 == 0)) std::this_thread::yield();
        st(&run->desc[c].w[0], w0);
    }
    void publish_full(int c, uint64_t w0, uint64_t w2, uint64_t w3, uint64_t total) {
        jitter_sleep(run->jitter, *rng);
        if (run->delay_full >= 0 && c == run->delay_full)     // test knob: successors see only the SPEC
            std::this_thread::sleep_for(std::chrono::milliseconds(30));
        st(&run->desc[c].w[2], w2);
        st(&run->desc[c].w[3], w3);
        if (run->jitter && ((*rng)() % 4 == 0)) std::this_thread::yield();
        st(&run->desc[c].w[0], w0);
        if (c == run->nchunks - 1) run->total.store(total);
    }
    template <class X> void crc(X& ex, ScanShared& S) { crc_phase(ex, S, run->shift.data()); }
    void emit_lane(ScanShared& S, int t) {
        unsigned of = 0;
        emit_lane_impl(S, t, &of);
        if (of) run->overflow.store(1);
    }
    void emit_lane_impl(ScanShared& S, int t, unsigned* of) { ::emit_lane(S, t, run->out, run->out_cap, of); }
    void summary(ScanShared& S) { write_summary(S, run->sums.data(), run->x8n.data()); }
};

static void run_chunk(EmuRun& R, int c, ScanShared& S, std::mt19937& rng) {
    int lo = 0, hi = (int)R.files.size() - 1;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if ((int)R.prefix[mid] <= c) lo = mid; else hi = mid - 1;
    }
    const FileRec& F = R.files[lo];
    const int cl = c - (int)F.first_chunk;
    S.C.cbase = (int64_t)cl * CLY_CHUNK;
    S.C.nrel = (int64_t)F.len - S.C.cbase;
    S.C.dlen = (int)(S.C.nrel < CLY_CHUNK ? S.C.nrel : CLY_CHUNK);
    S.C.win_len = (int)(S.C.nrel < CLY_WIN ? S.C.nrel : CLY_WIN);
    S.C.chunk = c;
    S.C.fidx = lo;
    S.C.fof = cl == 0;
    S.C.lof = cl == (int)F.nchunks - 1;
    S.C.fid = F.fid;
    S.C.gfile = F.base;
    HostExec ex;
    HostEnv env{&R, &F, &rng, R.epoch};
    chunk_body(ex, S, env);
}

static void build_shift_tables(std::vector<uint32_t>& h) {
    int levels = 0;
    while ((1 << levels) < CLY_NT) levels++;
    h.assign((size_t)1024 * (levels ? levels : 1), 0);
    for (int lvl = 0; lvl < levels; lvl++) {
        const uint32_t xm = cly_x8n((uint64_t)CLY_SUB << lvl);
        for (int bpos = 0; bpos < 4; bpos++)
            for (uint32_t i = 0; i < 256; i++) h[lvl * 1024 + bpos * 256 + i] = cly_multmodp(xm, i << (8 * bpos));
    }
}

struct cly_ctx {
    int dbg_on;
    std::vector<ChunkDbg> dbg;
    std::vector<ChunkSum> sums;
    std::vector<int> lanes;
};

extern "C" int cly_ctx_create(int device, cly_ctx** out) {
    (void)device;
    *out = new cly_ctx();
    (*out)->dbg_on = 0;
    return CLY_OK;
}
extern "C" int cly_dbg_enable(cly_ctx* c, int on) { c->dbg_on = on; return 0; }
extern "C" int cly_dbg_chunks(cly_ctx* c, void* dbg_out, void* sums_out, int max) {
    const int n = (int)c->sums.size() < max ? (int)c->sums.size() : max;
    if (dbg_out && !c->dbg.empty()) memcpy(dbg_out, c->dbg.data(), sizeof(ChunkDbg) * n);
    if (sums_out) memcpy(sums_out, c->sums.data(), sizeof(ChunkSum) * n);
    return n;
}
extern "C" int cly_dbg_trace(cly_ctx* c, int* out, int n) {
    memset(out, 0, sizeof(int) * n);
    for (int i = 0; i < (int)c->lanes.size() && 2048 + i < n; i++) out[2048 + i] = c->lanes[i];
    return n;
}
extern "C" int cly_dbg_sizes(int* out3) { out3[0] = sizeof(ChunkDbg); out3[1] = sizeof(ChunkSum); out3[2] = sizeof(ScanShared); return 0; }
extern "C" void cly_ctx_destroy(cly_ctx* c) { delete c; }
extern "C" uint64_t cly_scan_capacity(const cly_file* files, int nfiles) {
    uint64_t cap = 0;
    for (int i = 0; i < nfiles; i++) cap += files[i].len / 9 + 1;
    return cap;
}

extern "C" int cly_scan(cly_ctx* ctx, const cly_file* files, int nfiles, cly_tuple* out, uint64_t out_cap,
                        uint64_t* file_first, cly_file_result* res, uint64_t* needed, cly_stats* stats) {
    if (!ctx || (!files && nfiles) || nfiles < 0 || !res || !file_first) return CLY_ERR_ARG;
    if (nfiles == 0) { if (needed) *needed = 0; return CLY_OK; }
    EmuRun R;
    uint64_t nch = 0, bytes = 0;
    for (int i = 0; i < nfiles; i++) {
        if (files[i].len >= (1ull << 32)) return CLY_ERR_ARG;
        const uint32_t n = files[i].len ? (uint32_t)((files[i].len + CLY_CHUNK - 1) / CLY_CHUNK) : 1;
        R.files.push_back(FileRec{files[i].base, files[i].len, files[i].fid, (uint32_t)nch, n});
        R.prefix.push_back((uint32_t)nch);
        nch += n;
        bytes += files[i].len;
    }
    R.prefix.push_back((uint32_t)nch);
    R.nchunks = (int)nch;
    // stale descriptor words from an "earlier call" (other epoch) must be ignored
    R.desc.assign(nch, Desc{{0, 0, 0, 0}});
    R.epoch = 7;
    for (auto& d : R.desc) for (int k = 0; k < 4; k++) d.w[k] = ds_tag(6, 0x5a5a5a5a5a5aull) | ((uint64_t)(k & 1) << 46);
    R.sums.assign(nch, ChunkSum{});
    if (ctx->dbg_on) R.dbg.assign(nch, ChunkDbg{});
    if (ctx->dbg_on > 1) R.lanes.assign(4 * CLY_NT * 8, 0);
    build_shift_tables(R.shift);
    R.x8n.resize(CLY_CHUNK + 1);
    for (int n = 0; n <= CLY_CHUNK; n++) R.x8n[n] = cly_x8n((uint64_t)n);
    // emulated device tuple buffer (gaps allowed, compacted below)
    std::vector<cly_tuple> dev(cly_scan_capacity(files, nfiles) + 16);
    R.out = dev.data();
    R.out_cap = dev.size();
    const char* th = getenv("CLY_EMU_THREADS");
    const int nthreads = th ? atoi(th) : 8;
    const char* jt = getenv("CLY_EMU_JITTER");
    R.jitter = jt ? atoi(jt) : 0;
    const char* dfull = getenv("CLY_EMU_DELAY_FULL");
    R.delay_full = dfull ? atoi(dfull) : -1;
    std::atomic<int> ticket{0};
    std::vector<std::thread> pool;
    for (int k = 0; k < (nthreads > 0 ? nthreads : 1); k++) {
        pool.emplace_back([&R, &ticket, k]() {
            std::mt19937 rng(1234u + (unsigned)k);
            ScanShared* S = (ScanShared*)aligned_alloc(64, (sizeof(ScanShared) + 63) & ~size_t(63));
            std::vector<uint32_t> tab(CLY_TAB_WORDS);
            for (int t = 0; t < 256; t++) build_tab_lane(tab.data(), t, 256);
            for (;;) {
                const int c = ticket.fetch_add(1);
                if (c >= R.nchunks) break;
                memset(S, 0xA5, sizeof(ScanShared));     // stale LDS contents
                S->tab = tab.data();
                run_chunk(R, c, *S, rng);
            }
            free(S);
        });
    }
    for (auto& t : pool) t.join();
    ctx->sums = R.sums;
    ctx->dbg = R.dbg;
    ctx->lanes = R.lanes;
    if (getenv("CLY_EMU_STATS")) fprintf(stderr, "emu: %d chunks, %u look-back fallbacks, %u recoveries\n", R.nchunks, R.fallbacks.load(), R.recoveries.load());
    if (R.fail.load()) return CLY_ERR_DEVICE;
    if (R.overflow.load()) return CLY_ERR_CAPACITY;
    // k_fin
    uint64_t total = 0;
    for (int f = 0; f < nfiles; f++) {
        const FileRec& F = R.files[f];
        int64_t best = EVT_NONE;
        uint64_t bg = 0;
        int32_t bs = 0;
        for (uint32_t i = 0; i < F.nchunks; i++) {
            uint64_t g = 0;
            int32_t st = 0;
            const int64_t o = fin_chunk_event(R.sums.data(), (int)F.first_chunk, (int)F.nchunks, (int)i, &g, &st);
            if (o < best) { best = o; bg = g; bs = st; }
        }
        if (best == EVT_NONE) return CLY_ERR_DEVICE;     // every file ends in an event
        const uint64_t first = R.sums[F.first_chunk].p_excl;
        res[f].n_records = bg - first;
        res[f].end_offset = best;
        res[f].status = bs;
        res[f]._pad = 0;
        file_first[f] = first;
        total += res[f].n_records;
    }
    // compact per file (the device buffer may hold tuples past an ErrInvalidCRC)
    uint64_t need = 0;
    for (int f = 0; f < nfiles; f++) need += res[f].n_records;
    if (needed) *needed = need;
    if (stats) {
        memset(stats, 0, sizeof(*stats));
        stats->passes = 1; stats->n_chunks = (uint32_t)nch; stats->bytes = bytes; stats->records = total;
    }
    if (need > out_cap) return CLY_ERR_CAPACITY;
    uint64_t o = 0;
    for (int f = 0; f < nfiles; f++) {
        memcpy(out + o, dev.data() + file_first[f], sizeof(cly_tuple) * res[f].n_records);
        file_first[f] = o;
        o += res[f].n_records;
    }
    return CLY_OK;
}

extern "C" int cly_scan_device(cly_ctx*, const cly_file*, int, cly_tuple*, uint64_t, uint64_t*, cly_file_result*,
                               uint64_t*, cly_stats*, void*) {
    return CLY_ERR_DEVICE;
}
extern "C" const char* cly_strerror(int code) { return code == 0 ? "ok" : "error"; }
extern "C" const char* cly_build_info(void) {
    static char buf[160];
    snprintf(buf, sizeof(buf), "clyscan CPU EMULATOR (test only) NT=%d SUB=%d CHUNK=%d", CLY_NT, CLY_SUB, CLY_CHUNK);
    return buf;
}
