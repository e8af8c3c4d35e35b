// clyload.hip — the index load of NewCouloyDB on the device (host driver of
// libclyscan; include/clyload.h).
//
// Restates, from data files on disk to a queryable index:
//   NewCouloyDB -> loadDataFile (db.go:442-485: the `%09d.cly` files of the
//   directory, fids ascending, the last one the active file)
//   -> loadIndex (db.go:487-655: every record of every file in fid order,
//   tx buffering by txId, updateIndex, the TTL sweep).
// The files are mmap'd, copied to HBM, scanned (cly_scan_device) and the
// index state of every record (all five indexes) is rebuilt on the device
// (cly_index_device).  The tuples and states come back, and the host builds
// what updateIndex puts in the MemTables (meta/memTable.go:15-30) from the
// records the device marked as index entries: the String and ListMeta indexes
// as open-addressing tables over the mapped key bytes, and the per-key Hash
// (field), List (seq gob encoding) and Set (member hash) maps, keyed as
// ixkey.h derives them (the same code as the device's).
//
// The host inserts are timed separately from the device work.
#include <hip/hip_runtime.h>
#include <dirent.h>
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <mutex>
#include <thread>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/clyload.h"
#include "scan_core.h"
#include "ixkey.h"

extern "C" hipStream_t cly_ctx_stream_internal(cly_ctx* c);
extern "C" int cly_ctx_device_internal(cly_ctx* c);
extern "C" uint64_t cly_ix_hash_mask_internal(uint64_t n);
extern "C" hipError_t cly_ix_hash_ptr_internal(cly_ctx* ctx, uint64_t n, void** out);
#define LOAD_PIECE (64ull << 20)
#define LOAD_STAGE (8ull << 20)            // page-locked staging buffer (two per copy thread)
#define LOAD_THREADS_MAX 16
// process-wide staging buffers of the file copies (allocated on first use)
static std::mutex g_stage_mu;
static void* g_stage[2 * LOAD_THREADS_MAX];

struct Mapped {
    uint32_t fid;
    const uint8_t* p;
    uint64_t len;
};

// The String / ListMeta index: open-addressing tables of (key hash, tuple
// index), sharded by the hash's top bits so that one thread builds each shard;
// the key bytes stay in the mapped files.  The device already decided the one
// live record of every key (last writer wins), so inserts never meet an equal
// key and need no comparison.
struct FlatShard {
    std::vector<uint64_t> h;     // key hash | 1 (0 = empty)
    std::vector<uint64_t> ti;    // tuple index
    uint64_t mask = 0, n = 0;
};
static constexpr int FLAT_SHARD_BITS = 4;
static constexpr int FLAT_SHARDS = 1 << FLAT_SHARD_BITS;
struct FlatIndex {
    FlatShard sh[FLAT_SHARDS];
    uint64_t n = 0;
};
// shard = the top FLAT_SHARD_BITS of the hash's valid bits (the device hash keeps hbits)
static inline int flat_shard(uint64_t h, int hshift) { return (int)((h >> hshift) & (FLAT_SHARDS - 1)); }
// host array without value-initialisation (the device fills it)
template <class T> struct HostArr {
    std::unique_ptr<T[]> p;
    uint64_t n = 0;
    void alloc(uint64_t k) { p.reset(k ? new T[k] : nullptr); n = k; }
    T& operator[](uint64_t i) { return p[i]; }
    const T& operator[](uint64_t i) const { return p[i]; }
    uint64_t size() const { return n; }
    T* data() { return p.get(); }
};
struct cly_db {
    std::vector<Mapped> files;
    HostArr<cly_tuple> tuples;
    HostArr<uint8_t> state;
    HostArr<uint64_t> khash;     // the device index's key hash per record (String / ListMeta tables)
    uint64_t hmask = ~0ull;
    int hshift = 60;
    std::vector<uint64_t> first;
    FlatIndex str, listmeta;
    // getHashIndex / getListDataIndex / getSetIndex (index.go): realKey -> MemTable
    std::unordered_map<std::string, std::unordered_map<std::string, cly_pos>> hash, list, set;
};
[[maybe_unused]] static inline uint64_t key_hash(const uint8_t* p, uint64_t n) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (n * 0xBF58476D1CE4E5B9ull);      // FNV-style, 8 bytes a step
    uint64_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        memcpy(&w, p + i, 8);
        h = (h ^ w) * 0x100000001B3ull;
        h ^= h >> 29;
    }
    uint64_t w = 0;
    memcpy(&w, p + i, n - i);
    h = (h ^ w) * 0x100000001B3ull;
    h ^= h >> 32;
    h *= 0x94D049BB133111EBull;
    return (h ^ (h >> 31)) | 1;
}

// fn(t) on nthreads threads (t = 0 on the caller's)
template <class F> static void par_run(int nthreads, F fn) {
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; t++) th.emplace_back(fn, t);
    fn(0);
    for (auto& x : th) x.join();
}
static int load_threads() {
    return (int)std::min<unsigned>(LOAD_THREADS_MAX, std::max(1u, std::thread::hardware_concurrency()));
}

static double now_ms() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

static const uint8_t* file_of(const cly_db* db, uint32_t fid) {
    // fids ascending in `files`: binary search
    size_t lo = 0, hi = db->files.size();
    while (lo < hi) {
        const size_t mid = (lo + hi) / 2;
        if (db->files[mid].fid < fid) lo = mid + 1; else hi = mid;
    }
    return lo < db->files.size() && db->files[lo].fid == fid ? db->files[lo].p : nullptr;
}

// realKey of tuple t (parseLogRecordKey, db.go:706-710)
static const uint8_t* real_key_ptr(const cly_db* db, const cly_tuple& t, uint64_t& len) {
    const uint8_t* f = file_of(db, t.fid);
    const uint32_t tl = t.txid_len == 0xFF ? 0 : t.txid_len;
    len = t.key_size - tl;
    return f + t.offset + t.header_size + tl;
}
static std::string real_key(const cly_db* db, const cly_tuple& t) {
    uint64_t n;
    const uint8_t* p = real_key_ptr(db, t, n);
    return std::string((const char*)p, n);
}
static void flat_init(FlatShard& x, uint64_t n) {
    uint64_t cap = 16;
    while (cap < 2 * n) cap <<= 1;
    x.h.assign(cap, 0);
    x.ti.assign(cap, 0);
    x.mask = cap - 1;
    x.n = 0;
}
static void flat_put(FlatShard& x, uint64_t h, uint64_t ti) {
    uint64_t i = h & x.mask;
    while (x.h[i]) i = (i + 1) & x.mask;
    x.h[i] = h;
    x.ti[i] = ti;
    x.n++;
}
static void flat_build(cly_db* db, int nthreads, std::vector<uint64_t>& composite);
static int flat_get(const cly_db* db, const FlatIndex& xi, uint32_t kind, const uint8_t* key, uint64_t klen,
                    cly_pos* pos) {
    if (klen > 0xFFFFFFFFull) return CLY_DB_NOT_FOUND;
    const uint64_t h = (ixk_hash(kind, key, (uint32_t)klen) & db->hmask) | 1;
    const FlatShard& x = xi.sh[flat_shard(h, db->hshift)];
    if (!x.mask) return CLY_DB_NOT_FOUND;
    for (uint64_t i = h & x.mask; x.h[i]; i = (i + 1) & x.mask) {
        if (x.h[i] != h) continue;
        const cly_tuple& t = db->tuples[x.ti[i]];
        uint64_t n;
        const uint8_t* k = real_key_ptr(db, t, n);
        if (n == klen && memcmp(k, key, n) == 0) {
            if (pos) { pos->offset = t.offset; pos->fid = t.fid; pos->_pad = 0; }
            return CLY_OK;
        }
    }
    return CLY_DB_NOT_FOUND;
}

static int list_files(const char* dir, std::vector<Mapped>& out) {
    DIR* d = opendir(dir);
    if (!d) return CLY_ERR_ARG;
    struct dirent* e;
    std::vector<uint32_t> fids;
    while ((e = readdir(d))) {
        // data/dataFile.go:20-23 + public/preset.go:6: fmt.Sprintf("%09d", fid) + ".cly"
        const size_t n = strlen(e->d_name);
        if (n != 13 || strcmp(e->d_name + 9, ".cly") != 0) continue;
        bool digits = true;
        for (int i = 0; i < 9; i++) digits &= e->d_name[i] >= '0' && e->d_name[i] <= '9';
        if (digits) fids.push_back((uint32_t)strtoul(std::string(e->d_name, 9).c_str(), nullptr, 10));
    }
    closedir(d);
    std::sort(fids.begin(), fids.end());
    for (uint32_t fid : fids) {
        char path[4096];
        snprintf(path, sizeof(path), "%s/%09u.cly", dir, fid);
        const int fd = open(path, O_RDONLY);
        if (fd < 0) return CLY_ERR_ARG;
        struct stat sb;
        if (fstat(fd, &sb) != 0) { close(fd); return CLY_ERR_ARG; }
        Mapped m;
        m.fid = fid;
        m.len = (uint64_t)sb.st_size;
        m.p = nullptr;
        if (m.len) {
            void* p = mmap(nullptr, m.len, PROT_READ, MAP_PRIVATE, fd, 0);     // pages: faulted in by the copy threads
            if (p == MAP_FAILED) { close(fd); return CLY_ERR_ARG; }
            m.p = (const uint8_t*)p;
        }
        close(fd);
        out.push_back(m);
    }
    return CLY_OK;
}

// Two passes over the LIVE tuples, each split over `nthreads` threads: count
// the records per shard (the key hashes are the device index's, downloaded),
// then let thread t fill shards t, t+T, ...
static void flat_build(cly_db* db, int nthreads, std::vector<uint64_t>& composite) {
    const uint64_t need = db->tuples.size();
    std::vector<std::vector<uint64_t>> comp(nthreads);
    HostArr<uint64_t> hv;
    hv.alloc(need);
    std::vector<uint64_t> cnt((size_t)nthreads * 2 * FLAT_SHARDS, 0);
    auto hash_part = [&](int t) {
        const uint64_t a = need * t / nthreads, b = need * (t + 1) / nthreads;
        uint64_t* c = &cnt[(size_t)t * 2 * FLAT_SHARDS];
        for (uint64_t i = a; i < b; i++) {
            hv[i] = 0;
            const uint8_t st = db->state[i];
            if (st != CLY_IX_LIVE && st != CLY_IX_LOADONLY) continue;
            const uint32_t dt = db->tuples[i].data_type;
            if (dt == 1 || dt == 2 || dt == 4) { comp[t].push_back(i); continue; }    // Hash / List / Set
            if (st != CLY_IX_LIVE || (dt != 0 && dt != 3)) continue;               // String / ListMeta
            hv[i] = (db->khash[i] & db->hmask) | 1;
            c[(dt == 3) * FLAT_SHARDS + flat_shard(hv[i], db->hshift)]++;
        }
    };
    std::vector<uint64_t> boff((size_t)nthreads * 2 * FLAT_SHARDS + 1, 0);
    HostArr<uint64_t> bidx;
    auto scatter_part = [&](int t) {
        const uint64_t a = need * t / nthreads, b = need * (t + 1) / nthreads;
        uint64_t w[2 * FLAT_SHARDS];
        for (int ks = 0; ks < 2 * FLAT_SHARDS; ks++) w[ks] = boff[(size_t)ks * nthreads + t];
        for (uint64_t i = a; i < b; i++) {
            if (!hv[i]) continue;
            const int ks = (db->tuples[i].data_type == 3) * FLAT_SHARDS + flat_shard(hv[i], db->hshift);
            bidx[w[ks]++] = i;
        }
    };
    auto fill_part = [&](int t) {
        for (int kind = 0; kind < 2; kind++)
            for (int sh = t; sh < FLAT_SHARDS; sh += nthreads) {
                const int ks = kind * FLAT_SHARDS + sh;
                const uint64_t lo = boff[(size_t)ks * nthreads], hi = boff[(size_t)(ks + 1) * nthreads];
                FlatShard& x = (kind ? db->listmeta : db->str).sh[sh];
                flat_init(x, hi - lo);
                for (uint64_t j = lo; j < hi; j++) flat_put(x, hv[bidx[j]], bidx[j]);
            }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; t++) th.emplace_back(hash_part, t);
    hash_part(0);
    for (auto& x : th) x.join();
    th.clear();
    {
        // bucket the records by (kind, shard): exclusive offsets over (kind, shard, thread)
        uint64_t acc = 0;
        for (int ks = 0; ks < 2 * FLAT_SHARDS; ks++)
            for (int u = 0; u < nthreads; u++) {
                boff[(size_t)ks * nthreads + u] = acc;
                acc += cnt[(size_t)u * 2 * FLAT_SHARDS + ks];
            }
        boff[(size_t)nthreads * 2 * FLAT_SHARDS] = acc;
        bidx.alloc(acc);
    }
    for (int t = 1; t < nthreads; t++) th.emplace_back(scatter_part, t);
    scatter_part(0);
    for (auto& x : th) x.join();
    th.clear();
    for (int t = 1; t < nthreads; t++) th.emplace_back(fill_part, t);
    fill_part(0);
    for (auto& x : th) x.join();
    composite.clear();
    for (auto& v : comp) composite.insert(composite.end(), v.begin(), v.end());    // scan order
    db->str.n = db->listmeta.n = 0;
    for (int sh = 0; sh < FLAT_SHARDS; sh++) {
        db->str.n += db->str.sh[sh].n;
        db->listmeta.n += db->listmeta.sh[sh].n;
    }
}

extern "C" void cly_db_close(cly_db* db) {
    if (!db) return;
    for (Mapped& m : db->files) if (m.p) munmap((void*)m.p, m.len);
    delete db;
}

#define DCK(x) do { if ((x) != hipSuccess) { rc = CLY_ERR_DEVICE; goto done; } } while (0)

extern "C" int cly_db_open(cly_ctx* ctx, const char* dir, cly_db** out, cly_load_stats* st) {
    if (!ctx || !dir || !out) return CLY_ERR_ARG;
    *out = nullptr;
    cly_load_stats s;
    memset(&s, 0, sizeof(s));
    const double t0 = now_ms();
    cly_db* db = new cly_db();
    int rc = list_files(dir, db->files);
    const int nf = (int)db->files.size();
    uint8_t* d_bytes = nullptr;
    cly_tuple* d_tup = nullptr;
    uint8_t* d_state = nullptr;
    std::vector<cly_file> hf(nf ? nf : 1), df(nf ? nf : 1);
    std::vector<cly_file_result> res(nf ? nf : 1);
    uint64_t total = 0, need = 0, cap = 0;
    hipStream_t strm = cly_ctx_stream_internal(ctx);
    double t1, t2, t3, t4, t5;
    cly_index_result ir;
    if (rc != CLY_OK) goto done;
    t1 = now_ms();
    s.list_map_ms = t1 - t0;
    s.n_files = (uint64_t)nf;
    if (nf) s.active_fid = db->files[nf - 1].fid;
    DCK(hipSetDevice(cly_ctx_device_internal(ctx)));
    for (int i = 0; i < nf; i++) {
        hf[i].base = db->files[i].p; hf[i].len = db->files[i].len; hf[i].fid = db->files[i].fid;
        total += (hf[i].len + 4095) & ~4095ull;
        s.bytes += hf[i].len;
    }
    DCK(hipMalloc((void**)&d_bytes, total + 4096));
    {
        // the files' pages are faulted in and copied by load_threads() threads,
        // 64-MiB pieces each (pageable copies from several threads overlap)
        struct Piece { const uint8_t* src; uint8_t* dst; uint64_t len; };
        std::vector<Piece> pieces;
        uint64_t off = 0;
        for (int i = 0; i < nf; i++) {
            df[i] = hf[i];
            df[i].base = d_bytes + off;
            for (uint64_t a = 0; a < hf[i].len; a += LOAD_PIECE)
                pieces.push_back({hf[i].base + a, d_bytes + off + a, std::min<uint64_t>(LOAD_PIECE, hf[i].len - a)});
            off += (hf[i].len + 4095) & ~4095ull;
        }
        std::atomic<size_t> next(0);
        std::atomic<int> err(0);
        const int dev = cly_ctx_device_internal(ctx);
        const int nt = load_threads();
        std::lock_guard<std::mutex> lk(g_stage_mu);
        for (int k = 0; k < 2 * LOAD_THREADS_MAX; k++)          // (again after a failed allocation)
            if (!g_stage[k] && hipHostMalloc(&g_stage[k], LOAD_STAGE, hipHostMallocPortable) != hipSuccess) {
                g_stage[k] = nullptr;
                err = 1;
            }
        if (err) { rc = CLY_ERR_DEVICE; goto done; }
        par_run(nt, [&](int t) {
            // thread t: pieces through its two page-locked staging buffers
            // (CPU copy of one while the DMA of the other runs)
            if (hipSetDevice(dev) != hipSuccess) { err = 1; return; }
            hipStream_t ts = nullptr;
            hipEvent_t ev[2] = {nullptr, nullptr};
            if (hipStreamCreateWithFlags(&ts, hipStreamNonBlocking) != hipSuccess ||
                hipEventCreateWithFlags(&ev[0], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&ev[1], hipEventDisableTiming) != hipSuccess) { err = 1; return; }
            int b = 0;
            bool used[2] = {false, false};
            for (size_t k; (k = next.fetch_add(1)) < pieces.size();) {
                const Piece& pc = pieces[k];
                for (uint64_t a = 0; a < pc.len; a += LOAD_STAGE) {
                    const uint64_t n = std::min<uint64_t>(LOAD_STAGE, pc.len - a);
                    uint8_t* stg = (uint8_t*)g_stage[2 * t + b];
                    if (used[b] && hipEventSynchronize(ev[b]) != hipSuccess) err = 1;
                    memcpy(stg, pc.src + a, n);
                    if (hipMemcpyAsync(pc.dst + a, stg, n, hipMemcpyHostToDevice, ts) != hipSuccess ||
                        hipEventRecord(ev[b], ts) != hipSuccess) err = 1;
                    used[b] = true;
                    b ^= 1;
                }
            }
            if (hipStreamSynchronize(ts) != hipSuccess) err = 1;
            hipEventDestroy(ev[0]); hipEventDestroy(ev[1]);
            hipStreamDestroy(ts);
        });
        if (err) { rc = CLY_ERR_DEVICE; goto done; }
    }
    t2 = now_ms();
    s.h2d_ms = t2 - t1;
    cap = cly_scan_capacity(hf.data(), nf) + 16;
    DCK(hipMalloc((void**)&d_tup, sizeof(cly_tuple) * cap));
    db->first.resize(nf ? nf : 1);
    rc = cly_scan_device(ctx, df.data(), nf, d_tup, cap, db->first.data(), res.data(), &need, nullptr, nullptr);
    if (rc != CLY_OK) goto done;
    for (int i = 0; i < nf; i++)
        if (res[i].status < 0) { rc = res[i].status; goto done; }         // loadIndex returns the read error
    if (nf) s.write_off = res[nf - 1].end_offset;                         // db.go:632-634
    t3 = now_ms();
    s.scan_ms = t3 - t2;
    DCK(hipMalloc((void**)&d_state, need ? need : 1));
    rc = cly_index_device(ctx, df.data(), nf, d_tup, db->first.data(), res.data(), d_state, &ir, nullptr);
    if (rc != CLY_OK) goto done;
    db->tuples.alloc(need);
    db->state.alloc(need);
    db->khash.alloc(need);
    db->hmask = cly_ix_hash_mask_internal(need);
    db->hshift = 64 - __builtin_clzll(db->hmask | 15) - FLAT_SHARD_BITS;
    DCK(hipStreamSynchronize(strm));
    if (need) {
        // tuples, states and key hashes back, in pieces from several threads
        uint64_t* d_hash = nullptr;
        DCK(cly_ix_hash_ptr_internal(ctx, need, (void**)&d_hash));
        struct Piece { void* dst; const void* src; uint64_t len; };
        std::vector<Piece> pieces;
        auto add = [&](void* dst, const void* src, uint64_t len) {
            for (uint64_t a = 0; a < len; a += LOAD_PIECE)
                pieces.push_back({(uint8_t*)dst + a, (const uint8_t*)src + a, std::min<uint64_t>(LOAD_PIECE, len - a)});
        };
        add(db->tuples.data(), d_tup, sizeof(cly_tuple) * need);
        add(db->state.data(), d_state, need);
        add(db->khash.data(), d_hash, sizeof(uint64_t) * need);
        std::atomic<size_t> next(0);
        std::atomic<int> err(0);
        const int dev = cly_ctx_device_internal(ctx);
        std::lock_guard<std::mutex> lk(g_stage_mu);
        par_run(load_threads(), [&](int t) {
            // thread t: DMA into one staging buffer while the CPU copies the other out
            if (hipSetDevice(dev) != hipSuccess) { err = 1; return; }
            hipStream_t ts = nullptr;
            if (hipStreamCreateWithFlags(&ts, hipStreamNonBlocking) != hipSuccess) { err = 1; return; }
            struct Pend { uint8_t* dst; uint64_t n; int b; };
            Pend pend = {nullptr, 0, 0};
            hipEvent_t ev[2] = {nullptr, nullptr};
            if (hipEventCreateWithFlags(&ev[0], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&ev[1], hipEventDisableTiming) != hipSuccess) { err = 1; return; }
            int b = 0;
            auto drain = [&]() {
                if (!pend.dst) return;
                if (hipEventSynchronize(ev[pend.b]) != hipSuccess) err = 1;
                memcpy(pend.dst, g_stage[2 * t + pend.b], pend.n);
                pend.dst = nullptr;
            };
            for (size_t k; (k = next.fetch_add(1)) < pieces.size();) {
                const Piece& pc = pieces[k];
                for (uint64_t a = 0; a < pc.len; a += LOAD_STAGE) {
                    const uint64_t n = std::min<uint64_t>(LOAD_STAGE, pc.len - a);
                    if (hipMemcpyAsync(g_stage[2 * t + b], (const uint8_t*)pc.src + a, n, hipMemcpyDeviceToHost, ts) !=
                            hipSuccess || hipEventRecord(ev[b], ts) != hipSuccess) err = 1;
                    drain();
                    pend = {(uint8_t*)pc.dst + a, n, b};
                    b ^= 1;
                }
            }
            drain();
            hipEventDestroy(ev[0]); hipEventDestroy(ev[1]);
            hipStreamDestroy(ts);
        });
        if (err) { rc = CLY_ERR_DEVICE; goto done; }
    }
    t4 = now_ms();
    s.index_ms = t4 - t3;
    s.records = need;
    {
        // MemTable inserts (updateIndex, db.go:511-575) for the records the
        // device marked as index entries: String / ListMeta into the flat
        // tables, Hash / List / Set into realKey -> (field | seqBuf | hashKey) maps
        std::vector<uint64_t> composite;
        flat_build(db, std::min(FLAT_SHARDS, load_threads()), composite);
        for (uint64_t i : composite) {
            const cly_tuple& t = db->tuples[i];
            uint32_t off, len;
            ixk_input(t, off, len, false);
            const uint8_t* d = file_of(db, t.fid) + t.offset + t.header_size + off;
            IxKey k;
            if (!ixk_key(t.data_type, d, len, k)) continue;      // (the device rejected a panicking decode)
            cly_pos p;
            p.offset = t.offset; p.fid = t.fid; p._pad = 0;
            const uint8_t* r = d + k.r_off;
            if (t.data_type == 1) {              // realKey = R[0:la], field = R[la:]
                const uint32_t la = k.p[0] | ((uint32_t)k.p[1] << 8) | ((uint32_t)k.p[2] << 16) | ((uint32_t)k.p[3] << 24);
                db->hash[std::string((const char*)r, la)][std::string((const char*)r + la, k.r_len - la)] = p;
            } else if (t.data_type == 2) {       // realKey = R, seqBuf = P[1:]
                db->list[std::string((const char*)r, k.r_len)][std::string((const char*)k.p + 1, k.plen - 1)] = p;
            } else {                             // realKey = R, hashKey = P
                db->set[std::string((const char*)r, k.r_len)][std::string((const char*)k.p, 4)] = p;
            }
        }
        s.str_keys = db->str.n;
        s.listmeta_keys = db->listmeta.n;
        for (auto& kv : db->hash) s.hash_fields += kv.second.size();
        for (auto& kv : db->list) s.list_items += kv.second.size();
        for (auto& kv : db->set) s.set_members += kv.second.size();
    }
    t5 = now_ms();
    s.insert_ms = t5 - t4;
    s.total_ms = t5 - t0;
done:
    hipFree(d_bytes); hipFree(d_tup); hipFree(d_state);
    if (st) *st = s;
    if (rc != CLY_OK) { cly_db_close(db); return rc; }
    *out = db;
    return CLY_OK;
}

static int found(const cly_pos* src, cly_pos* pos) {
    if (pos) *pos = *src;
    return CLY_OK;
}

extern "C" int cly_db_get(cly_db* db, const uint8_t* key, uint64_t klen, cly_pos* pos) {
    if (!db) return CLY_ERR_ARG;
    return flat_get(db, db->str, 0, key, klen, pos);
}

extern "C" int cly_db_listmeta(cly_db* db, const uint8_t* key, uint64_t klen, cly_pos* pos) {
    if (!db) return CLY_ERR_ARG;
    return flat_get(db, db->listmeta, 3, key, klen, pos);
}

extern "C" int cly_db_hget(cly_db* db, const uint8_t* key, uint64_t klen, const uint8_t* field, uint64_t flen,
                           cly_pos* pos) {
    if (!db) return CLY_ERR_ARG;
    auto h = db->hash.find(std::string((const char*)key, klen));
    if (h == db->hash.end()) return CLY_DB_NOT_FOUND;
    auto it = h->second.find(std::string((const char*)field, flen));
    return it == h->second.end() ? CLY_DB_NOT_FOUND : found(&it->second, pos);
}

static int map_get(const std::unordered_map<std::string, std::unordered_map<std::string, cly_pos>>& m,
                   const uint8_t* key, uint64_t klen, const std::string& sub, cly_pos* pos) {
    auto h = m.find(std::string((const char*)key, klen));
    if (h == m.end()) return CLY_DB_NOT_FOUND;
    auto it = h->second.find(sub);
    return it == h->second.end() ? CLY_DB_NOT_FOUND : found(&it->second, pos);
}

extern "C" int cly_db_lget(cly_db* db, const uint8_t* key, uint64_t klen, const uint8_t* seq, uint64_t slen,
                           cly_pos* pos) {
    if (!db || slen > 0xFFFFFFFFull) return CLY_ERR_ARG;
    // the bytes as getListDataIndex(key).Get(seqBuf) takes them (seqBuf =
    // seq.GobEncode() of the caller's Float, txnList.go:250-262): not re-decoded
    return map_get(db->list, key, klen, std::string((const char*)seq, (size_t)slen), pos);
}

extern "C" int cly_db_sget(cly_db* db, const uint8_t* key, uint64_t klen, const uint8_t* member, uint64_t mlen,
                           cly_pos* pos) {
    if (!db || klen > 0xFFFFFFFFull || mlen > 0xFFFFFFFFull) return CLY_ERR_ARG;
    uint8_t hdr[20], hk[4];                      // hashMemberKey(key, member), txnSet.go:149-153
    int h = ixk_put_varint((int64_t)klen, hdr);
    h += ixk_put_varint((int64_t)mlen, hdr + h);
    uint32_t c = ixk_crc_bytes(0xFFFFFFFFu, hdr, (uint32_t)h);
    c = ixk_crc_bytes(c, key, (uint32_t)klen);
    c = ixk_crc_bytes(c, member, (uint32_t)mlen);
    ixk_be32(hk, ~c);
    return map_get(db->set, key, klen, std::string((const char*)hk, 4), pos);
}

// The index key updateIndex derives for a record of data type dtype from the
// decoded key bytes d[0:n] (ixkey.h): writes P || R to out; returns its length,
// -1 if the decode panics, -2 if dtype has no index, -3 if cap is too small.
extern "C" int64_t cly_index_key(uint32_t dtype, const uint8_t* d, uint64_t n, uint8_t* out, uint64_t cap,
                                 uint32_t* plen) {
    if (n > 0xFFFFFFFFull) return -3;
    IxKey k;
    if (!ixk_key(dtype, d, (uint32_t)n, k)) return k.panic ? -1 : -2;
    if ((uint64_t)k.plen + k.r_len > cap) return -3;
    memcpy(out, k.p, k.plen);
    memcpy(out + k.plen, d + k.r_off, k.r_len);
    if (plen) *plen = k.plen;
    return (int64_t)k.plen + k.r_len;
}

// getLogRecordByPos (db.go:680-704): the record at pos, its value.  The CRC
// was checked by the load; the header is decoded again here.
extern "C" int cly_db_value(cly_db* db, const cly_pos* pos, uint8_t* buf, uint64_t cap, uint64_t* vlen) {
    if (!db || !pos || !vlen) return CLY_ERR_ARG;
    const Mapped* m = nullptr;
    for (const Mapped& f : db->files) if (f.fid == pos->fid) m = &f;
    if (!m || pos->offset < 0 || (uint64_t)pos->offset >= m->len) return CLY_ERR_ARG;
    const Hdr h = step_hdr(m->p, pos->offset, (int64_t)m->len, pos->offset);
    if (h.status != REC_OK) return h.status;
    *vlen = h.vs;
    if (buf && cap >= h.vs) memcpy(buf, m->p + pos->offset + h.hsz + h.ks, h.vs);
    return (buf && cap < h.vs) ? CLY_ERR_CAPACITY : CLY_OK;
}
