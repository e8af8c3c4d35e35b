// clyload.hip — the index load of NewCouloyDB on the device (host driver of
// libclyscan; include/clyload.h).
//
// Restates, from the files of a data directory to a queryable index:
//   NewCouloyDB -> loadDataFile (db.go:442-485: the `*.cly` files, stems by
//   strconv.Atoi, fids ascending, the last one the active file)
//   -> loadIndexFromHintFile (merge.go:257-287: hint-index records into the
//   String index first) -> loadIndex (db.go:487-655: merge-finished checked,
//   every record of every file in fid order, tx buffering by txId,
//   updateIndex, the TTL sweep's db.Del).
// The files are mmap'd and copied to HBM; the hint file and the data files are
// scanned in one cly_scan_device call, the hint records' positions decoded on
// the device, and their tuples rewritten as String puts of their stored key
// (no txId) so that the device index rebuild (cly_index_device) applies them
// first and the data files' String records override them, last writer wins.
// The host records (offset, fid, header and key sizes, expiration: 24 B of
// each 48-B tuple) and the class bytes come back, and the host builds what updateIndex puts
// in the MemTables (meta/memTable.go:15-30) from the records the device
// marked as index entries: the String and ListMeta indexes as open-addressing
// tables over the mapped key bytes, and the per-key Hash (field), List (seq
// gob encoding) and Set (member hash) maps, keyed as ixkey.h derives them
// (the same code as the device's).  The TTL sweep's tombstones follow
// appendLogRecord's rotation rule (db.go:368-413).
//
// The host inserts are timed separately from the device work.
#include <hip/hip_runtime.h>
#include <dirent.h>
#include <errno.h>
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
extern "C" int cly_order_keys_internal(hipStream_t st, const cly_tuple* d_tup, uint64_t n, const uint8_t* d_state,
                                       uint32_t dt, const uint64_t* first, const uint64_t* bases, int nf,
                                       uint32_t** d_ord_out, uint64_t* m_out, uint32_t* rounds_out);
extern "C" int cly_scan_device_alloc_internal(cly_ctx* c, const cly_file* files, int nfiles, cly_tuple** d_out,
                                              uint64_t* cap, uint64_t* file_first, cly_file_result* res,
                                              uint64_t* needed);
#define LOAD_PIECE (64ull << 20)
#define LOAD_STAGE (8ull << 20)            // page-locked staging buffer (two per copy thread)
#define LOAD_THREADS_MAX 16
// process-wide staging buffers of the file copies (allocated on first use)
static std::mutex g_stage_mu;
static void* g_stage[2 * LOAD_THREADS_MAX];

// db->state bytes: the index state (low nibble) and the record's data type
// (high nibble; k_state_dt)
#define ST_STATE(b) ((uint8_t)((b) & 15))
#define ST_DT(b) ((uint32_t)((b) >> 4))
struct Mapped {
    uint32_t fid;
    const uint8_t* p;
    uint64_t len;
};
// Go's strconv.Atoi (64-bit int): an optional sign, decimal digits, no overflow
static bool go_atoi(const char* s, size_t n, int64_t& v) {
    size_t i = 0;
    bool neg = false;
    if (n && (s[0] == '+' || s[0] == '-')) { neg = s[0] == '-'; i = 1; }
    if (i == n) return false;
    uint64_t x = 0;
    for (; i < n; i++) {
        if (s[i] < '0' || s[i] > '9') return false;
        const uint64_t d = (uint64_t)(s[i] - '0');
        if (x > (UINT64_MAX - d) / 10) return false;
        x = x * 10 + d;
    }
    if (neg) { if (x > (uint64_t)INT64_MAX + 1) return false; v = (int64_t)(0 - x); }
    else { if (x > (uint64_t)INT64_MAX) return false; v = (int64_t)x; }
    return true;
}
// CRC-32/IEEE of a byte range (host; table-driven)
static uint32_t host_crc(const uint8_t* p, uint64_t n) {
    static uint32_t tab[256];
    static std::once_flag once;
    std::call_once(once, [] {
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t c = i;
            for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ CLY_POLY : c >> 1;
            tab[i] = c;
        }
    });
    uint32_t c = 0xFFFFFFFFu;
    for (uint64_t i = 0; i < n; i++) c = tab[(c ^ p[i]) & 0xff] ^ (c >> 8);
    return ~c;
}
// ReadLogRecord (data/dataFile.go:64-111) at off of a host buffer: the
// header, and REC_OK only if the CRC matches (else CLY_ERR_CRC)
static Hdr host_read_record(const uint8_t* p, uint64_t len, int64_t off) {
    Hdr h = step_hdr(p, off, (int64_t)len, off);
    if (h.status == REC_OK && host_crc(p + off + 4, (uint64_t)h.size - 4) != h.crc) h.status = CLY_ERR_CRC;
    return h;
}

// host array without value-initialisation (the device fills it): an
// anonymous mapping advised for transparent huge pages, so that the copy
// threads that first write it (the open's read-back, hundreds of MB) take a
// page fault per 2 MiB rather than per 4 KiB
template <class T> struct HostArr {
    T* p = nullptr;
    uint64_t n = 0, bytes = 0;
    HostArr() = default;
    HostArr(const HostArr&) = delete;
    HostArr& operator=(const HostArr&) = delete;
    ~HostArr() { release(); }
    void release() {
        if (p) munmap(p, bytes);
        p = nullptr; n = 0; bytes = 0;
    }
    void alloc(uint64_t k) {
        release();
        if (!k) return;
        const uint64_t b = (k * sizeof(T) + 4095) & ~4095ull;
        void* m = mmap(nullptr, b, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (m == MAP_FAILED) throw std::bad_alloc();
        if (b >= (2ull << 20)) madvise(m, b, MADV_HUGEPAGE);
        p = (T*)m; n = k; bytes = b;
    }
    T& operator[](uint64_t i) { return p[i]; }
    const T& operator[](uint64_t i) const { return p[i]; }
    uint64_t size() const { return n; }
    T* data() { return p; }
};
// The String / ListMeta index: open-addressing tables sharded by the key
// hash's top valid bits, built on the device (k_flat_count, k_flat_insert)
// and read back whole; the key bytes stay in the mapped files.  A slot is
// 8 B: 0 empty, else tag << 40 | (tuple index + 1), the tag 24 bits of a
// remix of the hash (a lookup compares keys only on equal tags); probing
// starts at hash & mask.  The device already decided the one live record of
// every key (last writer wins), so inserts never meet an equal key.
struct FlatShard {
    HostArr<uint64_t> s;
    uint64_t mask = 0, n = 0;    // (mask 0: no slots)
};
static constexpr int FLAT_SHARD_BITS = 4;
static constexpr int FLAT_SHARDS = 1 << FLAT_SHARD_BITS;
#define FLAT_TI_BITS 40
#define FLAT_TI_MASK ((1ull << FLAT_TI_BITS) - 1)
struct FlatIndex {
    FlatShard sh[FLAT_SHARDS];
    uint64_t n = 0;
};
// shard = the top FLAT_SHARD_BITS of the hash's valid bits (the device hash keeps hbits)
__host__ __device__ static inline int flat_shard(uint64_t h, int hshift) { return (int)((h >> hshift) & (FLAT_SHARDS - 1)); }
__host__ __device__ static inline uint64_t flat_tag(uint64_t h) { return (h * 0x9E3779B97F4A7C15ull) >> 40; }
// the slot's tuple index, or ~0 for an empty slot
static inline uint64_t flat_ti(uint64_t v) { return v ? (v & FLAT_TI_MASK) - 1 : ~0ull; }
// What the host keeps of a record for its lookups and enumerations (24 B; the
// 48-B tuple stays on the device): the file offset (below 2^48) with the
// header size in bits 48..54, "txId != 0" in bit 55 and the txId varint's
// length in bits 56..63; the expiration; the fid; the stored key's size.
// The data type is the class byte's high nibble (k_state_dt).
struct HostRec { uint64_t a; int64_t exp; uint32_t fid, ks; };
static_assert(sizeof(HostRec) == 24, "24-B host records");
#define HR_OFF_MASK ((1ull << 48) - 1)
static inline uint64_t hr_off(const HostRec& r) { return r.a & HR_OFF_MASK; }
static inline uint32_t hr_hsz(const HostRec& r) { return (uint32_t)(r.a >> 48) & 0x7Fu; }
static inline bool hr_tx(const HostRec& r) { return ((r.a >> 55) & 1u) != 0; }
static inline uint32_t hr_txl(const HostRec& r) { return (uint32_t)(r.a >> 56); }
struct cly_db {
    std::vector<Mapped> files;       // in loadIndex's order (fids as sort.Ints orders the stems)
    std::unordered_map<uint32_t, uint32_t> fid_ix;   // uint32(fid) -> its file
    Mapped hint = {0, nullptr, 0};   // hint-index (tuples 0 .. n_hint-1 are its records)
    uint64_t n_hint = 0;
    std::vector<cly_pos> hint_pos;   // DecodeLogRecordPos of each hint record's value
    std::vector<uint64_t> expired;   // tuple indices of the String winners the TTL sweep removed
    std::vector<cly_db_entry> it[6]; // cly_db_entries, built on first use
    bool it_built[6] = {false, false, false, false, false, false};
    HostArr<HostRec> recs;           // per tuple (scan order)
    HostArr<uint8_t> state;
    uint64_t hmask = ~0ull;
    int hshift = 60;
    std::vector<uint64_t> first;
    FlatIndex str, listmeta;
    // the String (0) and ListMeta (1) winners as tuple indices, ascending by
    // key (bytes.Compare; clyorder.hip): the BTree order of the enumeration
    HostArr<uint32_t> ord[2];
    uint64_t n_ord[2] = {0, 0};
    // the Hash / List / Set entries in (key, sub) order, built at the open
    std::vector<cly_db_entry> comp[3];
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
    const auto it = db->fid_ix.find(fid);
    return it == db->fid_ix.end() ? nullptr : db->files[it->second].p;
}

// realKey of tuple ti (parseLogRecordKey, db.go:706-710); a hint record's
// stored key as it is (strIndex.Put(logRecord.Key), merge.go:283)
static const uint8_t* real_key_ptr(const cly_db* db, uint64_t ti, uint64_t& len) {
    const HostRec& t = db->recs[ti];
    const uint8_t* f = ti < db->n_hint ? db->hint.p : file_of(db, t.fid);
    const uint32_t tl = hr_txl(t) == 0xFF ? 0 : hr_txl(t);
    len = t.ks - tl;
    return f + hr_off(t) + hr_hsz(t) + tl;
}
// the LogPos an index entry at tuple ti holds
static cly_pos pos_of(const cly_db* db, uint64_t ti) {
    if (ti < db->n_hint) return db->hint_pos[ti];
    cly_pos p;
    p.offset = (int64_t)hr_off(db->recs[ti]); p.fid = db->recs[ti].fid; p._pad = 0;
    return p;
}
// slots of a shard of n keys: a power of two >= 1.5 n (at least 16; none for no key)
static uint64_t flat_cap(uint64_t n) {
    if (!n) return 0;
    uint64_t cap = 16;
    while (cap < n + n / 2) cap <<= 1;
    return cap;
}
static int flat_get(const cly_db* db, const FlatIndex& xi, uint32_t kind, const uint8_t* key, uint64_t klen,
                    cly_pos* pos) {
    if (klen > 0xFFFFFFFFull) return CLY_DB_NOT_FOUND;
    const uint64_t h = (ixk_hash(kind, key, (uint32_t)klen) & db->hmask) | 1, tg = flat_tag(h);
    const FlatShard& x = xi.sh[flat_shard(h, db->hshift)];
    if (!x.mask) return CLY_DB_NOT_FOUND;
    for (uint64_t i = h & x.mask, v; (v = x.s[i]); i = (i + 1) & x.mask) {
        if ((v >> FLAT_TI_BITS) != tg) continue;
        uint64_t n;
        const uint64_t ti = flat_ti(v);
        const uint8_t* k = real_key_ptr(db, ti, n);
        if (n == klen && memcmp(k, key, n) == 0) {
            if (pos) *pos = pos_of(db, ti);
            return CLY_OK;
        }
    }
    return CLY_DB_NOT_FOUND;
}

static int map_file(const char* path, Mapped& m, bool& exists) {
    m.p = nullptr; m.len = 0;
    exists = false;
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return errno == ENOENT ? CLY_OK : CLY_ERR_ARG;
    exists = true;
    struct stat sb;
    if (fstat(fd, &sb) != 0 || S_ISDIR(sb.st_mode)) { close(fd); return CLY_ERR_ARG; }
    m.len = (uint64_t)sb.st_size;
    if (m.len) {
        void* p = mmap(nullptr, m.len, PROT_READ, MAP_PRIVATE, fd, 0);     // for the host's key reads
        if (p == MAP_FAILED) { close(fd); m.len = 0; return CLY_ERR_ARG; }
        m.p = (const uint8_t*)p;
        close(fd);
        return CLY_OK;
    }
    close(fd);
    return CLY_OK;
}
// loadDataFile's listing (db.go:442-470): entries ending in ".cly", stem =
// the name up to its first '.', fid = strconv.Atoi(stem) (failure: "the data
// dir maybe contaminated or damaged"), sort.Ints; the file read is
// GetDataFileName(uint32(fid)) = "%09d.cly" (absent: read as empty; the
// reference's OpenFile creates it empty).  A file listed twice (say "7.cly" and
// "000000007.cly", or "-1.cly" and "4294967295.cly": the same uint32 fid) is
// read at every place sort.Ints puts it, as loadDataFile/loadIndex do
// (db.go:449-464, 587-631): each place opens %09d of the uint32 fid, so every
// reading sees the same file, and transactions spanning the places resolve as
// the reference's do.
static int list_files(const char* dir, std::vector<Mapped>& out, std::unordered_map<uint32_t, uint32_t>& ix) {
    DIR* d = opendir(dir);
    if (!d) return CLY_ERR_ARG;
    struct dirent* e;
    std::vector<int64_t> fids;
    int rc = CLY_OK;
    while ((e = readdir(d))) {
        const size_t n = strlen(e->d_name);
        if (n < 4 || strcmp(e->d_name + n - 4, ".cly") != 0) continue;
        const char* dot = strchr(e->d_name, '.');
        int64_t v;
        if (!go_atoi(e->d_name, (size_t)(dot - e->d_name), v)) { rc = CLY_ERR_DIR; break; }
        fids.push_back(v);
    }
    closedir(d);
    if (rc != CLY_OK) return rc;
    std::sort(fids.begin(), fids.end());
    std::vector<uint32_t> order;                 // every listing, in sort.Ints order
    for (int64_t v : fids) order.push_back((uint32_t)v);
    for (uint32_t fid : order) {
        char path[4096];
        snprintf(path, sizeof(path), "%s/%09u.cly", dir, fid);
        Mapped m;
        bool exists;
        if (map_file(path, m, exists) != CLY_OK) return CLY_ERR_ARG;
        m.fid = fid;
        ix[fid] = (uint32_t)out.size();
        out.push_back(m);
    }
    return CLY_OK;
}

// The records the flat tables take: a String or ListMeta key's live record
// (dt 0 / 3; class byte = state | dt << 4, k_state_dt); -1 for the others
__device__ static inline int flat_ks(uint8_t b, uint64_t h, int hshift) {
    const uint32_t st = b & 15u, dt = b >> 4;
    if (st != CLY_IX_LIVE || (dt != 0 && dt != 3)) return -1;
    return (dt == 3 ? FLAT_SHARDS : 0) + flat_shard(h, hshift);
}
// keys per (kind, shard)
__global__ void k_flat_count(const uint8_t* __restrict__ state, const uint64_t* __restrict__ hash, uint64_t n,
                             uint64_t hmask, int hshift, unsigned long long* cnt) {
    __shared__ unsigned int c[2 * FLAT_SHARDS];
    if (threadIdx.x < 2 * FLAT_SHARDS) c[threadIdx.x] = 0;
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t b = state[i];
        if ((b & 15u) != CLY_IX_LIVE) continue;
        const int ks = flat_ks(b, (hash[i] & hmask) | 1, hshift);
        if (ks >= 0) atomicAdd(&c[ks], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 2 * FLAT_SHARDS && c[threadIdx.x]) atomicAdd(&cnt[threadIdx.x], (unsigned long long)c[threadIdx.x]);
}
// the inserts: linear probing from hash & mask, a slot claimed by CAS on 0
// (geo: per (kind, shard) its first slot and its mask)
__global__ void k_flat_insert(const uint8_t* __restrict__ state, const uint64_t* __restrict__ hash, uint64_t n,
                              uint64_t hmask, int hshift, const uint64_t* __restrict__ geo, unsigned long long* slots) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t b = state[i];
        if ((b & 15u) != CLY_IX_LIVE) continue;
        const uint64_t h = (hash[i] & hmask) | 1;
        const int ks = flat_ks(b, h, hshift);
        if (ks < 0) continue;
        const uint64_t base = geo[2 * ks], m = geo[2 * ks + 1];
        const unsigned long long v = (unsigned long long)((flat_tag(h) << FLAT_TI_BITS) | (i + 1));
        for (uint64_t j = h & m; atomicCAS(&slots[base + j], 0ull, v) != 0ull; j = (j + 1) & m) {}
    }
}
// Hash / List / Set records an index points at (scan order), from the class bytes
static void composite_list(const cly_db* db, int nthreads, std::vector<uint64_t>& composite) {
    const uint64_t need = db->state.size();
    std::vector<std::vector<uint64_t>> comp(nthreads);
    par_run(nthreads, [&](int t) {
        const uint64_t a = need * t / nthreads, b = need * (t + 1) / nthreads;
        for (uint64_t i = a; i < b; i++) {
            const uint8_t st = ST_STATE(db->state[i]);
            if (st != CLY_IX_LIVE && st != CLY_IX_LOADONLY) continue;
            const uint32_t dt = ST_DT(db->state[i]);
            if (dt == 1 || dt == 2 || dt == 4) comp[t].push_back(i);
        }
    });
    composite.clear();
    for (auto& v : comp) composite.insert(composite.end(), v.begin(), v.end());
}

extern "C" void cly_db_close(cly_db* db) {
    if (!db) return;
    for (Mapped& m : db->files) if (m.p) munmap((void*)m.p, m.len);
    if (db->hint.p) munmap((void*)db->hint.p, db->hint.len);
    delete db;
}

#define DCK(x) do { if ((x) != hipSuccess) { rc = CLY_ERR_DEVICE; goto done; } } while (0)

// The host table build's per-record class byte: the index state (low nibble)
// and the data type (high nibble, 7 for any type above 6), so that the build
// reads 1 B per record instead of the 48-B tuple
__global__ void k_state_dt(uint8_t* state, const cly_tuple* t, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t dt = t[i].data_type;
    state[i] = (uint8_t)(state[i] | ((dt < 7 ? dt : 7) << 4));
}

// The host records of the tuples (what lookups read; half the tuples' bytes
// over PCIe)
__global__ void k_host_rec(const cly_tuple* t, HostRec* r, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const cly_tuple x = t[i];
    HostRec o;
    o.a = ((uint64_t)x.offset & HR_OFF_MASK) | ((uint64_t)(x.header_size & 0x7Fu) << 48) |
          ((uint64_t)(x.tx_id != 0) << 55) | ((uint64_t)x.txid_len << 56);
    o.exp = x.expiration;
    o.fid = x.fid;
    o.ks = x.key_size;
    r[i] = o;
}
// A hint record's tuple as the index rebuild takes it: strIndex.Put of its
// stored key (no txId prefix, merge.go:283), whatever its types, no TTL
__global__ void k_hint_as_put(cly_tuple* t, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    t[i].tx_id = 0; t[i].txid_len = 0; t[i].type = 0; t[i].data_type = 0; t[i].expiration = 0;
}

// Page-locked staging buffers (two per copy thread), allocated once, each by
// the copy thread that first uses its slot (the threads' allocations run side
// by side); the caller holds g_stage_mu.
static bool stage_pair(int t) {
    for (int k = 2 * t; k < 2 * t + 2; k++)                // (again after a failed allocation)
        if (!g_stage[k] && hipHostMalloc(&g_stage[k], LOAD_STAGE, hipHostMallocPortable) != hipSuccess) {
            g_stage[k] = nullptr;
            return false;
        }
    return true;
}
// The pool's staging buffers, all of them, allocated by load_threads()
// threads side by side (include/clyload.h cly_load_prepare): an application
// that opens a database calls it at start-up, so that the first open finds
// them (allocating the 32 page-locked 8-MiB buffers inside the first open's
// copy cost it 15-25 ms, profiles/r5_*).  Scan-only users never pay for them;
// without it the open's copy threads allocate their own pair at first use.
// Tried once per process: a failure is remembered (the lazy path still tries
// per copy thread).
extern "C" int cly_load_prepare(void) {
    static int state = 0;                  // 0 not tried, 1 all allocated, 2 failed
    std::lock_guard<std::mutex> lk(g_stage_mu);
    if (state) return state == 1 ? CLY_OK : CLY_ERR_DEVICE;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) { state = 2; return CLY_ERR_DEVICE; }
    std::atomic<int> ok(0);
    const int nt = load_threads();
    par_run(nt, [&](int t) {
        if (hipSetDevice(dev) == hipSuccess && stage_pair(t)) ok++;
    });
    state = ok == nt ? 1 : 2;
    return state == 1 ? CLY_OK : CLY_ERR_DEVICE;
}
// The files' bytes to device dev: nt threads (staging buffers of threads t0 ..
// t0+nt-1) fault the mapped pages in and copy 64-MiB pieces through the
// page-locked staging buffers (CPU copy of one while the DMA of the other
// runs).  The caller holds g_stage_mu.
static int copy_to_device(int dev, const std::vector<cly_file>& hf, std::vector<cly_file>& df, uint8_t* d_bytes,
                          int t0, int nt) {
    struct Piece { const uint8_t* src; uint8_t* dst; uint64_t len; };
    std::vector<Piece> pieces;
    uint64_t off = 0;
    for (size_t i = 0; i < hf.size(); i++) {
        df[i] = hf[i];
        df[i].base = d_bytes + off;
        for (uint64_t a = 0; a < hf[i].len; a += LOAD_PIECE)
            pieces.push_back({hf[i].base + a, d_bytes + off + a, std::min<uint64_t>(LOAD_PIECE, hf[i].len - a)});
        off += (hf[i].len + 4095) & ~4095ull;
    }
    std::atomic<size_t> next(0);
    std::atomic<int> err(0);
    par_run(nt, [&](int t) {
        if (hipSetDevice(dev) != hipSuccess || !stage_pair(t0 + t)) { err = 1; return; }
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
                uint8_t* stg = (uint8_t*)g_stage[2 * (t0 + t) + b];
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
    return err ? CLY_ERR_DEVICE : CLY_OK;
}

// Device buffers back to host memory, in pieces from several threads (DMA
// into one staging buffer while the CPU copies the other out).
struct D2H { void* dst; const void* src; uint64_t len; };
static int copy_to_host(cly_ctx* ctx, const std::vector<D2H>& parts, int t0, int nt, bool lock = true) {
    struct Piece { void* dst; const void* src; uint64_t len; };
    std::vector<Piece> pieces;
    for (const D2H& x : parts)
        for (uint64_t a = 0; a < x.len; a += LOAD_PIECE)
            pieces.push_back({(uint8_t*)x.dst + a, (const uint8_t*)x.src + a, std::min<uint64_t>(LOAD_PIECE, x.len - a)});
    std::atomic<size_t> next(0);
    std::atomic<int> err(0);
    const int dev = cly_ctx_device_internal(ctx);
    std::unique_lock<std::mutex> lk(g_stage_mu, std::defer_lock);     // (lock = false: the caller holds it)
    if (lock) lk.lock();
    // (threads t0 .. t0+nt-1, each with its own two staging buffers)
    par_run(nt, [&, t0](int tl) {
        const int t = t0 + tl;
        if (hipSetDevice(dev) != hipSuccess || !stage_pair(t)) { err = 1; return; }
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
    return err ? CLY_ERR_DEVICE : CLY_OK;
}

// getNonMergeFileId (merge.go:240-255): the record at offset 0 of
// merge-finished must read and its value be an integer.
static int check_merge_finished(const char* dir) {
    char path[4096];
    snprintf(path, sizeof(path), "%s/merge-finished", dir);
    Mapped m;
    bool exists;
    if (map_file(path, m, exists) != CLY_OK) return CLY_ERR_MERGE_FIN;
    if (!exists) return CLY_OK;
    int rc = CLY_OK;
    const Hdr h = host_read_record(m.p, m.len, 0);
    if (h.status == CLY_ERR_CRC) rc = CLY_ERR_CRC;                                 // ErrInvalidCRC
    else if (h.status == CLY_ERR_TRUNC5 || h.status == CLY_ERR_VARINT) rc = h.status;    // the decode panics
    else if (h.status != REC_OK) rc = CLY_ERR_MERGE_FIN;                           // io.EOF: an error here
    else {
        int64_t v;
        if (!go_atoi((const char*)m.p + h.hsz + h.ks, h.vs, v)) rc = CLY_ERR_MERGE_FIN;
    }
    if (m.p) munmap((void*)m.p, m.len);
    return rc;
}

// EncodeLogRecord (data/logRecord.go:57-84) of db.Del's tombstone for key:
// {encodeKeyWithTxId(key, NO_TX_ID), LogRecordDeleted, String}
static std::vector<uint8_t> tombstone(const uint8_t* key, uint64_t klen) {
    std::vector<uint8_t> r(4 + 2 + 10 + 2 + 1 + klen);
    uint8_t* p = r.data();
    p[4] = 1; p[5] = 0;                                 // LogRecordDeleted, String
    int n = 6;
    n += ixk_put_varint((int64_t)klen + 1, p + n);      // key = 0x00 || key
    n += ixk_put_varint(0, p + n);
    n += ixk_put_varint(0, p + n);
    p[n] = 0x00;
    memcpy(p + n + 1, key, klen);
    r.resize(n + 1 + klen);
    const uint32_t c = host_crc(r.data() + 4, r.size() - 4);
    r[0] = (uint8_t)c; r[1] = (uint8_t)(c >> 8); r[2] = (uint8_t)(c >> 16); r[3] = (uint8_t)(c >> 24);
    return r;
}

// The index rebuild on the device (cly_index_device), then the String /
// ListMeta tables: keys per shard counted, slots laid out, inserts, and the
// class bytes, the slots and the hint positions read back on copy threads
// 0 .. nb-1 (the caller holds g_stage_mu).
static int flat_device(cly_ctx* ctx, cly_db* db, const cly_file* df, int nall, const cly_tuple* d_tup,
                       const std::vector<uint64_t>& first, const std::vector<cly_file_result>& res, uint8_t* d_state,
                       const cly_pos* d_hpos, uint64_t need, cly_index_result& ir, int nb, cly_load_stats& s) {
    hipStream_t strm = cly_ctx_stream_internal(ctx);
    if (nall) {
        const int rc = cly_index_device(ctx, df, nall, d_tup, first.data(), res.data(), d_state, &ir, nullptr);
        if (rc != CLY_OK) return rc;
    }
    if (!need) return hipStreamSynchronize(strm) == hipSuccess ? CLY_OK : CLY_ERR_DEVICE;
    if (need >= FLAT_TI_MASK) return CLY_ERR_ARG;                 // (a slot holds a 40-bit tuple index)
    int rc = CLY_OK;
    uint64_t* d_hash = nullptr;
    unsigned long long* d_cnt = nullptr;
    unsigned long long* d_slots = nullptr;
    uint64_t* d_geo = nullptr;
    uint32_t* d_ord[2] = {nullptr, nullptr};
    unsigned long long cnt[2 * FLAT_SHARDS];
    uint64_t geo[4 * FLAT_SHARDS], tot = 0;
    const unsigned grid = (unsigned)std::min<uint64_t>((need + 255) / 256, 8192);
    std::vector<D2H> parts = {{db->state.data(), d_state, need}};
    DCK(cly_ix_hash_ptr_internal(ctx, need, (void**)&d_hash));
    DCK(hipMalloc((void**)&d_cnt, sizeof(cnt) + sizeof(geo)));
    d_geo = (uint64_t*)(d_cnt + 2 * FLAT_SHARDS);
    DCK(hipMemsetAsync(d_cnt, 0, sizeof(cnt), strm));
    hipLaunchKernelGGL(k_state_dt, dim3((unsigned)((need + 255) / 256)), dim3(256), 0, strm, d_state, d_tup, need);
    hipLaunchKernelGGL(k_flat_count, dim3(grid), dim3(256), 0, strm, d_state, d_hash, need, db->hmask, db->hshift, d_cnt);
    DCK(hipGetLastError());
    DCK(hipMemcpyAsync(cnt, d_cnt, sizeof(cnt), hipMemcpyDeviceToHost, strm));
    DCK(hipStreamSynchronize(strm));
    for (int ks = 0; ks < 2 * FLAT_SHARDS; ks++) {
        const uint64_t cap = flat_cap(cnt[ks]);
        FlatShard& x = (ks >= FLAT_SHARDS ? db->listmeta : db->str).sh[ks % FLAT_SHARDS];
        x.s.alloc(cap);
        x.mask = cap ? cap - 1 : 0;
        x.n = cnt[ks];
        geo[2 * ks] = tot; geo[2 * ks + 1] = x.mask;
        if (cap) parts.push_back({x.s.data(), nullptr, cap * 8});     // (its source once the slots exist)
        tot += cap;
    }
    DCK(hipMalloc((void**)&d_slots, 8 * (tot ? tot : 1)));
    {
        size_t k = 1;
        for (int ks = 0; ks < 2 * FLAT_SHARDS; ks++)
            if (cnt[ks]) parts[k++].src = d_slots + geo[2 * ks];
    }
    DCK(hipMemsetAsync(d_slots, 0, 8 * tot, strm));
    DCK(hipMemcpyAsync(d_geo, geo, sizeof(uint64_t) * 4 * FLAT_SHARDS, hipMemcpyHostToDevice, strm));
    hipLaunchKernelGGL(k_flat_insert, dim3(grid), dim3(256), 0, strm, d_state, d_hash, need, db->hmask, db->hshift, d_geo,
                       d_slots);
    DCK(hipGetLastError());
    {
        // the MemTable order: String (dt 0) and ListMeta (dt 3) winners by key
        const double to = now_ms();
        std::vector<uint64_t> bases(nall);
        for (int i = 0; i < nall; i++) bases[i] = (uint64_t)(uintptr_t)df[i].base;
        for (int k = 0; k < 2; k++) {
            uint32_t rounds = 0;
            rc = cly_order_keys_internal(strm, d_tup, need, d_state, k ? 3u : 0u, first.data(), bases.data(), nall,
                                         &d_ord[k], &db->n_ord[k], &rounds);
            if (rc != CLY_OK) goto done;
            s.order_rounds = std::max(s.order_rounds, rounds);
            db->ord[k].alloc(db->n_ord[k]);
            if (db->n_ord[k]) parts.push_back({db->ord[k].data(), d_ord[k], sizeof(uint32_t) * db->n_ord[k]});
        }
        s.order_ms = now_ms() - to;
    }
    DCK(hipStreamSynchronize(strm));
    if (db->n_hint) parts.push_back({db->hint_pos.data(), d_hpos, sizeof(cly_pos) * db->n_hint});
    rc = copy_to_host(ctx, parts, 0, nb, false);
    db->str.n = db->listmeta.n = 0;
    for (int sh = 0; sh < FLAT_SHARDS; sh++) {
        db->str.n += db->str.sh[sh].n;
        db->listmeta.n += db->listmeta.sh[sh].n;
    }
done:
    hipFree(d_cnt); hipFree(d_slots); hipFree(d_ord[0]); hipFree(d_ord[1]);
    return rc;
}

extern "C" int cly_db_open(cly_ctx* ctx, const char* dir, cly_db** out, cly_load_stats* st) {
    return cly_db_open_multi(&ctx, 1, dir, nullptr, out, st);
}
extern "C" int cly_db_open_opts(cly_ctx* ctx, const char* dir, const cly_db_options* opt, cly_db** out,
                                cly_load_stats* st) {
    return cly_db_open_multi(&ctx, 1, dir, opt, out, st);
}

// One shard of the load: a contiguous range [f0, f1) of the open's files (the
// hint-index first when present, then the data files by fid), copied to its
// context's device and scanned there.
struct LoadShard {
    cly_ctx* ctx = nullptr;
    int dev = 0, f0 = 0, f1 = 0;
    uint8_t* d_bytes = nullptr;
    cly_tuple* d_tup = nullptr;
    uint64_t cap = 0, need = 0;
    std::vector<cly_file> df;
    std::vector<cly_file_result> res;
    std::vector<uint64_t> first;
    int rc = CLY_OK;
    double t_copy = 0, t_scan = 0;
};
static void shard_load(LoadShard& S, const std::vector<cly_file>& hf, int t0, int nt) {
    const int n = S.f1 - S.f0;
    const std::vector<cly_file> h(hf.begin() + S.f0, hf.begin() + S.f1);
    S.df.resize(n); S.res.resize(n); S.first.resize(n);
    if (hipSetDevice(S.dev) != hipSuccess) { S.rc = CLY_ERR_DEVICE; return; }
    uint64_t total = 0;
    for (const cly_file& f : h) total += (f.len + 4095) & ~4095ull;
    if (hipMalloc((void**)&S.d_bytes, total + 4096) != hipSuccess) { S.d_bytes = nullptr; S.rc = CLY_ERR_DEVICE; return; }
    S.rc = copy_to_device(S.dev, h, S.df, S.d_bytes, t0, nt);
    S.t_copy = now_ms();
    if (S.rc != CLY_OK) return;
    // the tuple buffer sized by the exact record count, once the link knows it
    S.rc = cly_scan_device_alloc_internal(S.ctx, S.df.data(), n, &S.d_tup, &S.cap, S.first.data(), S.res.data(), &S.need);
    S.t_scan = now_ms();
}
static void shard_free(LoadShard& S) {
    if (!S.d_bytes && !S.d_tup) return;
    if (hipSetDevice(S.dev) == hipSuccess) { hipFree(S.d_bytes); hipFree(S.d_tup); }
    S.d_bytes = nullptr; S.d_tup = nullptr;
}

extern "C" int cly_db_open_multi(cly_ctx* const* ctxs, int nctx, const char* dir, const cly_db_options* opt,
                                 cly_db** out, cly_load_stats* st) {
    if (!ctxs || nctx < 1 || nctx > LOAD_THREADS_MAX || !dir || !out) return CLY_ERR_ARG;
    for (int k = 0; k < nctx; k++) {
        if (!ctxs[k]) return CLY_ERR_ARG;
        for (int q = 0; q < k; q++) if (ctxs[q] == ctxs[k]) return CLY_ERR_ARG;   // one scan per context at a time
    }
    *out = nullptr;
    cly_ctx* ctx = ctxs[0];                      // the index is rebuilt on the first context
    cly_load_stats s;
    memset(&s, 0, sizeof(s));
    uint64_t dfs = opt && opt->data_file_size ? opt->data_file_size : (256ull << 20);
    if (dfs < 64) dfs = 64;                      // checkOptions (db.go:433-438)
    const bool apply = opt && (opt->flags & CLY_DB_APPLY_SWEEP);
    const double t0 = now_ms();
    cly_db* db = new cly_db();
    int rc = list_files(dir, db->files, db->fid_ix);
    const int nf = (int)db->files.size();
    const int dev0 = cly_ctx_device_internal(ctx);
    bool has_hint = false;
    int nall = 0;                                // hint (file 0 when present) + data files
    cly_tuple* d_tup = nullptr;                  // every tuple, in file order, on the first context's device
    bool own_tup = false;
    uint8_t* d_state = nullptr;
    cly_pos* d_hpos = nullptr;
    HostRec* d_hrec = nullptr;
    std::vector<cly_file> hf, df;
    std::vector<cly_file_result> res;
    std::vector<uint64_t> first;
    std::vector<LoadShard> sh(nctx);
    uint64_t need = 0;
    hipStream_t strm = cly_ctx_stream_internal(ctx);
    double t1, t2 = 0, t3, t4, t5;
    cly_index_result ir;
    if (rc != CLY_OK) goto done;
    {
        char path[4096];
        snprintf(path, sizeof(path), "%s/hint-index", dir);
        if (map_file(path, db->hint, has_hint) != CLY_OK) { rc = CLY_ERR_ARG; goto done; }
    }
    t1 = now_ms();
    s.list_map_ms = t1 - t0;
    s.n_files = (uint64_t)nf;
    nall = nf + (has_hint ? 1 : 0);
    hf.resize(nall);
    if (has_hint) { hf[0].base = db->hint.p; hf[0].len = db->hint.len; hf[0].fid = 0; hf[0]._pad = 0; }
    for (int i = 0; i < nf; i++) {
        cly_file& f = hf[i + (has_hint ? 1 : 0)];
        f.base = db->files[i].p; f.len = db->files[i].len; f.fid = db->files[i].fid; f._pad = 0;
        s.bytes += f.len;
    }
    {
        // contiguous file ranges balanced by bytes (each file weighs len + 4 KiB):
        // a file goes to the shard its weight's midpoint falls in; file 0 to
        // shard 0 (a single non-empty shard is then the first context's)
        uint64_t tot = 0, acc = 0;
        for (const cly_file& f : hf) tot += f.len + 4096;
        int f = 0;
        for (int k = 0; k < nctx; k++) {
            sh[k].ctx = ctxs[k];
            sh[k].dev = cly_ctx_device_internal(ctxs[k]);
            sh[k].f0 = f;
            const uint64_t target = tot / (uint64_t)nctx * (uint64_t)(k + 1) + (k + 1 == nctx ? tot : 0);
            while (f < nall && (f == 0 || acc + (hf[f].len + 4096) / 2 <= target)) acc += hf[f++].len + 4096;
            sh[k].f1 = f;
        }
        s.n_shards = 0;
        for (const LoadShard& S : sh) s.n_shards += S.f1 > S.f0;
    }
    if (nall) {
        // the shards in parallel, one host thread each (load_threads() copy
        // threads shared out), each on its own context's device and stream
        std::lock_guard<std::mutex> lk(g_stage_mu);
        const int nt = load_threads(), ntk = std::max(1, nt / (int)s.n_shards);
        std::vector<std::thread> th;
        int slot = 0;
        for (LoadShard& S : sh) {
            if (S.f1 == S.f0) continue;
            th.emplace_back(shard_load, std::ref(S), std::cref(hf), slot, ntk);
            slot += ntk;
        }
        for (auto& x : th) x.join();
        for (const LoadShard& S : sh) {
            if (S.f1 == S.f0) continue;
            if (S.rc != CLY_OK && rc == CLY_OK) rc = S.rc;
            t2 = std::max(t2, S.t_copy);
            s.tuple_slots += S.cap;
        }
        if (rc != CLY_OK) goto done;
    } else t2 = t1;
    s.h2d_ms = t2 - t1;
    // the shards' results in file order; their tuples gathered on the first
    // context's device (peer copies), whose index reads every shard's file bytes
    // in place (peer access when a shard is on another device)
    df.resize(nall); res.resize(nall); first.resize(nall);
    for (const LoadShard& S : sh) {
        for (int i = S.f0; i < S.f1; i++) {
            df[i] = S.df[i - S.f0];
            res[i] = S.res[i - S.f0];
            first[i] = need + S.first[i - S.f0];
        }
        need += S.need;
    }
    DCK(hipSetDevice(dev0));
    if (s.n_shards <= 1) {
        d_tup = sh[0].d_tup;
    } else {
        DCK(hipMalloc((void**)&d_tup, sizeof(cly_tuple) * (need + 16)));
        own_tup = true;
        uint64_t off = 0;
        for (const LoadShard& S : sh) {
            if (S.f1 == S.f0) continue;
            if (S.dev != dev0) {
                int can = 0;
                DCK(hipDeviceCanAccessPeer(&can, dev0, S.dev));
                if (!can) { rc = CLY_ERR_DEVICE; goto done; }
                const hipError_t e = hipDeviceEnablePeerAccess(S.dev, 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) { rc = CLY_ERR_DEVICE; goto done; }
                (void)hipGetLastError();
            }
            if (S.need) DCK(hipMemcpyPeerAsync(d_tup + off, dev0, S.d_tup, S.dev, sizeof(cly_tuple) * S.need, strm));
            off += S.need;
        }
    }
    // the errors in the reference's order: loadIndexFromHintFile first (its
    // loop: ReadLogRecord, then DecodeLogRecordPos of that record; merge.go:
    // 270-285), then loadIndex's merge-finished check (db.go:492-499), then
    // the data files in fid order
    if (has_hint) {
        db->n_hint = res[0].n_records;
        s.hint_records = db->n_hint;
        if (db->n_hint) {
            uint64_t bad = 0;
            DCK(hipMalloc((void**)&d_hpos, sizeof(cly_pos) * db->n_hint));
            rc = cly_hint_positions_device(ctx, df[0].base, d_tup, db->n_hint, d_hpos, &bad, nullptr);
            if (rc != CLY_OK) goto done;                                   // DecodeLogRecordPos panics
            hipLaunchKernelGGL(k_hint_as_put, dim3((unsigned)((db->n_hint + 255) / 256)), dim3(256), 0, strm, d_tup,
                               db->n_hint);
            DCK(hipGetLastError());
        }
        if (res[0].status < 0) { rc = res[0].status; goto done; }
    }
    if (nf) {
        rc = check_merge_finished(dir);          // (loadIndex returns early without data files)
        if (rc != CLY_OK) goto done;
    }
    for (int i = has_hint ? 1 : 0; i < nall; i++)
        if (res[i].status < 0) { rc = res[i].status; goto done; }         // loadIndex returns it
    if (nf) {
        s.active_fid_loaded = db->files[nf - 1].fid;
        s.write_off_loaded = res[nall - 1].end_offset;                    // db.go:632-634
    }
    DCK(hipStreamSynchronize(strm));
    t3 = now_ms();
    s.scan_ms = t3 - t2;
    DCK(hipMalloc((void**)&d_state, need ? need : 1));
    DCK(hipMalloc((void**)&d_hrec, sizeof(HostRec) * (need ? need : 1)));
    if (need) {
        hipLaunchKernelGGL(k_host_rec, dim3((unsigned)((need + 255) / 256)), dim3(256), 0, strm, d_tup, d_hrec, need);
        DCK(hipGetLastError());
        DCK(hipStreamSynchronize(strm));
    }
    db->recs.alloc(need);
    db->state.alloc(need);
    db->hint_pos.resize(db->n_hint);
    db->hmask = cly_ix_hash_mask_internal(need);
    db->hshift = 64 - __builtin_clzll(db->hmask | 15) - FLAT_SHARD_BITS;
    {
        // the host records (what lookups read) come back on copy threads nb..
        // from now on, beside the index rebuild and the tables' build on the
        // device and their read-back on threads 0 .. nb-1
        std::unique_lock<std::mutex> lk(g_stage_mu);
        const int nt = load_threads(), nb = std::max(1, nt / 2);
        int trc = CLY_OK;
        std::thread tcopy([&]() {
            if (need) trc = copy_to_host(ctx, {{db->recs.data(), d_hrec, sizeof(HostRec) * need}}, nb,
                                         std::max(1, nt - nb), false);
        });
        rc = flat_device(ctx, db, nall ? df.data() : nullptr, nall, d_tup, first, res, d_state, d_hpos, need, ir, nb, s);
        tcopy.join();
        if (rc == CLY_OK) rc = trc;
        if (rc != CLY_OK) goto done;
    }
    t4 = now_ms();
    s.index_ms = t4 - t3;
    s.records = need;
    {
        // MemTable inserts (updateIndex, db.go:511-575) for the records the
        // device marked as index entries: String / ListMeta are in the flat
        // tables already; Hash / List / Set go into realKey -> (field | seqBuf |
        // hashKey) maps
        std::vector<uint64_t> composite;
        composite_list(db, load_threads(), composite);
        for (uint64_t i : composite) {
            const HostRec& t = db->recs[i];
            const uint32_t dt = ST_DT(db->state[i]);
            // ixk_input: the stored key when applied at once (txId 0), else the realKey
            const uint32_t tl = hr_txl(t) == 0xFF ? 0u : hr_txl(t);
            const uint32_t off = hr_tx(t) ? tl : 0u, len = hr_tx(t) ? t.ks - tl : t.ks;
            const uint8_t* d = file_of(db, t.fid) + hr_off(t) + hr_hsz(t) + off;
            IxKey k;
            if (!ixk_key(dt, d, len, k)) continue;               // (the device rejected a panicking decode)
            cly_pos p;
            p.offset = (int64_t)hr_off(t); p.fid = t.fid; p._pad = 0;
            const uint8_t* r = d + k.r_off;
            if (dt == 1) {                       // realKey = R[0:la], field = R[la:]
                const uint32_t la = k.p[0] | ((uint32_t)k.p[1] << 8) | ((uint32_t)k.p[2] << 16) | ((uint32_t)k.p[3] << 24);
                db->hash[std::string((const char*)r, la)][std::string((const char*)r + la, k.r_len - la)] = p;
            } else if (dt == 2) {                // realKey = R, seqBuf = P[1:]
                db->list[std::string((const char*)r, k.r_len)][std::string((const char*)k.p + 1, k.plen - 1)] = p;
            } else {                             // realKey = R, hashKey = P
                db->set[std::string((const char*)r, k.r_len)][std::string((const char*)k.p, 4)] = p;
            }
        }
        // the per-key MemTables' fill order: keys ascending, subs ascending
        // inside a key (bytes.Compare; google/btree keeps the same order)
        const std::unordered_map<std::string, std::unordered_map<std::string, cly_pos>>* cm[3] = {&db->hash, &db->list,
                                                                                                   &db->set};
        for (int k = 0; k < 3; k++) {
            std::vector<cly_db_entry>& v = db->comp[k];
            v.clear();
            for (const auto& kv : *cm[k])
                for (const auto& sub : kv.second) {
                    cly_db_entry e;
                    memset(&e, 0, sizeof(e));
                    e.key = (const uint8_t*)kv.first.data(); e.key_len = kv.first.size();
                    e.sub = (const uint8_t*)sub.first.data(); e.sub_len = sub.first.size();
                    e.pos = sub.second;
                    v.push_back(e);
                }
            auto bcmp = [](const uint8_t* a, uint64_t na, const uint8_t* b, uint64_t nb) {
                const int c = memcmp(a, b, std::min(na, nb));
                return c ? c : (na < nb ? -1 : na > nb ? 1 : 0);
            };
            std::sort(v.begin(), v.end(), [&](const cly_db_entry& a, const cly_db_entry& b) {
                const int c = bcmp(a.key, a.key_len, b.key, b.key_len);
                return c ? c < 0 : bcmp(a.sub, a.sub_len, b.sub, b.sub_len) < 0;
            });
        }
        s.str_keys = db->str.n;
        s.listmeta_keys = db->listmeta.n;
        for (auto& kv : db->hash) s.hash_fields += kv.second.size();
        for (auto& kv : db->list) s.list_items += kv.second.size();
        for (auto& kv : db->set) s.set_members += kv.second.size();
    }
    {
        // the TTL sweep's db.Del (db.go:639-651, 186-215): a tombstone per swept
        // key appended by appendLogRecord's rule (db.go:368-413)
        for (uint64_t i = db->n_hint; i < need; i++)
            if (ST_STATE(db->state[i]) == CLY_IX_EXPIRED) db->expired.push_back(i);
        s.n_expired = db->expired.size();
        // db.Del refuses an empty key (db.go:186-188) and loadIndex returns
        // that error (db.go:646-649): the open fails (the reference may have
        // appended other keys' tombstones first, in Go map order; none here)
        for (uint64_t i : db->expired) {
            uint64_t kl;
            real_key_ptr(db, i, kl);
            if (kl == 0) { rc = CLY_ERR_KEY_EMPTY; goto done; }
        }
        uint32_t afid = s.active_fid_loaded;
        int64_t woff = s.write_off_loaded;
        int fd = -1;
        for (uint64_t i : db->expired) {
            uint64_t kl;
            const uint8_t* k = real_key_ptr(db, i, kl);
            const std::vector<uint8_t> rec = tombstone(k, kl);
            if ((uint64_t)woff + rec.size() > dfs) {                      // setActivityFile: fid + 1
                afid++; woff = 0; s.sweep_files++;
                if (fd >= 0) { close(fd); fd = -1; }
            }
            if (apply) {
                if (fd < 0) {
                    char path[4096];
                    snprintf(path, sizeof(path), "%s/%09u.cly", dir, afid);
                    fd = open(path, O_CREAT | O_RDWR | O_APPEND, 0644);    // driver/fileIO: O_APPEND
                    if (fd < 0) { rc = CLY_ERR_ARG; goto done; }
                }
                if (write(fd, rec.data(), rec.size()) != (ssize_t)rec.size()) { close(fd); rc = CLY_ERR_ARG; goto done; }
            }
            woff += (int64_t)rec.size();
        }
        if (fd >= 0) close(fd);
        s.active_fid = afid;
        s.write_off = woff;
    }
    t5 = now_ms();
    s.insert_ms = t5 - t4;
    s.total_ms = t5 - t0;
done:
    (void)hipSetDevice(dev0);
    if (own_tup) hipFree(d_tup);
    hipFree(d_state); hipFree(d_hpos); hipFree(d_hrec);
    for (LoadShard& S : sh) shard_free(S);
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

// getLogRecordByPos (db.go:680-704): the record at pos (ReadLogRecord, CRC
// included), its value; a LogRecordDeleted or an unknown fid is
// ErrKeyNotFound.
extern "C" int cly_db_value(cly_db* db, const cly_pos* pos, uint8_t* buf, uint64_t cap, uint64_t* vlen) {
    if (!db || !pos || !vlen) return CLY_ERR_ARG;
    *vlen = 0;
    const Mapped* m = nullptr;
    for (const Mapped& f : db->files) if (f.fid == pos->fid) m = &f;
    if (!m) return CLY_DB_NOT_FOUND;                                  // dataFile == nil
    if (pos->offset < 0) return CLY_ERR_OFFSET;                       // mmap ReadAt: invalid offset
    const Hdr h = host_read_record(m->p, m->len, pos->offset);
    if (h.status == CLY_END_EOF || h.status == CLY_END_ZERO || h.status == CLY_END_TORN) return CLY_DB_EOF;
    if (h.status != REC_OK) return h.status;                          // ErrInvalidCRC, the panics
    if (h.type == 1) return CLY_DB_NOT_FOUND;                         // LogRecordDeleted
    *vlen = h.vs;
    if (buf && cap >= h.vs) memcpy(buf, m->p + pos->offset + h.hsz + h.ks, h.vs);
    return (buf && cap < h.vs) ? CLY_ERR_CAPACITY : CLY_OK;
}

// ---------------------------------------------------------------------------
// Enumeration (cly_db_count / cly_db_entries), built on first use.
static void build_entries(cly_db* db, int kind) {
    std::vector<cly_db_entry>& v = db->it[kind];
    v.clear();
    // String / ListMeta: the device's key order (db->ord)
    auto ordered = [&](int k, bool str) {
        v.reserve(db->n_ord[k]);
        for (uint64_t j = 0; j < db->n_ord[k]; j++) {
            const uint64_t ti = db->ord[k][j];
            cly_db_entry e;
            memset(&e, 0, sizeof(e));
            e.key = real_key_ptr(db, ti, e.key_len);
            e.pos = pos_of(db, ti);
            e.expiration = str && ti >= db->n_hint ? db->recs[ti].exp : 0;
            v.push_back(e);
        }
    };
    switch (kind) {
        case CLY_IT_STRING: ordered(0, true); break;
        case CLY_IT_LISTMETA: ordered(1, false); break;
        case CLY_IT_HASH: v = db->comp[0]; break;
        case CLY_IT_LIST: v = db->comp[1]; break;
        case CLY_IT_SET: v = db->comp[2]; break;
        case CLY_IT_EXPIRED:
            for (uint64_t i : db->expired) {
                cly_db_entry e;
                memset(&e, 0, sizeof(e));
                e.key = real_key_ptr(db, i, e.key_len);
                e.pos = pos_of(db, i);
                e.expiration = db->recs[i].exp;
                v.push_back(e);
            }
            break;
    }
    db->it_built[kind] = true;
}
extern "C" uint64_t cly_db_count(cly_db* db, int kind) {
    if (!db || kind < 0 || kind > CLY_IT_EXPIRED) return 0;
    if (!db->it_built[kind]) build_entries(db, kind);
    return db->it[kind].size();
}
extern "C" uint64_t cly_db_entries(cly_db* db, int kind, uint64_t first, cly_db_entry* out, uint64_t n) {
    if (!db || !out || kind < 0 || kind > CLY_IT_EXPIRED) return 0;
    if (!db->it_built[kind]) build_entries(db, kind);
    const std::vector<cly_db_entry>& v = db->it[kind];
    uint64_t k = 0;
    for (; k < n && first + k < v.size(); k++) out[k] = v[first + k];
    return k;
}
