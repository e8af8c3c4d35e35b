// clyindex.hip — db.loadIndex's index rebuild on the device (gfx950), part of
// libclyscan.so (C-ABI: cly_index_device in include/clyscan.h).
//
// Reference (db.go:511-637): every record of the scan, in fid/offset order,
// goes through parseLogRecordKey (db.go:706-710); a record without a txId is
// applied to the index at once (updateIndex, db.go:511-575); a record with a
// txId is buffered until a TxnCommit marker of that txId applies the buffer in
// order (a TxnRollback marker drops it, TxnBegin is ignored).  For the String
// and ListMeta indexes the key is realKey itself; Hash/List/Set keys are
// composite (decodeFieldKey, decodeListKey + the big.Float gob re-encoding,
// hashMemberKey's CRC): ixkey.h derives them as (kind, P, R).  The last applied
// record of a key decides, Put -> index[key] = (fid, offset), Deleted -> key
// absent.  A winner whose key merge.go would look up differently (a Hash/List/
// Set record without a txId: loadIndex decodes its stored key, merge its
// realKey) is CLY_IX_LOADONLY: indexed, but not rewritten by a merge.
//
// Device pipeline:
//   k_ixclass   per record: class (applied now / tx data / tx marker / host / none)
//   select + radix sort of the tx records by txId (stable: scan order kept)
//   k_ixtx      per tx record: its next marker in the same txId (segmented
//               suffix scan), a committed data record is applied at its marker
//   select + keys-only radix sort of the applied records' packed keys (ix_pk:
//   hb hash bits | tombstone | record index; 8 B per record and pass)
//   segmented arg-max of the application order per hash group: the winner of
//   each key (k_ixwin); adjacent records of a group with different keys (a
//   hash collision) list the group for an exact one-thread resolution (k_ixcoll)
//   k_ixwinfix  the winners' final states from the flags k_ixclass kept
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_segmented_radix_sort.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "scan_core.h"
#include "ixkey.h"

extern "C" hipStream_t cly_ctx_stream_internal(cly_ctx* c);
extern "C" int64_t cly_ctx_now_internal(cly_ctx* c);
extern "C" int cly_ctx_device_internal(cly_ctx* c);
extern "C" hipError_t cly_ix_scratch_internal(cly_ctx* ctx, int k, size_t bytes, void** out);

#define IX_NONE 0xFFFFFFFFFFFFFFFFull
// record index of a hash-sorted entry: bit 31 carries "LogRecordDeleted" so that
// the winner's type needs no second (random) read of its tuple
#define IX_DEL 0x80000000u
#define IX_WIN 7                     // a key's winner, its final state not yet decided (k_ixwinfix)
#define IXI(x) ((x) & 0x7fffffffu)
enum { K_NONE = 0, K_APPLY = 1, K_TXDATA = 2, K_COMMIT = 3, K_ROLLBACK = 4 };

__device__ __forceinline__ int ix_file(const uint64_t* first, int nfiles, uint64_t i) {
    int lo = 0, hi = nfiles - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (first[mid] <= i) lo = mid; else hi = mid - 1;
    }
    return lo;
}
// realKey of tuple t (parseLogRecordKey: key[n:], n = 0 for a short varint)
__device__ __forceinline__ const uint8_t* ix_rkey(const uint64_t* bases, int f, const cly_tuple& t, uint32_t& len) {
    len = t.key_size - t.txid_len;
    return (const uint8_t*)bases[f] + t.offset + t.header_size + t.txid_len;
}
// 64-bit hash of (index, key): ixkey.h's ixk_hash
__device__ __forceinline__ uint64_t ix_hash(uint32_t index_kind, const uint8_t* k, uint32_t len) {
    return ixk_hash(index_kind, k, len);
}

// Key signature (16 B): the first min(len, 15) realKey bytes, zero-padded, and
// in byte 15 the length (len <= 15) or 0x80 (longer), with the data type in
// bits 4-6.  Injective for keys of <= 15 bytes, so two such records name the
// same key iff their signatures are equal; equal signatures of longer keys
// still need the byte comparison.  k_ixwin reads one 16-B signature per sorted
// record instead of two tuples and two keys.
#define IX_SIG_LONG 0x80u
// ix_hash and the signature together.  A key of <= 15 bytes comes in as at most
// five aligned dword loads (none past the dword of its last byte) joined by
// alignbyte; the hash is ix_hash's, computed from those words.
__device__ __forceinline__ uint64_t ix_hash_sig(uint32_t kind, const uint8_t* k, uint32_t len, uint4& sig) {
    uint32_t v[4];
    uint64_t h;
    if (len <= 15) {
        const uintptr_t a = (uintptr_t)k;
        const uint32_t* base = (const uint32_t*)(a & ~(uintptr_t)3);
        const uint32_t sh = (uint32_t)(a & 3);
        const uint32_t nd = (sh + len + 3) >> 2;
        uint32_t d[5];
        #pragma unroll
        for (int j = 0; j < 5; j++) d[j] = (uint32_t)j < nd ? base[j] : 0u;
        #pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t w = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh);
            const uint32_t lo = 4u * i;
            const uint32_t m = len >= lo + 4 ? 0xffffffffu : (len <= lo ? 0u : (1u << (8 * (len - lo))) - 1u);
            v[i] = w & m;
        }
        h = 0xcbf29ce484222325ull ^ ((uint64_t)kind << 56) ^ len;
        uint64_t tail = v[0] | ((uint64_t)v[1] << 32);
        if (len >= 8) {
            h = (h ^ tail) * 0x100000001b3ull;
            h ^= h >> 29;
            tail = v[2] | ((uint64_t)v[3] << 32);
        }
        h = (h ^ tail) * 0x100000001b3ull;
        h ^= h >> 32;
        h *= 0xd6e8feb86659fd93ull;
        h ^= h >> 32;
    } else {
        h = ix_hash(kind, k, len);
        #pragma unroll
        for (int i = 0; i < 4; i++)
            v[i] = k[4 * i] | ((uint32_t)k[4 * i + 1] << 8) | ((uint32_t)k[4 * i + 2] << 16) |
                   (i < 3 ? (uint32_t)k[4 * i + 3] << 24 : 0u);
    }
    sig = make_uint4(v[0], v[1], v[2], v[3] | (((len <= 15 ? len : IX_SIG_LONG) | ((kind & 7u) << 4)) << 24));
    return h;
}
__device__ __forceinline__ bool ix_sig_long(const uint4& s) { return (s.w >> 24) & IX_SIG_LONG; }

__device__ __forceinline__ bool ix_composite(uint32_t dt) { return dt == 1 || dt == 2 || dt == 4; }
// the key bytes of tuple t as stored
__device__ __forceinline__ const uint8_t* ix_key_bytes(const uint64_t* bases, int f, const cly_tuple& t) {
    return (const uint8_t*)bases[f] + t.offset + t.header_size;
}
// the index key of a Hash/List/Set record (ixkey.h) under loadIndex's decode
// (merge = false) or merge.go's (merge = true)
__device__ __forceinline__ bool ix_ckey(const uint64_t* bases, int f, const cly_tuple& t, bool merge, IxKey& k,
                                        const uint8_t*& d) {
    uint32_t off, len;
    ixk_input(t, off, len, merge);
    d = ix_key_bytes(bases, f, t) + off;
    ixk_key(t.data_type, d, len, k);
    return !k.panic;
}
__device__ __forceinline__ bool ix_ckey_eq(const IxKey& a, const uint8_t* da, const IxKey& b, const uint8_t* db) {
    if (a.kind != b.kind || a.plen != b.plen || a.r_len != b.r_len) return false;
    for (uint32_t q = 0; q < a.plen; q++) if (a.p[q] != b.p[q]) return false;
    for (uint32_t q = 0; q < a.r_len; q++) if (da[a.r_off + q] != db[b.r_off + q]) return false;
    return true;
}
// hash and signature of a composite key: ix_hash of R folded with P; the
// signature is never injective (IX_SIG_LONG): equal ones are compared exactly
__device__ __forceinline__ uint64_t ix_hash_ckey(const IxKey& k, const uint8_t* d, uint4& sig) {
    uint64_t h = ix_hash(k.kind, d + k.r_off, k.r_len);
    uint32_t pw[5] = {0, 0, 0, 0, 0};
    for (uint32_t q = 0; q < k.plen; q++) pw[q >> 2] |= (uint32_t)k.p[q] << (8 * (q & 3));
    #pragma unroll
    for (int j = 0; j < 5; j += 2) {
        const uint64_t w = pw[j] | (j + 1 < 5 ? (uint64_t)pw[j + 1] << 32 : 0ull);
        h = (h ^ w ^ ((uint64_t)k.plen << 58)) * 0x100000001b3ull;
        h ^= h >> 29;
    }
    h *= 0xd6e8feb86659fd93ull;
    h ^= h >> 32;
    sig = make_uint4(pw[0], pw[1], k.r_len, (pw[2] & 0xffffffu) | ((IX_SIG_LONG | ((k.kind & 7u) << 4)) << 24));
    return h;
}

__device__ __forceinline__ bool ix_expired(const cly_tuple& t, int64_t now_ns) {
    return t.data_type == 0 && t.expiration != 0 && t.expiration <= now_ns;
}
// flags of an applied record (its del byte): what a winner's final state needs
// of its tuple, so that k_ixwinfix reads bytes in scan order instead of tuples
#define IXF_DEL 1u          // LogRecordDeleted
#define IXF_EXP 2u          // a String put expired at the context's clock (TTL sweep)
#define IXF_CHK 4u          // Hash/List/Set without a txId: ix_win_state compares the two decodes
// hash, signature and flags of applied record i; returns the tombstone bit
__device__ __forceinline__ bool ix_apply_one(const cly_tuple& t, uint64_t i, const uint64_t* first,
                                             const uint64_t* bases, int nfiles, uint64_t* hash, uint8_t* del,
                                             uint4* ksig, uint64_t hash_mask, uint32_t* bad, int64_t now_ns) {
    const int f = ix_file(first, nfiles, i);
    uint4 sg;
    if (ix_composite(t.data_type)) {
        IxKey k;
        const uint8_t* d;
        if (!ix_ckey(bases, f, t, false, k, d)) atomicOr(bad, 2u);     // updateIndex's decode panics
        hash[i] = ix_hash_ckey(k, d, sg) & hash_mask;
    } else {
        uint32_t len;
        const uint8_t* k = ix_rkey(bases, f, t, len);
        hash[i] = ix_hash_sig(t.data_type, k, len, sg) & hash_mask;
    }
    const bool dl = t.type == 1;
    del[i] = (dl ? IXF_DEL : 0u) | (ix_expired(t, now_ns) ? IXF_EXP : 0u) |
             (ix_composite(t.data_type) && t.tx_id == 0 && t.txid_len != 0 ? IXF_CHK : 0u);
    ksig[i] = sg;
    return dl;
}

// Sort key of an applied record (one u64, sorted keys-only): hb bits of its
// key hash above the tombstone bit and ib bits of its record index, so that
// the radix sort moves 8 B per record and pass and sorts only the hb hash bits
// (stable: scan order inside a hash group).  hb is narrower than the table
// hash (ix_hash_mask): equal sort hashes of different keys are collisions,
// which k_ixwin detects from the key signatures and k_ixcoll resolves exactly.
__device__ __forceinline__ uint64_t ix_pk(uint64_t hash, uint32_t i, bool del, uint32_t ib, uint32_t hb) {
    return ((hash & ((1ull << hb) - 1)) << (ib + 1)) | ((uint64_t)del << ib) | i;
}
__device__ __forceinline__ uint64_t ix_pk_h(uint64_t pk, uint32_t ib) { return pk >> (ib + 1); }
// the record index with IX_DEL, as the selection values before
__device__ __forceinline__ uint32_t ix_pk_s(uint64_t pk, uint32_t ib) {
    return (uint32_t)(pk & ((1ull << ib) - 1)) | (((pk >> ib) & 1) ? IX_DEL : 0u);
}
// application order of record i: scan order for a record without a txId
// (k_ixclass writes none), its commit marker's position for a tx data record
__device__ __forceinline__ uint64_t ix_order(const uint8_t* cls, const uint64_t* order, uint32_t i) {
    return cls[i] == 1 /* K_APPLY */ ? ((uint64_t)i << 32) | i : order[i];
}

struct IxTot { unsigned long long n_live, n_applied, n_loadonly, n_coll, n_tx, n_now, n_mpanic, n_chead; uint32_t bad, _pad; };

// sum of a and b over the workgroup (256 threads), one atomic per counter
__device__ __forceinline__ void ix_wg_add2(unsigned long long a, unsigned long long b, unsigned long long* da,
                                           unsigned long long* db) {
    __shared__ unsigned long long sh[2][4];
    for (int d = 32; d >= 1; d >>= 1) { a += __shfl_xor(a, d, 64); b += __shfl_xor(b, d, 64); }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sh[0][w] = a; sh[1][w] = b; }
    __syncthreads();
    if (threadIdx.x < 2) {
        const unsigned long long v = sh[threadIdx.x][0] + sh[threadIdx.x][1] + sh[threadIdx.x][2] + sh[threadIdx.x][3];
        if (v) atomicAdd(threadIdx.x == 0 ? da : db, v);
    }
}

// class of each record (every data type 0..4 is indexed; others: no-op)
__global__ void __launch_bounds__(256)
k_ixclass(const cly_tuple* __restrict__ tup, uint64_t n, uint8_t* cls, uint8_t* state, uint8_t* txflag, IxTot* tot,
          const uint64_t* __restrict__ first, const uint64_t* __restrict__ bases, int nfiles, uint64_t* hash,
          uint8_t* apflag, uint8_t* del, uint4* ksig, uint64_t* pk, uint64_t hash_mask, uint32_t ib, uint32_t hb,
          int64_t now_ns) {
    unsigned long long ntx = 0, nnow = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const cly_tuple t = tup[i];
        uint8_t c = K_NONE;
        if (t.txid_len == 0xFF) atomicOr(&tot->bad, 1u);          // parseLogRecordKey panics
        const bool idx = t.data_type <= 4;                         // String Hash List ListMeta Set
        if (t.tx_id == 0) {                                        // updateIndex at once
            if (idx) c = K_APPLY;
        } else if (t.type == 2) c = K_COMMIT;                      // LogRecordTxnCommit
        else if (t.type == 3) c = K_ROLLBACK;                      // LogRecordTxnRollback
        else if (t.type != 4 && idx) c = K_TXDATA;                 // buffered (Begin ignored)
        // merge.go:101-126 decodes every Hash/List/Set record's realKey
        if (ix_composite(t.data_type) && t.txid_len != 0xFF) {
            IxKey k;
            const uint8_t* d;
            if (!ix_ckey(bases, ix_file(first, nfiles, i), t, true, k, d)) atomicAdd(&tot->n_mpanic, 1ull);
        }
        cls[i] = c;
        state[i] = CLY_IX_DEAD;
        const bool tx = c == K_TXDATA || c == K_COMMIT || c == K_ROLLBACK;
        txflag[i] = tx;
        ntx += tx;
        nnow += c == K_APPLY;
        // a record without a txId is applied now: order = scan order (implicit,
        // ix_order), its hash, signature and tombstone bit come from this same
        // pass over the tuples
        if (c == K_APPLY) {
            const bool dl = ix_apply_one(t, i, first, bases, nfiles, hash, del, ksig, hash_mask, &tot->bad, now_ns);
            pk[i] = ix_pk(hash[i], (uint32_t)i, dl, ib, hb);
        }
        apflag[i] = c == K_APPLY;
    }
    ix_wg_add2(ntx, nnow, &tot->n_tx, &tot->n_now);
}

// per tx record (sorted by txId, scan order within): element of the segmented
// suffix scan = (txId, position of the nearest marker at or after it)
struct TxNext { uint64_t tx; uint64_t mpos; };
struct TxNextOp {
    __device__ __forceinline__ TxNext operator()(const TxNext& a, const TxNext& b) const {
        // a precedes b in scan order (the scan runs backwards over the sorted records)
        if (b.tx != a.tx) return b;
        return TxNext{b.tx, b.mpos != IX_NONE ? b.mpos : a.mpos};
    }
};
__global__ void __launch_bounds__(256)
k_ixtxin(const uint64_t* __restrict__ stx, const uint32_t* __restrict__ sidx, const uint8_t* __restrict__ cls,
         uint64_t m, TxNext* rev) {
    for (uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x; p < m; p += (uint64_t)gridDim.x * 256) {
        const uint32_t i = sidx[p];
        const uint8_t c = cls[i];
        rev[m - 1 - p] = TxNext{stx[p], (c == K_COMMIT || c == K_ROLLBACK) ? p : IX_NONE};
    }
}
// committed tx data records get their application order (marker position, own position)
__global__ void __launch_bounds__(256)
k_ixtx(const uint32_t* __restrict__ sidx, const uint8_t* __restrict__ cls, uint64_t m, const TxNext* __restrict__ nxt,
       uint64_t* order, uint8_t* state) {
    for (uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x; p < m; p += (uint64_t)gridDim.x * 256) {
        const uint32_t i = sidx[p];
        const uint8_t c = cls[i];
        if (c != K_TXDATA) continue;
        const uint64_t mp = nxt[m - 1 - p].mpos;
        const bool committed = mp != IX_NONE && cls[sidx[mp]] == K_COMMIT;
        if (committed) order[i] = ((uint64_t)sidx[mp] << 32) | i;
    }
}
// applied records (now and at commit): order, hash
__global__ void __launch_bounds__(256)
k_ixapply(const cly_tuple* __restrict__ tup, uint64_t n, const uint8_t* __restrict__ cls,
          const uint64_t* __restrict__ order, const uint64_t* __restrict__ first, const uint64_t* __restrict__ bases,
          int nfiles, uint64_t* hash, uint8_t* apflag, uint8_t* del, uint4* ksig, uint64_t hash_mask,
          uint32_t* bad, int64_t now_ns) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        if (cls[i] != K_TXDATA || order[i] == IX_NONE) continue;   // K_APPLY: done by k_ixclass
        ix_apply_one(tup[i], i, first, bases, nfiles, hash, del, ksig, hash_mask, bad, now_ns);
        apflag[i] = 1;
    }
}
// arg-max of the order per hash group (segmented, forward)
struct GMax { uint64_t h; uint64_t order; uint32_t idx; uint32_t head; };
struct GMaxOp {
    __device__ __forceinline__ GMax operator()(const GMax& a, const GMax& b) const {
        if (b.h != a.h) return b;
        return b.order > a.order ? b : GMax{b.h, a.order, a.idx, a.head};
    }
};
__global__ void __launch_bounds__(256)
k_ixgin(const uint64_t* __restrict__ spk, uint32_t ib, const uint8_t* __restrict__ cls,
        const uint64_t* __restrict__ order, uint64_t m, GMax* g) {
    for (uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x; q < m; q += (uint64_t)gridDim.x * 256) {
        const uint64_t v = spk[q];
        const uint32_t i = IXI(ix_pk_s(v, ib));
        g[q] = GMax{ix_pk_h(v, ib), ix_order(cls, order, i), i, (uint32_t)q};
    }
}
__device__ __forceinline__ bool ix_same_key(const cly_tuple* tup, const uint64_t* first, const uint64_t* bases,
                                            int nfiles, uint32_t a, uint32_t b) {
    const cly_tuple ta = tup[a], tb = tup[b];
    if (ta.data_type != tb.data_type) return false;
    if (ix_composite(ta.data_type)) {
        IxKey x, y;
        const uint8_t *dx, *dy;
        ix_ckey(bases, ix_file(first, nfiles, a), ta, false, x, dx);
        ix_ckey(bases, ix_file(first, nfiles, b), tb, false, y, dy);
        return ix_ckey_eq(x, dx, y, dy);
    }
    uint32_t la, lb;
    const uint8_t* ka = ix_rkey(bases, ix_file(first, nfiles, a), ta, la);
    const uint8_t* kb = ix_rkey(bases, ix_file(first, nfiles, b), tb, lb);
    if (la != lb) return false;
    for (uint32_t q = 0; q < la; q++) if (ka[q] != kb[q]) return false;
    return true;
}
// state of a key's winner w: LIVE, or LOADONLY when merge.go's lookup (the
// realKey decoded, merge.go:101-126) names another key than loadIndex's (the
// stored key decoded, for a Hash/List/Set record without a txId)
__device__ __forceinline__ uint8_t ix_win_state(const cly_tuple* tup, const uint64_t* first, const uint64_t* bases,
                                                int nfiles, uint32_t w) {
    const cly_tuple t = tup[w];
    if (!ix_composite(t.data_type) || t.tx_id != 0 || t.txid_len == 0) return CLY_IX_LIVE;
    const int f = ix_file(first, nfiles, w);
    IxKey x, y;
    const uint8_t *dx, *dy;
    ix_ckey(bases, f, t, false, x, dx);
    if (!ix_ckey(bases, f, t, true, y, dy)) return CLY_IX_LOADONLY;
    return ix_ckey_eq(x, dx, y, dy) ? CLY_IX_LIVE : CLY_IX_LOADONLY;
}
// group ends: the winner (max order) decides the key; adjacent different keys
// inside a group mark a hash collision (resolved exactly by k_ixcoll)
__global__ void __launch_bounds__(256)
k_ixwin(const uint64_t* __restrict__ spk, uint32_t ib, const GMax* __restrict__ g, uint64_t m,
        const cly_tuple* __restrict__ tup, const uint64_t* __restrict__ first, const uint64_t* __restrict__ bases,
        int nfiles, const uint4* __restrict__ ksig, uint8_t* state, uint8_t* coll, uint32_t* heads, IxTot* tot) {
    unsigned long long ncoll = 0;
    const int lane = threadIdx.x & 63;
    // whole waves over consecutive entries: an entry loads its signature once
    // (when a neighbour shares its hash) and the next lane takes it by shuffle
    for (uint64_t qw = (uint64_t)blockIdx.x * 256 + (threadIdx.x & ~63u); qw < m; qw += (uint64_t)gridDim.x * 256) {
        const uint64_t q = qw + lane;
        const bool in = q < m;
        uint64_t vq = 0, hq = 0;
        bool eqL = false, eqR = false;
        if (in) {
            vq = spk[q];
            hq = ix_pk_h(vq, ib);
            eqL = q > 0 && ix_pk_h(spk[q - 1], ib) == hq;
            eqR = q + 1 < m && ix_pk_h(spk[q + 1], ib) == hq;
        }
        uint4 sa = make_uint4(0, 0, 0, 0);
        if (eqL || eqR) sa = ksig[IXI(ix_pk_s(vq, ib))];
        uint4 sb;
        sb.x = __shfl_up(sa.x, 1, 64);
        sb.y = __shfl_up(sa.y, 1, 64);
        sb.z = __shfl_up(sa.z, 1, 64);
        sb.w = __shfl_up(sa.w, 1, 64);
        // a collided group's head is listed once (the first differing entry to
        // set its coll byte) for k_ixcoll
        bool push = false;
        uint64_t h0 = 0;
        if (in) {
            if (lane == 0 && eqL) sb = ksig[IXI(ix_pk_s(spk[q - 1], ib))];
            bool differ = false;
            if (eqL) {
                differ = sa.x != sb.x || sa.y != sb.y || sa.z != sb.z || sa.w != sb.w;
                if (!differ && ix_sig_long(sa))
                    differ = !ix_same_key(tup, first, bases, nfiles, IXI(ix_pk_s(vq, ib)), IXI(ix_pk_s(spk[q - 1], ib)));
            }
            if (differ) {
                h0 = q;
                while (h0 > 0 && ix_pk_h(spk[h0 - 1], ib) == hq) h0--;
                const uint32_t bit = 1u << (8 * (h0 & 3));
                push = !(atomicOr((uint32_t*)(coll + (h0 & ~3ull)), bit) & bit);
                ncoll++;
            }
            // the group's last entry decides (g == nullptr: no tx record was
            // applied, so the application order is the scan order, which the
            // stable sort keeps inside a group: the last wins)
            if (!eqR) {
                const uint32_t sq = ix_pk_s(vq, ib);
                const uint32_t w = g ? g[q].idx : IXI(sq);
                const bool deleted = g ? tup[w].type == 1 : (sq & IX_DEL) != 0;
                // LogRecordDeleted -> key absent; a String key whose winning put expired is
                // db.Del'd by loadIndex's TTL sweep (db.go:639-651: not exp.After(now))
                // (the winner's final state from its flags: k_ixwinfix, in scan order;
                // random byte stores: a bitmap of atomicOr measured 2x slower)
                if (!deleted) state[w] = IX_WIN;
            }
        }
        const uint64_t bm = __ballot(push);
        if (bm) {
            const int l0 = __builtin_ctzll(bm);
            uint32_t base = 0;
            if (lane == l0) base = (uint32_t)atomicAdd(&tot->n_chead, (unsigned long long)__popcll(bm));
            base = __shfl(base, l0, 64);
            if (push) heads[base + __popcll(bm & ((1ull << lane) - 1))] = (uint32_t)h0;
        }
    }
    // one atomic per wave (a collision per record of a narrow hash is common)
    for (int d = 32; d >= 1; d >>= 1) ncoll += __shfl_xor(ncoll, d, 64);
    if ((threadIdx.x & 63) == 0 && ncoll) atomicAdd(&tot->n_coll, ncoll);
}
// the winners' states (LIVE, LOADONLY or EXPIRED) in scan order: the tuples
// read as consecutive runs instead of one line per sorted winner
__global__ void __launch_bounds__(256)
k_ixwinfix(const cly_tuple* __restrict__ tup, uint64_t n, const uint64_t* __restrict__ first,
           const uint64_t* __restrict__ bases, int nfiles, const uint8_t* __restrict__ flg, uint8_t* state) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        if (state[i] != IX_WIN) continue;
        const uint32_t f = flg[i];
        state[i] = (f & IXF_EXP) ? (uint8_t)CLY_IX_EXPIRED
                 : (f & IXF_CHK) ? ix_win_state(tup, first, bases, nfiles, (uint32_t)i) : (uint8_t)CLY_IX_LIVE;
    }
}
// exact resolution of a collided hash group (one thread): per distinct key the max order
__global__ void __launch_bounds__(256)
k_ixcoll(const uint64_t* __restrict__ spk, uint32_t ib, const uint8_t* __restrict__ cls,
         const uint64_t* __restrict__ order, uint64_t m,
         const cly_tuple* __restrict__ tup, const uint64_t* __restrict__ first, const uint64_t* __restrict__ bases,
         int nfiles, const uint4* __restrict__ ksig, const uint64_t* __restrict__ hash, const uint8_t* __restrict__ flg,
         uint8_t* state, const uint32_t* __restrict__ heads, uint64_t nheads) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= nheads) return;
    const uint64_t q0 = heads[t];
    const uint64_t h0 = ix_pk_h(spk[q0], ib);
    uint64_t q1 = q0 + 1;
    while (q1 < m && ix_pk_h(spk[q1], ib) == h0) q1++;
    for (uint64_t a = q0; a < q1; a++) state[IXI(ix_pk_s(spk[a], ib))] = CLY_IX_DEAD;
    for (uint64_t a = q0; a < q1; a++) {
        const uint32_t ia = IXI(ix_pk_s(spk[a], ib));
        const uint64_t oa = ix_order(cls, order, ia);
        const uint4 sa = ksig[ia];
        bool best = true;
        for (uint64_t b = q0; b < q1 && best; b++) {
            const uint32_t ibb = IXI(ix_pk_s(spk[b], ib));
            if (b == a || ix_order(cls, order, ibb) <= oa) continue;
            // same key: equal signatures (exact for keys of <= 15 bytes), else
            // equal table hashes and the bytes
            const uint4 sb = ksig[ibb];
            if (sa.x != sb.x || sa.y != sb.y || sa.z != sb.z || sa.w != sb.w) continue;
            if (!ix_sig_long(sa) || (hash[ia] == hash[ibb] && ix_same_key(tup, first, bases, nfiles, ia, ibb)))
                best = false;
        }
        const uint32_t f = flg[ia];
        if (best && !(f & IXF_DEL))
            state[ia] = (f & IXF_EXP) ? (uint8_t)CLY_IX_EXPIRED
                      : (f & IXF_CHK) ? ix_win_state(tup, first, bases, nfiles, ia) : (uint8_t)CLY_IX_LIVE;
    }
}
// counts: one atomic per workgroup and counter (a wave-level atomic on one
// address from every wave serialises in L2)
__global__ void __launch_bounds__(256)
k_ixcount(const uint8_t* __restrict__ state, const uint8_t* __restrict__ flag, uint64_t n, IxTot* tot) {
    __shared__ unsigned long long sh[3][4];
    unsigned long long live = 0, host = 0, ap = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        live += state[i] == CLY_IX_LIVE || state[i] == CLY_IX_LOADONLY;
        host += state[i] == CLY_IX_LOADONLY;
        ap += flag[i];
    }
    for (int d = 32; d >= 1; d >>= 1) {
        live += __shfl_xor(live, d, 64);
        host += __shfl_xor(host, d, 64);
        ap += __shfl_xor(ap, d, 64);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sh[0][w] = live; sh[1][w] = host; sh[2][w] = ap; }
    __syncthreads();
    if (threadIdx.x < 3) {
        const unsigned long long v = sh[threadIdx.x][0] + sh[threadIdx.x][1] + sh[threadIdx.x][2] + sh[threadIdx.x][3];
        unsigned long long* dst = threadIdx.x == 0 ? &tot->n_live : threadIdx.x == 1 ? &tot->n_loadonly : &tot->n_applied;
        if (v) atomicAdd(dst, v);
    }
}

// the txIds of the selected tx records
__global__ void __launch_bounds__(256)
k_ixgathertx(const cly_tuple* __restrict__ tup, const uint32_t* __restrict__ sel, uint64_t m, uint64_t* dst) {
    for (uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x; p < m; p += (uint64_t)gridDim.x * 256)
        dst[p] = (uint64_t)tup[sel[p]].tx_id;
}
// sort keys of the selected applied records
__global__ void __launch_bounds__(256)
k_ixgatherd(const uint64_t* __restrict__ hash, const uint32_t* __restrict__ sel, const uint8_t* __restrict__ del,
            uint64_t m, uint64_t* dst, uint32_t ib, uint32_t hb) {
    for (uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x; p < m; p += (uint64_t)gridDim.x * 256) {
        const uint32_t i = sel[p];
        dst[p] = ix_pk(hash[i], i, (del[i] & IXF_DEL) != 0, ib, hb);
    }
}

// ---------------------------------------------------------------------------
#define ICK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "clyindex: %s failed: %s\n", #x, hipGetErrorString(e_)); rc = CLY_ERR_DEVICE; goto done; } } while (0)

// The key hash keeps hbits = log2(n) + 24 bits (multiple of 8, 32..64):
// expected colliding pairs n^2 / 2^(hbits+1) <= 2^-25 n stay ~0, and the radix
// sort makes hbits/8 passes instead of 8.  Test hook: CLY_IX_HASH_MASK (hex)
// narrows the hash so that collisions (resolved exactly by k_ixcoll) are common.
static uint64_t ix_hash_mask(uint64_t n, int& hbits) {
    int lg = 0;
    while (lg < 63 && (1ull << lg) < n) lg++;
    hbits = (lg + 24 + 7) & ~7;
    if (hbits < 32) hbits = 32;
    if (hbits > 64) hbits = 64;
    uint64_t hm = hbits == 64 ? ~0ull : (1ull << hbits) - 1;
    const char* e = getenv("CLY_IX_HASH_MASK");
    if (e && *e) { hm = strtoull(e, nullptr, 16); hbits = hm ? 64 - __builtin_clzll(hm) : 1; }
    return hm;
}
extern "C" uint64_t cly_ix_hash_mask_internal(uint64_t n) { int hb; return ix_hash_mask(n, hb); }
// Sort-key geometry (ix_pk): ib = ceil(log2 n) index bits, hb = log2(n) + 8
// hash bits (at most 63 - ib, at most the table hash's width): expected
// colliding pairs n^2 / 2^(hb+1) <= n / 512, each resolved exactly; the radix
// sort makes ceil(hb / 8) passes of 8 B per record (C4: 5 passes, before 7
// passes of a 12-B key-value pair).
static void ix_pk_bits(uint64_t n, int hbits, uint32_t& ib, uint32_t& hb) {
    int lg = 0;
    while (lg < 63 && (1ull << lg) < n) lg++;
    ib = lg ? (uint32_t)lg : 1u;
    int h = lg + 8;
    if (h > 63 - (int)ib) h = 63 - (int)ib;
    if (h > hbits) h = hbits;
    hb = (uint32_t)h;
}
// The device buffer of the key hashes of the last cly_index_device call of
// this context (n values: the records applied to an index; others undefined).
extern "C" hipError_t cly_ix_hash_ptr_internal(cly_ctx* ctx, uint64_t n, void** out) {
    return cly_ix_scratch_internal(ctx, 13, sizeof(uint64_t) * n, out);
}

static unsigned ix_grid(uint64_t n) { const uint64_t b = (n + 255) / 256; return (unsigned)(b < 16384 ? (b ? b : 1) : 16384); }

extern "C" int cly_index_device(cly_ctx* ctx, const cly_file* files, int nfiles, const cly_tuple* d_tuples,
                                const uint64_t* file_first, const cly_file_result* res, uint8_t* d_state,
                                cly_index_result* ir, void* stream_v) {
    if (!ctx || !ir || nfiles < 0 || (nfiles && (!files || !file_first || !res))) return CLY_ERR_ARG;
    memset(ir, 0, sizeof(*ir));
    const int64_t now_ns = cly_ctx_now_internal(ctx);
    uint64_t n = 0;
    for (int i = 0; i < nfiles; i++) {
        if (res[i].status < 0) return res[i].status;           // loadIndex returns the scan's error
        if (file_first[i] != n) return CLY_ERR_ARG;
        n += res[i].n_records;
    }
    if (n == 0) return CLY_OK;
    if (n >= (1ull << 31) || !d_state) return CLY_ERR_ARG;
    if (hipSetDevice(cly_ctx_device_internal(ctx)) != hipSuccess) return CLY_ERR_DEVICE;
    hipStream_t st = stream_v ? (hipStream_t)stream_v : cly_ctx_stream_internal(ctx);
    int rc = CLY_OK;
    uint64_t* h_fb = (uint64_t*)malloc(sizeof(uint64_t) * (2 * (size_t)nfiles + 2));
    for (int i = 0; i < nfiles; i++) { h_fb[i] = file_first[i]; h_fb[nfiles + 1 + i] = (uint64_t)files[i].base; }
    h_fb[nfiles] = n;
    uint64_t *d_fb = nullptr, *d_txkey = nullptr, *d_k2 = nullptr, *d_order = nullptr, *d_hash = nullptr;
    uint32_t *d_sel = nullptr, *d_sidx = nullptr;
    uint8_t *d_cls = nullptr, *d_flag = nullptr, *d_coll = nullptr, *d_del = nullptr, *d_apflag = nullptr;
    uint4* d_ksig = nullptr;
    uint64_t hm = ~0ull;
    TxNext *d_rev = nullptr, *d_nxt = nullptr;
    GMax *d_g = nullptr, *d_g2 = nullptr;
    IxTot* d_tot = nullptr;
    IxTot h_tot;
    unsigned long long* d_nsel = nullptr;
    unsigned long long h_nsel = 0;
    void* d_tmp = nullptr;
    size_t tmp_bytes = 0, need = 0;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const unsigned grid = ix_grid(n);
    rocprim::counting_iterator<uint32_t> cnt(0);
    uint64_t m = 0, m2 = 0;
    int hbits = 64;
    uint32_t ib = 1, hb = 1;
    uint64_t* d_pk = nullptr;
    const uint64_t* d_first = nullptr;
    const uint64_t* d_bases = nullptr;
    ICK(hipEventCreateWithFlags(&e0, hipEventDisableSystemFence));     // (timing only)
    ICK(hipEventCreateWithFlags(&e1, hipEventDisableSystemFence));
    ICK(cly_ix_scratch_internal(ctx, 0, sizeof(uint64_t) * (2 * (size_t)nfiles + 2), (void**)&d_fb));
    d_first = d_fb;
    d_bases = d_fb + nfiles + 1;
    ICK(cly_ix_scratch_internal(ctx, 1, sizeof(IxTot), (void**)&d_tot));
    ICK(cly_ix_scratch_internal(ctx, 2, sizeof(unsigned long long), (void**)&d_nsel));
    ICK(cly_ix_scratch_internal(ctx, 3, n, (void**)&d_cls));
    ICK(cly_ix_scratch_internal(ctx, 4, n, (void**)&d_flag));
    ICK(cly_ix_scratch_internal(ctx, 5, n + 4, (void**)&d_coll));     // (k_ixwin sets bytes by word atomics)
    ICK(cly_ix_scratch_internal(ctx, 6, n, (void**)&d_del));
    ICK(cly_ix_scratch_internal(ctx, 7, n, (void**)&d_apflag));
    ICK(cly_ix_scratch_internal(ctx, 9, sizeof(uint4) * n, (void**)&d_ksig));
    ICK(cly_ix_scratch_internal(ctx, 10, sizeof(uint64_t) * n, (void**)&d_txkey));
    ICK(cly_ix_scratch_internal(ctx, 11, sizeof(uint64_t) * n, (void**)&d_k2));
    ICK(cly_ix_scratch_internal(ctx, 12, sizeof(uint64_t) * n, (void**)&d_order));
    ICK(cly_ix_scratch_internal(ctx, 13, sizeof(uint64_t) * n, (void**)&d_hash));
    ICK(cly_ix_scratch_internal(ctx, 14, sizeof(uint32_t) * n, (void**)&d_sel));
    ICK(cly_ix_scratch_internal(ctx, 15, sizeof(uint32_t) * n, (void**)&d_sidx));
    ICK(cly_ix_scratch_internal(ctx, 16, sizeof(TxNext) * n, (void**)&d_rev));
    ICK(cly_ix_scratch_internal(ctx, 17, sizeof(TxNext) * n, (void**)&d_nxt));
    ICK(cly_ix_scratch_internal(ctx, 18, sizeof(GMax) * n, (void**)&d_g));
    ICK(cly_ix_scratch_internal(ctx, 19, sizeof(GMax) * n, (void**)&d_g2));
    ICK(cly_ix_scratch_internal(ctx, 21, sizeof(uint64_t) * n, (void**)&d_pk));
    // temp storage: the largest of the select / sort / scan needs
    ICK(rocprim::select(nullptr, need, cnt, d_flag, d_sel, d_nsel, (size_t)n, st));
    tmp_bytes = need;
    ICK(rocprim::radix_sort_pairs(nullptr, need, d_k2, d_txkey, d_sel, d_sidx, (size_t)n, 0u, 64u, st));
    if (need > tmp_bytes) tmp_bytes = need;
    ICK(rocprim::radix_sort_keys(nullptr, need, d_k2, d_txkey, (size_t)n, 0u, 64u, st));
    if (need > tmp_bytes) tmp_bytes = need;
    ICK(rocprim::inclusive_scan(nullptr, need, d_rev, d_nxt, (size_t)n, TxNextOp(), st));
    if (need > tmp_bytes) tmp_bytes = need;
    ICK(rocprim::inclusive_scan(nullptr, need, d_g, d_g2, (size_t)n, GMaxOp(), st));
    if (need > tmp_bytes) tmp_bytes = need;
    ICK(cly_ix_scratch_internal(ctx, 20, tmp_bytes, &d_tmp));
    ICK(hipMemcpyAsync(d_fb, h_fb, sizeof(uint64_t) * (2 * (size_t)nfiles + 1), hipMemcpyHostToDevice, st));
    ICK(hipMemsetAsync(d_tot, 0, sizeof(IxTot), st));
    ICK(hipMemsetAsync(d_coll, 0, n + 4, st));
    ICK(hipEventRecord(e0, st));
    hm = ix_hash_mask(n, hbits);
    ix_pk_bits(n, hbits, ib, hb);
    k_ixclass<<<grid, 256, 0, st>>>(d_tuples, n, d_cls, d_state, d_flag, d_tot, d_first, d_bases, nfiles, d_hash,
                                    d_apflag, d_del, d_ksig, d_pk, hm, ib, hb, now_ns);
    ICK(hipMemcpyAsync(&h_tot, d_tot, sizeof(IxTot), hipMemcpyDeviceToHost, st));
    ICK(hipStreamSynchronize(st));
    // ---- transactions: tx records sorted by txId (stable: scan order within a txId)
    if (h_tot.n_tx) {
        size_t tb = tmp_bytes;
        ICK(rocprim::select(d_tmp, tb, cnt, d_flag, d_sel, d_nsel, (size_t)n, st));
        ICK(hipMemcpyAsync(&h_nsel, d_nsel, sizeof(h_nsel), hipMemcpyDeviceToHost, st));
        ICK(hipStreamSynchronize(st));
        m = h_nsel;
    }
    if (m) {
        // (tx data records' application orders: k_ixtx; the others stay IX_NONE)
        ICK(hipMemsetAsync(d_order, 0xff, sizeof(uint64_t) * n, st));
        k_ixgathertx<<<ix_grid(m), 256, 0, st>>>(d_tuples, d_sel, m, d_k2);
        {
            size_t tb = tmp_bytes;
            // sorted txIds into d_txkey (free after the gather; d_hash holds k_ixclass's hashes)
            ICK(rocprim::radix_sort_pairs(d_tmp, tb, d_k2, d_txkey, d_sel, d_sidx, (size_t)m, 0u, 64u, st));
        }
        k_ixtxin<<<ix_grid(m), 256, 0, st>>>(d_txkey, d_sidx, d_cls, m, d_rev);
        {
            size_t tb = tmp_bytes;
            ICK(rocprim::inclusive_scan(d_tmp, tb, d_rev, d_nxt, (size_t)m, TxNextOp(), st));
        }
        k_ixtx<<<ix_grid(m), 256, 0, st>>>(d_sidx, d_cls, m, d_nxt, d_order, d_state);
    }
    // ---- applied records: hash, sort, winner per key
    // (records without a txId were hashed by k_ixclass; committed tx data here)
    if (m) k_ixapply<<<grid, 256, 0, st>>>(d_tuples, n, d_cls, d_order, d_first, d_bases, nfiles, d_hash, d_apflag,
                                           d_del, d_ksig, hm, &d_tot->bad, now_ns);
    if (m == 0 && h_tot.n_now == n) {
        m2 = n;                                                 // every record applied: no select
    } else {
        size_t tb = tmp_bytes;
        ICK(rocprim::select(d_tmp, tb, cnt, d_apflag, d_sel, d_nsel, (size_t)n, st));
        ICK(hipMemcpyAsync(&h_nsel, d_nsel, sizeof(h_nsel), hipMemcpyDeviceToHost, st));
        ICK(hipStreamSynchronize(st));
        m2 = h_nsel;
    }
    if (m2) {
        // every record applied now: k_ixclass wrote the sort keys in place;
        // otherwise build the selected records' keys
        const bool ident = m == 0 && m2 == n;
        if (!ident) k_ixgatherd<<<ix_grid(m2), 256, 0, st>>>(d_hash, d_sel, d_del, m2, d_k2, ib, hb);
        {
            // sorted keys into d_txkey (free after the tx phase)
            size_t tb = tmp_bytes;
            ICK(rocprim::radix_sort_keys(d_tmp, tb, ident ? d_pk : d_k2, d_txkey, (size_t)m2, ib + 1u, ib + 1u + hb,
                                         st));
        }
        if (m) {                    // tx records: application order != scan order, arg-max per group
            k_ixgin<<<ix_grid(m2), 256, 0, st>>>(d_txkey, ib, d_cls, d_order, m2, d_g);
            size_t tb = tmp_bytes;
            ICK(rocprim::inclusive_scan(d_tmp, tb, d_g, d_g2, (size_t)m2, GMaxOp(), st));
        }
        // (d_sel is free after the sort: the collided groups' heads)
        k_ixwin<<<ix_grid(m2), 256, 0, st>>>(d_txkey, ib, m ? d_g2 : nullptr, m2, d_tuples, d_first, d_bases,
                                             nfiles, d_ksig, d_state, d_coll, d_sel, d_tot);
        ICK(hipMemcpyAsync(&h_tot, d_tot, sizeof(IxTot), hipMemcpyDeviceToHost, st));
        ICK(hipStreamSynchronize(st));
        if (h_tot.n_chead)
            k_ixcoll<<<(unsigned)((h_tot.n_chead + 255) / 256), 256, 0, st>>>(
                d_txkey, ib, d_cls, d_order, m2, d_tuples, d_first, d_bases, nfiles, d_ksig, d_hash, d_del, d_state,
                d_sel, h_tot.n_chead);
        k_ixwinfix<<<ix_grid(n), 256, 0, st>>>(d_tuples, n, d_first, d_bases, nfiles, d_del, d_state);
    }
    k_ixcount<<<ix_grid(n) < 1024 ? ix_grid(n) : 1024, 256, 0, st>>>(d_state, d_apflag, n, d_tot);
    ICK(hipGetLastError());
    ICK(hipEventRecord(e1, st));
    ICK(hipMemcpyAsync(&h_tot, d_tot, sizeof(IxTot), hipMemcpyDeviceToHost, st));
    ICK(hipStreamSynchronize(st));
    if (h_tot.bad) { rc = CLY_ERR_VARINT; goto done; }
    ir->n_live = h_tot.n_live;
    ir->n_applied = h_tot.n_applied;
    ir->n_host = 0;
    ir->n_loadonly = h_tot.n_loadonly;
    ir->n_merge_panic = h_tot.n_mpanic;
    ir->n_collisions = h_tot.n_coll;
    {
        float ms = 0;
        ICK(hipEventElapsedTime(&ms, e0, e1));
        ir->index_ms = ms;
    }
done:
    hipStreamSynchronize(st);                     // (the buffers stay in the context's scratch)
    if (e0) hipEventDestroy(e0);
    if (e1) hipEventDestroy(e1);
    free(h_fb);
    return rc;
}

// Host-memory entry: scan the files (host memory) on the device and rebuild
// the String/ListMeta index state of every record; state[i] per record in scan
// order (n_out = records).
extern "C" int cly_index(cly_ctx* ctx, const cly_file* files, int nfiles, uint8_t* state, uint64_t cap,
                         uint64_t* n_out, cly_index_result* ir) {
    if (!ctx || !ir || !n_out || nfiles < 0 || (nfiles && !files)) return CLY_ERR_ARG;
    memset(ir, 0, sizeof(*ir));
    *n_out = 0;
    if (hipSetDevice(cly_ctx_device_internal(ctx)) != hipSuccess) return CLY_ERR_DEVICE;
    hipStream_t st = cly_ctx_stream_internal(ctx);
    int rc = CLY_OK;
    uint64_t total = 0;
    for (int i = 0; i < nfiles; i++) {
        if (files[i].len >= (1ULL << 32)) return CLY_ERR_ARG;
        total += (files[i].len + 4095) & ~4095ULL;
    }
    const int nf = nfiles ? nfiles : 1;
    cly_file* df = (cly_file*)calloc(nf, sizeof(cly_file));
    uint64_t* first = (uint64_t*)calloc(nf, sizeof(uint64_t));
    cly_file_result* res = (cly_file_result*)calloc(nf, sizeof(cly_file_result));
    uint8_t *d_bytes = nullptr, *d_state = nullptr;
    cly_tuple* d_tup = nullptr;
    uint64_t need = 0, cap_t = 0, T = 0, off = 0;
    ICK(hipMalloc((void**)&d_bytes, total + 4096));
    for (int i = 0; i < nfiles; i++) {
        df[i] = files[i];
        df[i].base = d_bytes + off;
        if (files[i].len) ICK(hipMemcpyAsync(d_bytes + off, files[i].base, files[i].len, hipMemcpyHostToDevice, st));
        off += (files[i].len + 4095) & ~4095ULL;
    }
    cap_t = cly_scan_capacity(files, nfiles) + 16;
    ICK(hipMalloc((void**)&d_tup, sizeof(cly_tuple) * cap_t));
    rc = cly_scan_device(ctx, df, nfiles, d_tup, cap_t, first, res, &need, nullptr, nullptr);
    if (rc != CLY_OK) goto done;
    for (int i = 0; i < nfiles; i++) {
        if (res[i].status < 0) { rc = res[i].status; goto done; }
        if (first[i] != T && res[i].n_records)
            ICK(hipMemcpyAsync(d_tup + T, d_tup + first[i], sizeof(cly_tuple) * res[i].n_records,
                               hipMemcpyDeviceToDevice, st));
        first[i] = T;
        T += res[i].n_records;
    }
    *n_out = T;
    if (T > cap) { rc = CLY_ERR_CAPACITY; goto done; }
    ICK(hipMalloc((void**)&d_state, T + 1));
    rc = cly_index_device(ctx, df, nfiles, d_tup, first, res, d_state, ir, nullptr);
    if (rc != CLY_OK) goto done;
    if (T) ICK(hipMemcpyAsync(state, d_state, T, hipMemcpyDeviceToHost, st));
    ICK(hipStreamSynchronize(st));
done:
    hipStreamSynchronize(st);
    hipFree(d_bytes); hipFree(d_tup); hipFree(d_state);
    free(df); free(first); free(res);
    return rc;
}
