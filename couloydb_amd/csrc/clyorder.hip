// clyorder.hip — the MemTable order of the String and ListMeta indexes after a
// device load (part of libclyscan; used by clyload.hip's cly_db_open).
//
// The reference's default MemTable is a BTree ordered by bytes.Compare of the
// key (options.go:33 -> meta/btree.go:21-29, Item.Less at :64-66), and
// MemTable.Iterator (meta/memTable.go:25-26) walks it in that order.  The load
// driver's winners (one per key, the record an index entry points at) come out
// of the device index in scan order; here they are sorted by their realKey
// bytes so that the caller can fill (or build bottom-up) its BTree in
// ascending order.
//
// Round 0: a 128-bit sort key per winner — realKey bytes 0..14 big-endian,
// zero-padded, then the length class min(len, 16) — by two stable LSD radix
// sorts (bytes 8..14 + class, then bytes 0..7).  Keys of at most 15 bytes are
// then totally ordered: a key that is a proper prefix of another has zero
// padding where the other has its next bytes, and a smaller class when those
// are zero too, which is bytes.Compare's "shorter first".  Adjacent winners
// with equal round-0 keys of class 16 (16+ bytes, equal first 15) form runs;
// round r >= 1 compares bytes 15 + 7(r-1) .. +7 (class min(remaining, 8),
// 8 = more follow) inside the runs only, by a segmented radix sort, until no
// run is left.  Winners hold distinct keys, so the order is total.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_segmented_radix_sort.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <stdint.h>
#include <stdio.h>

#include "scan_core.h"

#define OCK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "clyorder: %s failed: %s\n", #x, hipGetErrorString(e_)); rc = CLY_ERR_DEVICE; goto done; } } while (0)

// realKey of tuple ti: the file holding it (the last file whose first tuple
// index is <= ti; empty files share their successor's first index and come
// before it), then key[txId varint length:] (db.go:706-710)
__device__ __forceinline__ const uint8_t* ord_key(const cly_tuple* __restrict__ tup, const uint64_t* __restrict__ first,
                                                  const uint64_t* __restrict__ bases, int nf, uint32_t ti, uint32_t& len) {
    int lo = 0, hi = nf - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (first[mid] <= ti) lo = mid; else hi = mid - 1;
    }
    const cly_tuple& t = tup[ti];
    const uint32_t tl = t.txid_len == 0xFF ? 0u : t.txid_len;
    len = t.key_size - tl;
    return (const uint8_t*)bases[lo] + t.offset + t.header_size + tl;
}
// bytes [off, off + nb) of a key of length len, big-endian, zero past its end
__device__ __forceinline__ uint64_t ord_be(const uint8_t* k, uint32_t len, uint32_t off, uint32_t nb) {
    uint64_t v = 0;
    for (uint32_t q = 0; q < nb; q++) v = (v << 8) | (off + q < len ? k[off + q] : 0u);
    return v;
}
// winners of one data type (state byte = index state | dt << 4, k_state_dt)
__global__ void k_ord_flag(const uint8_t* __restrict__ state, uint64_t n, uint32_t dt, uint8_t* flag) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) flag[i] = (state[i] & 15u) == CLY_IX_LIVE && (uint32_t)(state[i] >> 4) == dt;
}
// round 0 keys: k1 = bytes 8..14 << 8 | min(len, 16), k0 = bytes 0..7; pos = j
__global__ void k_ord_key0(const uint32_t* __restrict__ sel, uint64_t m, const cly_tuple* __restrict__ tup,
                           const uint64_t* __restrict__ fb, int nf, uint64_t* k0, uint64_t* k1, uint32_t* pos) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    uint32_t len;
    const uint8_t* k = ord_key(tup, fb + nf, fb, nf, sel[j], len);
    k0[j] = ord_be(k, len, 0, 8);
    k1[j] = (ord_be(k, len, 8, 7) << 8) | (len < 16u ? len : 16u);
    pos[j] = (uint32_t)j;
}
__global__ void k_ord_gather(const uint64_t* __restrict__ src, const uint32_t* __restrict__ perm, uint64_t m,
                             uint64_t* dst) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < m) dst[j] = src[perm[j]];
}
// final round-0 order: winners' tuple indices, the sorted k1 (tie test) and
// the ties (equal 128-bit key of class 16 as the winner before)
__global__ void k_ord_fin0(const uint32_t* __restrict__ sel, const uint32_t* __restrict__ perm, uint64_t m,
                           const uint64_t* __restrict__ k0s, const uint64_t* __restrict__ k1, uint32_t* ord,
                           uint8_t* tie, unsigned long long* nties) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    ord[j] = sel[perm[j]];
    bool t = false;
    if (j > 0) {
        const uint64_t a = k1[perm[j]], b = k1[perm[j - 1]];
        t = k0s[j] == k0s[j - 1] && a == b && (a & 0xffu) == 16u;
    }
    tie[j] = t;
    if (t) atomicAdd(nties, 1ull);
}
// positions in runs: a tie or followed by one
__global__ void k_ord_inrun(const uint8_t* __restrict__ tie, uint64_t m, uint8_t* inrun) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < m) inrun[j] = tie[j] || (j + 1 < m && tie[j + 1]);
}
// round r keys of the run members: bytes 15 + 7 (r - 1) .. + 7 << 8 | class
__global__ void k_ord_keyr(const uint32_t* __restrict__ P, uint64_t np, const uint32_t* __restrict__ ord,
                           const uint8_t* __restrict__ tie, const cly_tuple* __restrict__ tup,
                           const uint64_t* __restrict__ fb, int nf, uint32_t off, uint64_t* key, uint32_t* val,
                           uint8_t* start) {
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= np) return;
    const uint32_t ti = ord[P[c]];
    uint32_t len;
    const uint8_t* k = ord_key(tup, fb + nf, fb, nf, ti, len);
    const uint32_t rem = len > off ? len - off : 0u;
    key[c] = (ord_be(k, len, off, 7) << 8) | (rem < 8u ? rem : 8u);
    val[c] = ti;
    start[c] = !tie[P[c]];
}
// the runs, sorted, back into place; the ties left for the next round
__global__ void k_ord_scatter(const uint32_t* __restrict__ P, uint64_t np, const uint64_t* __restrict__ ks,
                              const uint32_t* __restrict__ vs, const uint8_t* __restrict__ start, uint32_t* ord,
                              uint8_t* tie, unsigned long long* nties) {
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= np) return;
    ord[P[c]] = vs[c];
    const bool t = !start[c] && ks[c] == ks[c - 1] && (ks[c] & 0xffu) == 8u;
    tie[P[c]] = t;
    if (t) atomicAdd(nties, 1ull);
}
static inline unsigned ogrid(uint64_t n) { return (unsigned)((n + 255) / 256); }

// The winners of data type dt (String 0, ListMeta 3) among the n tuples,
// sorted by bytes.Compare of their realKeys: *d_ord (hipMalloc'd, the caller
// frees it) holds *m tuple indices.  first/bases: per file (nf) the index of
// its first tuple and its bytes on the device.
extern "C" int cly_order_keys_internal(hipStream_t st, const cly_tuple* d_tup, uint64_t n, const uint8_t* d_state,
                                       uint32_t dt, const uint64_t* first, const uint64_t* bases, int nf,
                                       uint32_t** d_ord_out, uint64_t* m_out, uint32_t* rounds_out) {
    int rc = CLY_OK;
    *d_ord_out = nullptr; *m_out = 0;
    if (rounds_out) *rounds_out = 0;
    if (n >= (1ull << 32)) return CLY_ERR_ARG;                 // (u32 tuple indices)
    uint8_t *d_flag = nullptr, *d_tie = nullptr, *d_aux = nullptr;
    uint32_t *d_sel = nullptr, *d_pa = nullptr, *d_pb = nullptr, *d_ord = nullptr, *d_vb = nullptr;
    uint64_t *d_k0 = nullptr, *d_k1 = nullptr, *d_ka = nullptr, *d_fb = nullptr;
    unsigned long long* d_cnt = nullptr;                       // [0] selected, [1] ties, [2] segment starts
    void* d_tmp = nullptr;
    size_t tmp_bytes = 0, need = 0;
    unsigned long long h_cnt[3] = {0, 0, 0};
    uint64_t m = 0;
    uint32_t rounds = 0;
    OCK(hipMalloc((void**)&d_cnt, sizeof(h_cnt)));
    OCK(hipMalloc((void**)&d_fb, sizeof(uint64_t) * 2 * (nf ? nf : 1)));
    OCK(hipMemcpyAsync(d_fb, bases, sizeof(uint64_t) * nf, hipMemcpyHostToDevice, st));
    OCK(hipMemcpyAsync(d_fb + nf, first, sizeof(uint64_t) * nf, hipMemcpyHostToDevice, st));
    OCK(hipMemsetAsync(d_cnt, 0, sizeof(h_cnt), st));
    OCK(hipMalloc((void**)&d_flag, n ? n : 1));
    OCK(hipMalloc((void**)&d_sel, sizeof(uint32_t) * (n ? n : 1)));
    OCK(rocprim::select(nullptr, need, rocprim::counting_iterator<uint32_t>(0), d_flag, d_sel,
                                      d_cnt, (size_t)n, st));
    tmp_bytes = need;
    OCK(rocprim::radix_sort_pairs(nullptr, need, d_k1, d_ka, d_pa, d_pb, (size_t)n, 0u, 64u, st));
    if (need > tmp_bytes) tmp_bytes = need;
    OCK(hipMalloc(&d_tmp, tmp_bytes ? tmp_bytes : 1));
    if (n) {
        hipLaunchKernelGGL(k_ord_flag, dim3(ogrid(n)), dim3(256), 0, st, d_state, n, dt, d_flag);
        OCK(rocprim::select(d_tmp, need = tmp_bytes, rocprim::counting_iterator<uint32_t>(0), d_flag,
                                          d_sel, d_cnt, (size_t)n, st));
        OCK(hipMemcpyAsync(h_cnt, d_cnt, sizeof(h_cnt), hipMemcpyDeviceToHost, st));
        OCK(hipStreamSynchronize(st));
    }
    m = h_cnt[0];
    OCK(hipMalloc((void**)&d_ord, sizeof(uint32_t) * (m ? m : 1)));
    if (m) {
        OCK(hipMalloc((void**)&d_k0, sizeof(uint64_t) * m));
        OCK(hipMalloc((void**)&d_k1, sizeof(uint64_t) * m));
        OCK(hipMalloc((void**)&d_ka, sizeof(uint64_t) * m));
        OCK(hipMalloc((void**)&d_pa, sizeof(uint32_t) * m));
        OCK(hipMalloc((void**)&d_pb, sizeof(uint32_t) * m));
        OCK(hipMalloc((void**)&d_tie, m));
        hipLaunchKernelGGL(k_ord_key0, dim3(ogrid(m)), dim3(256), 0, st, d_sel, m, d_tup, d_fb, nf, d_k0, d_k1, d_pa);
        // LSD: by k1 (stable), then by k0 (stable): the 128-bit order
        OCK(rocprim::radix_sort_pairs(d_tmp, need = tmp_bytes, d_k1, d_ka, d_pa, d_pb, (size_t)m, 0u, 64u, st));
        hipLaunchKernelGGL(k_ord_gather, dim3(ogrid(m)), dim3(256), 0, st, d_k0, d_pb, m, d_ka);
        OCK(rocprim::radix_sort_pairs(d_tmp, need = tmp_bytes, d_ka, d_k0, d_pb, d_pa, (size_t)m, 0u, 64u, st));
        hipLaunchKernelGGL(k_ord_fin0, dim3(ogrid(m)), dim3(256), 0, st, d_sel, d_pa, m, d_k0, d_k1, d_ord, d_tie,
                           d_cnt + 1);
        OCK(hipGetLastError());
        OCK(hipMemcpyAsync(h_cnt, d_cnt, sizeof(h_cnt), hipMemcpyDeviceToHost, st));
        OCK(hipStreamSynchronize(st));
        // refinement rounds over the runs of equal 15-byte prefixes of long keys
        // (d_k0/d_k1/d_ka/d_pa/d_pb/d_sel/d_flag reused as round scratch)
        for (uint32_t off = 15; h_cnt[1]; off += 7) {
            rounds++;
            uint8_t* d_inrun = d_flag;
            uint32_t* d_P = d_sel;
            hipLaunchKernelGGL(k_ord_inrun, dim3(ogrid(m)), dim3(256), 0, st, d_tie, m, d_inrun);
            OCK(hipMemsetAsync(d_cnt, 0, sizeof(h_cnt), st));
            OCK(rocprim::select(d_tmp, need = tmp_bytes, rocprim::counting_iterator<uint32_t>(0),
                                              d_inrun, d_P, d_cnt, (size_t)m, st));
            OCK(hipMemcpyAsync(h_cnt, d_cnt, sizeof(h_cnt), hipMemcpyDeviceToHost, st));
            OCK(hipStreamSynchronize(st));
            const uint64_t np = h_cnt[0];
            uint64_t* d_key = d_k0;
            uint64_t* d_keys = d_k1;
            uint32_t* d_val = d_pa;
            uint32_t* d_vals = d_pb;
            if (!d_aux) OCK(hipMalloc((void**)&d_aux, m + 1));
            if (!d_vb) OCK(hipMalloc((void**)&d_vb, sizeof(uint32_t) * (m + 1)));
            hipLaunchKernelGGL(k_ord_keyr, dim3(ogrid(np)), dim3(256), 0, st, d_P, np, d_ord, d_tie, d_tup, d_fb, nf,
                               off, d_key, d_val, d_aux);
            // segment begins: the run starts among the members (+ np at the end)
            OCK(rocprim::select(d_tmp, need = tmp_bytes, rocprim::counting_iterator<uint32_t>(0),
                                              d_aux, d_vb, d_cnt + 2, (size_t)np, st));
            OCK(hipMemcpyAsync(h_cnt, d_cnt, sizeof(h_cnt), hipMemcpyDeviceToHost, st));
            OCK(hipStreamSynchronize(st));
            const uint64_t nseg = h_cnt[2];
            const uint32_t np32 = (uint32_t)np;
            OCK(hipMemcpyAsync(d_vb + nseg, &np32, sizeof(uint32_t), hipMemcpyHostToDevice, st));
            size_t sneed = 0;
            OCK(rocprim::segmented_radix_sort_pairs(nullptr, sneed, d_key, d_keys, d_val, d_vals, (unsigned)np,
                                                        (unsigned)nseg, d_vb, d_vb + 1, 0u, 64u, st));
            if (sneed > tmp_bytes) {
                OCK(hipStreamSynchronize(st));
                hipFree(d_tmp);
                d_tmp = nullptr;
                tmp_bytes = sneed;
                OCK(hipMalloc(&d_tmp, tmp_bytes));
            }
            OCK(rocprim::segmented_radix_sort_pairs(d_tmp, sneed, d_key, d_keys, d_val, d_vals, (unsigned)np,
                                                        (unsigned)nseg, d_vb, d_vb + 1, 0u, 64u, st));
            OCK(hipMemsetAsync(d_cnt + 1, 0, sizeof(unsigned long long), st));
            hipLaunchKernelGGL(k_ord_scatter, dim3(ogrid(np)), dim3(256), 0, st, d_P, np, d_keys, d_vals, d_aux,
                               d_ord, d_tie, d_cnt + 1);
            OCK(hipGetLastError());
            OCK(hipMemcpyAsync(h_cnt, d_cnt, sizeof(h_cnt), hipMemcpyDeviceToHost, st));
            OCK(hipStreamSynchronize(st));
            if (off > (1u << 31)) { rc = CLY_ERR_DEVICE; goto done; }     // (never: keys are < 4 GiB)
        }
    }
    OCK(hipStreamSynchronize(st));
    *d_ord_out = d_ord;
    d_ord = nullptr;
    *m_out = m;
    if (rounds_out) *rounds_out = rounds;
done:
    hipStreamSynchronize(st);
    hipFree(d_flag); hipFree(d_tie); hipFree(d_aux); hipFree(d_sel); hipFree(d_pa); hipFree(d_pb); hipFree(d_ord);
    hipFree(d_vb); hipFree(d_k0); hipFree(d_k1); hipFree(d_ka); hipFree(d_fb); hipFree(d_cnt); hipFree(d_tmp);
    return rc;
}
