// clygen.hip — GPU writer of synthetic CouloyDB data files (include/clygen.h).
// One wavefront encodes one record: lanes write contiguous byte ranges and
// compute raw CRC-32 registers that are shifted into place with GF(2)
// multiplication (crc_gf.h) and XOR-reduced across the wave.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/clygen.h"
#include "crc_gf.h"

static inline int uvarint_len(uint64_t ux) { int n = 1; while (ux >= 0x80) { ux >>= 7; n++; } return n; }
static inline uint64_t zigzag(int64_t x) { uint64_t ux = (uint64_t)x << 1; return x < 0 ? ~ux : ux; }

extern "C" uint64_t cly_gen_record_size(int64_t tx_id, uint32_t value_len) {
    const uint64_t klen = (uint64_t)uvarint_len(zigzag(tx_id)) + 9;
    return 6 + uvarint_len(zigzag((int64_t)klen)) + uvarint_len(zigzag((int64_t)value_len)) + 1 + klen + value_len;
}

extern "C" uint64_t cly_gen_layout(cly_gen_rec* recs, uint64_t nrecs, uint64_t data_file_size,
                                   uint64_t align, uint64_t* file_off, uint64_t* file_len,
                                   uint32_t max_files, uint32_t* nfiles) {
    uint32_t f = 0;
    uint64_t write_off = 0, base = 0;
    if (max_files == 0) return 0;
    file_off[0] = 0;
    for (uint64_t i = 0; i < nrecs; i++) {
        const uint64_t size = cly_gen_record_size(recs[i].tx_id, recs[i].value_len);
        if (write_off + size > data_file_size && write_off > 0) {      // db.go:376 rotation
            file_len[f] = write_off;
            base += (write_off + align - 1) / align * align;
            if (++f >= max_files) { *nfiles = f; return base; }
            file_off[f] = base;
            write_off = 0;
        }
        recs[i].dst = base + write_off;
        write_off += size;
    }
    file_len[f] = write_off;
    *nfiles = f + 1;
    return base + (write_off + align - 1) / align * align;
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

struct RecView {
    uint8_t hdr[32];
    int hlen;           // header bytes incl. crc placeholder
    int klen;           // key bytes
    uint8_t key[20];
    uint64_t size;
};

__device__ __forceinline__ uint8_t byte_at(const RecView& r, const cly_gen_rec& g, uint64_t seed, uint64_t j) {
    if (j < (uint64_t)r.hlen) return r.hdr[j];
    j -= r.hlen;
    if (j < (uint64_t)r.klen) return r.key[j];
    j -= r.klen;
    switch (g.value_mode) {
        case CLYGEN_VALUE_KEYZERO:
            return j < 9 ? r.key[r.klen - 9 + j] : 0;
        case CLYGEN_VALUE_ALNUM: {
            const char cs[] = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789";
            uint64_t v = splitmix64(seed ^ ((uint64_t)g.key_index << 20) ^ j);
            return (uint8_t)cs[v % 62];
        }
        default: {
            uint64_t v = splitmix64(seed ^ ((uint64_t)g.key_index * 0x100000001B3ull) ^ (j >> 3));
            return (uint8_t)(v >> (8 * (j & 7)));
        }
    }
}

__global__ void __launch_bounds__(256) k_gen_encode(uint8_t* __restrict__ buf, const cly_gen_rec* __restrict__ recs,
                                                    uint64_t nrecs, uint64_t seed) {
    const uint64_t ridx = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (ridx >= nrecs) return;
    const cly_gen_rec g = recs[ridx];
    RecView r;
    // key = varint(tx_id) || %09d(key_index)   (batch.go:120-127, bytex.GetTestKey)
    int kl = 0;
    {
        uint64_t ux = (uint64_t)g.tx_id << 1;
        if (g.tx_id < 0) ux = ~ux;
        while (ux >= 0x80) { r.key[kl++] = (uint8_t)(ux | 0x80); ux >>= 7; }
        r.key[kl++] = (uint8_t)ux;
        uint32_t k = g.key_index;
        for (int d = 8; d >= 0; d--) { r.key[kl + d] = (uint8_t)('0' + k % 10); k /= 10; }
        kl += 9;
    }
    r.klen = kl;
    // header (logRecord.go:59-68); crc bytes filled at the end
    int h = 4;
    r.hdr[h++] = g.type;
    r.hdr[h++] = g.dtype;
    const int64_t vals[3] = {kl, (int64_t)g.value_len, 0};
    for (int v = 0; v < 3; v++) {
        uint64_t ux = (uint64_t)vals[v] << 1;
        if (vals[v] < 0) ux = ~ux;
        while (ux >= 0x80) { r.hdr[h++] = (uint8_t)(ux | 0x80); ux >>= 7; }
        r.hdr[h++] = (uint8_t)ux;
    }
    r.hlen = h;
    r.size = (uint64_t)h + kl + g.value_len;
    // bytes [4, size): lane ranges, raw CRC per lane
    const uint64_t body = r.size - 4;
    const uint64_t per = (body + 63) / 64;
    uint64_t lo = 4 + per * lane, hi = lo + per;
    if (lo > r.size) lo = r.size;
    if (hi > r.size) hi = r.size;
    uint32_t s = 0;
    uint8_t* dst = buf + g.dst;
    for (uint64_t j = lo; j < hi; j++) {
        const uint8_t b = byte_at(r, g, seed, j);
        dst[j] = b;
        s = cly_crc_byte_bitwise(s, b);
    }
    // shift this lane's register to the record end, XOR-reduce across the wave
    uint32_t contrib = (hi > lo) ? cly_shift(s, r.size - hi) : 0;
    if (lane == 0) contrib ^= cly_shift(0xFFFFFFFFu, body);   // init's contribution
    for (int off = 32; off > 0; off >>= 1) contrib ^= __shfl_xor(contrib, off, 64);
    if (lane == 0) {
        const uint32_t crc = ~contrib;                       // logRecord.go:80-81
        dst[0] = (uint8_t)crc; dst[1] = (uint8_t)(crc >> 8);
        dst[2] = (uint8_t)(crc >> 16); dst[3] = (uint8_t)(crc >> 24);
    }
}

extern "C" int cly_gen_encode(uint8_t* d_buf, const cly_gen_rec* d_recs, uint64_t nrecs, uint64_t seed) {
    if (!nrecs) return 0;
    const uint64_t blocks = (nrecs + 3) / 4;
    // a launch's work-item count (grid x block) must stay below 2^32
    const uint64_t per = 1u << 22;
    for (uint64_t b0 = 0; b0 < blocks; b0 += per) {
        const uint64_t nb = blocks - b0 < per ? blocks - b0 : per;
        hipLaunchKernelGGL(k_gen_encode, dim3((unsigned)nb), dim3(256), 0, 0, d_buf, d_recs + b0 * 4,
                           nrecs - b0 * 4, seed);
    }
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) { fprintf(stderr, "clygen: %s\n", hipGetErrorString(e)); return -11; }
    return 0;
}
