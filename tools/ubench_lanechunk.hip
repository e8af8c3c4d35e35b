// Microbenchmark for the per-lane-chunk scan layout (not part of the product).
// Each lane owns a contiguous chunk of C bytes and streams it through a
// slicing-by-4 CRC register (LDS tables, 16 replicas, bank-skewed); loads are
// per-lane 16-B pieces (64 different cache lines per wave instruction).
// Compared with a coalesced read of the same bytes.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/ub tools/ubench_lanechunk.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define LDS __attribute__((address_space(3)))
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define POLY 0xEDB88320u

__device__ __forceinline__ void init_tables(LDS uint32_t* t) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) {
        uint32_t cv = i;
        for (int k = 0; k < 8; k++) cv = (cv & 1) ? (cv >> 1) ^ POLY : cv >> 1;
        for (int tt = 0; tt < 4; tt++) {
            for (int r = 0; r < 16; r++) t[i * 64 + tt * 16 + r] = cv;
            uint32_t tl = cv & 0xff;
            for (int k = 0; k < 8; k++) tl = (tl & 1) ? (tl >> 1) ^ POLY : tl >> 1;
            cv = (cv >> 8) ^ tl;
        }
    }
    __syncthreads();
}
struct CL { uint32_t oe, oo, s0, s1, s2, s3; };
__device__ __forceinline__ CL crc_lane(int lane) {
    const uint32_t r4 = (uint32_t)(lane & 15) * 4, h = (uint32_t)(lane >> 4) & 1u;
    CL c;
    c.oe = r4 + 64 * h; c.oo = r4 + 64 * (1 - h);
    c.s0 = 0x0c0c0000u | ((4u + (3u - (0u ^ h))) << 8);
    c.s1 = 0x0c0c0000u | ((4u + (3u - (1u ^ h))) << 8);
    c.s2 = 0x0c0c0000u | ((4u + (3u - (2u ^ h))) << 8);
    c.s3 = 0x0c0c0000u | ((4u + (3u - (3u ^ h))) << 8);
    return c;
}
__device__ __forceinline__ uint32_t crc_word(const LDS uint8_t* sm, uint32_t x, const CL& c) {
    const uint32_t a0 = __builtin_amdgcn_perm(x, c.oe, c.s0), a1 = __builtin_amdgcn_perm(x, c.oo, c.s1);
    const uint32_t a2 = __builtin_amdgcn_perm(x, c.oe, c.s2), a3 = __builtin_amdgcn_perm(x, c.oo, c.s3);
    return *(const LDS uint32_t*)(sm + a0) ^ *(const LDS uint32_t*)(sm + a1) ^
           *(const LDS uint32_t*)(sm + a2 + 128) ^ *(const LDS uint32_t*)(sm + a3 + 128);
}

template <int C, int B, int NB, int MODE>   // chunk bytes, burst bytes, bursts in flight; MODE 0 crc+nt 1 crc 2 loads only 3 crc only
__global__ void __launch_bounds__(512, 2) k_lane(const uint8_t* __restrict__ data, uint64_t n, uint32_t* out) {
    __shared__ __attribute__((aligned(16))) uint32_t tab[16384];
    init_tables((LDS uint32_t*)tab);
    const LDS uint8_t* sm = (const LDS uint8_t*)tab;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const CL cl = crc_lane(lane);
    const uint64_t ntile = n / (64ull * C);
    constexpr int P = B / 16;                 // pieces per burst
    constexpr int NBU = C / B;
    for (uint64_t t = (uint64_t)blockIdx.x * 8 + wave; t < ntile; t += (uint64_t)gridDim.x * 8) {
        const u32x4* src = (const u32x4*)(data + t * 64ull * C + (uint64_t)lane * C);
        u32x4 buf[NB][P];
        #pragma unroll
        for (int b = 0; b < NB - 1; b++)
            #pragma unroll
            for (int p = 0; p < P; p++) buf[b][p] = MODE == 3 ? (u32x4){(uint32_t)p, (uint32_t)t, 0u, (uint32_t)lane} : MODE == 0 ? __builtin_nontemporal_load(src + b * P + p) : src[b * P + p];
        uint32_t s = 0;
        #pragma unroll NB
        for (int b = 0; b < NBU; b++) {
            if (b + NB - 1 < NBU) {
                #pragma unroll
                for (int p = 0; p < P; p++) buf[(b + NB - 1) % NB][p] = MODE == 3 ? (u32x4){(uint32_t)p, (uint32_t)b, s, (uint32_t)lane} : MODE == 0 ? __builtin_nontemporal_load(src + (b + NB - 1) * P + p) : src[(b + NB - 1) * P + p];
            }
            #pragma unroll
            for (int p = 0; p < P; p++) {
                const u32x4 v = buf[b % NB][p];
                if (MODE == 2) { s = s ^ v.x ^ v.y ^ v.z ^ v.w; continue; }
                s = crc_word(sm, s ^ v.x, cl);
                s = crc_word(sm, s ^ v.y, cl);
                s = crc_word(sm, s ^ v.z, cl);
                s = crc_word(sm, s ^ v.w, cl);
            }
        }
        out[t * 64 + lane] = s;
    }
}

// coalesced read baseline: each wave reads 1 KiB per instruction, xor-reduces
__global__ void __launch_bounds__(512, 2) k_coal(const uint8_t* __restrict__ data, uint64_t n, uint32_t* out) {
    const u32x4* s4 = (const u32x4*)data;
    const uint64_t nv = n / 16;
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 512 + threadIdx.x; i < nv; i += (uint64_t)gridDim.x * 512 * 4) {
        u32x4 v[4];
        #pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t j = i + (uint64_t)k * gridDim.x * 512;
            v[k] = j < nv ? __builtin_nontemporal_load(s4 + j) : (u32x4){0, 0, 0, 0};
        }
        #pragma unroll
        for (int k = 0; k < 4; k++) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_fill(uint8_t* d, uint64_t n) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i < n / 8; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = i * 0x9E3779B97F4A7C15ull + 0x434C59;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        ((uint64_t*)d)[i] = z ^ (z >> 31);
    }
}

static uint32_t cpu_raw(const uint8_t* p, int n) {
    static uint32_t T[256];
    if (!T[1]) for (int i = 0; i < 256; i++) { uint32_t c = i; for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ POLY : c >> 1; T[i] = c; }
    uint32_t s = 0;
    for (int i = 0; i < n; i++) s = T[(s ^ p[i]) & 0xff] ^ (s >> 8);
    return s;
}

template <int C, int B, int NB, int MODE>
void run(const uint8_t* d, uint64_t n, uint32_t* out, int grid, const char* name, const std::vector<uint8_t>& head) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int w = 0; w < 2; w++) hipLaunchKernelGGL((k_lane<C, B, NB, MODE>), dim3(grid), dim3(512), 0, 0, d, n, out);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    const int it = 10;
    for (int w = 0; w < it; w++) hipLaunchKernelGGL((k_lane<C, B, NB, MODE>), dim3(grid), dim3(512), 0, 0, d, n, out);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= it;
    uint32_t o[4]; CK(hipMemcpy(o, out, 16, hipMemcpyDeviceToHost));
    int ok = 1;
    for (int l = 0; l < 4; l++) ok &= o[l] == cpu_raw(head.data() + (size_t)l * C, C);
    printf("%-20s mode %d C=%5d B=%4d NB=%d: %.3f ms  %.0f GB/s  crc %s\n", name, MODE, C, B, NB, ms, n / ms / 1e6, ok ? "ok" : "BAD");
}

int main() {
    const uint64_t n = 4294966272ull & ~((1ull << 20) - 1);
    uint8_t* d; uint32_t* out;
    CK(hipMalloc(&d, n)); CK(hipMalloc(&out, n / 16 + 1024));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, d, n);
    CK(hipDeviceSynchronize());
    std::vector<uint8_t> head(4 * 4096);
    CK(hipMemcpy(head.data(), d, head.size(), hipMemcpyDeviceToHost));
    int ncu = 0; CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const int grid = ncu * 2;
    {
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        for (int w = 0; w < 2; w++) hipLaunchKernelGGL(k_coal, dim3(grid * 4), dim3(512), 0, 0, d, n, out);
        CK(hipEventRecord(e0));
        for (int w = 0; w < 10; w++) hipLaunchKernelGGL(k_coal, dim3(grid * 4), dim3(512), 0, 0, d, n, out);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 10;
        printf("coalesced read               %.3f ms  %.0f GB/s\n", ms, n / ms / 1e6);
    }
    run<2048, 128, 1, 0>(d, n, out, grid, "lane chunk", head);
    run<2048, 128, 1, 1>(d, n, out, grid, "lane chunk", head);
    run<2048, 128, 1, 2>(d, n, out, grid, "lane chunk", head);
    run<2048, 128, 1, 3>(d, n, out, grid, "lane chunk", head);
    run<2048, 128, 2, 1>(d, n, out, grid, "lane chunk", head);
    run<2048, 128, 2, 2>(d, n, out, grid, "lane chunk", head);
    run<2048, 256, 1, 1>(d, n, out, grid, "lane chunk", head);
    run<2048, 256, 1, 2>(d, n, out, grid, "lane chunk", head);
    run<2048, 64, 2, 1>(d, n, out, grid, "lane chunk", head);
    run<2048, 64, 2, 2>(d, n, out, grid, "lane chunk", head);
    run<1024, 128, 1, 1>(d, n, out, grid, "lane chunk", head);
    run<1024, 128, 2, 1>(d, n, out, grid, "lane chunk", head);
    run<1024, 128, 2, 0>(d, n, out, grid, "lane chunk", head);
    run<1024, 128, 3, 1>(d, n, out, grid, "lane chunk", head);
    run<1024, 128, 2, 2>(d, n, out, grid, "lane chunk", head);
    run<1024, 128, 2, 3>(d, n, out, grid, "lane chunk", head);
    return 0;
}
