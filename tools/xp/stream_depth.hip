// Microbenchmark (not product): streaming 4-KiB blocks per wave with D blocks in
// flight and W units of CRC-like work per block, to find k_scan's latency/issue floor.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define TILE_BLK 16
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mk(const void* p, uint32_t n) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)n, 0x00020000);
}
__device__ __forceinline__ void issue(__amdgpu_buffer_rsrc_t r, uint32_t bs, int lane, u32x4 (&e)[4]) {
  const uint32_t off = bs + 64u * (lane & 15) + 16u * (lane >> 4);
#pragma unroll
  for (int k = 0; k < 4; k++) e[k] = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(off + 1024u * k), 0, 0);
}
template <int WORK>
__device__ __forceinline__ uint32_t work(const __attribute__((address_space(3))) uint32_t* tab, const u32x4 (&e)[4], uint32_t acc, int lane) {
  uint32_t w[16];
#pragma unroll
  for (int k = 0; k < 4; k++) { w[4*k] = e[k].x; w[4*k+1] = e[k].y; w[4*k+2] = e[k].z; w[4*k+3] = e[k].w; }
  if (WORK == 0) { uint32_t x = acc; for (int k = 0; k < 16; k++) x ^= w[k]; return x; }
  uint32_t R = 0;
  const uint32_t r4 = (lane & 15) * 4;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const uint32_t x = R ^ w[k];
    const uint32_t a0 = ((x & 0xff) << 8) | r4, a1 = (((x >> 8) & 0xff) << 8) | (r4 + 64);
    const uint32_t a2 = (((x >> 16) & 0xff) << 8) | r4, a3 = ((x >> 24) << 8) | (r4 + 64);
    R = tab[a0 >> 2] ^ tab[a1 >> 2] ^ tab[(a2 + 128) >> 2] ^ tab[(a3 + 128) >> 2];
  }
  if (WORK >= 2) {   // extra dependent integer work (~WORK*40 VALU)
    uint32_t y = R;
#pragma unroll
    for (int i = 0; i < 20 * WORK; i++) y = __builtin_amdgcn_alignbyte(y, y ^ (uint32_t)i, 1) + w[i & 15];
    R ^= y;
  }
  return acc ^ R;
}
template <int D, int WORK, int WAVES>
__global__ void __launch_bounds__(64 * WAVES) kstream(const uint8_t* buf, uint32_t ntiles, uint32_t* out) {
  __shared__ uint32_t tab[37000];   // 148 KB: one workgroup per CU, as k_scan
  for (int i = threadIdx.x; i < 16384; i += blockDim.x) tab[i] = i * 2654435761u;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t acc = 0;
  const auto* T = (const __attribute__((address_space(3))) uint32_t*)tab;
  for (uint32_t t = blockIdx.x * WAVES + wv; t < ntiles; t += gridDim.x * WAVES) {
    const auto r = mk(buf + (uint64_t)t * TILE_BLK * 4096, TILE_BLK * 4096);
    if (D == 1) {
      u32x4 e[4];
      issue(r, 0, lane, e);
#pragma unroll 1
      for (int m = 0; m < TILE_BLK; m++) {
        u32x4 c[4] = {e[0], e[1], e[2], e[3]};
        if (m + 1 < TILE_BLK) issue(r, (m + 1) * 4096, lane, e);
        acc = work<WORK>(T, c, acc, lane);
      }
    } else {
      u32x4 e0[4], e1[4];
      issue(r, 0, lane, e0);
      issue(r, 4096, lane, e1);
#pragma unroll 1
      for (int m = 0; m < TILE_BLK; m += 2) {
        u32x4 c[4] = {e0[0], e0[1], e0[2], e0[3]};
        if (m + 2 < TILE_BLK) issue(r, (m + 2) * 4096, lane, e0);
        acc = work<WORK>(T, c, acc, lane);
        u32x4 d[4] = {e1[0], e1[1], e1[2], e1[3]};
        if (m + 3 < TILE_BLK) issue(r, (m + 3) * 4096, lane, e1);
        acc = work<WORK>(T, d, acc, lane);
      }
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
template <int D, int WORK, int WAVES>
void run(const uint8_t* buf, uint32_t ntiles, uint32_t* out, const char* name) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const int grid = 256;
  for (int i = 0; i < 3; i++) kstream<D, WORK, WAVES><<<grid, 64 * WAVES>>>(buf, ntiles, out);
  hipEventRecord(a);
  const int reps = 10;
  for (int i = 0; i < reps; i++) kstream<D, WORK, WAVES><<<grid, 64 * WAVES>>>(buf, ntiles, out);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b); ms /= reps;
  double bytes = (double)ntiles * TILE_BLK * 4096;
  printf("%-28s D=%d WORK=%d WAVES=%2d  %.3f ms  %.2f TB/s\n", name, D, WORK, WAVES, ms, bytes / ms / 1e9);
}
int main() {
  const uint32_t ntiles = 65536;     // 4 GiB
  uint8_t* buf; uint32_t* out;
  hipMalloc(&buf, (size_t)ntiles * TILE_BLK * 4096);
  hipMemset(buf, 0x5a, (size_t)ntiles * TILE_BLK * 4096);
  hipMalloc(&out, 256 * 1024 * 4);
  run<1, 0, 16>(buf, ntiles, out, "floor");
  run<2, 0, 16>(buf, ntiles, out, "floor");
  run<1, 0, 8>(buf, ntiles, out, "floor");
  run<2, 0, 8>(buf, ntiles, out, "floor");
  run<1, 1, 16>(buf, ntiles, out, "crc");
  run<2, 1, 16>(buf, ntiles, out, "crc");
  run<2, 1, 12>(buf, ntiles, out, "crc");
  run<2, 1, 8>(buf, ntiles, out, "crc");
  run<1, 4, 16>(buf, ntiles, out, "crc+160");
  run<2, 4, 16>(buf, ntiles, out, "crc+160");
  run<2, 4, 12>(buf, ntiles, out, "crc+160");
  run<1, 8, 16>(buf, ntiles, out, "crc+320");
  run<2, 8, 16>(buf, ntiles, out, "crc+320");
  run<2, 8, 12>(buf, ntiles, out, "crc+320");
  return 0;
}
