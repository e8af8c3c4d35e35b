// Microbenchmark (not product): does waiting for the next block's loads with
// vmcnt(0) -- which also waits for the stores issued after them -- cost k_scan's
// store streams?  Each wave streams 4-KiB blocks (one in flight), runs the
// CRC-like table chain, stores a 16-B entry from 16 lanes and a 4-B register
// from every lane per block (k_scan's compact entries and segment registers),
// and waits for its next block: mode 0 as the compiler places the wait (the two
// stores are unconditional, so it counts them: vmcnt(2), they stay in flight),
// mode 4 with a vmcnt(0) added at the top (what a data-dependent number of
// stores makes the compiler emit: the wait covers the stores too), mode 3
// without the stores.  Checksums of the loaded words are printed side by side.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define LDSP __attribute__((address_space(3)))
#define NBLK 16
#define WAVES 16
typedef __amdgpu_buffer_rsrc_t rsrc_t;
__device__ __forceinline__ rsrc_t mk(const void* p, uint32_t n) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)n, 0x00020000);
}
template <int MODE>  // 0: counted wait (compiler), 3: no stores, 4: vmcnt(0) at the top
__global__ void __launch_bounds__(64 * WAVES) kwait(const uint8_t* buf, uint32_t ntiles, uint32_t* rec, uint32_t* seg,
                                                    uint32_t* out) {
  __shared__ uint32_t tab[16384];
  for (int i = threadIdx.x; i < 16384; i += blockDim.x) tab[i] = i * 2654435761u;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t r4 = (lane & 15) * 4;
  uint32_t acc = 0;
  for (uint32_t t = blockIdx.x * WAVES + wv; t < ntiles; t += gridDim.x * WAVES) {
    const rsrc_t r = mk(buf + (uint64_t)t * NBLK * 4096, NBLK * 4096);
    const rsrc_t trs = mk(rec + (uint64_t)t * 512 * 4, 512 * 16);
    const rsrc_t srs = mk(seg + (uint64_t)t * 1024, 1024 * 4);
    const uint32_t off0 = 64u * (lane & 15) + 16u * (lane >> 4);
    u32x4 e0, e1, e2, e3;
    e0 = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off0, 0, 0);
    e1 = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(off0 + 1024), 0, 0);
    e2 = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(off0 + 2048), 0, 0);
    e3 = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(off0 + 3072), 0, 0);
    uint32_t tcnt = 0;
#pragma unroll 1
    for (int m = 0; m < NBLK; m++) {
      if (MODE == 4) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      uint32_t w[16] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w, e2.x, e2.y, e2.z, e2.w, e3.x, e3.y, e3.z, e3.w};
      if (m + 1 < NBLK) {
        const uint32_t o = off0 + (m + 1) * 4096u;
        e0 = __builtin_amdgcn_raw_buffer_load_b128(r, (int)o, 0, 0);
        e1 = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(o + 1024), 0, 0);
        e2 = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(o + 2048), 0, 0);
        e3 = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(o + 3072), 0, 0);
      }
      uint32_t R = 0;
#pragma unroll
      for (int k = 0; k < 16; k++) {
        const uint32_t x = R ^ w[k];
        R = tab[((x & 0xff) << 6 | r4) >> 2 & 16383] ^ tab[(((x >> 8) & 0xff) << 6 | (r4 + 64)) >> 2 & 16383] ^
            tab[(((x >> 16) & 0xff) << 6 | r4) >> 2 & 16383] ^ tab[((x >> 24) << 6 | (r4 + 64)) >> 2 & 16383];
      }
      acc ^= R + w[(m + lane) & 15];
      if (MODE != 3) {
        // one entry store (16 lanes, 256 B), one segment-register store (every lane), both after the loads
        const uint32_t eo = lane < 16 ? ((tcnt + lane) & 511) * 16u : 0x40000000u;   // out of range: dropped
        __builtin_amdgcn_raw_buffer_store_b128((u32x4){R, w[0], w[1], (uint32_t)m}, trs, (int)eo, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32(R, srs, (int)((m * 64 + lane) * 4), 0, 0);
      }
      tcnt += 15;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
__global__ void kfill(uint32_t* p, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = (uint32_t)(i * 0x9E3779B97F4A7C15ull >> 29);
}
template <int MODE>
void run(const uint8_t* buf, uint32_t ntiles, uint32_t* rec, uint32_t* seg, uint32_t* out, uint32_t* h) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  for (int i = 0; i < 3; i++) kwait<MODE><<<256, 64 * WAVES>>>(buf, ntiles, rec, seg, out);
  (void)hipEventRecord(a);
  const int reps = 10;
  for (int i = 0; i < reps; i++) kwait<MODE><<<256, 64 * WAVES>>>(buf, ntiles, rec, seg, out);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  ms /= reps;
  (void)hipMemcpy(h, out, 256 * 1024 * 4, hipMemcpyDeviceToHost);
  uint32_t cs = 0;
  for (int i = 0; i < 256 * 1024; i++) cs = cs * 31 + h[i];
  printf("mode %d  %.3f ms  %.2f TB/s  checksum %08x\n", MODE, ms, (double)ntiles * NBLK * 4096 / ms / 1e9, cs);
}
int main() {
  const uint32_t ntiles = 65536;
  uint8_t* buf;
  uint32_t *out, *rec, *seg;
  (void)hipMalloc(&buf, (size_t)ntiles * NBLK * 4096);
  kfill<<<4096, 256>>>((uint32_t*)buf, (uint64_t)ntiles * NBLK * 1024);
  (void)hipMalloc(&out, 256 * 1024 * 4);
  (void)hipMalloc(&rec, (size_t)ntiles * 512 * 16);
  (void)hipMalloc(&seg, (size_t)ntiles * 1024 * 4);
  static uint32_t h[256 * 1024];
  for (int rep = 0; rep < 2; rep++) {
    run<0>(buf, ntiles, rec, seg, out, h);
    run<4>(buf, ntiles, rec, seg, out, h);
    run<3>(buf, ntiles, rec, seg, out, h);
  }
  return 0;
}
