// Microbenchmark (not product): k_scan's per-block skeleton built up feature by
// feature (transpose, LDS stage, CRC, segment-register store, snapshots, stride
// round) over 4 GiB of 276-B "records", one 16-wave workgroup per CU.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
#define LDSP __attribute__((address_space(3)))
#define NBLK 16
#define WAVES 16
#define STG_BYTES (64 * 80 + 32)
#define F_TR 1
#define F_STG 2
#define F_CRC 4
#define F_SEG 8
#define F_SNAP 16
#define F_STRIDE 32
#define F_X3 64      // bitop3 xor in the CRC
#define F_NOST 128
#define F_SEGT 256
#define F_NT 512
#define F_SEGAFT 1024
#define F_SEG4 2048     // segment registers stored as one b128 per lane every 4 blocks
#define F_R8 4096       // 8 CRC table replicas (32 KB) instead of 16
#define F_SNK 8192      // compact entries through a 1-KiB LDS sink per wave, flushed as whole 1-KiB stores
#define F_E8 16384      // compact entries of 8 B
#define F_SEGH 32768    // segment registers at 128-B granularity (even lanes store)
#define F_SEGQ 65536    // ... at 256-B granularity (lanes % 4 == 0 store)
#define F_KS 131072     // no segment registers stored: a segmented Kogge-Stone scan of the
                        // segments' registers over the lanes (A^(64 2^l) by nibble tables)
                        // and the register entering a record start's word (A^(4k) by four
                        // nibble matrices) -- k_scan checking every record itself
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mk(const void* p, uint32_t n) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)n, 0x00020000);
}
__device__ __forceinline__ uint32_t dppsl1(uint32_t old, uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x130, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t rdl(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
__device__ __forceinline__ void swap32(uint32_t& a, uint32_t& b) { auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false); a = r[0]; b = r[1]; }
__device__ __forceinline__ void swap16(uint32_t& a, uint32_t& b) { auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false); a = r[0]; b = r[1]; }
__device__ __forceinline__ uint32_t wave_add_incl(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
  return v;
}
template <int F>
__device__ __forceinline__ uint32_t crc_word(const LDSP uint8_t* sm, uint32_t x, uint32_t oe, uint32_t oo, uint32_t s0,
                                             uint32_t s1, uint32_t s2, uint32_t s3, uint32_t nxt) {
  const uint32_t a0 = __builtin_amdgcn_perm(x, oe, s0), a1 = __builtin_amdgcn_perm(x, oo, s1);
  const uint32_t a2 = __builtin_amdgcn_perm(x, oe, s2), a3 = __builtin_amdgcn_perm(x, oo, s3);
  const uint32_t t0 = *(const LDSP uint32_t*)(sm + a0), t1 = *(const LDSP uint32_t*)(sm + a1);
  const uint32_t t2 = *(const LDSP uint32_t*)(sm + a2 + 128), t3 = *(const LDSP uint32_t*)(sm + a3 + 128);
  if (F & F_X3) return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(t0, t1, nxt, 0x96), t2, t3, 0x96);
  return t0 ^ t1 ^ t2 ^ t3 ^ nxt;
}
__device__ __forceinline__ uint32_t nib_mul(const LDSP uint32_t* T, uint32_t x) {
  uint32_t y = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) y ^= T[j * 16 + ((x >> (4 * j)) & 15u)];
  return y;
}
template <int F>
__global__ void __launch_bounds__(64 * WAVES) kskel(const uint8_t* buf, uint32_t ntiles, uint32_t* rec, uint32_t* seg,
                                                    uint32_t* snap, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[65536 + 256 + WAVES * (STG_BYTES + 256) + ((F & F_SNK) ? WAVES * 2048 : 0) + ((F & F_KS) ? 10 * 512 : 0)];
  for (int i = threadIdx.x; i < 16384; i += blockDim.x) ((LDSP uint32_t*)smem)[i] = i * 2654435761u;
  LDSP uint32_t* kst = (LDSP uint32_t*)(smem + 65536 + 256 + WAVES * (STG_BYTES + 256) + ((F & F_SNK) ? WAVES * 2048 : 0));
  if (F & F_KS) for (int i = threadIdx.x; i < 10 * 128; i += blockDim.x) kst[i] = i * 0x9E3779B9u;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  LDSP uint8_t* sm = (LDSP uint8_t*)smem;
  LDSP uint32_t* stg = (LDSP uint32_t*)(sm + 65536 + 256 + wv * STG_BYTES);
  LDSP uint32_t* mkk = (LDSP uint32_t*)(sm + 65536 + 256 + WAVES * STG_BYTES + wv * 256);
  LDSP u32x4* sv = (LDSP u32x4*)stg;
  LDSP u32x4* snk = (LDSP u32x4*)(sm + 65536 + 256 + WAVES * (STG_BYTES + 256)) + wv * 128;
  LDSP uint32_t* segl = nullptr;
  const uint32_t r4 = (F & F_R8) ? (lane & 7) * 4 : (lane & 15) * 4, h = (lane >> 4) & 1;
  const uint32_t oe = r4 + 64 * h, oo = r4 + 64 * (1 - h);
  const uint32_t s0 = 0x0c0c0000u | ((4u + (3u - (0u ^ h))) << 8), s1 = 0x0c0c0000u | ((4u + (3u - (1u ^ h))) << 8);
  const uint32_t s2 = 0x0c0c0000u | ((4u + (3u - (2u ^ h))) << 8), s3 = 0x0c0c0000u | ((4u + (3u - (3u ^ h))) << 8);
  uint32_t acc = 0;
  for (uint32_t t = blockIdx.x * WAVES + wv; t < ntiles; t += gridDim.x * WAVES) {
    const uint32_t tb = t * NBLK * 4096;
    const auto r = mk(buf + (uint64_t)tb, NBLK * 4096 + 32);
    const auto trs = mk(rec + (uint64_t)t * 512 * 4, 512 * 16);
    const auto srs = mk(seg + (uint64_t)t * 1024, 1024 * 4);
    const auto nrs = mk(snap + (uint64_t)t * 516, 513 * 4);
    u32x4 e[4], hl = {0, 0, 0, 0};
    const uint32_t off0 = 64u * (lane & 15) + 16u * (lane >> 4);
#pragma unroll
    for (int k = 0; k < 4; k++) e[k] = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(off0 + 1024u * k), 0, 0);
    if ((F & F_STG) && lane < 2) hl = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(4096 + 16 * lane), 0, 0);
    uint32_t X = (t * 37u) % 276u, tcnt = 0, nb = 0, Rp = 0, sq[4] = {0, 0, 0, 0}, sk = 0, gcar = 0;
#pragma unroll 1
    for (int m = 0; m < NBLK; m++) {
      const uint32_t bs = m * 4096;
      if (F & F_TR) {
#pragma unroll
        for (int c = 0; c < 4; c++) {
          uint32_t a0 = e[0][c], a1 = e[1][c], a2 = e[2][c], a3 = e[3][c];
          swap32(a0, a2); swap32(a1, a3); swap16(a0, a1); swap16(a2, a3);
          e[0][c] = a0; e[1][c] = a1; e[2][c] = a2; e[3][c] = a3;
        }
      }
      uint32_t w[16];
#pragma unroll
      for (int k = 0; k < 4; k++) { w[4*k] = e[k].x; w[4*k+1] = e[k].y; w[4*k+2] = e[k].z; w[4*k+3] = e[k].w; }
      const u32x4 hc = hl;
      const bool segl_on = (F & F_SEGQ) ? (lane & 3) == 0 : (F & F_SEGH) ? (lane & 1) == 0 : true;
      const int segdiv = (F & F_SEGQ) ? 4 : (F & F_SEGH) ? 2 : 1;
      if ((F & F_SEG) && !(F & (F_SEGT | F_SEGAFT | F_SEG4)) && m > 0 && segl_on) __builtin_amdgcn_raw_buffer_store_b32(Rp, srs, (int)(((m - 1) * (64 / segdiv) + lane / segdiv) * 4), 0, (F & F_NT) ? 2 : 0);
      if ((F & F_SEGT) && m > 0) segl[(m - 1) * 64 + lane] = Rp;
      if (m + 1 < NBLK) {
#pragma unroll
        for (int k = 0; k < 4; k++) e[k] = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(bs + 4096 + off0 + 1024u * k), 0, 0);
        if ((F & F_STG) && lane < 2) hl = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(bs + 8192 + 16 * lane), 0, 0);
      }
      if (F & F_SNAP) mkk[lane] = 0;
      if (F & F_STG) {
        const uint32_t t0x = rdl(hc.x, 0), t0y = rdl(hc.y, 0), t0z = rdl(hc.z, 0), t0w = rdl(hc.w, 0);
#pragma unroll
        for (int k = 0; k < 4; k++) sv[5 * lane + k] = (u32x4){w[4*k], w[4*k+1], w[4*k+2], w[4*k+3]};
        const u32x4 nx = (u32x4){dppsl1(t0x, w[0]), dppsl1(t0y, w[1]), dppsl1(t0z, w[2]), dppsl1(t0w, w[3])};
        sv[5 * lane + 4] = nx;
        if (lane == 63) { sv[5 * lane + 5] = nx; sv[5 * lane + 6] = (u32x4){rdl(hc.x, 1), rdl(hc.y, 1), rdl(hc.z, 1), rdl(hc.w, 1)}; }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      if (F & F_STRIDE) {
        // lanes k: records at X + 276 k inside the block; header words from the stage
        const uint32_t k = lane, P = X + 276u * k;
        const bool act = P < 4096u;
        const uint32_t Pc = act ? P : X;
        const uint32_t d = Pc >> 2;
        const LDSP uint32_t* q = stg + d + ((d >> 4) << 2);
        const uint32_t w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3], w4 = q[4], sh = Pc & 3;
        const uint32_t crc = __builtin_amdgcn_alignbyte(w1, w0, sh), h1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
        const uint32_t h2 = __builtin_amdgcn_alignbyte(w3, w2, sh), h3 = __builtin_amdgcn_alignbyte(w4, w3, sh);
        const bool match = act && ((h1 ^ 0x5a5a5a5au) & 0x00ffffffu) != 1u && ((h2 ^ h3) != 7u);
        const uint64_t bm = __ballot(!match);
        const uint32_t kb = bm ? (uint32_t)__ffsll((long long)bm) - 1 : 64u;
        if (k < kb && (F & F_NOST)) acc ^= crc + P;
        if ((F & F_SNK) && k < kb) snk[(sk + k) & 127] = (u32x4){crc, 0x11, 0x100, P | 0x4000000};
        if (k < kb && !(F & (F_NOST | F_SNK)) && !(F & F_E8)) {
          __builtin_amdgcn_raw_buffer_store_b128((u32x4){crc, 0x11, 0x100, (P - 0) | 0x4000000}, trs, (int)(((tcnt + k) & 511) * 16u), 0, (F & F_NT) ? 2 : 0);
        }
        if (k < kb && !(F & (F_NOST | F_SNK)) && (F & F_E8)) {
          __builtin_amdgcn_raw_buffer_store_b64((u32x2){crc, (P - 0) | 0x4000000}, trs, (int)(((tcnt + k) & 511) * 8u), 0, 0);
        }
        if (k < kb) {
          if (F & F_SNAP) {
            const uint32_t pw = (P >> 2) + ((P & 3) ? 1 : 0);
            if (pw < 1024) __atomic_fetch_or(mkk + (pw >> 4), 1u << (pw & 15u), __ATOMIC_RELAXED);
          }
        }
        const uint32_t lastc = rdl(crc, (int)kb - 1);
        acc ^= lastc;
        tcnt += kb;
        X = X + kb * 276u - 4096u;
        if (F & F_SNK) {
          sk += kb;
          if (sk >= 64) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint32_t b0 = (tcnt - sk) & ~63u;
            __builtin_amdgcn_raw_buffer_store_b128(snk[((tcnt - sk) + lane) & 127], trs, (int)(((b0 + lane) * 16u) & 8191u), 0, 0);
            sk -= 64;
          }
        }
      }
      if (F & F_CRC) {
        uint32_t R = 0;
        uint32_t x = w[0];
#pragma unroll
        for (int k = 0; k < 16; k++) {
          const uint32_t enter = x ^ w[k];   // the register entering word k
          const uint32_t nx = crc_word<F>(sm, x, oe, oo, s0, s1, s2, s3, k < 15 ? w[k + 1] : 0u);
          w[k] = enter;
          x = nx;
        }
        R = x;
        Rp = R;
        if ((F & F_SEGAFT)) __builtin_amdgcn_raw_buffer_store_b32(R, srs, (int)((m * 64 + lane) * 4), 0, 0);
        if (F & F_SEG4) {
          sq[m & 3] = R;
          if ((m & 3) == 3) __builtin_amdgcn_raw_buffer_store_b128((u32x4){sq[0], sq[1], sq[2], sq[3]}, srs, (int)(((m >> 2) * 64 + lane) * 16), 0, 0);
        }
        if (F & F_KS) {
          // segmented inclusive scan of (reset, register) over the lanes
          uint32_t v = R, rf = ((lane * 7 + m) % 5 == 0) ? 1u : 0u;
#pragma unroll
          for (int l = 0; l < 6; l++) {
            const int d = 1 << l;
            const uint32_t vp = (uint32_t)__shfl_up((int)v, d, 64), rp = (uint32_t)__shfl_up((int)rf, d, 64);
            if (lane >= d && !rf) { v = nib_mul(kst + l * 128, vp) ^ v; rf = rp; }
          }
          uint32_t gin = (uint32_t)__shfl_up((int)v, 1, 64);
          if (lane == 0) gin = gcar;
          gcar = rdl(v, 63);
          // the register entering the segment's first record start (word k): A^(4k) gin ^ w[k]
          if (rf) {
            const uint32_t k = (uint32_t)(lane & 15);
            uint32_t x = gin;
            if (k & 1) x = nib_mul(kst + 6 * 128, x);
            if (k & 2) x = nib_mul(kst + 7 * 128, x);
            if (k & 4) x = nib_mul(kst + 8 * 128, x);
            if (k & 8) x = nib_mul(kst + 9 * 128, x);
            acc ^= x ^ w[k & 15];
          }
          acc ^= v;
        }
        acc ^= R;
      } else {
#pragma unroll
        for (int k = 0; k < 16; k++) acc ^= w[k];
      }
      if (F & F_SNAP) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t mm = mkk[lane];
        if (__ballot(mm != 0u)) {
#pragma unroll
          for (int k = 0; k < 4; k++) sv[5 * lane + k] = (u32x4){w[4*k], w[4*k+1], w[4*k+2], w[4*k+3]};
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          const uint32_t c = (uint32_t)__builtin_popcount(mm), incl = wave_add_incl(c);
          uint32_t rr = nb + incl - c, qq = mm;
          nb += rdl(incl, 63);
          while (__ballot(qq != 0u)) {
            if (qq) {
              const uint32_t kk = (uint32_t)__builtin_ctz(qq);
              qq &= qq - 1u;
              __builtin_amdgcn_raw_buffer_store_b32(stg[20u * (uint32_t)lane + kk], nrs, (int)((rr & 511) * 4u), 0, 0);
              rr++;
            }
          }
        }
      }
    }
    if ((F & F_SEG) && !(F & (F_SEGT | F_SEGAFT | F_SEG4))) __builtin_amdgcn_raw_buffer_store_b32(Rp, srs, (int)((15 * 64 + lane) * 4), 0, 0);
    if ((F & F_SNK) && sk) __builtin_amdgcn_raw_buffer_store_b128(snk[lane], trs, (int)((((tcnt - sk) & ~63u) + lane) * 16u & 8191u), 0, 0);
    if (F & F_SEGT) {
      segl[15 * 64 + lane] = Rp;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int k = 0; k < 4; k++) __builtin_amdgcn_raw_buffer_store_b128(((LDSP u32x4*)segl)[k * 64 + lane], srs, (int)((k * 64 + lane) * 16), 0, 0);
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
template <int F>
void run(const uint8_t* buf, uint32_t ntiles, uint32_t* rec, uint32_t* seg, uint32_t* snap, uint32_t* out) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int i = 0; i < 3; i++) kskel<F><<<256, 64 * WAVES>>>(buf, ntiles, rec, seg, snap, out);
  hipEventRecord(a);
  const int reps = 10;
  for (int i = 0; i < reps; i++) kskel<F><<<256, 64 * WAVES>>>(buf, ntiles, rec, seg, snap, out);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b); ms /= reps;
  printf("F=%4d tr=%d stg=%d crc=%d seg=%d snap=%d stride=%d x3=%d  %.3f ms  %.2f TB/s\n", F, !!(F & 1), !!(F & 2), !!(F & 4),
         !!(F & 8), !!(F & 16), !!(F & 32), !!(F & 64), ms, (double)ntiles * NBLK * 4096 / ms / 1e9);
}
int main() {
  const uint32_t ntiles = 65536;
  uint8_t* buf; uint32_t *out, *rec, *seg, *snap;
  hipMalloc(&buf, (size_t)ntiles * NBLK * 4096 + 65536);
  hipMemset(buf, 0x5a, (size_t)ntiles * NBLK * 4096 + 65536);
  hipMalloc(&out, 256 * 1024 * 4);
  hipMalloc(&rec, (size_t)ntiles * 512 * 16);
  hipMalloc(&seg, (size_t)ntiles * 1024 * 4);
  hipMalloc(&snap, (size_t)ntiles * 516 * 4);
#define R(F) run<F>(buf, ntiles, rec, seg, snap, out)
  for (int rep = 0; rep < 2; rep++) {
    R(7 + 64); R(127); R(127 - 8); R(127 - 8 + F_KS); R(127 - 8 - 16); R(127 - 8 - 16 + F_KS); R(127 + F_KS);
  }
  return 0;
}
