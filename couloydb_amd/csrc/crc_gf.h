// crc_gf.h — CRC-32/IEEE arithmetic shared by host and device code of
// libclyscan (the product library; not the oracle).
//
// Register convention: the reflected CRC-32 register `s` that Go's
// crc32.Update keeps between bytes (init 0xFFFFFFFF, final = ~s), i.e. the
// checksum of data/logRecord.go:80 and :141-143 is ~reg(0xFFFFFFFF, bytes).
// Processing one zero byte is the linear map A: s -> T0[s & 0xff] ^ (s >> 8).
// A^L (L zero bytes) equals multiplication by x^(8L) mod P in the reflected
// polynomial representation (bit 31 = x^0); that identity is what lets a
// long record's CRC be assembled from independently computed pieces.
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#define CLY_HD __host__ __device__ __forceinline__
#else
#define CLY_HD static inline
#endif

#define CLY_POLY 0xEDB88320u

// a * b mod P, reflected representation (bit 31 = x^0).  Bounded loop: no
// forward-progress assumptions for the optimizer to exploit when a == 0.
CLY_HD uint32_t cly_multmodp(uint32_t a, uint32_t b) {
    uint32_t p = 0;
    for (int k = 31; k >= 0; k--) {
        if (a & (1u << k)) p ^= b;
        b = (b & 1) ? (b >> 1) ^ CLY_POLY : b >> 1;
    }
    return p;
}

// x^(8*nbytes) mod P, by square-and-multiply over x^(2^k).
CLY_HD uint32_t cly_x8n(uint64_t nbytes) {
    uint32_t p = 1u << 31;          // x^0
    uint32_t sq = 1u << 23;         // x^8 (one byte)
    while (nbytes) {
        if (nbytes & 1) p = cly_multmodp(sq, p);
        sq = cly_multmodp(sq, sq);
        nbytes >>= 1;
    }
    return p;
}

// Register after L zero bytes: A^L s.
CLY_HD uint32_t cly_shift(uint32_t s, uint64_t nbytes) {
    return nbytes ? cly_multmodp(cly_x8n(nbytes), s) : s;
}

// One byte through the register without a table (bitwise).
CLY_HD uint32_t cly_crc_byte_bitwise(uint32_t s, uint8_t b) {
    s ^= b;
    for (int k = 0; k < 8; k++) s = (s & 1) ? (s >> 1) ^ CLY_POLY : s >> 1;
    return s;
}
