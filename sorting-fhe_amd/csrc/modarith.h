// Word-size modular arithmetic for RNS-CKKS residues (primes < 2^61).
//
// Shared by the host code, the gfx950 HIP kernels and (re-stated in plain C)
// the oracle.  Every routine returns the canonical representative in [0, q)
// unless its name says "lazy", so any two correct implementations agree
// bit-for-bit.
//
// The reference gets this arithmetic from OpenFHE 1.1.4 (external, not
// vendored).  The algorithms are the published ones:
//   * Shoup multiplication by a precomputed constant  w' = floor(w 2^64 / q)
//   * Barrett reduction of a 128-bit product with mu = floor(2^(2b) / q),
//     b = bit length of q (HAC 14.42 / OpenFHE NativeInteger::ModMulFast).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define SF_HD __host__ __device__ __forceinline__
#else
#define SF_HD static inline
#endif

typedef uint64_t u64;
typedef unsigned __int128 u128;

SF_HD u64 sf_mulhi(u64 a, u64 b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul64hi(a, b);
#else
    return (u64)(((u128)a * b) >> 64);
#endif
}

SF_HD u64 sf_add(u64 a, u64 b, u64 q) {
    u64 r = a + b;
    return r >= q ? r - q : r;
}
SF_HD u64 sf_sub(u64 a, u64 b, u64 q) { return a >= b ? a - b : a + q - b; }
SF_HD u64 sf_neg(u64 a, u64 q) { return a ? q - a : 0; }

// Shoup: a * w mod q for a < 2^64, w < q, wp = floor(w * 2^64 / q).
SF_HD u64 sf_mul_shoup_lazy(u64 a, u64 w, u64 wp, u64 q) {
    u64 hi = sf_mulhi(a, wp);
    return a * w - hi * q;  // in [0, 2q)
}
SF_HD u64 sf_mul_shoup(u64 a, u64 w, u64 wp, u64 q) {
    u64 r = sf_mul_shoup_lazy(a, w, wp, q);
    return r >= q ? r - q : r;
}

// Barrett constants for a prime q with bit length b (q < 2^61):
//   mu = floor(2^(2b) / q)  (fits in b+1 bits).
typedef struct {
    u64 q;
    u64 mu;
    u64 r64;     // 2^64 mod q
    uint32_t b;  // bit length of q
    uint32_t pad;
} sf_barrett;

// Reduce a 128-bit value z to [0, q).  Precondition: z < 2^(b+63) so that
// z >> (b-1) fits a word; the estimate never overshoots, and the final loop
// runs at most 2 + z / 2^(2b) times (one or two for a single product, ~18
// for the widest lazy sum of products).  The loop is capped: operands that
// break the precondition (non-canonical residues) give a wrong result in
// bounded time instead of ~2^24 iterations per word on the GPU.
SF_HD u64 sf_reduce128(u64 zlo, u64 zhi, const sf_barrett* m) {
    const uint32_t b = m->b;
    // x = z >> (b-1)
    u64 x = (zhi << (65 - b)) | (zlo >> (b - 1));
    // qhat = (x * mu) >> (b+1)
    u64 plo = x * m->mu;
    u64 phi = sf_mulhi(x, m->mu);
    u64 qhat = (phi << (63 - b)) | (plo >> (b + 1));
    u64 r = zlo - qhat * m->q;
    for (int it = 0; r >= m->q && it < 64; ++it) r -= m->q;
    return r;
}

// Reduce any 128-bit value (e.g. a lazily accumulated sum of products):
// reduce the high word mod q, fold it with 2^64 mod q, then Barrett.
SF_HD u64 sf_reduce128_acc(u64 zlo, u64 zhi, const sf_barrett* m) {
    u64 h = sf_reduce128(zhi, 0, m);
    u64 tlo = h * m->r64;
    u64 thi = sf_mulhi(h, m->r64);
    u64 lo = tlo + zlo;
    u64 hi = thi + (lo < tlo ? 1 : 0);
    return sf_reduce128(lo, hi, m);
}

SF_HD u64 sf_mul(u64 a, u64 b, const sf_barrett* m) {
    u64 lo = a * b;
    u64 hi = sf_mulhi(a, b);
    return sf_reduce128(lo, hi, m);
}

SF_HD u64 sf_shoup_precomp(u64 w, u64 q) {
    return (u64)(((u128)w << 64) / q);
}

SF_HD u64 sf_pow(u64 a, u64 e, const sf_barrett* m) {
    u64 r = 1 % m->q;
    while (e) {
        if (e & 1) r = sf_mul(r, a, m);
        a = sf_mul(a, a, m);
        e >>= 1;
    }
    return r;
}

static inline sf_barrett sf_make_barrett(u64 q) {
    sf_barrett m;
    uint32_t b = 64 - (uint32_t)__builtin_clzll(q);
    m.q = q;
    m.b = b;
    m.pad = 0;
    u128 num = (u128)1 << (2 * b);
    m.mu = (u64)(num / q);
    m.r64 = (u64)((((u128)1) << 64) % q);
    return m;
}

SF_HD uint32_t sf_brev(uint32_t x, uint32_t bits) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __brev(x) >> (32 - bits);
#else
    uint32_t r = 0;
    for (uint32_t i = 0; i < bits; ++i) r |= ((x >> i) & 1u) << (bits - 1 - i);
    return r;
#endif
}
