// gs_rng.h -- counter-based random streams of the native (non-replay) mode.
//
// Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11) keyed by
// (seed_lo, seed_hi ^ global_chain), counter (c0, c1, c2, c3).  The same
// streams are restated in oracle/harmonic.py (philox4x32_10, u53,
// box_muller, gamma_native) so native-mode results are checkable bit-for-bit
// up to libm rounding.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gs {

enum : uint32_t {
    TAG_CR = 1, TAG_GAMMA_N = 2, TAG_GAMMA_U = 3, TAG_GAMMA_BOOST = 4,
    TAG_IW_N = 5, TAG_TN = 6, TAG_MH_U = 7
};

struct Key { uint32_t k0, k1; };

__device__ __forceinline__ Key chain_key(uint32_t seed_lo, uint32_t seed_hi, uint32_t chain) {
    return Key{seed_lo, seed_hi ^ chain};
}

__device__ __forceinline__ uint4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, Key k) {
    uint32_t k0 = k.k0, k1 = k.k1;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        const uint32_t n0 = hi1 ^ c1 ^ k0;
        const uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return make_uint4(c0, c1, c2, c3);
}

// uniform in (0, 1): 53 random bits + half an ulp
__device__ __forceinline__ double u53(uint32_t a, uint32_t b) {
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6) + 0.5) * (1.0 / 9007199254740992.0);
}

__device__ __forceinline__ void box_muller(uint4 w, double& z0, double& z1) {
    const double u1 = u53(w.x, w.y);
    const double u2 = u53(w.z, w.w);
    const double r = sqrt(-2.0 * log(u1));
    double sn, cs;
    sincos(2.0 * M_PI * u2, &sn, &cs);
    z0 = r * cs;
    z1 = r * sn;
}

__device__ __forceinline__ double normal1(Key k, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
    double z0, z1;
    box_muller(philox(c0, c1, c2, c3, k), z0, z1);
    return z0;
}

__device__ __forceinline__ double uniform1(Key k, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
    const uint4 w = philox(c0, c1, c2, c3, k);
    return u53(w.x, w.y);
}

// Marsaglia & Tsang (2000) Gamma(alpha, 1); alpha < 1 via the boost
// G(alpha) = G(alpha + 1) U^(1/alpha).  Attempt j uses counter
// (b, spec | j << 8, TAG | sub << 8, it).  Acceptance > 95 % for alpha >= 1.
__device__ inline double gamma_mt(double alpha, Key k, uint32_t b, uint32_t spec, uint32_t it, uint32_t sub) {
    const double a = alpha >= 1.0 ? alpha : alpha + 1.0;
    const double d = a - 1.0 / 3.0;
    const double c = 1.0 / sqrt(9.0 * d);
    double g = 0.0;
    for (uint32_t j = 0; j < (1u << 20); ++j) {
        const uint32_t cc = spec | (j << 8);
        const double x = normal1(k, b, cc, TAG_GAMMA_N | (sub << 8), it);
        const double u = uniform1(k, b, cc, TAG_GAMMA_U | (sub << 8), it);
        const double t = 1.0 + c * x;
        if (t <= 0.0) continue;
        const double v = t * t * t;
        if (u < 1.0 - 0.0331 * (x * x) * (x * x) || log(u) < 0.5 * x * x + d * (1.0 - v + log(v))) {
            g = d * v;
            break;
        }
    }
    if (alpha < 1.0) {
        const double ub = uniform1(k, b, spec, TAG_GAMMA_BOOST | (sub << 8), it);
        g = g * exp(log(ub) / alpha);
    }
    return g;
}

}  // namespace gs
