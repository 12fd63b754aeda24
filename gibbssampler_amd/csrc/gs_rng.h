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
#include "gs_bm_tables.h"

namespace gs {

enum : uint32_t {
    TAG_CR = 1, TAG_GAMMA_N = 2, TAG_GAMMA_U = 3, TAG_GAMMA_BOOST = 4,
    TAG_IW_N = 5, TAG_TN = 6, TAG_MH_U = 7
};

struct Key { uint32_t k0, k1; };

__device__ __forceinline__ Key chain_key(uint32_t seed_lo, uint32_t seed_hi, uint32_t chain) {
    return Key{seed_lo, seed_hi ^ chain};
}

// UKEY: the key is wave-uniform (one chain per workgroup), so the round key can
// sit in an SGPR and each Philox word costs one gfx950 three-input XOR
// (v_bitop3, truth table 0x96); with a per-lane key the plain two-XOR form.
template <bool UKEY = false>
__device__ __forceinline__ uint4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, Key k) {
    uint32_t k0 = k.k0, k1 = k.k1;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        // one v_mad_u64_u32 per product (hi:lo in a register pair)
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0, n2;
        if constexpr (UKEY) {
            // the builtin rather than inline asm: the hazard recognizer treats an
            // asm block conservatively (an s_nop after each pair in the sweep)
            n0 = __builtin_amdgcn_bitop3_b32(hi1, c1, k0, 0x96);
            n2 = __builtin_amdgcn_bitop3_b32(hi0, c3, k1, 0x96);
        } else {
            n0 = hi1 ^ c1 ^ k0;
            n2 = hi0 ^ c3 ^ k1;
        }
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return make_uint4(c0, c1, c2, c3);
}

// uniform in (0, 1): 53 random bits + half an ulp
__device__ __forceinline__ double u53(uint32_t a, uint32_t b) {
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6) + 0.5) * (1.0 / 9007199254740992.0);
}

// ln(x) for normal finite x > 0 (the Box-Muller radius): x = m 2^e with
// m in [sqrt(1/2), sqrt(2)); ln m = 2 atanh(s), s = (m-1)/(m+1), |s| < 0.172;
// the atanh series through s^21 is below 2.5e-17 relative; m - 1 is exact.
__device__ __forceinline__ double bm_log(double x) {
    int e;
    double m = frexp(x, &e);
    if (m < 0.70710678118654752440) { m *= 2.0; e -= 1; }
    const double f = m - 1.0;
    const double sv = f / (2.0 + f);
    const double s2 = sv * sv;
    double p = 0.047619047619047616;
    p = fma(p, s2, 0.05263157894736842);
    p = fma(p, s2, 0.058823529411764705);
    p = fma(p, s2, 0.06666666666666667);
    p = fma(p, s2, 0.07692307692307693);
    p = fma(p, s2, 0.09090909090909091);
    p = fma(p, s2, 0.1111111111111111);
    p = fma(p, s2, 0.14285714285714285);
    p = fma(p, s2, 0.2);
    p = fma(p, s2, 0.3333333333333333);
    const double ts = 2.0 * sv;
    const double lnm = fma(ts * s2, p, ts);
    const double de = (double)e;
    return fma(de, 0.6931471805599453, fma(de, 2.3190468138462996e-17, lnm));
}

// sin and cos of 2 pi u for u in (0, 1): u = q/4 + y exactly (|y| <= 1/8),
// Taylor polynomials of sin(2 pi y) / cos(2 pi y) (|2 pi y| <= pi/4,
// truncation < 5e-17), then the quadrant rotation.
__device__ __forceinline__ void bm_sincos2pi(double u, double& sn, double& cs) {
    const double q = rint(4.0 * u);
    const double y = fma(q, -0.25, u);
    const double y2 = y * y;
    double ps = 0.10422916220813984;
    ps = fma(ps, y2, -0.7181223017785006);
    ps = fma(ps, y2, 3.819952584848282);
    ps = fma(ps, y2, -15.09464257682299);
    ps = fma(ps, y2, 42.058693944897655);
    ps = fma(ps, y2, -76.70585975306139);
    ps = fma(ps, y2, 81.60524927607506);
    ps = fma(ps, y2, -41.34170224039976);
    ps = fma(ps, y2, 6.283185307179586);
    const double sy = ps * y;
    double pc = -0.03638284114254567;
    pc = fma(pc, y2, 0.28200596845579123);
    pc = fma(pc, y2, -1.714390711088672);
    pc = fma(pc, y2, 7.903536371318469);
    pc = fma(pc, y2, -26.4262567833744);
    pc = fma(pc, y2, 60.24464137187666);
    pc = fma(pc, y2, -85.45681720669373);
    pc = fma(pc, y2, 64.9393940226683);
    pc = fma(pc, y2, -19.739208802178716);
    const double cy = fma(pc, y2, 1.0);
    const int k = (int)q & 3;
    const double a = (k & 1) ? cy : sy;
    const double b = (k & 1) ? sy : cy;
    sn = (k & 2) ? -a : a;
    cs = ((k + 1) & 2) ? -b : b;
}

// sqrt(x) for the Box-Muller radius x = -2 ln u1, u1 in (0, 1]: x is +-0 or
// lies in [2^-53, 75], never below the 2^-767 where the compiler's fp64 sqrt
// expansion rescales its argument (by 2^256 in, 2^-128 out).  This is that
// expansion (rsq seed, one Goldschmidt step, a Newton correction) without the
// rescaling, whose scale factors are 2^0 on this range, and without its second
// Newton correction: the rsq seed is good to ~2^-22, the Goldschmidt step
// doubles that and the Newton step leaves <= 1 ulp (r06: the correctly-rounded
// second correction cost two fp64 FMAs per normal pair, 1.7 % of the headline
// step, tools/lib_ab.py; the native streams are checked against the oracle's
// libm Box-Muller at 1e-10).  Its +-0 / +inf class select becomes a clamp of
// the seed: for x > 0 here rsq(x) <= 2^26.5 < 2^30 (no change), and for x = +-0
// the clamped seed carries the signed zero through every step (g0 = x 2^30 =
// +-0, ..., g2 = +-0 = x, what the select returned).
__device__ __forceinline__ double bm_sqrt_radius(double x) {
    const double y0 = fmin(fabs(__builtin_amdgcn_rsq(x)), 1073741824.0);
    const double g0 = x * y0;
    const double h0 = y0 * 0.5;
    const double r0 = fma(-h0, g0, 0.5);
    const double g1 = fma(g0, r0, g0);
    const double h1 = fma(h0, r0, h0);
    const double d0 = fma(-g1, g1, x);
    return fma(d0, h1, g1);
}

__device__ __forceinline__ void box_muller(uint4 w, double& z0, double& z1) {
    const double u1 = u53(w.x, w.y);
    const double u2 = u53(w.z, w.w);
    const double r = bm_sqrt_radius(-2.0 * bm_log(u1));
    double sn, cs;
    bm_sincos2pi(u2, sn, cs);
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

// Two independent Gamma draws with the streams of gamma_mt(alpha0, k, b, spec0,
// it, sub) and gamma_mt(alpha1, k, b, spec1, it, sub), bit-identical to those
// two calls, run in lockstep: attempt j of both in one loop iteration, so the
// two rejection chains overlap instead of following one another (the
// inverse-Wishart's two Bartlett factors).
__device__ inline void gamma_mt_pair(double alpha0, double alpha1, Key k, uint32_t b, uint32_t spec0, uint32_t spec1,
                                     uint32_t it, uint32_t sub, double& g0, double& g1) {
    const double al[2] = {alpha0, alpha1};
    const double a[2] = {alpha0 >= 1.0 ? alpha0 : alpha0 + 1.0, alpha1 >= 1.0 ? alpha1 : alpha1 + 1.0};
    const uint32_t sp[2] = {spec0, spec1};
    double d[2], c[2], g[2] = {0.0, 0.0};
    bool done[2] = {false, false};
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        d[q] = a[q] - 1.0 / 3.0;
        c[q] = 1.0 / sqrt(9.0 * d[q]);
    }
    for (uint32_t j = 0; j < (1u << 20) && !(done[0] && done[1]); ++j) {
        // both attempts unconditionally (pure functions of the counters), so
        // their Philox / Box-Muller chains interleave; a finished draw ignores its
        // later attempts
        double x[2], u[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const uint32_t cc = sp[q] | (j << 8);
            x[q] = normal1(k, b, cc, TAG_GAMMA_N | (sub << 8), it);
            u[q] = uniform1(k, b, cc, TAG_GAMMA_U | (sub << 8), it);
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const double t = 1.0 + c[q] * x[q];
            const double v = t * t * t;
            const bool acc = t > 0.0 && (u[q] < 1.0 - 0.0331 * (x[q] * x[q]) * (x[q] * x[q]) ||
                                         log(u[q]) < 0.5 * x[q] * x[q] + d[q] * (1.0 - v + log(v)));
            if (acc && !done[q]) {
                g[q] = d[q] * v;
                done[q] = true;
            }
        }
    }
#pragma unroll
    for (int q = 0; q < 2; ++q)
        if (al[q] < 1.0) {
            const double ub = uniform1(k, b, sp[q], TAG_GAMMA_BOOST | (sub << 8), it);
            g[q] = g[q] * exp(log(ub) / al[q]);
        }
    g0 = g[0];
    g1 = g[1];
}

// ---- table-driven fp64 Box-Muller for the CR sweep ------------------------
// The tables (gs_bm_tables.h, correctly rounded) are staged in LDS (a 16-B
// aligned array: each cell is one 16-B read) once per workgroup: tab[0..1023] = {c_k, -ln c_k} (512 cells of the frexp mantissa
// [1/2, 1)), tab[1024..1535] = {sin, cos}(2 pi (k + 1/2) / 256).  Every
// operation is fp64; the table cells bound the polynomial arguments (|r| <
// 1.09e-3 for the log1p, |phi| <= pi / 256 for the trigonometric remainder), so
// low degrees reach ~1 ulp: log1p truncated after r^5 / 5 (relative error <
// r^5 / 6 < 2.6e-16), sin after phi^5, cos after phi^6 (< 1e-17 absolute).
// r06: the cells follow the frexp mantissa directly (the r05 table covered
// [sqrt(1/2), sqrt(2)), which needed a compare, a select, an ldexp and an
// exponent fix-up per draw, and a float->int index) and are twice as many, and
// the trig cells are centred, and the log returns -2 ln u (the radius argument,
// the factor folded into its constants): 11 instructions fewer per normal pair.
constexpr int BM_LOG_DOUBLES = 2 * BM_LOG_CELLS;
constexpr int BM_TAB_DOUBLES = BM_LOG_DOUBLES + 512;

__device__ __forceinline__ void bm_stage_tables(double* tab) {
    for (int k = threadIdx.x; k < BM_LOG_DOUBLES; k += blockDim.x) tab[k] = BM_LOG_TAB[k];
    for (int k = threadIdx.x; k < 512; k += blockDim.x) tab[BM_LOG_DOUBLES + k] = BM_TRIG_TAB[k];
}

// -2 ln(x 2^-53) for x = K + 1/2 in [1/2, 2^53) (u53's uniform before its exact
// 2^-53 scaling, which becomes an integer exponent offset): the Box-Muller radius
// argument directly.  x = m 2^e, m in [1/2, 1); the cell of m is the top 9
// mantissa bits -- a bit field of x's high word (x and m share the mantissa);
// -2 ln x = e (-2 ln 2) + 2 ln c_k - 2 log1p(m c_k - 1), the last term as
// r (-2 + r (1 + r (-2/3 + r (1/2 - 2/5 r)))).  e <= 0 and ln m < 0 have one
// sign, and the last cell (m -> 1) has c = 1 exactly, so nothing cancels.
__device__ __forceinline__ double bm_m2log_tab(double x, const double* __restrict__ tab) {
    int e;
    const double m = frexp(x, &e);
    e -= 53;
    // byte offset of cell k's {c_k, 2 ln c_k} pair: ((hi >> 11) & 511) * 16
    static_assert(BM_LOG_CELLS == 512, "the bit field below assumes 9 index bits");
    const uint32_t off = ((uint32_t)__double2hiint(x) >> 7) & 0x1FF0u;
    const double2 cv = *reinterpret_cast<const double2*>(reinterpret_cast<const char*>(tab) + off);
    const double r = fma(m, cv.x, -1.0);
    double q = fma(r, -0.4, 0.5);
    q = fma(q, r, -0.6666666666666666);
    q = fma(q, r, 1.0);
    q = fma(q, r, -2.0);
    const double de = (double)e;
    return fma(de, -1.3862943611198906, fma(de, -4.638093627692599e-17, cv.y + q * r));
}

// sin, cos of 2 pi u for u = (K + 0.5) 2^-53, K = (wz >> 5) 2^26 + (ww >> 6):
// cell k = the top 8 bits (wz >> 24), the remainder angle measured from the
// cell's centre, phi = (K' + 0.5 - 2^44) 2 pi 2^-53 with K' the low 45 bits
__device__ __forceinline__ void bm_sincos_tab(uint32_t wz, uint32_t ww, const double* __restrict__ tab,
                                              double& sn, double& cs) {
    const uint32_t k = wz >> 24;
    // 2^52 + K' as a double from its bits (hi word 0x433 | K' >> 32, lo word the
    // low 32 bits of K'), less 2^52 + 2^44: K' - 2^44, exact; then one fma
    // (y + 1/2) 2 pi 2^-53 (the power-of-two scaling folded into the constant)
    const uint32_t kh = (wz >> 5) & 0x7FFFFu;                      // K' = kh 2^26 + (ww >> 6)
    const uint32_t lo = __builtin_amdgcn_alignbit(kh, ww, 6);      // (kh << 26) | (ww >> 6)
    const uint32_t hi = ((wz >> 11) & 0x1FFFu) | 0x43300000u;      // 0x433 | kh >> 6
    const double y = __hiloint2double((int)hi, (int)lo) - 4521191813414912.0;
    constexpr double S = 6.283185307179586 / 9007199254740992.0;
    const double ph = fma(y, S, 0.5 * S);
    const double p2 = ph * ph;
    const double ps = fma(p2, 8.333333333333333e-3, -0.16666666666666666);
    const double sph = fma(ph * p2, ps, ph);
    double pc = fma(p2, -1.388888888888889e-3, 4.1666666666666664e-2);
    pc = fma(pc, p2, -0.5);
    const double cph = fma(pc, p2, 1.0);
    const double2 tv = reinterpret_cast<const double2*>(tab + BM_LOG_DOUBLES)[k];     // 16-B aligned tab
    const double sk = tv.x, ck = tv.y;
    sn = fma(sk, cph, ck * sph);
    cs = fma(ck, cph, -(sk * sph));
}

__device__ __forceinline__ void box_muller_tab(uint4 w, const double* __restrict__ tab, double& z0, double& z1) {
    // u1 = x 2^-53 (u53), x = K + 1/2 formed exactly as u53 forms it
    const double x = (double)(w.x >> 5) * 67108864.0 + (double)(w.y >> 6) + 0.5;
    const double r = bm_sqrt_radius(bm_m2log_tab(x, tab));
    double sn, cs;
    bm_sincos_tab(w.z, w.w, tab, sn, cs);
    z0 = r * cs;
    z1 = r * sn;
}

}  // namespace gs
