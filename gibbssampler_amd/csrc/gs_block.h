// gs_block.h -- per-l prior / CR-operator algebra shared by the translation
// units of libgibbs_hip.so (full-sky sweep, masked CR).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include "gibbs_capi.h"

namespace gs_block {
constexpr double PI = 3.14159265358979323846;
constexpr int NP = GS_NPARAM;
}

// ============================================================================
// device helpers
// ============================================================================
__device__ __forceinline__ double var_from_dl(double D, int ell) {
    // generate_var_cl (utils.py:126-129): D*2*pi/(l(l+1)), l=0 keeps D_0
    return ell == 0 ? D : D * 2.0 * gs_block::PI / (double)(ell * (ell + 1));
}

__device__ __forceinline__ double dl_at(const double* __restrict__ dl_chain, const int* __restrict__ ell2bin,
                                        int maxbins, int Lp1, int sp, int ell) {
    const int b = ell2bin[sp * Lp1 + ell];
    return b < 0 ? 0.0 : dl_chain[sp * maxbins + b];
}

// iteration counter of the counter-based streams: a host value, or (for
// hipGraph replay) a device base word plus the step's offset within the
// captured graph (host); the graph's last step advances the base by the
// number of steps it holds, so only one launch per replay takes a ticket
struct IterArg {
    uint32_t host;
    const uint32_t* dev;
    __device__ __forceinline__ uint32_t get() const { return dev ? *dev + host : host; }
};

// lower Cholesky of the TE block of C and the B entry, zero-variance rule
struct CovChol { double a00, a10, a11, aB; };

__device__ __forceinline__ CovChol cov_chol_teb(double tt, double ee, double te, double bb) {
    CovChol c;
    if (tt != 0.0) {
        c.a00 = sqrt(tt);
        c.a10 = te / c.a00;
        c.a11 = sqrt(fmax(ee - c.a10 * c.a10, 0.0));
    } else {
        c.a00 = 0.0; c.a10 = 0.0; c.a11 = sqrt(ee);
    }
    c.aB = sqrt(bb);
    return c;
}

// ============================================================================
// per-(chain, l) CR operator
// ============================================================================
// MODE 0 centered (CenteredGibbs.py:324-351):   Sigma = (C^+ + diag(b^2 k))^-1, M = Sigma diag(b k)
// MODE 1 non-centered (NonCenteredGibbs.py:141-174): Sigma = (I + A^T diag(b^2 k) A)^-1,
//                                                   M = Sigma A^T diag(b k), A = chol(C)
// the D_l of every spectrum at this l (for the operator below): the bin
// indices, then the values, each group issued together and unconditionally (an
// unbinned l reads bin 0 and drops it) -- two memory latencies in all
template <int F>
__device__ __forceinline__ void block_params_load(int chain, int ell, int L, int maxbins, const double* __restrict__ dl,
                                                  const int* __restrict__ ell2bin,
                                                  double (&dq)[F == 1 ? 1 : (F == 2 ? 2 : 4)]) {
    const int Lp1 = L + 1;
    constexpr int NS = F == 1 ? 1 : (F == 2 ? 2 : 4);
    const double* dlc = dl + (long long)chain * NS * maxbins;
    int bq[NS];
#pragma unroll
    for (int q = 0; q < NS; ++q) bq[q] = ell2bin[q * Lp1 + ell];
#pragma unroll
    for (int q = 0; q < NS; ++q) dq[q] = dlc[q * maxbins + max(bq[q], 0)];
#pragma unroll
    for (int q = 0; q < NS; ++q) dq[q] = bq[q] < 0 ? 0.0 : dq[q];
}

// the operator from this l's binned D_l (dq) and beam b
template <int F, int MODE>
__device__ __forceinline__ void block_params_from(int ell, double b, const double (&dq)[F == 1 ? 1 : (F == 2 ? 2 : 4)],
                                                  double k0, double k1, double k2, double (&p)[gs_block::NP]) {
    const double kap[3] = {k0, k1, k2};
#pragma unroll
    for (int q = 0; q < gs_block::NP; ++q) p[q] = 0.0;
    if constexpr (F != 3) {
#pragma unroll
        for (int f = 0; f < F; ++f) {
            const double v = var_from_dl(dq[f], ell);
            double sig, M;
            if constexpr (MODE == 0) {
                const double iv = v != 0.0 ? 1.0 / v : 0.0;
                sig = 1.0 / (kap[f] * b * b + iv);
                M = sig * (kap[f] * b);
            } else {
                sig = 1.0 / (1.0 + kap[f] * b * b * v);
                M = sig * (sqrt(v) * b * kap[f]);
            }
            p[f] = M;
            p[F + f] = sqrt(sig);
        }
    } else {
        const double tt = var_from_dl(dq[0], ell);
        const double ee = var_from_dl(dq[1], ell);
        const double bb = var_from_dl(dq[2], ell);
        const double te = var_from_dl(dq[3], ell);
        const double p0 = b * b * k0, p1 = b * b * k1, p2 = b * b * k2;
        double s00, s11, s01, s22, M00, M01, M10, M11, M22;
        if constexpr (MODE == 0) {
            double it, ie, ite;
            if (tt != 0.0 && ee != 0.0) {
                const double det = tt * ee - te * te;
                it = ee / det; ie = tt / det; ite = -te / det;
            } else {
                it = tt != 0.0 ? 1.0 / tt : 0.0;
                ie = ee != 0.0 ? 1.0 / ee : 0.0;
                ite = 0.0;
            }
            const double q00 = it + p0, q11 = ie + p1, q01 = ite;
            const double det = q00 * q11 - q01 * q01;
            s00 = q11 / det; s11 = q00 / det; s01 = -q01 / det;
            const double ib = bb != 0.0 ? 1.0 / bb : 0.0;
            s22 = 1.0 / (ib + p2);
            M00 = s00 * (b * k0); M01 = s01 * (b * k1);
            M10 = s01 * (b * k0); M11 = s11 * (b * k1);
            M22 = s22 * (b * k2);
        } else {
            const CovChol A = cov_chol_teb(tt, ee, te, bb);
            // Q = I + A^T P A, A = [[a00, 0], [a10, a11]]
            const double q00 = 1.0 + A.a00 * A.a00 * p0 + A.a10 * A.a10 * p1;
            const double q01 = A.a10 * A.a11 * p1;
            const double q11 = 1.0 + A.a11 * A.a11 * p1;
            const double det = q00 * q11 - q01 * q01;
            s00 = q11 / det; s11 = q00 / det; s01 = -q01 / det;
            s22 = 1.0 / (1.0 + A.aB * A.aB * p2);
            // M = S A^T diag(b k): A^T = [[a00, a10], [0, a11]]
            const double bt = b * k0, be = b * k1;
            const double c00 = A.a00 * bt, c01 = A.a10 * be, c11 = A.a11 * be;   // A^T diag(bk)
            M00 = s00 * c00; M01 = s00 * c01 + s01 * c11;
            M10 = s01 * c00; M11 = s01 * c01 + s11 * c11;
            M22 = s22 * (A.aB * b * k2);
        }
        const double l00 = sqrt(s00);
        const double l10 = s01 / l00;
        const double l11 = sqrt(fmax(s11 - l10 * l10, 0.0));
        p[0] = M00; p[1] = M01; p[2] = M10; p[3] = M11; p[4] = M22;
        p[5] = l00; p[6] = l10; p[7] = l11; p[8] = sqrt(s22); p[9] = 0.0;
    }
}

// the operator of one (chain, l) into registers (the CR sweep computes its own
// lanes' operators this way; block_params_at stores them)
template <int F, int MODE>
__device__ __forceinline__ void block_params_compute(int chain, int ell, int L, int maxbins,
                                                     const double* __restrict__ dl, const int* __restrict__ ell2bin,
                                                     const double* __restrict__ bl, double k0, double k1, double k2,
                                                     double (&p)[gs_block::NP]) {
    double dq[F == 1 ? 1 : (F == 2 ? 2 : 4)];
    block_params_load<F>(chain, ell, L, maxbins, dl, ell2bin, dq);
    block_params_from<F, MODE>(ell, bl[ell], dq, k0, k1, k2, p);
}

template <int F, int MODE>
__device__ __forceinline__ void block_params_at(int g, int L, int nchains, int maxbins, const double* __restrict__ dl,
                                                const int* __restrict__ ell2bin, const double* __restrict__ bl,
                                                double k0, double k1, double k2, double* __restrict__ params) {
    const int Lp1 = L + 1;
    if (g >= nchains * Lp1) return;
    double p[gs_block::NP];
    block_params_compute<F, MODE>(g / Lp1, g % Lp1, L, maxbins, dl, ell2bin, bl, k0, k1, k2, p);
    double* o = params + (long long)g * gs_block::NP;
    constexpr int NW = F == 3 ? gs_block::NP : 2 * F;
#pragma unroll
    for (int q = 0; q < NW; ++q) o[q] = p[q];
}

