// gs_aux.h -- the masked aux-variable step's per-pixel v | s update as the pixel
// operation of the fused ring stage (gs_sht_aux_pass_batch, gs_sht.hip), shared
// by gs_masked.hip (its k_mc_v computes the same expressions through mc_aux_pixel).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "gs_rng.h"

namespace gs {

constexpr uint32_t TAG_AUX_V = 8;

// v | s (CenteredGibbs.py:693-700; over-relaxed 797-802) and the s | v input
// y = v + N^-1 d (711-713) of one pixel of one field row: Abs = (A b s)[pixel]
struct GsAuxPix {
    const double* ninv;      // [F][Npix] shared by the batch
    const double* dpix;      // [F][Npix]
    double* v;               // [B][F][Npix] (read when over, always written)
    const double* zv;        // replay normals [B] x zvs, [F][Npix] each (nullptr: Philox)
    long long zvs;
    long long npix;
    double mu[3];
    int rows[3];
    int F, over;
    double alpha;
    uint32_t slo, shi, chain, sub, iter;
};

// the pixel's loads (split from the arithmetic so a caller can issue the loads
// of several pixels before the first use; mc_aux_pixel = apply(load))
struct GsAuxPre { double ni, dp, vo, zr; };
__device__ __forceinline__ GsAuxPre mc_aux_load(const GsAuxPix& a, int b, int k, long long p) {
    const long long g = (long long)k * a.npix + p;
    const long long cb = (long long)b * a.F * a.npix;
    GsAuxPre q;
    q.ni = a.ninv[g];
    q.dp = a.dpix[g];
    q.vo = a.over ? a.v[cb + g] : 0.0;
    q.zr = a.zv ? a.zv[(long long)b * a.zvs + g] : 0.0;
    return q;
}
__device__ __forceinline__ double mc_aux_apply(const GsAuxPix& a, int b, int k, long long p, const GsAuxPre& q,
                                               double Abs) {
    const long long g = (long long)k * a.npix + p;
    const long long cb = (long long)b * a.F * a.npix;
    const int row = a.rows[k];
    const double mu = row == 0 ? a.mu[0] : (row == 1 ? a.mu[1] : a.mu[2]);
    const double gam = mu - q.ni;
    const double mean = gam * Abs;
    double z;
    if (a.zv) z = q.zr;
    else z = normal1(chain_key(a.slo, a.shi, a.chain + b), (uint32_t)p, (uint32_t)row, TAG_AUX_V | (a.sub << 8), a.iter);
    double vn;
    if (!a.over) vn = z * sqrt(gam) + mean;
    else vn = mean + a.alpha * (q.vo - mean) + sqrt(1.0 - a.alpha * a.alpha) * z * sqrt(gam);
    a.v[cb + g] = vn;
    return vn + q.ni * q.dp;
}
__device__ __forceinline__ double mc_aux_pixel(const GsAuxPix& a, int b, int k, long long p, double Abs) {
    return mc_aux_apply(a, b, k, p, mc_aux_load(a, b, k, p), Abs);
}

}  // namespace gs
