// gs_masked.hip -- masked (pixel-domain) constrained-realization steps on gfx950.
//
// Device versions of the reference's masked CR samplers (EB class
// PolarizedCenteredConstrainedRealization, CenteredGibbs.py:241-850), TEB
// generalised for the auxiliary-variable scheme:
//   a9  sample_gibbs_change_variable   CenteredGibbs.py:676-729
//   a10 overrelaxation_sampler         CenteredGibbs.py:733-825
//   a11 sample_mala (+ gradient, log density, log proposal) 494-603
//   a12 the dispatch ladder of sample  CenteredGibbs.py:828-850
// A context runs a batch of B chains (chains chain0 .. chain0 + B - 1 on the same
// data): every per-chain array is [B][...] contiguous, every pixel- and slot-wise
// kernel carries the chain in blockIdx.y, and each transform is ONE batched SHT
// over the B maps (gs_sht_*_batch) -- so B small-map chains fill the GPU that
// one leaves mostly idle.  Chain b of a batch does exactly the arithmetic of a
// one-chain context with chain id chain0 + b (bit-identical for the same
// resolved sht_mode -- the table and recurrence Legendre stages agree to
// ~1e-12, not bit for bit -- tested).  The MALA
// accept test reduces its eight sums in a fixed order (bitwise reproducible).
//
// Per-pixel arrays are [F][Npix] over the field rows (F = 2: Q, U; F = 3:
// T, Q, U); a_lm are real m-major [F][(L+1)^2].  Native draws: pixel normals
// Philox(c0 = pixel, c1 = map row (0 T, 1 Q, 2 U), c2 = TAG_AUX_V | sub << 8,
// c3 = iteration); slot normals are the CR stream of the full-sky sweep with
// substep SUB_S + 2k (+1 for the second over-relaxed s draw) or SUB_MALA;
// the MALA uniform is Philox(0, call, TAG_MALA_U, iteration).  The same
// streams are restated in oracle/masked.py (NativeDraws).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include <cmath>
#include <string>
#include <vector>
#include <algorithm>
#include <cstdlib>

#include "gibbs_capi.h"
#include "gs_rng.h"
#include "gs_common.h"
#include "gs_block.h"
#include "gs_aux.h"

// library-internal SHT entry points (gs_sht.hip)
extern "C" long long gs_sht_phi_plane(const gs_sht* p);
extern "C" int gs_sht_synth_blocks(gs_sht* p, int nmap, int nfield, const double* alm_real, const int* blk, int K,
                                   const int* blk_lmax, double* phib, double* maps, void* stream, int parseval);
extern "C" int gs_sht_register_weights(gs_sht* p, const double* weights, int wnc, void* stream);
extern "C" int gs_sht_blocks_parseval(const gs_sht* p, int nfield, int ncomp_total);
extern "C" int gs_sht_parseval_maps(gs_sht* p, int ncomp, double* maps, void* stream);
extern "C" int gs_sht_ring_class_counts(const gs_sht* p, int counts[3]);
extern "C" int gs_sht_aux_pass_batch(gs_sht* p, int nmap, int ncomp, const double* alm_in, const double* bl,
                                     const void* aux, double* alm_out, void* stream);

using namespace gs;
using gs_detail::set_error;

namespace {

constexpr double PI = 3.14159265358979323846;
constexpr uint32_t TAG_MALA_U = 9;
constexpr uint32_t TAG_RJ_U = 10;   // RJPO accept uniform: Philox(0, 0, TAG_RJ_U, iteration)
constexpr int SUB_S = 16;
constexpr int SUB_V_INIT = 255;
constexpr int SUB_MALA = 200;
constexpr int SUB_PCG_S = 250;     // CR substep of the PCG's C^-1/2 slot normals
constexpr int SUB_PCG_V = 254;     // TAG_AUX_V substep of the PCG's pixel normals
constexpr int NSUM = 8;
constexpr int RED_BLOCK = 256;

inline unsigned nblocks(long long n, int bs) { return (unsigned)std::max<long long>(1, (n + bs - 1) / bs); }
inline hipStream_t S(void* s) { return (hipStream_t)s; }

struct Rows { int r[3]; };

// (l, m) of complex index i (healpy m-major)
__device__ __forceinline__ void cidx_lm(int L, long long i, int& l, int& m) {
    const double b = 2.0 * L + 3.0;
    m = (int)floor((b - sqrt(fmax(b * b - 8.0 * (double)i, 0.0))) / 2.0);
    m = max(0, min(m, L));
    while (m > 0 && (long long)m * (2 * L + 3 - m) / 2 > i) --m;
    while (m < L && (long long)(m + 1) * (2 * L + 2 - m) / 2 <= i) ++m;
    l = (int)(i - (long long)m * (2 * L + 1 - m) / 2);
}

// x = b_l s (real layout, per field)
__global__ void k_mc_beam(int L, int F, const double* __restrict__ bl, const double* __restrict__ s,
                          double* __restrict__ x) {
    const long long NR = (long long)(L + 1) * (L + 1);
    const long long nlm = (long long)(L + 1) * (L + 2) / 2;
    const long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (g >= F * nlm) return;
    const int f = (int)(g / nlm);
    const long long i = g % nlm;
    int l, m;
    cidx_lm(L, i, l, m);
    const double b = bl[l];
    if (m == 0) { x[f * NR + l] = b * s[f * NR + l]; return; }
    const long long r = 2 * i - (L + 1);
    x[f * NR + r] = b * s[f * NR + r];
    x[f * NR + r + 1] = b * s[f * NR + r + 1];
}

// v | s (CenteredGibbs.py:693-700; over-relaxed 797-802) and the s | v input
// y = v + N^-1 d (711-713), per pixel and field row
// (mc_aux_pixel, gs_aux.h: the fused ring stage of gs_sht_aux_pass_batch runs the
// same expressions, so both give the same bits)
__global__ void k_mc_v(GsAuxPix a, const double* __restrict__ Abs, double* __restrict__ y) {
    const long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (g >= a.F * a.npix) return;
    // chain b of the batch (blockIdx.y): its maps
    const int b = blockIdx.y;
    const long long cb = (long long)b * a.F * a.npix;
    const int k = (int)(g / a.npix);
    const long long p = g % a.npix;
    y[cb + g] = mc_aux_pixel(a, b, k, p, Abs[cb + g]);
}

__device__ __forceinline__ void slot_normals(const double* __restrict__ zs, long long NR, int F, long long r, int nv,
                                             Key key, long long i, uint32_t sub, uint32_t iter, double (&z)[3][2]) {
#pragma unroll
    for (int f = 0; f < 3; ++f) {
        if (f >= F) break;
        if (zs) {
            z[f][0] = zs[f * NR + r];
            z[f][1] = nv == 2 ? zs[f * NR + r + 1] : 0.0;
        } else {
            box_muller(philox((uint32_t)i, (uint32_t)f, TAG_CR | (sub << 8), iter, key), z[f][0], z[f][1]);
        }
    }
}

// s | v (CenteredGibbs.py:703-726; over-relaxed 778-781): per slot
// s = mean + L z with mean = M d_eff, d_eff = complex_to_real(map2alm(y)) / mu_f,
// (M, L) the centered per-l block for kappa_f = mu_f / w; over-relaxed
// s' = mean + alpha (s - mean) + sqrt(1 - alpha^2) L z
template <int F>
__global__ void k_mc_s(int L, const double* __restrict__ params, const double* __restrict__ r_alm, double imu0,
                       double imu1, double imu2, const double* __restrict__ zs, long long zss, uint32_t seed_lo,
                       uint32_t seed_hi, uint32_t chain, uint32_t sub, uint32_t iter, int over, double alpha,
                       double* __restrict__ s) {
    const long long NR = (long long)(L + 1) * (L + 1);
    const long long nlm = (long long)(L + 1) * (L + 2) / 2;
    const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i >= nlm) return;
    params += (long long)blockIdx.y * (L + 1) * GS_NPARAM;
    r_alm += (long long)blockIdx.y * F * NR;
    s += (long long)blockIdx.y * F * NR;
    if (zs) zs += (long long)blockIdx.y * zss;
    chain += blockIdx.y;
    int l, m;
    cidx_lm(L, i, l, m);
    const long long r = m == 0 ? l : 2 * i - (L + 1);
    const int nv = m == 0 ? 1 : 2;
    const double* p = params + (long long)l * GS_NPARAM;
    const double imu[3] = {imu0, imu1, imu2};
    double z[3][2];
    slot_normals(zs, NR, F, r, nv, chain_key(seed_lo, seed_hi, chain), i, sub, iter, z);
    const double c1 = sqrt(1.0 - alpha * alpha);
    for (int c = 0; c < nv; ++c) {
        double d[3], mean[3], fl[3];
#pragma unroll
        for (int f = 0; f < F; ++f) d[f] = r_alm[f * NR + r + c] * imu[f];
        if constexpr (F != 3) {
#pragma unroll
            for (int f = 0; f < F; ++f) { mean[f] = p[f] * d[f]; fl[f] = p[F + f] * z[f][c]; }
        } else {
            mean[0] = p[0] * d[0] + p[1] * d[1];
            mean[1] = p[2] * d[0] + p[3] * d[1];
            mean[2] = p[4] * d[2];
            fl[0] = p[5] * z[0][c];
            fl[1] = p[6] * z[0][c] + p[7] * z[1][c];
            fl[2] = p[8] * z[2][c];
        }
#pragma unroll
        for (int f = 0; f < F; ++f) {
            double* sp = s + f * NR + r + c;
            *sp = over ? mean[f] + alpha * (*sp - mean[f]) + c1 * fl[f] : fl[f] + mean[f];
        }
    }
}

__global__ void k_set_one(int n, int32_t* a) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) a[i] = 1;
}

__global__ void k_mc_mul(long long n, const double* __restrict__ a, const double* __restrict__ b,
                         double* __restrict__ out) {
    const long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (g < n) out[g] = a[g] * b[g];
}

// per-slot inverse prior variance (zero-variance rule) of field f at l (EB)
__device__ __forceinline__ double inv_prior(const double* __restrict__ dl, int L, int f, int l) {
    const double v = var_from_dl(dl[f * (L + 1) + l], l);
    return v != 0.0 ? 1.0 / v : 0.0;
}

// grad = -C^+ s - (b / w) r + g2,  r = complex_to_real(map2alm(N^-1 A b s))  (494-520)
__global__ void k_mc_grad(int L, int F, const double* __restrict__ dl, const double* __restrict__ bl,
                          const double* __restrict__ s, const double* __restrict__ r_alm, const double* __restrict__ g2,
                          double inv_w, double* __restrict__ grad) {
    const long long NR = (long long)(L + 1) * (L + 1);
    const long long nlm = (long long)(L + 1) * (L + 2) / 2;
    const long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (g >= F * nlm) return;
    const long long cb = (long long)blockIdx.y * F * NR;
    dl += (long long)blockIdx.y * (F == 3 ? 4 : F) * (L + 1);
    s += cb; r_alm += cb; grad += cb;
    const int f = (int)(g / nlm);
    const long long i = g % nlm;
    int l, m;
    cidx_lm(L, i, l, m);
    const long long r = m == 0 ? l : 2 * i - (L + 1);
    const int nv = m == 0 ? 1 : 2;
    const double ip = inv_prior(dl, L, f, l);
    for (int c = 0; c < nv; ++c) {
        const long long o = f * NR + r + c;
        grad[o] = -ip * s[o] + -(r_alm[o] * inv_w * bl[l]) + g2[o];
    }
}

// s_new = s + tau sigma grad + sqrt(2 tau sigma) z  (523-527), sigma = p[F+f]^2
__global__ void k_mc_propose(int L, int F, const double* __restrict__ params, const double* __restrict__ s,
                             const double* __restrict__ grad, double tau, const double* __restrict__ zm,
                             uint32_t seed_lo, uint32_t seed_hi, uint32_t chain, uint32_t sub, uint32_t iter,
                             double* __restrict__ snew) {
    const long long NR = (long long)(L + 1) * (L + 1);
    const long long nlm = (long long)(L + 1) * (L + 2) / 2;
    const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i >= nlm) return;
    const long long cb = (long long)blockIdx.y * F * NR;
    params += (long long)blockIdx.y * (L + 1) * GS_NPARAM;
    s += cb; grad += cb; snew += cb;
    if (zm) zm += cb;
    chain += blockIdx.y;
    int l, m;
    cidx_lm(L, i, l, m);
    const long long r = m == 0 ? l : 2 * i - (L + 1);
    const int nv = m == 0 ? 1 : 2;
    double z[3][2];
    slot_normals(zm, NR, F, r, nv, chain_key(seed_lo, seed_hi, chain), i, sub, iter, z);
    for (int f = 0; f < F; ++f) {
        const double sq = params[(long long)l * GS_NPARAM + F + f];
        const double sig = sq * sq;
        for (int c = 0; c < nv; ++c) {
            const long long o = f * NR + r + c;
            snew[o] = s[o] + tau * sig * grad[o] + sqrt(2.0 * tau * sig) * z[f][c];
        }
    }
}

// MALA sums (fixed-order partials per block):
//  0: sum C^+ s0^2   1: sum C^+ s1^2   2: s0 . g2   3: s1 . g2
//  4: sum (s0 - s1 - tau sig g1)^2 / (2 tau sig)   5: sum (s1 - s0 - tau sig g0)^2 / (2 tau sig)
//  6: sum N^-1 pix0^2   7: sum N^-1 pix1^2
// The last two from the maps pix = A b s (p0, p1), or -- p0 = nullptr, harmonic
// inputs r0, r1 = map2alm(N^-1 A b s) of the fused operator -- as (1/w) (b s) . r:
// A^T = map2alm / w exactly (real layout), so sum N^-1 pix^2 = (b s)^T A^T N^-1 A
// (b s); the same sum in other rounding, without the maps
__global__ __launch_bounds__(RED_BLOCK) void k_mc_sums(int L, int F, long long npix, const double* __restrict__ dl,
                                                       const double* __restrict__ params, double tau,
                                                       const double* __restrict__ s0, const double* __restrict__ s1,
                                                       const double* __restrict__ g0, const double* __restrict__ g1,
                                                       const double* __restrict__ g2, const double* __restrict__ ninv,
                                                       const double* __restrict__ p0, const double* __restrict__ p1,
                                                       double* __restrict__ partial, const double* __restrict__ r0,
                                                       const double* __restrict__ r1, const double* __restrict__ bl,
                                                       double inv_w) {
    const long long NR = (long long)(L + 1) * (L + 1);
    const long long nslot = F * NR, npx = F * npix;
    const bool harm = p0 == nullptr;
    {
        const long long cb = (long long)blockIdx.y * nslot, pb = (long long)blockIdx.y * npx;
        dl += (long long)blockIdx.y * (F == 3 ? 4 : F) * (L + 1);
        params += (long long)blockIdx.y * (L + 1) * GS_NPARAM;
        s0 += cb; s1 += cb; g0 += cb; g1 += cb;
        if (harm) { r0 += cb; r1 += cb; } else { p0 += pb; p1 += pb; }
        partial += (long long)blockIdx.y * gridDim.x * NSUM;
    }
    double a[NSUM] = {0, 0, 0, 0, 0, 0, 0, 0};
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x; g < nslot; g += stride) {
        const int f = (int)(g / NR);
        const long long r = g % NR;
        int l;
        if (r <= L) l = (int)r;
        else { int m; cidx_lm(L, (r + L + 1) / 2, l, m); }
        const double ip = inv_prior(dl, L, f, l);
        const double sq = params[(long long)l * GS_NPARAM + F + f];
        const double ts = tau * (sq * sq);
        const double x0 = s0[g], x1 = s1[g];
        a[0] += ip * x0 * x0;
        a[1] += ip * x1 * x1;
        a[2] += x0 * g2[g];
        a[3] += x1 * g2[g];
        const double e01 = x0 - x1 - ts * g1[g];
        const double e10 = x1 - x0 - ts * g0[g];
        a[4] += e01 * e01 / (2.0 * ts);
        a[5] += e10 * e10 / (2.0 * ts);
        if (harm) {
            a[6] += ((bl[l] * x0) * r0[g]) * inv_w;
            a[7] += ((bl[l] * x1) * r1[g]) * inv_w;
        }
    }
    for (long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x; !harm && g < npx; g += stride) {
        const double q0 = p0[g], q1 = p1[g];
        a[6] += q0 * q0 * ninv[g];
        a[7] += q1 * q1 * ninv[g];
    }
    __shared__ double red[NSUM][RED_BLOCK];
#pragma unroll
    for (int k = 0; k < NSUM; ++k) red[k][threadIdx.x] = a[k];
    __syncthreads();
    for (int h = RED_BLOCK / 2; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h)
#pragma unroll
            for (int k = 0; k < NSUM; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + h];
        __syncthreads();
    }
    if (threadIdx.x < NSUM) partial[blockIdx.x * NSUM + threadIdx.x] = red[threadIdx.x][0];
}

// accept with log u < log pi(s1) + log q(s0|s1) - log pi(s0) - log q(s1|s0) (577-603)
// fixed-order sum of N rows of per-block partials over one workgroup of
// RED_BLOCK threads: thread t sums blocks t, t + RED_BLOCK, ... in order, then
// a fixed tree in LDS (deterministic; loads spread over the workgroup instead
// of one thread's dependent chain)
template <int N>
__device__ __forceinline__ void block_sums(int nblk, const double* __restrict__ partial, int stride, double (&t)[N]) {
    __shared__ double red[N][RED_BLOCK];
    double v[N];
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] = 0.0;
    for (int b = threadIdx.x; b < nblk; b += RED_BLOCK)
#pragma unroll
        for (int k = 0; k < N; ++k) v[k] += partial[(long long)b * stride + k];
#pragma unroll
    for (int k = 0; k < N; ++k) red[k][threadIdx.x] = v[k];
    __syncthreads();
    for (int h = RED_BLOCK / 2; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h)
#pragma unroll
            for (int k = 0; k < N; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + h];
        __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < N; ++k) t[k] = red[k][0];
}

__global__ void k_mc_accept(int nblk, const double* __restrict__ partial, long long nslot, const double* __restrict__ um,
                            uint32_t seed_lo, uint32_t seed_hi, uint32_t chain, uint32_t call, uint32_t iter,
                            int32_t* __restrict__ flag, int32_t* __restrict__ accept,
                            double* __restrict__ log_ratio) {
    // chain b = blockIdx.y of the batch (one workgroup per chain)
    const int b = blockIdx.y;
    partial += (long long)b * nblk * NSUM;
    if (um) um += b;
    chain += b;
    flag += b;
    if (accept) accept += b;
    if (log_ratio) log_ratio += b;
    double t[NSUM];
    block_sums<NSUM>(nblk, partial, NSUM, t);
    if (threadIdx.x == 0) {
        const double lp1 = -0.5 * t[1] + -0.5 * t[7] + t[3];
        const double lp0 = -0.5 * t[0] + -0.5 * t[6] + t[2];
        const double lr = lp1 + (-0.5 * t[4]) - (lp0 + (-0.5 * t[5]));
        const double u = um ? um[0] : uniform1(chain_key(seed_lo, seed_hi, chain), 0u, call, TAG_MALA_U, iter);
        const int acc = log(u) < lr ? 1 : 0;
        *flag = acc;
        if (accept) *accept = acc;
        if (log_ratio) *log_ratio = lr;
    }
}

// dst <- src when the accept flag is set: the whole grid moves the map (the
// accept workgroup alone took ~257 us for the 4.2 MB of an N_side 256 EB map)
__global__ void k_select_copy(long long n, const int32_t* __restrict__ flag, const double* __restrict__ src,
                              double* __restrict__ dst) {
    if (!flag[blockIdx.y]) return;
    src += (long long)blockIdx.y * n;
    dst += (long long)blockIdx.y * n;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x; g < n; g += stride) dst[g] = src[g];
}

// RJPO (CenteredGibbs.py:606-674): per-block partials of (rhs - Q x) . (s - x)
// with y = Q x, in a fixed order (grid-stride per thread, then an LDS tree)
__global__ __launch_bounds__(RED_BLOCK) void k_rj_dot(long long n, const double* __restrict__ rhs,
                                                      const double* __restrict__ y, const double* __restrict__ s,
                                                      const double* __restrict__ x, double* __restrict__ partial) {
    {
        const long long cb = (long long)blockIdx.y * n;
        rhs += cb; y += cb; s += cb; x += cb;
        partial += (long long)blockIdx.y * gridDim.x;
    }
    double a = 0.0;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x; g < n; g += stride)
        a += (rhs[g] - y[g]) * (s[g] - x[g]);
    __shared__ double red[RED_BLOCK];
    red[threadIdx.x] = a;
    __syncthreads();
    for (int h = RED_BLOCK / 2; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

// log_proba = -sum (rhs - Q x) . (s_old - x) (:664-669); accept when
// log u < log_proba (:670), then s <- x (the PCG solution), else s stays
__global__ __launch_bounds__(RED_BLOCK) void k_rj_accept(int nblk, const double* __restrict__ partial, long long n,
                                                         const double* __restrict__ um, uint32_t seed_lo,
                                                         uint32_t seed_hi, uint32_t chain, uint32_t iter,
                                                         int32_t* __restrict__ flag,
                                                         int32_t* __restrict__ accept, double* __restrict__ log_ratio) {
    const int b = blockIdx.y;
    partial += (long long)b * nblk;
    if (um) um += b;
    chain += b;
    flag += b;
    if (accept) accept += b;
    if (log_ratio) log_ratio += b;
    double t[1];
    block_sums<1>(nblk, partial, 1, t);
    if (threadIdx.x == 0) {
        const double lr = -t[0];
        const double u = um ? um[0] : uniform1(chain_key(seed_lo, seed_hi, chain), 0u, 0u, TAG_RJ_U, iter);
        const int acc = log(u) < lr ? 1 : 0;
        *flag = acc;
        if (accept) *accept = acc;
        if (log_ratio) *log_ratio = lr;
    }
}

// ---------------------------------------------------------------------------
// f1: PCG CR (CenteredGibbs.py:448-491) -- Q x = C^+ x + b A^T N^-1 A b x
// ---------------------------------------------------------------------------
// prior pseudo-inverse factors at l: EB per field sqrt(inv_var); TEB the lower
// factor A^+ = [[i00, 0], [t10, i11]] of the TE block (C^+ = (A^+)^T A^+) and iB
struct PriorPinv { double i00, t10, i11, iB, ie, ib; };

template <int F>
__device__ __forceinline__ PriorPinv prior_pinv(const double* __restrict__ dl, int L, int l) {
    PriorPinv q{0, 0, 0, 0, 0, 0};
    if constexpr (F != 3) {
        const double ve = var_from_dl(dl[l], l);
        q.ie = ve != 0.0 ? sqrt(1.0 / ve) : 0.0;
        if constexpr (F == 2) {
            const double vb = var_from_dl(dl[(L + 1) + l], l);
            q.ib = vb != 0.0 ? sqrt(1.0 / vb) : 0.0;
        }
    } else {
        const double tt = var_from_dl(dl[l], l), ee = var_from_dl(dl[(L + 1) + l], l);
        const double bb = var_from_dl(dl[2 * (L + 1) + l], l), te = var_from_dl(dl[3 * (L + 1) + l], l);
        const CovChol A = cov_chol_teb(tt, ee, te, bb);
        q.i00 = A.a00 != 0.0 ? 1.0 / A.a00 : 0.0;
        q.i11 = A.a11 != 0.0 ? 1.0 / A.a11 : 0.0;
        q.t10 = -A.a10 * q.i00 * q.i11;
        q.iB = A.aB != 0.0 ? 1.0 / A.aB : 0.0;
    }
    return q;
}

// y = sqrt(N^-1) z per pixel (the pixel half of the fluctuations, 467-471)
__global__ void k_pcg_zpix(long long npix, int F, Rows rows, const double* __restrict__ ninv,
                           const double* __restrict__ zv, uint32_t seed_lo, uint32_t seed_hi, uint32_t chain,
                           uint32_t iter, double* __restrict__ y) {
    const long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (g >= F * npix) return;
    y += (long long)blockIdx.y * F * npix;
    if (zv) zv += (long long)blockIdx.y * F * npix;
    chain += blockIdx.y;
    const int k = (int)(g / npix);
    const long long p = g % npix;
    const double z = zv ? zv[g]
                        : normal1(chain_key(seed_lo, seed_hi, chain), (uint32_t)p, (uint32_t)rows.r[k],
                                  TAG_AUX_V | ((uint32_t)SUB_PCG_V << 8), iter);
    y[g] = z * sqrt(ninv[g]);
}

// rhs = b A^T N^-1 d (g2) + b * map2alm(y, iter=3) * Npix/4pi + (A^+)^T z_slot
template <int F>
__global__ void k_pcg_rhs(int L, const double* __restrict__ dl, const double* __restrict__ bl,
                          const double* __restrict__ g2, const double* __restrict__ r_alm, double resc,
                          const double* __restrict__ zs, uint32_t seed_lo, uint32_t seed_hi, uint32_t chain,
                          uint32_t iter, double* __restrict__ rhs) {
    const long long NR = (long long)(L + 1) * (L + 1);
    const long long nlm = (long long)(L + 1) * (L + 2) / 2;
    const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i >= nlm) return;
    {
        const long long cb = (long long)blockIdx.y * F * NR;
        dl += (long long)blockIdx.y * (F == 3 ? 4 : F) * (L + 1);
        r_alm += cb; rhs += cb;
        if (zs) zs += cb;
        chain += blockIdx.y;
    }
    int l, m;
    cidx_lm(L, i, l, m);
    const long long r = m == 0 ? l : 2 * i - (L + 1);
    const int nv = m == 0 ? 1 : 2;
    double z[3][2];
    slot_normals(zs, NR, F, r, nv, chain_key(seed_lo, seed_hi, chain), i, SUB_PCG_S, iter, z);
    const PriorPinv q = prior_pinv<F>(dl, L, l);
    const double b = bl[l];
    for (int c = 0; c < nv; ++c) {
        double h[3];
        if constexpr (F != 3) { h[0] = q.ie * z[0][c]; h[1] = q.ib * (F == 2 ? z[1][c] : 0.0); }
        else { h[0] = q.i00 * z[0][c] + q.t10 * z[1][c]; h[1] = q.i11 * z[1][c]; h[2] = q.iB * z[2][c]; }
#pragma unroll
        for (int f = 0; f < F; ++f) {
            const long long o = f * NR + r + c;
            rhs[o] = g2[o] + (r_alm[o] * resc * b + h[f]);
        }
    }
}

// Device-resident CG state (one solve at a time per context).  The scalars of
// the recurrence live on the device; every iteration kernel reads them there
// and returns at once when the solve has converged, so the host launches whole
// batches of iterations and reads the state once per batch, never per iteration.
struct PcgState {
    double bn, rz, rn, alpha, beta, tol;
    int it, done, maxiter, pad;
};

// z = Sigma r at one slot (all fields), Sigma = L L^T the centered block for
// kappa_f = nbar_f / w (the per-l "diag_cl" preconditioner of qcinv's chain,
// CenteredGibbs.py:282)
template <int F>
__device__ __forceinline__ void pcg_prec_slot(const double* __restrict__ p, const double (&r)[3], double (&z)[3]) {
    if constexpr (F != 3) {
#pragma unroll
        for (int f = 0; f < F; ++f) z[f] = p[F + f] * p[F + f] * r[f];
    } else {
        const double t0 = p[5] * r[0] + p[6] * r[1], t1 = p[7] * r[1];        // L^T r
        z[0] = p[5] * t0;
        z[1] = p[6] * t0 + p[7] * t1;
        z[2] = p[8] * p[8] * r[2];
    }
}

// fixed-order block reduction of NV per-thread sums -> partial[block][NV]
template <int NV>
__device__ __forceinline__ void block_partial(const double (&v)[NV], double* __restrict__ partial) {
    __shared__ double red[NV][RED_BLOCK];
#pragma unroll
    for (int k = 0; k < NV; ++k) red[k][threadIdx.x] = v[k];
    __syncthreads();
    for (int h = RED_BLOCK / 2; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h)
#pragma unroll
            for (int k = 0; k < NV; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + h];
        __syncthreads();
    }
    if (threadIdx.x == 0)
#pragma unroll
        for (int k = 0; k < NV; ++k) partial[(long long)blockIdx.x * NSUM + k] = red[k][0];
}

// q = C^+ x + (b / w) r,  r = complex_to_real(map2alm(N^-1 A b x)); with
// partial != NULL also the per-block sums of x . q (the CG's p . Q p)
template <int F>
__global__ __launch_bounds__(RED_BLOCK) void k_pcg_qdot(int L, const double* __restrict__ dl,
                                                        const double* __restrict__ bl, const double* __restrict__ x,
                                                        const double* __restrict__ r_alm, double inv_w,
                                                        double* __restrict__ out, double* __restrict__ partial,
                                                        const PcgState* __restrict__ st) {
    const long long NR = (long long)(L + 1) * (L + 1);
    const long long nlm = (long long)(L + 1) * (L + 2) / 2;
    {
        const int b = blockIdx.y;
        const long long cb = (long long)b * F * NR;
        dl += (long long)b * (F == 3 ? 4 : F) * (L + 1);
        x += cb; r_alm += cb; out += cb;
        if (partial) partial += (long long)b * gridDim.x * NSUM;
        if (st) st += b;
    }
    if (st && st->done) return;
    double acc[1] = {0.0};
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nlm; i += (long long)gridDim.x * blockDim.x) {
        int l, m;
        cidx_lm(L, i, l, m);
        const long long r = m == 0 ? l : 2 * i - (L + 1);
        const int nv = m == 0 ? 1 : 2;
        const PriorPinv q = prior_pinv<F>(dl, L, l);
        const double bw = bl[l] * inv_w;
        for (int c = 0; c < nv; ++c) {
            double cx[3];
            if constexpr (F != 3) {
                cx[0] = q.ie * q.ie * x[r + c];
                if constexpr (F == 2) cx[1] = q.ib * q.ib * x[NR + r + c];
            } else {
                const double xt = x[r + c], xe = x[NR + r + c];
                const double y0 = q.i00 * xt, y1 = q.t10 * xt + q.i11 * xe;
                cx[0] = q.i00 * y0 + q.t10 * y1;
                cx[1] = q.i11 * y1;
                cx[2] = q.iB * q.iB * x[2 * NR + r + c];
            }
#pragma unroll
            for (int f = 0; f < F; ++f) {
                const double o = cx[f] + r_alm[f * NR + r + c] * bw;
                out[f * NR + r + c] = o;
                acc[0] += x[f * NR + r + c] * o;
            }
        }
    }
    if (partial) block_partial<1>(acc, partial);
}

// initial residual: z = M r, p = z, per-block sums of (rhs . rhs, r . z, r . r)
template <int F>
__global__ __launch_bounds__(RED_BLOCK) void k_pcg_init(int L, const double* __restrict__ params,
                                                        const double* __restrict__ rhs, const double* __restrict__ rr,
                                                        double* __restrict__ z, double* __restrict__ pdir,
                                                        double* __restrict__ partial) {
    const long long NR = (long long)(L + 1) * (L + 1);
    {
        const long long cb = (long long)blockIdx.y * F * NR;
        params += (long long)blockIdx.y * (L + 1) * GS_NPARAM;
        rhs += cb; rr += cb; z += cb; pdir += cb;
        partial += (long long)blockIdx.y * gridDim.x * NSUM;
    }
    double acc[3] = {0.0, 0.0, 0.0};
    for (long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x; g < NR; g += (long long)gridDim.x * blockDim.x) {
        int l;
        if (g <= L) l = (int)g;
        else { int m; cidx_lm(L, (g + L + 1) / 2, l, m); }
        double rv[3] = {0, 0, 0}, zv[3] = {0, 0, 0};
#pragma unroll
        for (int f = 0; f < F; ++f) rv[f] = rr[f * NR + g];
        pcg_prec_slot<F>(params + (long long)l * GS_NPARAM, rv, zv);
#pragma unroll
        for (int f = 0; f < F; ++f) {
            z[f * NR + g] = zv[f];
            pdir[f * NR + g] = zv[f];
            const double b = rhs[f * NR + g];
            acc[0] += b * b;
            acc[1] += rv[f] * zv[f];
            acc[2] += rv[f] * rv[f];
        }
    }
    block_partial<3>(acc, partial);
}

// alpha = rz / p.Qp from k_pcg_qdot's partials (slot 0), computed by every
// workgroup in the fixed order of k_pcg_scal (the same block_sums at the same
// block size: the same alpha bits, one launch fewer per CG iteration); then
// x += alpha p; r -= alpha q; z = M r; per-block sums of (r . z, r . r) into
// slots PCG_UPD_SLOT.. (disjoint from the slot the other workgroups still read)
constexpr int PCG_UPD_SLOT = 4;
template <int F>
__global__ __launch_bounds__(RED_BLOCK) void k_pcg_upd(int L, int nb, const double* __restrict__ params,
                                                       const double* __restrict__ p, const double* __restrict__ q,
                                                       double* __restrict__ x, double* __restrict__ rr,
                                                       double* __restrict__ z, double* __restrict__ partial,
                                                       PcgState* __restrict__ st) {
    {
        const long long cb = (long long)blockIdx.y * F * (long long)(L + 1) * (L + 1);
        params += (long long)blockIdx.y * (L + 1) * GS_NPARAM;
        p += cb; q += cb; x += cb; rr += cb; z += cb;
        partial += (long long)blockIdx.y * gridDim.x * NSUM;
        st += blockIdx.y;
    }
    if (st->done) return;
    double pq[1];
    block_sums<1>(nb, partial, NSUM, pq);
    const double a = st->rz / pq[0];
    if (blockIdx.x == 0 && threadIdx.x == 0) st->alpha = a;
    const long long NR = (long long)(L + 1) * (L + 1);
    double acc[2] = {0.0, 0.0};
    for (long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x; g < NR; g += (long long)gridDim.x * blockDim.x) {
        int l;
        if (g <= L) l = (int)g;
        else { int m; cidx_lm(L, (g + L + 1) / 2, l, m); }
        double rv[3] = {0, 0, 0}, zv[3] = {0, 0, 0};
#pragma unroll
        for (int f = 0; f < F; ++f) {
            const long long o = f * NR + g;
            x[o] += a * p[o];
            rv[f] = rr[o] - a * q[o];
            rr[o] = rv[f];
        }
        pcg_prec_slot<F>(params + (long long)l * GS_NPARAM, rv, zv);
#pragma unroll
        for (int f = 0; f < F; ++f) {
            z[f * NR + g] = zv[f];
            acc[0] += rv[f] * zv[f];
            acc[1] += rv[f] * rv[f];
        }
    }
    block_partial<2>(acc, partial + PCG_UPD_SLOT);
}

// the CG scalars from the block partials (fixed order), on the device:
// MODE 0 init (bn, rz, rn, done), 1 alpha = rz / p.Qp (the CG loop folds it into
// k_pcg_upd), 2 beta / rz / rn / it / done
template <int MODE>
__global__ __launch_bounds__(RED_BLOCK) void k_pcg_scal(int nblk, const double* __restrict__ partial,
                                                        PcgState* __restrict__ st, double tol, int maxiter) {
    partial += (long long)blockIdx.y * nblk * NSUM;         // chain b: one workgroup
    st += blockIdx.y;
    if (MODE != 0 && st->done) return;
    constexpr int NV = MODE == 0 ? 3 : (MODE == 1 ? 1 : 2);
    double t[NV];
    block_sums<NV>(nblk, partial + (MODE == 2 ? PCG_UPD_SLOT : 0), NSUM, t);
    if (threadIdx.x != 0) return;
    if constexpr (MODE == 0) {
        st->bn = sqrt(t[0]);
        st->rz = t[1];
        st->rn = sqrt(t[2]);
        st->tol = tol;
        st->maxiter = maxiter;
        st->it = 0;
        st->alpha = st->beta = 0.0;
        st->done = (0 < maxiter && st->rn > tol * st->bn) ? 0 : 1;
    } else if constexpr (MODE == 1) {
        st->alpha = st->rz / t[0];
    } else {
        st->beta = t[0] / st->rz;
        st->rz = t[0];
        st->rn = sqrt(t[1]);
        st->it += 1;
        st->done = (st->it < st->maxiter && st->rn > st->tol * st->bn) ? 0 : 1;
    }
}

// p = z + beta p (after the iteration's last scalar update)
__global__ void k_pcg_dir(long long n, const PcgState* __restrict__ st, const double* __restrict__ z,
                          double* __restrict__ p) {
    st += blockIdx.y;
    if (st->done) return;
    z += (long long)blockIdx.y * n;
    p += (long long)blockIdx.y * n;
    const double b = st->beta;
    for (long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x; g < n; g += (long long)gridDim.x * blockDim.x)
        p[g] = z[g] + b * p[g];
}

__global__ __launch_bounds__(RED_BLOCK) void k_dot2_finish(int nblk, const double* __restrict__ partial,
                                                           double* __restrict__ out) {
    partial += (long long)blockIdx.y * nblk * 2;
    out += 2 * blockIdx.y;
    double t[2];
    block_sums<2>(nblk, partial, 2, t);
    if (threadIdx.x == 0) {
        out[0] = t[0];
        out[1] = t[1];
    }
}

// y = a - y (the residual of an initial guess)
__global__ void k_sub_from(long long n, const double* __restrict__ a, double* __restrict__ y) {
    const long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (g < n) y[g] = a[g] - y[g];
}

// ---------------------------------------------------------------------------
// f2: pixel-domain non-centered likelihood (NonCenteredGibbs.py:333-355)
// ---------------------------------------------------------------------------
// out = C^(dir/2) in per slot: dir = +1 the centered map C^1/2 s_nc (EB
// sqrt(var), TEB chol(C)); dir = -1 the non-centered map C^+1/2 s (EB
// sqrt(inv_var) (NonCenteredGibbs.py:236-237, ASIS.py:185-189), TEB A^+)
template <int F>
__global__ void k_mc_center(int L, const double* __restrict__ dl, int dir, const double* __restrict__ in,
                            double* __restrict__ out) {
    const long long NR = (long long)(L + 1) * (L + 1);
    const long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (g >= NR) return;
    dl += (long long)blockIdx.y * (F == 3 ? 4 : F) * (L + 1);
    in += (long long)blockIdx.y * F * NR;
    out += (long long)blockIdx.y * F * NR;
    int l;
    if (g <= L) l = (int)g;
    else { int m; cidx_lm(L, (g + L + 1) / 2, l, m); }
    if constexpr (F != 3) {
        for (int f = 0; f < F; ++f) {
            const double v = var_from_dl(dl[f * (L + 1) + l], l);
            const double fac = dir > 0 ? sqrt(v) : (v != 0.0 ? sqrt(1.0 / v) : 0.0);
            out[f * NR + g] = fac * in[f * NR + g];
        }
    } else {
        const double tt = var_from_dl(dl[l], l), ee = var_from_dl(dl[(L + 1) + l], l);
        const double bb = var_from_dl(dl[2 * (L + 1) + l], l), te = var_from_dl(dl[3 * (L + 1) + l], l);
        const CovChol A = cov_chol_teb(tt, ee, te, bb);
        const double x0 = in[g], x1 = in[NR + g], x2 = in[2 * NR + g];
        if (dir > 0) {
            out[g] = A.a00 * x0;
            out[NR + g] = A.a10 * x0 + A.a11 * x1;
            out[2 * NR + g] = A.aB * x2;
        } else {
            const double i00 = A.a00 != 0.0 ? 1.0 / A.a00 : 0.0, i11 = A.a11 != 0.0 ? 1.0 / A.a11 : 0.0;
            const double t10 = -A.a10 * i00 * i11, iB = A.aB != 0.0 ? 1.0 / A.aB : 0.0;
            out[g] = i00 * x0;
            out[NR + g] = t10 * x0 + i11 * x1;
            out[2 * NR + g] = iB * x2;
        }
    }
}

// partial sums of N^-1 (d - m)^2 over all field rows
// synalm: a_lm = b_l C_l^1/2 z per real slot (F = 1: TT; 2: EE, BB; 3: TEB with
// the (T, E) Cholesky factor of [[TT, TE], [TE, EE]]); cl holds C_l (not D_l)
template <int F>
__global__ void k_synalm(int L, const double* __restrict__ cl, const double* __restrict__ beam,
                         const double* __restrict__ z, double* __restrict__ out) {
    const long long NR = (long long)(L + 1) * (L + 1);
    const long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (g >= NR) return;
    int l;
    if (g <= L) l = (int)g;
    else { int m; cidx_lm(L, (g + L + 1) / 2, l, m); }
    const int Lp1 = L + 1;
    if constexpr (F == 3) {
        const CovChol A = cov_chol_teb(cl[l], cl[Lp1 + l], cl[3 * Lp1 + l], cl[2 * Lp1 + l]);
        const double x0 = z[g], x1 = z[NR + g], x2 = z[2 * NR + g];
        out[g] = beam[l] * (A.a00 * x0);
        out[NR + g] = beam[Lp1 + l] * (A.a10 * x0 + A.a11 * x1);
        out[2 * NR + g] = beam[2 * Lp1 + l] * (A.aB * x2);
    } else {
        for (int f = 0; f < F; ++f)
            out[f * NR + g] = beam[f * Lp1 + l] * (sqrt(fmax(cl[f * Lp1 + l], 0.0)) * z[f * NR + g]);
    }
}

__global__ __launch_bounds__(RED_BLOCK) void k_mc_resid(long long n, const double* __restrict__ d,
                                                        const double* __restrict__ m, const double* __restrict__ w,
                                                        double* __restrict__ partial) {
    m += (long long)blockIdx.y * n;                          // chain b's model map (d, w shared)
    partial += (long long)blockIdx.y * gridDim.x * 2;
    double s0 = 0.0;
    for (long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x; g < n; g += (long long)gridDim.x * blockDim.x) {
        const double r = d[g] - m[g];
        s0 += r * r * w[g];
    }
    __shared__ double red[RED_BLOCK];
    red[threadIdx.x] = s0;
    __syncthreads();
    for (int h = RED_BLOCK / 2; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
        __syncthreads();
    }
    if (threadIdx.x == 0) { partial[2 * blockIdx.x] = red[0]; partial[2 * blockIdx.x + 1] = 0.0; }
}

__global__ void k_mc_halfneg(int nb, const double* __restrict__ two, double* __restrict__ out) {
    for (int b = threadIdx.x; b < nb; b += blockDim.x) out[b] = -0.5 * two[2 * b];
}

// f4: temperature full-sky CR from pixel data (CenteredGibbs.py:108-132 centered,
// NonCenteredGibbs.py:22-38 non-centered): per real slot, with g2 = b
// adjoint_synthesis_hp(N^-1 d), f = b adjoint_synthesis_hp(sqrt(N^-1) z_pix)
// (= b r Npix/4pi, r = map2alm(y, iter 3)) and kap = N^-1[0] Npix/4pi,
//   centered:     s = (g2 + C^+1/2 z + f) / (C^+ + kap b^2)      (C^+ zero for l < 2: mask_inversion)
//   non-centered: s = (sqrt(C) (g2 + f) + z) / (1 + C kap b^2)
template <int NC>
__global__ void k_tt_fullsky(int L, const double* __restrict__ dl, const double* __restrict__ bl,
                             const double* __restrict__ g2, const double* __restrict__ r_alm, double resc, double kap,
                             const double* __restrict__ zs, uint32_t seed_lo, uint32_t seed_hi, uint32_t chain,
                             uint32_t iter, double* __restrict__ s) {
    const long long NR = (long long)(L + 1) * (L + 1);
    const long long nlm = (long long)(L + 1) * (L + 2) / 2;
    const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i >= nlm) return;
    dl += (long long)blockIdx.y * (L + 1);
    r_alm += (long long)blockIdx.y * NR;
    s += (long long)blockIdx.y * NR;
    if (zs) zs += (long long)blockIdx.y * NR;
    chain += blockIdx.y;
    int l, m;
    cidx_lm(L, i, l, m);
    const long long r = m == 0 ? l : 2 * i - (L + 1);
    const int nv = m == 0 ? 1 : 2;
    double z[3][2];
    slot_normals(zs, NR, 1, r, nv, chain_key(seed_lo, seed_hi, chain), i, SUB_PCG_S, iter, z);
    const double v = var_from_dl(dl[l], l);
    const double b = bl[l];
    for (int c = 0; c < nv; ++c) {
        const double f = b * (r_alm[r + c] * resc);
        if constexpr (NC) {
            const double sv = sqrt(v);
            const double sig = 1.0 / (1.0 + v * kap * b * b);
            s[r + c] = sig * (sv * g2[r + c]) + sig * (z[0][c] + sv * f);
        } else {
            const double iv = (l >= 2 && v != 0.0) ? 1.0 / v : 0.0;
            const double sig = 1.0 / (iv + kap * b * b);
            s[r + c] = sig * g2[r + c] + sig * (z[0][c] * sqrt(iv) + f);
        }
    }
}

// ---------------------------------------------------------------------------
// f2, one Metropolis sweep without per-block SHTs (NonCenteredGibbs.py:401-445
// with the pixel likelihood of :333-355).  The current model map m = A b C^1/2
// s_nc is linear in the per-l factors C^1/2, and every block k changes one
// field's factors on its own l-range, so with y_k = A b (C_prop^1/2 -
// C_cur^1/2) s_nc (restricted to block k) and the residual r = d - m,
//   lik(accepted set S + k) - lik(S) = <N^-1 (r - sum_{j in S} y_j), y_k> - <N^-1 y_k, y_k> / 2
//                                    = g_k - sum_{j in S} G_kj - G_kk / 2,
// g_k = <N^-1 r, y_k>, G_kj = <N^-1 y_k, y_j>.  All y_k come from ONE block
// synthesis (gs_sht_synth_blocks: the Legendre recurrence shared by every
// block), G from one weighted Gram pass, and the blocks are then decided in
// the reference's order by one workgroup -- no host round trip per block.
// ---------------------------------------------------------------------------
constexpr int F2_GSUB = 32;          // elements per LDS stage of the Gram pass
constexpr int F2_RMAX = 176;         // rows (blocks + residual) per Gram pass
// dynamic LDS k_f2_decide may use: 160 KB less its static arrays (5 x F2_RMAX words + 1)
constexpr size_t F2_DECIDE_LDS = 160 * 1024 - (2 * sizeof(double) + 3 * sizeof(int)) * F2_RMAX - 64;
constexpr long long F2_CHUNK = 2048; // elements per Gram workgroup

// delta a (real layout) of blocks [k0, k0 + kn) and their local block table;
// blockIdx.y = chain (per-chain D_l [F][L+1], s_nc / da [F][(L+1)^2]; chain 0's
// threads write the shared local table)
template <int F>
__global__ void k_f2_delta(int L, int k0, int kn, const int* __restrict__ blk, const double* __restrict__ dl_cur,
                           const double* __restrict__ dl_prop, const double* __restrict__ bl,
                           const double* __restrict__ s_nc, double* __restrict__ da, int* __restrict__ blk_local) {
    const long long NR = (long long)(L + 1) * (L + 1);
    const long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    dl_cur += (long long)b * F * (L + 1);
    dl_prop += (long long)b * F * (L + 1);
    s_nc += (long long)b * F * NR;
    da += (long long)b * F * NR;
    if (g <= L && b == 0) {
#pragma unroll
        for (int f = 0; f < F; ++f) {
            const int b = blk[f * (L + 1) + g];
            blk_local[f * (L + 1) + g] = (b >= k0 && b < k0 + kn) ? b - k0 : -1;
        }
    }
    if (g >= NR) return;
    int l;
    if (g <= L) l = (int)g;
    else { int m; cidx_lm(L, (g + L + 1) / 2, l, m); }
#pragma unroll
    for (int f = 0; f < F; ++f) {
        const int b = blk[f * (L + 1) + l];
        double v = 0.0;
        if (b >= k0 && b < k0 + kn) {
            const double cp = sqrt(var_from_dl(dl_prop[f * (L + 1) + l], l));
            const double cc = sqrt(var_from_dl(dl_cur[f * (L + 1) + l], l));
            v = bl[l] * ((cp - cc) * s_nc[f * NR + g]);
        }
        da[f * NR + g] = v;
    }
}

// r = d - m per chain (blockIdx.y; d shared)
__global__ void k_f2_resid(long long n, const double* __restrict__ d, const double* __restrict__ m,
                           double* __restrict__ r) {
    const long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    const long long o = blockIdx.y * n;
    if (g < n) r[o + g] = d[g] - m[o + g];
}

// each chain's copy of the group's block l_max (the batched ring stage indexes
// its comps chain-major)
__global__ void k_f2_rep_lmax(int nb, int kn, const int* __restrict__ lmax, int* __restrict__ out) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g < nb * kn) out[g] = lmax[g % kn];
}

// Lower triangle of the R x R weighted Gram matrix of rows 0..R-2 = Y, R-1 = r,
// over one chunk of F2_CHUNK elements, on the fp64 matrix cores
// (v_mfma_f64_16x16x4_f64).  Every row is staged once per element (times
// sqrt(N^-1)) in LDS, S[element][row]: thread t stages element column t % 32
// and rows t / 32 + 8 j, all of a stage's loads issued together and the next
// stage's issued before this stage's MFMAs (one memory latency per stage,
// hidden).  The triangle is cut into 16 x 16 tiles (I >= J), tile pairs dealt
// round-robin to the 4 waves, one accumulator tile per owned pair; per k-step
// of 4 staged elements a pair costs two 8-B LDS reads -- lane l holds row
// 16 I + (l & 15) (A) / 16 J + (l & 15) (B) of element 4 s + (l >> 4) -- and one
// MFMA (1024 FMAs).  The r02/r03 VALU form (4 x 4 blocks per thread, 4 x 16-B
// LDS reads per 16 FMAs) was LDS-bound at about half the FMA rate: 1182 us
// against 736 us here at N_side 256 / 136 rows.  D layout (gfx950 f64): row
// (l >> 4) + 4 reg, col l & 15.  Per-chunk partials [chunk][nblk4][16] (4 x 4
// blocks of the lower triangle), summed in chunk order by k_f2_gram_finish.
typedef double f64x4 __attribute__((ext_vector_type(4)));
constexpr int F2_TMAX = (F2_RMAX + 15) / 16;
// T = 16-row tiles of this group (compile-time: the pair loop and the staging
// are branch-free, so a k-step's LDS reads are issued together ahead of its
// MFMAs).  A wave's slots past the last pair repeat its previous pair and are
// not stored.
template <int T>
__global__ __launch_bounds__(256) void k_f2_gram_mfma(int R, long long n, const double* __restrict__ Y,
                                                      const double* __restrict__ r, const double* __restrict__ w,
                                                      double* __restrict__ partial, const int* __restrict__ live) {
    // chain blockIdx.y: rows Y + y (R - 1) n, residual r + y n, partials after the
    // gridDim.x chunks of each earlier chain (w shared).  Workgroup x sums chunk
    // live[x]: the chunks with a nonzero weight (a chunk without adds exact
    // zeros, so the list leaves every bit of G)
    Y += (long long)blockIdx.y * (R - 1) * n;
    r += (long long)blockIdx.y * n;
    partial += (long long)blockIdx.y * gridDim.x * (((R + 3) / 4) * ((R + 3) / 4 + 1) / 2) * 16;
    const int chunk = live[blockIdx.x];
    constexpr int SROW = F2_RMAX + 6;
    static_assert(16 * F2_TMAX <= SROW, "tile rows exceed the staged column");
    constexpr int NPAIR = T * (T + 1) / 2;
    constexpr int PPW = (NPAIR + 3) / 4;
    constexpr int ROWS = 16 * T;
    constexpr int LPT = (ROWS + 7) / 8;
    __shared__ __attribute__((aligned(16))) double S[F2_GSUB][SROW];
    const int nb4 = (R + 3) / 4;
    const int nblk4 = nb4 * (nb4 + 1) / 2;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    GS_ASSERT(R <= ROWS && R > ROWS - 16);
    int ti[PPW], tj[PPW];
#pragma unroll
    for (int q = 0; q < PPW; ++q) {
        const int p0 = wave + 4 * q;
        const int p = p0 < NPAIR ? p0 : p0 - 4;
        int i = 0;
        while ((i + 1) * (i + 2) / 2 <= p) ++i;
        ti[q] = i;
        tj[q] = p - i * (i + 1) / 2;
    }
    f64x4 acc[PPW];
#pragma unroll
    for (int q = 0; q < PPW; ++q) acc[q] = f64x4{0.0, 0.0, 0.0, 0.0};
    const long long e0 = (long long)chunk * F2_CHUNK, e1 = min(n, e0 + F2_CHUNK);
    const int c = tid & (F2_GSUB - 1), r0 = tid / F2_GSUB;
    double v[LPT], sw;
    auto issue = [&](long long es) {
        const long long e = es + c;
        const bool ein = e < e1;
        const long long ec = ein ? e : e1 - 1;
        sw = w[ec];
#pragma unroll
        for (int j = 0; j < LPT; ++j) {
            const int row = r0 + 8 * j;
            const int rr = min(row, R - 1);
            v[j] = rr < R - 1 ? Y[(long long)rr * n + ec] : r[ec];
        }
        if (!ein) sw = 0.0;
    };
    issue(e0);
    const int rl = lane & 15, kq = lane >> 4;
    for (long long es = e0; es < e1; es += F2_GSUB) {
        const double s = sqrt(sw);
#pragma unroll
        for (int j = 0; j < LPT; ++j) {
            const int row = r0 + 8 * j;
            if (row < ROWS) S[c][row] = row < R ? v[j] * s : 0.0;
        }
        __syncthreads();
        if (es + F2_GSUB < e1) issue(es + F2_GSUB);
#pragma unroll
        for (int ks = 0; ks < F2_GSUB / 4; ++ks) {
            const double* col = &S[4 * ks + kq][rl];
            double a[PPW], b[PPW];
#pragma unroll
            for (int q = 0; q < PPW; ++q) { a[q] = col[16 * ti[q]]; b[q] = col[16 * tj[q]]; }
#pragma unroll
            for (int q = 0; q < PPW; ++q) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[q], b[q], acc[q], 0, 0, 0);
        }
        __syncthreads();
    }
    double* po = partial + (long long)blockIdx.x * nblk4 * 16;
#pragma unroll
    for (int q = 0; q < PPW; ++q) {
        if (wave + 4 * q >= NPAIR) break;                    // repeated slot
        const int gj = 16 * tj[q] + rl;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int gi = 16 * ti[q] + kq + 4 * g;
            const int bi = gi >> 2, bj = gj >> 2;
            if (bi < nb4 && bj <= bi)
                po[(long long)(bi * (bi + 1) / 2 + bj) * 16 + (gi & 3) * 4 + (gj & 3)] = acc[q][g];
        }
    }
}

template <int T>
void launch_gram_mfma_t(int Tr, unsigned nchunk, unsigned nch, hipStream_t st, int R, long long n, const double* Y,
                        const double* r, const double* w, double* part, const int* live) {
    if constexpr (T <= F2_TMAX) {
        if (Tr == T) {
            hipLaunchKernelGGL(k_f2_gram_mfma<T>, dim3(nchunk, nch), dim3(256), 0, st, R, n, Y, r, w, part, live);
            return;
        }
        launch_gram_mfma_t<T + 1>(Tr, nchunk, nch, st, R, n, Y, r, w, part, live);
    }
}

// chain blockIdx.y: its partials (nchunk chunks) -> G + y R R
__global__ void k_f2_gram_finish(int R, int nchunk, const double* __restrict__ partial, double* __restrict__ G) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= R * R) return;
    const int i = g / R, j = g % R;
    if (j > i) return;
    const int nb4 = (R + 3) / 4;
    const int nblk4 = nb4 * (nb4 + 1) / 2;
    partial += (long long)blockIdx.y * nchunk * nblk4 * 16;
    G += (long long)blockIdx.y * R * R;
    const int b = (i / 4) * (i / 4 + 1) / 2 + j / 4;
    const double* pp = partial + (long long)b * 16 + (i % 4) * 4 + (j % 4);
    const long long cs = (long long)nblk4 * 16;
    // chunks in order, 16 loads issued before their sums (the last group's
    // extra loads clamped and dropped): one memory latency per 16 chunks
    // instead of one per chunk (768 chunks at N_side 256: 284 us before)
    double s = 0.0;
    for (int c0 = 0; c0 < nchunk; c0 += 16) {
        double v[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) v[t] = pp[(long long)min(c0 + t, nchunk - 1) * cs];
#pragma unroll
        for (int t = 0; t < 16; ++t)
            if (c0 + t < nchunk) s += v[t];
    }
    G[g] = s;
}

// the decisions of blocks k0 .. k0+kn-1 in order (NonCenteredGibbs.py:427-442):
// log u < (g_k - sum_{j accepted} G_kj - G_kk / 2) + sum log r; after an
// acceptance later attempts see delta = 0 (the proposal IS the state).
// One workgroup; corr[k] = sum over accepted j < k of G_kj, accumulated in
// decision order.  Everything that does not depend on earlier decisions --
// the lower triangle of G, each block's sum of log proposal ratios and the
// log accept uniforms -- is staged in LDS in parallel first, so the serial
// chain of decisions touches LDS only (it was a chain of global-memory
// latencies per block: 236 us for 135 blocks at N_side 256).
// One workgroup per chain (blockIdx.x; per-chain G [R][R], spectra [F][maxbins],
// uniforms / flags [K][n_iter] with K = kacc blocks, taken [kn]): the chains'
// serial decision chains run side by side
__global__ __launch_bounds__(256) void k_f2_decide(int kn, int R, const double* __restrict__ G, int k0, int n_iter,
                                                   const int* __restrict__ blk_field,
                                                   const int* __restrict__ blk_bins, int maxbins,
                                                   const double* __restrict__ logr, const double* __restrict__ u_acc,
                                                   const double* __restrict__ prop, double* __restrict__ binned,
                                                   int32_t* __restrict__ accept_out, double* __restrict__ taken_out,
                                                   int lu_lds, int nspec, int kacc) {
    {
        const long long b = blockIdx.x;
        G += b * R * R;
        logr += b * nspec * maxbins;
        prop += b * nspec * maxbins;
        binned += b * nspec * maxbins;
        u_acc += b * kacc * n_iter;
        accept_out += b * kacc * n_iter;
        taken_out += b * kn;
    }
    extern __shared__ __attribute__((aligned(16))) double Gl[];      // [R (R + 1) / 2] lower triangle,
                                                                     // then (lu_lds) [kn][n_iter] log u
    __shared__ double corr[F2_RMAX];
    __shared__ double lrs[F2_RMAX];
    __shared__ int bfield[F2_RMAX], blo[F2_RMAX], bhi[F2_RMAX];
    __shared__ int taken_s;
    GS_ASSERT(kn < F2_RMAX && R == kn + 1);
    const int tid = threadIdx.x;
    const int ntri = R * (R + 1) / 2;
    double* lu = Gl + ntri;
    // the log uniforms go to LDS when they fit beside the triangle (the host
    // decides); otherwise the serial chain takes them from global memory
    if (lu_lds)
        for (int t = tid; t < kn * n_iter; t += blockDim.x) lu[t] = log(u_acc[(long long)k0 * n_iter + t]);
    for (int t = tid; t < ntri; t += blockDim.x) {
        int i = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
        while ((i + 1) * (i + 2) / 2 <= t) ++i;
        while (i * (i + 1) / 2 > t) --i;
        Gl[t] = G[(long long)i * R + (t - i * (i + 1) / 2)];
    }
    for (int k = tid; k < kn; k += blockDim.x) {
        corr[k] = 0.0;
        const int kg = k0 + k, f = blk_field[kg];
        const int lo = blk_bins[2 * kg], hi = blk_bins[2 * kg + 1];
        GS_ASSERT(lo >= 0 && hi <= maxbins && lo <= hi);
        bfield[k] = f; blo[k] = lo; bhi[k] = hi;
        double sl = 0.0;
        for (int b = lo; b < hi; ++b) sl += logr[f * maxbins + b];
        lrs[k] = sl;
    }
    __syncthreads();
    const int rl = (R - 1) * R / 2;                        // row R - 1 (the residual) of the triangle
    for (int k = 0; k < kn; ++k) {
        if (tid == 0) {
            const int kg = k0 + k, f = bfield[k];
            const double delta = (Gl[rl + k] - corr[k]) - 0.5 * Gl[k * (k + 1) / 2 + k];
            bool taken = false;
            for (int att = 0; att < n_iter; ++att) {
                const double l_u = lu_lds ? lu[k * n_iter + att] : log(u_acc[(long long)kg * n_iter + att]);
                const bool acc = l_u < (taken ? 0.0 : delta) + lrs[k];
                taken = taken || acc;
                accept_out[(long long)kg * n_iter + att] = acc ? 1 : 0;
            }
            taken_s = taken ? 1 : 0;
            taken_out[k] = taken ? 1.0 : 0.0;
            (void)f;
        }
        __syncthreads();
        if (taken_s) {
            for (int j = k + 1 + tid; j < kn; j += blockDim.x) corr[j] += Gl[j * (j + 1) / 2 + k];
            if (tid == 0) bfield[k] = -1 - bfield[k];          // mark taken (field kept, encoded)
        }
        __syncthreads();
    }
    // the accepted blocks' proposals into the binned spectra, all blocks in
    // parallel (their bins are disjoint), off the serial decision chain
    for (int k = 0; k < kn; ++k) {
        if (bfield[k] >= 0) continue;
        const int f = -1 - bfield[k];
        for (int b = blo[k] + tid; b < bhi[k]; b += blockDim.x) binned[f * maxbins + b] = prop[f * maxbins + b];
    }
}

// r -= sum over accepted blocks of y_k (before the next group of blocks); chain
// blockIdx.y (Y [kn][n], taken [kn], r [n] per chain)
__global__ void k_f2_update(long long n, int kn, const double* __restrict__ Y, const double* __restrict__ taken,
                            double* __restrict__ r) {
    const long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    Y += (long long)blockIdx.y * kn * n;
    taken += (long long)blockIdx.y * kn;
    r += (long long)blockIdx.y * n;
    if (g >= n) return;
    double v = r[g];
    for (int k = 0; k < kn; ++k)
        if (taken[k] != 0.0) v -= Y[(long long)k * n + g];
    r[g] = v;
}

}  // namespace

// ============================================================================
// context
// ============================================================================
struct gs_masked {
    int L = 0, nside = 0, F = 0, n_gibbs = 1, nblk = 0;
    int B = 1;                       // chains of the batch
    long long npix = 0, NR = 0, nlm = 0;
    long long FR = 0, FP = 0;        // per-chain strides: F (L+1)^2 slots, F Npix pixels
    int nspec = 2;                   // D_l rows per chain (1, 2 or 4)
    double w = 0, alpha = -0.995, tau = 0.02, noise_pol0 = 1.0;
    double mu[3] = {0, 0, 0};
    double nbar[3] = {0, 0, 0};      // mean N^-1 per map row (PCG preconditioner)
    double ninv0[3] = {0, 0, 0};     // N^-1 of pixel 0 per map row (the TT closed forms' noise level)
    double mu_eps = 1e-14;
    int adj_iter = 0;
    Rows rows{{1, 2, 0}};
    gs_sht* sht = nullptr;
    // shared by the batch (one data set): beam, data maps, N^-1, b A^T N^-1 d
    double *bl = nullptr, *dpix = nullptr, *ninv = nullptr, *g2 = nullptr;
    // per chain ([B][...])
    double *params = nullptr, *params_mala = nullptr;
    int* ell2bin = nullptr;
    double *x = nullptr, *Abs = nullptr, *y = nullptr, *r = nullptr, *r1 = nullptr;
    double *grad0 = nullptr, *grad1 = nullptr, *snew = nullptr, *pix0 = nullptr, *pix1 = nullptr, *vtmp = nullptr;
    double *partial = nullptr, *lr = nullptr;
    int32_t* accd = nullptr;         // the last MALA / RJPO accept decisions (device, [B])
    double *pr = nullptr, *pz = nullptr, *pp = nullptr, *pq = nullptr, *params_pcg = nullptr, *dots = nullptr;
    double* pcgs = nullptr;          // PcgState [B] of the device CG
    int pcg_syncs = 0;               // host synchronisations of the last solve
    int pcg_launched = 0;            // CG iterations launched by the last solve (>= every chain's count)
    long long pcg_work = 0;          // chain-iterations transformed by the last solve (compaction: sum of active)
    int* pcg_act = nullptr;          // [B] the unconverged chains of the running solve
    // f2 block MH workspace (f2_nb chains at a time; allocated on first use, grown as needed)
    double *f2_da = nullptr, *f2_r = nullptr, *f2_Y = nullptr, *f2_phib = nullptr, *f2_part = nullptr,
           *f2_G = nullptr, *f2_taken = nullptr;
    int *f2_blk = nullptr, *f2_lmaxb = nullptr;
    int* f2_live = nullptr;          // Gram chunks with a nonzero N^-1 (set at create)
    int f2_nlive = 0;
    int f2_cap = 0;                  // blocks per chain the Y / phib buffers hold
    int f2_nb = 0;                   // chains the buffers hold
};

namespace {

void mc_free(gs_masked* c) {
    if (c->sht) gs_sht_destroy(c->sht);
    double* bufs[] = {c->bl, c->dpix, c->ninv, c->g2, c->params, c->params_mala, c->x, c->Abs, c->y, c->r, c->r1,
                      c->grad0, c->grad1, c->snew, c->pix0, c->pix1, c->vtmp, c->partial, c->lr,
                      c->pr, c->pz, c->pp, c->pq, c->params_pcg, c->dots, c->pcgs, c->f2_da, c->f2_r, c->f2_Y,
                      c->f2_phib, c->f2_part, c->f2_G, c->f2_taken};
    for (double* b : bufs)
        if (b) (void)hipFree(b);
    if (c->ell2bin) (void)hipFree(c->ell2bin);
    if (c->accd) (void)hipFree(c->accd);
    if (c->f2_blk) (void)hipFree(c->f2_blk);
    if (c->f2_lmaxb) (void)hipFree(c->f2_lmaxb);
    if (c->f2_live) (void)hipFree(c->f2_live);
    if (c->pcg_act) (void)hipFree(c->pcg_act);
    delete c;
}

template <typename T>
int mc_alloc(T** p, size_t n) {
    GS_CHECK(hipMalloc((void**)p, std::max<size_t>(n, 1) * sizeof(T)));
    GS_CHECK(hipMemset(*p, 0, std::max<size_t>(n, 1) * sizeof(T)));
    return 0;
}

// centered per-l blocks of a plan-less model: kappa_f for unbinned D_l
// [B][nspec][L+1] -> params [B][L+1][NP]
template <int F>
__global__ void k_mc_params(int L, int nch, const double* __restrict__ dl, const int* __restrict__ ell2bin,
                            const double* __restrict__ bl, double k0, double k1, double k2, double* __restrict__ params) {
    block_params_at<F, GS_MODE_CENTERED>(blockIdx.x * blockDim.x + threadIdx.x, L, nch, L + 1, dl, ell2bin, bl, k0, k1,
                                         k2, params);
}

int mc_params(gs_masked* c, int nch, const double* dl, const double* kap, double* out, hipStream_t st) {
    const dim3 g(nblocks((long long)nch * (c->L + 1), 256)), b(256);
    if (c->F == 1)
        hipLaunchKernelGGL(k_mc_params<1>, g, b, 0, st, c->L, nch, dl, c->ell2bin, c->bl, kap[0], kap[1], kap[2], out);
    else if (c->F == 2)
        hipLaunchKernelGGL(k_mc_params<2>, g, b, 0, st, c->L, nch, dl, c->ell2bin, c->bl, kap[0], kap[1], kap[2], out);
    else
        hipLaunchKernelGGL(k_mc_params<3>, g, b, 0, st, c->L, nch, dl, c->ell2bin, c->bl, kap[0], kap[1], kap[2], out);
    GS_LAUNCH_CHECK("k_mc_params");
    return 0;
}

// maps of b s for nch chains (the beam applied on the transform's input load)
int mc_synth(gs_masked* c, int nch, const double* s, double* out, hipStream_t st) {
    return gs_sht_alm2map_batch(c->sht, nch, c->F, GS_ALM_REAL, s, c->bl, out, st);
}

// one v | s pass (plain or over-relaxed) for the whole batch; zv: chain 0's
// replay normals of this pass, zvs their chain stride
GsAuxPix aux_args(const gs_masked* c, int over, double* v, const double* zv, long long zvs, uint32_t slo,
                  uint32_t shi, uint32_t chain, uint32_t sub, uint32_t it) {
    GsAuxPix a;
    a.ninv = c->ninv; a.dpix = c->dpix; a.v = v; a.zv = zv; a.zvs = zvs; a.npix = c->npix;
    for (int k = 0; k < 3; ++k) { a.mu[k] = c->mu[k]; a.rows[k] = c->rows.r[k]; }
    a.F = c->F; a.over = over; a.alpha = c->alpha;
    a.slo = slo; a.shi = shi; a.chain = chain; a.sub = sub; a.iter = it;
    return a;
}

int mc_v(gs_masked* c, int over, const double* s, double* v, const double* zv, long long zvs, uint32_t slo,
         uint32_t shi, uint32_t chain, uint32_t sub, uint32_t it, hipStream_t st) {
    if (mc_synth(c, c->B, s, c->Abs, st)) return -1;
    hipLaunchKernelGGL(k_mc_v, dim3(nblocks(c->FP, 256), c->B), dim3(256), 0, st,
                       aux_args(c, over, v, zv, zvs, slo, shi, chain, sub, it), c->Abs, c->y);
    GS_LAUNCH_CHECK("k_mc_v");
    return 0;
}

// the s | v analysis r = map2alm(y): iter 0 explicit for EB/TEB
// (CenteredGibbs.py:717,773,812), healpy's default iter = 3 for TT (:208)
int mc_anal(gs_masked* c, hipStream_t st) {
    return gs_sht_map2alm_batch(c->sht, c->B, c->F, GS_ALM_REAL, c->y, nullptr, c->r, c->adj_iter, st);
}

// v | s and the s | v analysis it feeds: one fused pass where the plan has one
// (tables, merged ring stage, iter 0: gs_sht_aux_pass_batch, the maps A b s and
// y never leave LDS), else mc_v + mc_anal -- the same bits either way
int mc_vs(gs_masked* c, int over, const double* s, double* v, const double* zv, long long zvs, uint32_t slo,
          uint32_t shi, uint32_t chain, uint32_t sub, uint32_t it, hipStream_t st) {
    if (c->adj_iter == 0) {
        const GsAuxPix a = aux_args(c, over, v, zv, zvs, slo, shi, chain, sub, it);
        const int rc = gs_sht_aux_pass_batch(c->sht, c->B, c->F, s, c->bl, &a, c->r, st);
        if (rc <= 0) return rc;
    }
    if (mc_v(c, over, s, v, zv, zvs, slo, shi, chain, sub, it, st)) return -1;
    return mc_anal(c, st);
}

// s | v from the analysis in c->r (k_mc_s)
int mc_s_update(gs_masked* c, int over, double* s, const double* zs, long long zss, uint32_t slo, uint32_t shi,
                uint32_t chain, uint32_t sub, uint32_t it, hipStream_t st) {
    double imu[3] = {0, 0, 0};
    for (int k = 0; k < c->F; ++k) imu[k] = 1.0 / c->mu[c->rows.r[k]];
    const dim3 g(nblocks(c->nlm, 256), c->B), b(256);
    if (c->F == 1)
        hipLaunchKernelGGL(k_mc_s<1>, g, b, 0, st, c->L, c->params, c->r, imu[0], imu[1], imu[2], zs, zss, slo, shi,
                           chain, sub, it, over, c->alpha, s);
    else if (c->F == 2)
        hipLaunchKernelGGL(k_mc_s<2>, g, b, 0, st, c->L, c->params, c->r, imu[0], imu[1], imu[2], zs, zss, slo, shi,
                           chain, sub, it, over, c->alpha, s);
    else
        hipLaunchKernelGGL(k_mc_s<3>, g, b, 0, st, c->L, c->params, c->r, imu[0], imu[1], imu[2], zs, zss, slo, shi,
                           chain, sub, it, over, c->alpha, s);
    GS_LAUNCH_CHECK("k_mc_s");
    return 0;
}

// the MALA gradient without its map: r = map2alm(N^-1 A b s) from the fused
// operator pass (gs_sht_apply_weighted_batch; the map stays in LDS on the table
// path), kept in rbuf for the data term of the log density (k_mc_sums harmonic)
int mc_gradient_r(gs_masked* c, const double* dl, const double* s, double* grad, double* rbuf, hipStream_t st) {
    if (gs_sht_apply_weighted_batch(c->sht, c->B, c->F, s, c->bl, c->ninv, c->pix0, rbuf, st)) return -1;
    hipLaunchKernelGGL(k_mc_grad, dim3(nblocks(c->F * c->nlm, 256), c->B), dim3(256), 0, st, c->L, c->F, dl, c->bl, s,
                       rbuf, c->g2, 1.0 / c->w, grad);
    GS_LAUNCH_CHECK("k_mc_grad");
    return 0;
}

int mc_gradient(gs_masked* c, const double* dl, const double* s, double* grad, double* pix, hipStream_t st) {
    if (mc_synth(c, c->B, s, pix, st)) return -1;
    // map2alm(N^-1 A b s), N^-1 applied on the ring stage's pixel load
    if (gs_sht_map2alm_batch(c->sht, c->B, c->F, GS_ALM_REAL, pix, c->ninv, c->r, 0, st)) return -1;
    hipLaunchKernelGGL(k_mc_grad, dim3(nblocks(c->F * c->nlm, 256), c->B), dim3(256), 0, st, c->L, c->F, dl, c->bl, s,
                       c->r, c->g2, 1.0 / c->w, grad);
    GS_LAUNCH_CHECK("k_mc_grad");
    return 0;
}

}  // namespace

extern "C" {

int gs_masked_create(const gs_masked_desc* desc, const double* maps, const double* inv_noise, gs_masked** out) {
    if (!desc || !maps || !inv_noise || !out) return set_error("gs_masked_create: null argument");
    *out = nullptr;
    if (desc->nfields < 1 || desc->nfields > 3)
        return set_error("gs_masked_create: nfields must be 1 (T), 2 (EB) or 3 (TEB)");
    if (desc->adj_iter < 0 || desc->adj_iter > 16) return set_error("gs_masked_create: adj_iter out of range");
    if (desc->nchains < 0 || desc->nchains > 4096) return set_error("gs_masked_create: nchains out of range");
    if (desc->sht_mode < 0 || desc->sht_mode > 2) return set_error("gs_masked_create: sht_mode must be 0, 1 or 2");
    if (!desc->bl) return set_error("gs_masked_create: null beam");
    gs_masked* c = new gs_masked();
    c->L = desc->lmax; c->nside = desc->nside; c->F = desc->nfields;
    c->B = std::max(1, desc->nchains);
    c->n_gibbs = std::max(1, desc->n_gibbs);
    c->alpha = desc->alpha; c->tau = desc->tau; c->noise_pol0 = desc->noise_pol0;
    c->mu_eps = desc->mu_eps > 0.0 ? desc->mu_eps : 1e-14;
    c->adj_iter = desc->adj_iter;
    c->npix = 12LL * c->nside * c->nside;
    c->NR = (long long)(c->L + 1) * (c->L + 1);
    c->nlm = (long long)(c->L + 1) * (c->L + 2) / 2;
    c->FR = c->F * c->NR;
    c->FP = c->F * c->npix;
    c->nspec = c->F == 3 ? 4 : c->F;
    c->w = 4.0 * PI / (double)c->npix;
    c->rows = c->F == 2 ? Rows{{1, 2, 0}} : Rows{{0, 1, 2}};      // F = 1: the T row
    c->nblk = (int)std::min<long long>(512, nblocks(std::max(c->F * c->NR, c->F * c->npix), RED_BLOCK));
    if (gs_sht_create(c->nside, c->L, &c->sht)) { mc_free(c); return -1; }
    if (gs_sht_reserve(c->sht, c->B, nullptr)) { mc_free(c); return -1; }
    // the Legendre stage: matrix-core tables for batches (auto: >= 4 chains,
    // when the plan is a small-map one and the table fits its budget)
    if (desc->sht_mode == 2 || (desc->sht_mode == 0 && c->B >= 4)) {
        if (gs_sht_set_mfma(c->sht, 1)) {
            if (desc->sht_mode == 2) { mc_free(c); return -1; }
            (void)gs_last_error();          // auto: keep the on-the-fly kernels
        }
    }
    const long long FR = c->FR, FP = c->FP;
    const size_t B = (size_t)c->B;
    int rc = 0;
    rc |= mc_alloc(&c->bl, c->L + 1);
    rc |= mc_alloc(&c->dpix, FP);
    rc |= mc_alloc(&c->ninv, FP);
    rc |= mc_alloc(&c->g2, FR);
    rc |= mc_alloc(&c->params, B * (c->L + 1) * GS_NPARAM);
    rc |= mc_alloc(&c->params_mala, B * (c->L + 1) * GS_NPARAM);
    rc |= mc_alloc(&c->ell2bin, (size_t)4 * (c->L + 1));
    rc |= mc_alloc(&c->x, B * FR);
    rc |= mc_alloc(&c->Abs, B * FP);
    rc |= mc_alloc(&c->y, B * FP);
    rc |= mc_alloc(&c->r, B * FR);
    rc |= mc_alloc(&c->r1, B * FR);
    rc |= mc_alloc(&c->grad0, B * FR);
    rc |= mc_alloc(&c->grad1, B * FR);
    rc |= mc_alloc(&c->snew, B * FR);
    rc |= mc_alloc(&c->pix0, B * FP);
    rc |= mc_alloc(&c->pix1, B * FP);
    rc |= mc_alloc(&c->vtmp, B * FP);
    rc |= mc_alloc(&c->partial, B * c->nblk * NSUM);
    rc |= mc_alloc(&c->lr, B);
    rc |= mc_alloc(&c->accd, B);
    rc |= mc_alloc(&c->pr, B * FR);
    rc |= mc_alloc(&c->pz, B * FR);
    rc |= mc_alloc(&c->pp, B * FR);
    rc |= mc_alloc(&c->pq, B * FR);
    rc |= mc_alloc(&c->params_pcg, B * (c->L + 1) * GS_NPARAM);
    rc |= mc_alloc(&c->dots, 2 * B);
    rc |= mc_alloc(&c->pcgs, B * (sizeof(PcgState) / sizeof(double)));
    rc |= mc_alloc(&c->pcg_act, B);
    if (rc) { mc_free(c); return -1; }
    std::vector<int> e2b((size_t)4 * (c->L + 1));
    for (int sp = 0; sp < 4; ++sp)
        for (int l = 0; l <= c->L; ++l) e2b[(size_t)sp * (c->L + 1) + l] = l;
    // field rows of the caller's [3][Npix] maps; mu = max(N^-1) + 1e-14 (CenteredGibbs.py:276)
    std::vector<double> host((size_t)c->npix);
    bool ok = hipMemcpy(c->bl, desc->bl, (c->L + 1) * sizeof(double), hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(c->ell2bin, e2b.data(), e2b.size() * sizeof(int), hipMemcpyHostToDevice) == hipSuccess;
    for (int k = 0; ok && k < c->F; ++k) {
        const int row = c->rows.r[k];
        ok = hipMemcpy(c->dpix + k * c->npix, maps + row * c->npix, c->npix * sizeof(double),
                       hipMemcpyDeviceToDevice) == hipSuccess &&
             hipMemcpy(c->ninv + k * c->npix, inv_noise + row * c->npix, c->npix * sizeof(double),
                       hipMemcpyDeviceToDevice) == hipSuccess &&
             hipMemcpy(host.data(), inv_noise + row * c->npix, c->npix * sizeof(double), hipMemcpyDeviceToHost) ==
                 hipSuccess;
        if (ok) {
            c->mu[row] = *std::max_element(host.begin(), host.end()) + c->mu_eps;
            c->ninv0[row] = host[0];
            double acc = 0.0;
            for (double v : host) acc += v;
            c->nbar[row] = acc / (double)c->npix;
        }
    }
    if (!ok) { mc_free(c); return set_error("gs_masked_create: copy failed"); }
    {
        // the f2 Gram pass's chunks (F2_CHUNK elements of [field][pixel]) holding a
        // nonzero weight: the others add exact zeros and are not launched
        std::vector<double> w((size_t)c->F * c->npix);
        ok = hipMemcpy(w.data(), c->ninv, w.size() * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess;
        std::vector<int> live;
        for (size_t e0 = 0; ok && e0 < w.size(); e0 += F2_CHUNK) {
            bool any = false;
            for (size_t e = e0; e < std::min(w.size(), e0 + (size_t)F2_CHUNK) && !any; ++e) any = w[e] != 0.0;
            if (any) live.push_back((int)(e0 / F2_CHUNK));
        }
        if (live.empty()) live.push_back(0);
        ok = ok && mc_alloc(&c->f2_live, live.size()) == 0 &&
             hipMemcpy(c->f2_live, live.data(), live.size() * sizeof(int), hipMemcpyHostToDevice) == hipSuccess;
        c->f2_nlive = (int)live.size();
        if (!ok) { mc_free(c); return set_error("gs_masked_create: chunk list failed"); }
    }
    // N^-1 never changes for the context: its ring classes are computed once
    // (support skip, constant-ring operator and f2 Parseval forms)
    if (gs_sht_register_weights(c->sht, c->ninv, c->F, nullptr)) { mc_free(c); return -1; }
    // second_part_grad = b * complex_to_real(map2alm(N^-1 d)) * Npix/(4 pi)  (CenteredGibbs.py:298-306)
    const long long n = c->F * c->npix;
    hipLaunchKernelGGL(k_mc_mul, dim3(nblocks(n, 256)), dim3(256), 0, 0, n, c->ninv, c->dpix, c->y);
    if (gs_sht_map2alm(c->sht, c->F, GS_ALM_REAL, c->y, c->r, c->adj_iter, nullptr)) { mc_free(c); return -1; }
    hipLaunchKernelGGL(k_mc_beam, dim3(nblocks(c->F * c->nlm, 256)), dim3(256), 0, 0, c->L, c->F, c->bl, c->r, c->g2);
    const long long nr = c->F * c->NR;
    std::vector<double> g2h((size_t)nr);
    if (hipMemcpy(g2h.data(), c->g2, nr * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) {
        mc_free(c);
        return set_error("gs_masked_create: setup failed");
    }
    const double resc = (double)c->npix / (4.0 * PI);
    for (auto& v : g2h) v *= resc;
    if (hipMemcpy(c->g2, g2h.data(), nr * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) {
        mc_free(c);
        return set_error("gs_masked_create: setup failed");
    }
    *out = c;
    return 0;
}

int gs_masked_ring_classes(const gs_masked* c, int* counts) {
    if (!c || !counts) return set_error("gs_masked_ring_classes: null argument");
    return gs_sht_ring_class_counts(c->sht, counts);
}

int gs_masked_destroy(gs_masked* c) {
    if (c) mc_free(c);
    return 0;
}

int gs_masked_info(const gs_masked* c, double* mu3, double* second_part_grad) {
    if (!c) return set_error("null masked context");
    if (mu3)
        for (int k = 0; k < 3; ++k) mu3[k] = c->mu[k];
    if (second_part_grad)
        GS_CHECK(hipMemcpy(second_part_grad, c->g2, c->F * c->NR * sizeof(double), hipMemcpyDeviceToDevice));
    return 0;
}

int gs_masked_nchains(const gs_masked* c) { return c ? c->B : set_error("null masked context"); }

int gs_masked_sht_tables(const gs_masked* c) {
    if (!c) return set_error("null masked context");
    int on = 0;
    if (gs_sht_mfma_info(c->sht, &on, nullptr)) return -1;
    return on;
}

int gs_masked_gradient(gs_masked* c, const double* dl, const double* s, double* grad, double* pix, void* stream) {
    if (!c) return set_error("null masked context");
    if (!dl || !s || !grad || !pix) return set_error("gs_masked_gradient: null argument");
    return mc_gradient(c, dl, s, grad, pix, S(stream));
}

// ---- f1 PCG ----------------------------------------------------------------
// A Q p for the batch, without its dot product (partial == nullptr) or with the
// per-block p . Q p of every chain
// chains act[0 .. na) of a [B][n] array <-> a compact [na][n] one
__global__ void k_gather_chains(long long n, const int* __restrict__ act, const double* __restrict__ src,
                                double* __restrict__ dst) {
    const long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (g < n) dst[blockIdx.y * n + g] = src[(long long)act[blockIdx.y] * n + g];
}
__global__ void k_scatter_chains(long long n, const int* __restrict__ act, const double* __restrict__ src,
                                 double* __restrict__ dst) {
    const long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (g < n) dst[(long long)act[blockIdx.y] * n + g] = src[blockIdx.y * n + g];
}

// na < B (the batched CG's unconverged chains act[0 .. na)): only their maps are
// transformed -- gathered into a compact batch (map b of a batch is bit-identical
// to the same map transformed alone, so a chain's result does not depend on
// which others still run), the results scattered back; converged chains' r is
// not updated (their update kernels no longer read it)
static int pcg_apply(gs_masked* c, const double* dl, const double* x, double* out, double* partial, int nb,
                     const PcgState* state, hipStream_t st, int na = -1, const int* act = nullptr) {
    // r = map2alm(N^-1 A b x): one fused operator pass (the maps stay in LDS on
    // the table path; bit-identical to alm2map_beamed + map2alm_weighted)
    if (na >= 0 && na < c->B) {
        const long long n = c->FR;
        hipLaunchKernelGGL(k_gather_chains, dim3(nblocks(n, 256), na), dim3(256), 0, st, n, act, x, c->snew);
        if (gs_sht_apply_weighted_batch(c->sht, na, c->F, c->snew, c->bl, c->ninv, c->pix0, c->grad1, st)) return -1;
        hipLaunchKernelGGL(k_scatter_chains, dim3(nblocks(n, 256), na), dim3(256), 0, st, n, act, c->grad1, c->r);
        GS_LAUNCH_CHECK("pcg compact apply");
    } else if (gs_sht_apply_weighted_batch(c->sht, c->B, c->F, x, c->bl, c->ninv, c->pix0, c->r, st)) {
        return -1;
    }
    const dim3 g(partial ? nb : nblocks(c->nlm, RED_BLOCK), c->B), b(RED_BLOCK);
    const double iw = 1.0 / c->w;
    if (c->F == 1) hipLaunchKernelGGL(k_pcg_qdot<1>, g, b, 0, st, c->L, dl, c->bl, x, c->r, iw, out, partial, state);
    else if (c->F == 2) hipLaunchKernelGGL(k_pcg_qdot<2>, g, b, 0, st, c->L, dl, c->bl, x, c->r, iw, out, partial, state);
    else hipLaunchKernelGGL(k_pcg_qdot<3>, g, b, 0, st, c->L, dl, c->bl, x, c->r, iw, out, partial, state);
    GS_LAUNCH_CHECK("k_pcg_qdot");
    return 0;
}

int gs_masked_pcg_rhs(gs_masked* c, const double* dl, const double* zv, const double* zs, uint64_t seed,
                      uint32_t iteration, int chain, double* rhs, void* stream) {
    if (!c) return set_error("null masked context");
    if (!dl || !rhs) return set_error("gs_masked_pcg_rhs: null argument");
    const hipStream_t st = S(stream);
    const uint32_t slo = (uint32_t)(seed & 0xFFFFFFFFu), shi = (uint32_t)(seed >> 32), ch = (uint32_t)chain;
    hipLaunchKernelGGL(k_pcg_zpix, dim3(nblocks(c->FP, 256), c->B), dim3(256), 0, st, c->npix, c->F, c->rows, c->ninv,
                       zv, slo, shi, ch, iteration, c->y);
    GS_LAUNCH_CHECK("k_pcg_zpix");
    // adjoint_synthesis_hp: map2alm with healpy's default iter = 3 (utils.py:89,104)
    if (gs_sht_map2alm_batch(c->sht, c->B, c->F, GS_ALM_REAL, c->y, nullptr, c->r, 3, st)) return -1;
    const dim3 g(nblocks(c->nlm, 256), c->B), b(256);
    const double resc = (double)c->npix / (4.0 * PI);
    if (c->F == 1)
        hipLaunchKernelGGL(k_pcg_rhs<1>, g, b, 0, st, c->L, dl, c->bl, c->g2, c->r, resc, zs, slo, shi, ch,
                           iteration, rhs);
    else if (c->F == 2)
        hipLaunchKernelGGL(k_pcg_rhs<2>, g, b, 0, st, c->L, dl, c->bl, c->g2, c->r, resc, zs, slo, shi, ch,
                           iteration, rhs);
    else
        hipLaunchKernelGGL(k_pcg_rhs<3>, g, b, 0, st, c->L, dl, c->bl, c->g2, c->r, resc, zs, slo, shi, ch,
                           iteration, rhs);
    GS_LAUNCH_CHECK("k_pcg_rhs");
    return 0;
}

// Preconditioned CG on the device, every chain of the batch at once.  One
// iteration = one batched A Q p (two SHTs over the B maps) with the fused
// p . Q p partials, alpha per chain on the device, the fused update /
// preconditioner / (r . z, r . r) pass, beta / rz / rn / convergence per chain,
// the new directions.  Every kernel reads its chain's scalars from the device
// state and returns at once after that chain converged (a converged chain's x
// no longer changes, so each chain follows exactly its one-chain solve), so the
// host launches whole batches of iterations and reads the B states once per
// batch: the batch length follows the slowest chain's residual decay (its
// predicted remaining iterations, 1..64) -- never one host round trip per
// iteration (the qcinv loop, CenteredGibbs.py:484-488, synchronised per
// iteration).  The transforms of a converged chain keep running until the
// batch's last chain converges (their results are not used).
int gs_masked_pcg_solve(gs_masked* c, const double* dl, const double* rhs, double* x, int x_is_guess, double tol,
                        int maxiter, int* iters, double* rel_residual, void* stream) {
    if (!c) return set_error("null masked context");
    if (!dl || !rhs || !x) return set_error("gs_masked_pcg_solve: null argument");
    if (maxiter < 0) return set_error("gs_masked_pcg_solve: maxiter < 0");
    const hipStream_t st = S(stream);
    const long long n = c->FR;
    const int B = c->B;
    PcgState* dst = reinterpret_cast<PcgState*>(c->pcgs);
    // preconditioner: centered per-l block with kappa_f = nbar_f / w ("diag_cl")
    double kap[3] = {0, 0, 0};
    for (int k = 0; k < c->F; ++k) kap[k] = c->nbar[c->rows.r[k]] / c->w;
    if (mc_params(c, B, dl, kap, c->params_pcg, st)) return -1;
    const int nb = (int)std::min<long long>(c->nblk, nblocks(c->nlm, RED_BLOCK));
    if (x_is_guess) {
        if (pcg_apply(c, dl, x, c->pr, nullptr, 0, nullptr, st)) return -1;
        hipLaunchKernelGGL(k_sub_from, dim3(nblocks(B * n, 256)), dim3(256), 0, st, B * n, rhs, c->pr);   // r = rhs - Qx
        GS_LAUNCH_CHECK("k_sub_from");
    } else {
        GS_CHECK(hipMemsetAsync(x, 0, B * n * sizeof(double), st));
        GS_CHECK(hipMemcpyAsync(c->pr, rhs, B * n * sizeof(double), hipMemcpyDeviceToDevice, st));
    }
    const dim3 gb(nb, B), bb(RED_BLOCK), g1(1, B);
#define GS_PI(FF) hipLaunchKernelGGL((k_pcg_init<FF>), gb, bb, 0, st, c->L, c->params_pcg, rhs, c->pr, c->pz, c->pp, \
                                     c->partial)
    if (c->F == 1) GS_PI(1); else if (c->F == 2) GS_PI(2); else GS_PI(3);
#undef GS_PI
    hipLaunchKernelGGL(k_pcg_scal<0>, g1, bb, 0, st, nb, c->partial, dst, tol, maxiter);
    GS_LAUNCH_CHECK("k_pcg_init");
    // the unconverged chains as of the last state read
    int na = B;
    const bool compact = B > 1;
    auto iteration = [&]() -> int {
        if (pcg_apply(c, dl, c->pp, c->pq, c->partial, nb, dst, st, na, c->pcg_act)) return -1;
#define GS_PU(FF) hipLaunchKernelGGL((k_pcg_upd<FF>), gb, bb, 0, st, c->L, nb, c->params_pcg, c->pp, c->pq, x, c->pr, \
                                     c->pz, c->partial, dst)
        if (c->F == 1) GS_PU(1); else if (c->F == 2) GS_PU(2); else GS_PU(3);
#undef GS_PU
        hipLaunchKernelGGL(k_pcg_scal<2>, g1, bb, 0, st, nb, c->partial, dst, tol, maxiter);
        hipLaunchKernelGGL(k_pcg_dir, gb, bb, 0, st, n, dst, c->pz, c->pp);
        GS_LAUNCH_CHECK("pcg iteration");
        return 0;
    };
    std::vector<PcgState> h((size_t)B);
    auto read_state = [&]() -> int {
        GS_CHECK(hipMemcpyAsync(h.data(), dst, B * sizeof(PcgState), hipMemcpyDeviceToHost, st));
        GS_CHECK(hipStreamSynchronize(st));
        return 0;
    };
    auto all_done = [&]() {
        for (const auto& q : h)
            if (!q.done) return false;
        return true;
    };
    if (read_state()) return -1;
    int launched = 0, batch = 8;
    c->pcg_work = 0;
    std::vector<double> rn_prev((size_t)B);
    for (int b = 0; b < B; ++b) rn_prev[b] = h[b].rn;
    c->pcg_syncs = 1;
    while (!all_done() && launched < maxiter) {
        const int k = std::max(1, std::min(batch, maxiter - launched));
        for (int j = 0; j < k; ++j)
            if (iteration()) return -1;
        launched += k;
        c->pcg_work += (long long)k * na;
        if (read_state()) return -1;
        ++c->pcg_syncs;
        if (all_done()) break;
        if (compact) {
            std::vector<int> act;
            for (int b = 0; b < B; ++b)
                if (!h[b].done) act.push_back(b);
            if ((int)act.size() < na) {
                GS_CHECK(hipMemcpyAsync(c->pcg_act, act.data(), act.size() * sizeof(int), hipMemcpyHostToDevice, st));
                GS_CHECK(hipStreamSynchronize(st));      // (act is host-pageable and goes out of scope)
                na = (int)act.size();
            }
        }
        // predicted remaining iterations of each unconverged chain from its
        // residual's decay over this batch: the next batch runs until the slowest
        // is due (one chain), or -- compacting -- until the first is due, so a
        // chain that converges drops out of the transforms within a few iterations
        double rem_max = 1.0, rem_min = 64.0;
        for (int b = 0; b < B; ++b) {
            if (h[b].done) continue;
            const double rate = rn_prev[b] > 0.0 && h[b].rn > 0.0 ? std::pow(h[b].rn / rn_prev[b], 1.0 / k) : 0.5;
            const double want = h[b].tol * h[b].bn;
            double rem = 64.0;
            if (rate < 1.0 && rate > 0.0 && h[b].rn > want) rem = std::log(want / h[b].rn) / std::log(rate);
            rem_max = std::max(rem_max, rem);
            rem_min = std::min(rem_min, rem);
        }
        const double due = compact ? std::max(1.0, rem_min) : rem_max;
        batch = (int)std::max(1.0, std::min(64.0, std::floor(due)));
        for (int b = 0; b < B; ++b) rn_prev[b] = h[b].rn;
    }
    c->pcg_launched = launched;
    for (int b = 0; b < B; ++b) {
        if (iters) iters[b] = h[b].it;
        if (rel_residual) rel_residual[b] = h[b].bn > 0 ? h[b].rn / h[b].bn : 0.0;
    }
    return 0;
}

int gs_masked_pcg_apply(gs_masked* c, const double* dl, const double* x, double* out, void* stream) {
    if (!c) return set_error("null masked context");
    if (!dl || !x || !out) return set_error("gs_masked_pcg_apply: null argument");
    return pcg_apply(c, dl, x, out, nullptr, 0, nullptr, S(stream));
}

int gs_masked_rj_accept(gs_masked* c, const double* dl, const double* rhs, const double* x, double* s,
                        const double* um, uint64_t seed, uint32_t iteration, int chain, int32_t* accept,
                        double* log_ratio, void* stream) {
    if (!c) return set_error("null masked context");
    if (!dl || !rhs || !x || !s) return set_error("gs_masked_rj_accept: null argument");
    const hipStream_t st = S(stream);
    const long long n = c->FR;
    if (pcg_apply(c, dl, x, c->pr, nullptr, 0, nullptr, st)) return -1;          // Q x (fwd_op, :655)
    const int nb = (int)std::min<long long>(c->nblk, nblocks(n, RED_BLOCK));
    hipLaunchKernelGGL(k_rj_dot, dim3(nb, c->B), dim3(RED_BLOCK), 0, st, n, rhs, c->pr, s, x, c->partial);
    GS_LAUNCH_CHECK("k_rj_dot");
    hipLaunchKernelGGL(k_rj_accept, dim3(1, c->B), dim3(RED_BLOCK), 0, st, nb, c->partial, n, um,
                       (uint32_t)(seed & 0xFFFFFFFFu), (uint32_t)(seed >> 32), (uint32_t)chain, iteration, c->accd,
                       accept, log_ratio);
    GS_LAUNCH_CHECK("k_rj_accept");
    hipLaunchKernelGGL(k_select_copy, dim3(nblocks(n, 256), c->B), dim3(256), 0, st, n, c->accd, x, s);
    GS_LAUNCH_CHECK("k_select_copy");
    return 0;
}

int gs_masked_pcg_info(const gs_masked* c, int* host_syncs) {
    if (!c) return set_error("null masked context");
    if (host_syncs) *host_syncs = c->pcg_syncs;
    return 0;
}

int gs_masked_pcg_info2(const gs_masked* c, int* host_syncs, int* launched) {
    if (!c) return set_error("null masked context");
    if (host_syncs) *host_syncs = c->pcg_syncs;
    if (launched) *launched = c->pcg_launched;
    return 0;
}

int gs_masked_pcg_work(const gs_masked* c, long long* chain_iterations) {
    if (!c || !chain_iterations) return set_error("gs_masked_pcg_work: null argument");
    *chain_iterations = c->pcg_work;
    return 0;
}

// ---- f2 --------------------------------------------------------------------
static int masked_center(gs_masked* c, int nch, const double* dl, int dir, const double* in, double* out,
                         hipStream_t st) {
    const dim3 g(nblocks(c->NR, 256), nch), b(256);
    if (c->F == 1) hipLaunchKernelGGL(k_mc_center<1>, g, b, 0, st, c->L, dl, dir, in, out);
    else if (c->F == 2) hipLaunchKernelGGL(k_mc_center<2>, g, b, 0, st, c->L, dl, dir, in, out);
    else hipLaunchKernelGGL(k_mc_center<3>, g, b, 0, st, c->L, dl, dir, in, out);
    GS_LAUNCH_CHECK("k_mc_center");
    return 0;
}

int gs_masked_center(gs_masked* c, const double* dl, int dir, const double* in, double* out, void* stream) {
    if (!c) return set_error("null masked context");
    if (!dl || !in || !out) return set_error("gs_masked_center: null argument");
    return masked_center(c, c->B, dl, dir, in, out, S(stream));
}

int gs_synalm(int lmax, int nfields, const double* cl, const double* beam, const double* z, double* alm,
              void* stream) {
    if (lmax < 0 || nfields < 1 || nfields > 3) return set_error("gs_synalm: bad lmax / nfields");
    if (!cl || !beam || !z || !alm) return set_error("gs_synalm: null argument");
    const long long NR = (long long)(lmax + 1) * (lmax + 1);
    const dim3 g(nblocks(NR, 256)), b(256);
    if (nfields == 1) hipLaunchKernelGGL(k_synalm<1>, g, b, 0, S(stream), lmax, cl, beam, z, alm);
    else if (nfields == 2) hipLaunchKernelGGL(k_synalm<2>, g, b, 0, S(stream), lmax, cl, beam, z, alm);
    else hipLaunchKernelGGL(k_synalm<3>, g, b, 0, S(stream), lmax, cl, beam, z, alm);
    GS_LAUNCH_CHECK("k_synalm");
    return 0;
}

int gs_masked_nc_loglik(gs_masked* c, const double* dl, const double* s_nc, double* lik, void* stream) {
    if (!c) return set_error("null masked context");
    if (!dl || !s_nc || !lik) return set_error("gs_masked_nc_loglik: null argument");
    const hipStream_t st = S(stream);
    if (masked_center(c, c->B, dl, +1, s_nc, c->snew, st)) return -1;
    if (mc_synth(c, c->B, c->snew, c->pix1, st)) return -1;
    const long long n = c->FP;
    const int nb = (int)std::min<long long>(c->nblk, nblocks(n, RED_BLOCK));
    hipLaunchKernelGGL(k_mc_resid, dim3(nb, c->B), dim3(RED_BLOCK), 0, st, n, c->dpix, c->pix1, c->ninv, c->partial);
    hipLaunchKernelGGL(k_dot2_finish, dim3(1, c->B), dim3(RED_BLOCK), 0, st, nb, c->partial, c->dots);
    hipLaunchKernelGGL(k_mc_halfneg, dim3(1), dim3(64), 0, st, c->B, c->dots, lik);
    GS_LAUNCH_CHECK("k_mc_resid");
    return 0;
}

// blocks of one group: bounded by the Gram pass (F2_RMAX - 1) and by the
// workspace budget (GS_F2_GROUP_BYTES, default 6 GiB: the phase planes and
// maps of every block of a group are resident at once)
static int f2_group(const gs_masked* c) {
    const long long nco = c->F == 1 ? 1 : 2;
    const long long per = nco * (2 * gs_sht_phi_plane(c->sht) * 16 + c->npix * 8);
    long long budget = 6LL << 30;
    if (const char* e = gs_detail::option("GS_F2_GROUP_BYTES")) budget = std::max(1LL, atoll(e));
    return (int)std::max(1LL, std::min<long long>(F2_RMAX - 1, budget / std::max(per, 1LL)));
}

// chains per f2 pass: every chain of a pass holds its block group's phase planes,
// maps and Gram partials at once (GS_F2_BATCH_BYTES, default 64 GiB, of which
// each chain takes f2_chain_bytes); the passes run in chain order
static long long f2_chain_bytes(const gs_masked* c, int kcap) {
    const long long nco = c->F == 1 ? 1 : 2;
    const long long n = (long long)c->F * c->npix;
    const long long nchunk = (n + F2_CHUNK - 1) / F2_CHUNK;
    const long long nb4 = (kcap + 1 + 3) / 4;
    return (long long)kcap * (nco * 2 * gs_sht_phi_plane(c->sht) * 16 + n * 8) + nchunk * nb4 * (nb4 + 1) / 2 * 128 +
           (long long)(kcap + 1) * (kcap + 1) * 8 + n * 8 + (long long)c->F * c->NR * 8;
}

// the budget is also capped at 3/4 of what the device can give the workspace
// (its free memory plus the f2 buffers this context holds, which are freed
// before the new ones are allocated), so a batch on a smaller or shared GPU
// runs in more passes instead of failing its allocation
static int f2_chains_per_pass(const gs_masked* c, int kcap) {
    long long budget = 64LL << 30;
    if (const char* e = gs_detail::option("GS_F2_BATCH_BYTES")) budget = std::max(1LL, atoll(e));
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess) {
        const long long held = c->f2_cap > 0 ? (long long)c->f2_nb * f2_chain_bytes(c, c->f2_cap) : 0;
        budget = std::min(budget, ((long long)fr + held) / 4 * 3);
    } else {
        (void)hipGetLastError();
    }
    return (int)std::max(1LL, std::min<long long>(c->B, budget / std::max(1LL, f2_chain_bytes(c, kcap))));
}

static void f2_release(gs_masked* c) {
    double* bufs[] = {c->f2_Y, c->f2_phib, c->f2_part, c->f2_G, c->f2_taken, c->f2_da, c->f2_r};
    for (double* b : bufs)
        if (b) (void)hipFree(b);
    if (c->f2_lmaxb) (void)hipFree(c->f2_lmaxb);
    c->f2_Y = c->f2_phib = c->f2_part = c->f2_G = c->f2_taken = c->f2_da = c->f2_r = nullptr;
    c->f2_lmaxb = nullptr;
    c->f2_cap = 0;
    c->f2_nb = 0;
}

// the f2 workspace for NB chains of kcap blocks; on an allocation failure the
// chains per pass are halved (down to 1) instead of failing the sweep.
// Returns the chains per pass, or -1 when even one chain does not fit.
static int f2_reserve(gs_masked* c, int kcap, int NB) {
    if (c->f2_cap >= kcap && c->f2_nb >= NB) return c->f2_nb;
    const int F = c->F, nco = F == 1 ? 1 : 2;
    const long long n = (long long)F * c->npix;
    const long long nchunk = (n + F2_CHUNK - 1) / F2_CHUNK;
    const int nb4max = (kcap + 1 + 3) / 4;
    for (;;) {
        f2_release(c);
        const size_t nb = (size_t)NB;
        int rc = 0;
        rc |= mc_alloc(&c->f2_Y, nb * kcap * n);
        rc |= mc_alloc(&c->f2_phib, nb * kcap * nco * 2 * gs_sht_phi_plane(c->sht) * 2);
        rc |= mc_alloc(&c->f2_part, nb * nchunk * (nb4max * (nb4max + 1) / 2) * 16);
        rc |= mc_alloc(&c->f2_G, nb * (kcap + 1) * (kcap + 1));
        rc |= mc_alloc(&c->f2_taken, nb * kcap);
        rc |= mc_alloc(&c->f2_da, nb * F * c->NR);
        rc |= mc_alloc(&c->f2_r, nb * n);
        rc |= mc_alloc(&c->f2_lmaxb, nb * kcap);
        if (!rc) {
            c->f2_cap = kcap;
            c->f2_nb = NB;
            return NB;
        }
        (void)hipGetLastError();
        f2_release(c);
        if (NB == 1) return -1;
        NB = (NB + 1) / 2;
    }
}

// one pass over nb chains (pointers at the pass's first chain; chain-0-relative
// scratch): every launch carries the pass's chains in its grid, each chain's
// arithmetic that of a one-chain sweep (bit-identical)
static int pixel_mh_pass(gs_masked* c, int nb, int K, int n_iter, int maxbins, const int* blk, const int* blk_lmax,
                         const int* blk_field, const int* blk_bins, const double* s_nc, const double* dl_cur,
                         const double* dl_prop, const double* logr, const double* u_acc, const double* prop_binned,
                         double* binned, int32_t* accept_out, hipStream_t st) {
    const int F = c->F;
    const int KG = f2_group(c);
    const long long n = (long long)F * c->npix;
    const long long nchunk = (n + F2_CHUNK - 1) / F2_CHUNK;
    // the rows on constant-weight ring pairs in Parseval coordinates (their
    // weighted sums over pixels are those over the coordinates; no ring DFT for
    // the block maps there): decided per plan and block grouping, not per batch,
    // so a chain's sums do not depend on how many chains share its pass
    const int nco = F == 1 ? 1 : 2;
    const int kn_last = K - KG * ((K - 1) / KG);
    const int pv = kn_last * nco >= 2 ? gs_sht_blocks_parseval(c->sht, F, kn_last * nco) : 0;
    // residual of the current state: r = d - A b C_cur^1/2 s_nc
    if (masked_center(c, nb, dl_cur, +1, s_nc, c->snew, st)) return -1;
    if (mc_synth(c, nb, c->snew, c->pix1, st)) return -1;
    hipLaunchKernelGGL(k_f2_resid, dim3(nblocks(n, 256), nb), dim3(256), 0, st, n, c->dpix, c->pix1, c->f2_r);
    GS_LAUNCH_CHECK("k_f2_resid");
    if (pv && gs_sht_parseval_maps(c->sht, nb * F, c->f2_r, st)) return -1;
    for (int k0 = 0; k0 < K; k0 += KG) {
        const int kn = std::min(KG, K - k0);
        const int R = kn + 1;
        const dim3 gd(nblocks(std::max<long long>(c->NR, c->L + 1), 256), nb), bd(256);
        if (F == 1)
            hipLaunchKernelGGL(k_f2_delta<1>, gd, bd, 0, st, c->L, k0, kn, blk, dl_cur, dl_prop, c->bl, s_nc, c->f2_da,
                               c->f2_blk);
        else
            hipLaunchKernelGGL(k_f2_delta<2>, gd, bd, 0, st, c->L, k0, kn, blk, dl_cur, dl_prop, c->bl, s_nc, c->f2_da,
                               c->f2_blk);
        GS_LAUNCH_CHECK("k_f2_delta");
        hipLaunchKernelGGL(k_f2_rep_lmax, dim3(nblocks((long long)nb * kn, 256)), dim3(256), 0, st, nb, kn,
                           blk_lmax + k0, c->f2_lmaxb);
        GS_LAUNCH_CHECK("k_f2_rep_lmax");
        if (gs_sht_synth_blocks(c->sht, nb, F, c->f2_da, c->f2_blk, kn, c->f2_lmaxb, c->f2_phib, c->f2_Y, st, pv))
            return -1;
        launch_gram_mfma_t<1>((R + 15) / 16, (unsigned)c->f2_nlive, (unsigned)nb, st, R, n, c->f2_Y, c->f2_r,
                              c->ninv, c->f2_part, c->f2_live);
        GS_LAUNCH_CHECK("k_f2_gram_mfma");
        hipLaunchKernelGGL(k_f2_gram_finish, dim3(nblocks((long long)R * R, 256), nb), dim3(256), 0, st, R,
                           c->f2_nlive, c->f2_part, c->f2_G);
        GS_LAUNCH_CHECK("k_f2_gram_finish");
        // dynamic LDS: G's lower triangle (<= 124.6 KB at F2_RMAX rows), plus the
        // log uniforms when they fit in what the static arrays leave of 160 KB
        const size_t tri = (size_t)R * (R + 1) / 2 * sizeof(double);
        const size_t lus = (size_t)kn * n_iter * sizeof(double);
        const int lu_lds = tri + lus <= F2_DECIDE_LDS ? 1 : 0;
        const size_t dlds = tri + (lu_lds ? lus : 0);
        if (dlds > F2_DECIDE_LDS) return set_error("gs_masked_pixel_mh: Gram triangle exceeds the decision LDS");
        if (dlds > 64 * 1024 &&                 // the triangle of G beyond 64 KB of dynamic LDS
            hipFuncSetAttribute((const void*)k_f2_decide, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dlds) !=
                hipSuccess) {
            (void)hipGetLastError();
            return set_error("gs_masked_pixel_mh: cannot raise k_f2_decide's dynamic LDS limit");
        }
        hipLaunchKernelGGL(k_f2_decide, dim3(nb), dim3(256), dlds, st, kn, R, c->f2_G, k0, n_iter, blk_field, blk_bins,
                           maxbins, logr, u_acc, prop_binned, binned, accept_out, c->f2_taken, lu_lds, F, K);
        GS_LAUNCH_CHECK("k_f2_decide");
        if (k0 + kn < K) {
            hipLaunchKernelGGL(k_f2_update, dim3(nblocks(n, 256), nb), dim3(256), 0, st, n, kn, c->f2_Y, c->f2_taken,
                               c->f2_r);
            GS_LAUNCH_CHECK("k_f2_update");
        }
    }
    return 0;
}

// the batch: passes of f2_chains_per_pass chains (one pass for a whole batch
// whose workspace fits the budget), each launch of a pass serving all its chains
int gs_masked_pixel_mh(gs_masked* c, int K, int n_iter, int maxbins, const int* blk, const int* blk_lmax,
                       const int* blk_field, const int* blk_bins, const double* s_nc, const double* dl_cur,
                       const double* dl_prop, const double* logr, const double* u_acc, const double* prop_binned,
                       double* binned, int32_t* accept_out, void* stream) {
    if (!c) return set_error("null masked context");
    if (c->F != 1 && c->F != 2)
        return set_error("gs_masked_pixel_mh: the pixel-domain NC likelihood is defined for T or EB "
                         "(NonCenteredClsSampler / PolarizationNonCenteredClsSampler)");
    if (K < 0 || n_iter < 1 || maxbins < 1) return set_error("gs_masked_pixel_mh: K / n_iter / maxbins out of range");
    if (K == 0) return 0;
    if (!blk || !blk_lmax || !blk_field || !blk_bins || !s_nc || !dl_cur || !dl_prop || !logr || !u_acc ||
        !prop_binned || !binned || !accept_out)
        return set_error("gs_masked_pixel_mh: null argument");
    const hipStream_t st = S(stream);
    const int F = c->F;
    const int KG = f2_group(c);
    const int kcap = std::min(K, KG);
    const int NB = f2_reserve(c, kcap, f2_chains_per_pass(c, kcap));
    if (NB < 1) return set_error("gs_masked_pixel_mh: the f2 workspace of one chain does not fit in device memory");
    if (!c->f2_blk && mc_alloc(&c->f2_blk, (size_t)F * (c->L + 1))) return -1;
    const long long dls = (long long)F * (c->L + 1), bins = (long long)F * maxbins, acc = (long long)K * n_iter;
    for (int b = 0; b < c->B; b += NB) {
        const int nb = std::min(NB, c->B - b);
        if (pixel_mh_pass(c, nb, K, n_iter, maxbins, blk, blk_lmax, blk_field, blk_bins, s_nc + b * c->FR,
                          dl_cur + b * dls, dl_prop + b * dls, logr + b * bins, u_acc + b * acc,
                          prop_binned + b * bins, binned + b * bins, accept_out + b * acc, st))
            return -1;
    }
    return 0;
}

int gs_masked_tt_fullsky(gs_masked* c, int noncentered, const double* dl, const double* zv, const double* zs,
                         uint64_t seed, uint32_t iteration, int chain, double* s_out, void* stream) {
    if (!c) return set_error("null masked context");
    if (c->F != 1) return set_error("gs_masked_tt_fullsky: temperature-only context required");
    if (!dl || !s_out) return set_error("gs_masked_tt_fullsky: null argument");
    const hipStream_t st = S(stream);
    const uint32_t slo = (uint32_t)(seed & 0xFFFFFFFFu), shi = (uint32_t)(seed >> 32), ch = (uint32_t)chain;
    hipLaunchKernelGGL(k_pcg_zpix, dim3(nblocks(c->npix, 256), c->B), dim3(256), 0, st, c->npix, 1, c->rows, c->ninv,
                       zv, slo, shi, ch, iteration, c->y);
    GS_LAUNCH_CHECK("k_pcg_zpix");
    if (gs_sht_map2alm_batch(c->sht, c->B, 1, GS_ALM_REAL, c->y, nullptr, c->r, 3, st)) return -1;
    const double resc = (double)c->npix / (4.0 * PI);
    const double kap = c->ninv0[0] * resc;
    const dim3 g(nblocks(c->nlm, 256), c->B), b(256);
    if (noncentered)
        hipLaunchKernelGGL(k_tt_fullsky<1>, g, b, 0, st, c->L, dl, c->bl, c->g2, c->r, resc, kap, zs, slo, shi, ch,
                           iteration, s_out);
    else
        hipLaunchKernelGGL(k_tt_fullsky<0>, g, b, 0, st, c->L, dl, c->bl, c->g2, c->r, resc, kap, zs, slo, shi, ch,
                           iteration, s_out);
    GS_LAUNCH_CHECK("k_tt_fullsky");
    return 0;
}

int gs_masked_cr(gs_masked* c, int kind, const double* dl, double* s, double* v, const double* zv, const double* zs,
                 const double* zm, const double* um, uint64_t seed, uint32_t iteration, int chain, int32_t* accept,
                 double* log_ratio, void* stream) {
    if (!c) return set_error("null masked context");
    if (!dl || !s) return set_error("gs_masked_cr: null argument");
    if (kind < GS_MCR_AUX || kind > GS_MCR_AUX_MALA) return set_error("gs_masked_cr: bad kind");
    if ((kind == GS_MCR_MALA || kind == GS_MCR_AUX_MALA) && c->F != 2)
        return set_error("gs_masked_cr: MALA is defined for the EB model only (CenteredGibbs.py:560-603)");
    const hipStream_t st = S(stream);
    const uint32_t slo = (uint32_t)(seed & 0xFFFFFFFFu), shi = (uint32_t)(seed >> 32), ch = (uint32_t)chain;
    const long long FP = c->FP, FR = c->FR;
    const int B = c->B;
    double* vv = v ? v : c->vtmp;
    if (kind != GS_MCR_MALA) {
        const double kap[3] = {c->mu[c->rows.r[0]] / c->w, c->F >= 2 ? c->mu[c->rows.r[1]] / c->w : 0.0,
                               c->F == 3 ? c->mu[c->rows.r[2]] / c->w : 0.0};
        if (mc_params(c, B, dl, kap, c->params, st)) return -1;
        if (kind == GS_MCR_OVERRELAX) {
            // v | s plain, then n_gibbs x (s | v, v | s, s | v) over-relaxed; replay
            // normals per chain: zv [B][1 + n_gibbs][F][Npix], zs [B][2 n_gibbs][F][NR]
            const long long zvs = (1LL + c->n_gibbs) * FP, zss = 2LL * c->n_gibbs * FR;
            // CenteredGibbs.py:733-825: v | s, then per iteration s | v, v | s, s | v.  The
            // s | v that opens iteration k > 0 follows the one that closed k - 1 with
            // v unchanged: the reference transforms the same map again
            // (map2alm(v + N^-1 d), :763-765 = :810-812); here that analysis is the
            // one already in c->r (deterministic: the same bits), so each iteration
            // costs one v | s pass and one analysis instead of one and two
            if (mc_vs(c, 0, s, vv, zv, zvs, slo, shi, ch, SUB_V_INIT, iteration, st)) return -1;
            for (int k = 0; k < c->n_gibbs; ++k) {
                const double* zs1 = zs ? zs + (2LL * k) * FR : nullptr;
                const double* zs2 = zs ? zs + (2LL * k + 1) * FR : nullptr;
                const double* zvk = zv ? zv + (1LL + k) * FP : nullptr;
                if (mc_s_update(c, 1, s, zs1, zss, slo, shi, ch, SUB_S + 2 * k, iteration, st)) return -1;
                if (mc_vs(c, 1, s, vv, zvk, zvs, slo, shi, ch, k, iteration, st)) return -1;
                if (mc_s_update(c, 1, s, zs2, zss, slo, shi, ch, SUB_S + 2 * k + 1, iteration, st)) return -1;
            }
        } else {
            // replay normals per chain: zv [B][n_gibbs][F][Npix], zs [B][n_gibbs][F][NR]
            const long long zvs = (long long)c->n_gibbs * FP, zss = (long long)c->n_gibbs * FR;
            for (int k = 0; k < c->n_gibbs; ++k) {
                if (mc_vs(c, 0, s, vv, zv ? zv + k * FP : nullptr, zvs, slo, shi, ch, k, iteration, st)) return -1;
                if (mc_s_update(c, 0, s, zs ? zs + k * FR : nullptr, zss, slo, shi, ch, SUB_S + 2 * k, iteration, st))
                    return -1;
            }
        }
        if (kind != GS_MCR_AUX_MALA) {
            // the auxiliary-variable samplers always accept (CenteredGibbs.py:729,825)
            if (accept) {
                hipLaunchKernelGGL(k_set_one, dim3(1), dim3(64), 0, st, B, accept);
                GS_LAUNCH_CHECK("k_set_one");
            }
            return 0;
        }
    }
    // MALA (CenteredGibbs.py:560-603): sigma from the full-sky kappa of noise_pol[0];
    // replay zm [B][F][NR], um [B]
    const double km = (double)c->npix / (4.0 * PI * c->noise_pol0);
    const double kapm[3] = {km, km, km};
    if (mc_params(c, B, dl, kapm, c->params_mala, st)) return -1;
    // the two gradients through the fused operator (no maps); the log densities'
    // data terms sum_pix N^-1 pix^2 from the operator's output (k_mc_sums)
    if (mc_gradient_r(c, dl, s, c->grad0, c->r, st)) return -1;
    const uint32_t call = 0;
    hipLaunchKernelGGL(k_mc_propose, dim3(nblocks(c->nlm, 256), B), dim3(256), 0, st, c->L, c->F, c->params_mala, s,
                       c->grad0, c->tau, zm, slo, shi, ch, (uint32_t)(SUB_MALA + call), iteration, c->snew);
    GS_LAUNCH_CHECK("k_mc_propose");
    if (mc_gradient_r(c, dl, c->snew, c->grad1, c->r1, st)) return -1;
    hipLaunchKernelGGL(k_mc_sums, dim3(c->nblk, B), dim3(RED_BLOCK), 0, st, c->L, c->F, c->npix, dl, c->params_mala,
                       c->tau, s, c->snew, c->grad0, c->grad1, c->g2, c->ninv, nullptr, nullptr, c->partial, c->r,
                       c->r1, c->bl, 1.0 / c->w);
    GS_LAUNCH_CHECK("k_mc_sums");
    hipLaunchKernelGGL(k_mc_accept, dim3(1, B), dim3(256), 0, st, c->nblk, c->partial, FR, um, slo, shi, ch, call,
                       iteration, c->accd, accept, log_ratio ? log_ratio : c->lr);
    GS_LAUNCH_CHECK("k_mc_accept");
    hipLaunchKernelGGL(k_select_copy, dim3(nblocks(FR, 256), B), dim3(256), 0, st, FR, c->accd, c->snew, s);
    GS_LAUNCH_CHECK("k_select_copy");
    return 0;
}

}  // extern "C"
