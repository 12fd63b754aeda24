// gs_kernels.hip -- MI355X (gfx950) kernels and C-ABI of the Gibbs hot path.
//
// Data layout in HBM (DESIGN.md "Layout"):
//   d_alm   [F][NR]                 NR = (L+1)^2, real m-major (utils.py:49-76)
//   s       [nchains][F][NR]
//   params  [nchains][L+1][GS_NPARAM]   per-l CR operator (M, Lchol)
//   stats   [nchains][nstat][L+1]       per-l sufficient statistics
//   dl      [nchains][nspec][maxbins]   binned D_l
//
// The CR sweep is tiled over the (l, m) triangle: one wave owns 64
// consecutive l (lanes) and a range of m rows, so each lane keeps its l's
// operator in registers and accumulates its l's statistics without atomics;
// per-(task, l) partial sums are reduced in a fixed order by k_stats_finish
// (bitwise reproducible).  Row m of a tile is one contiguous 16-B-per-lane
// segment of every field, so every load/store wave-instruction is coalesced.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include <string>
#include <vector>
#include <cstring>
#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>

#include "gibbs_capi.h"
#include "gs_rng.h"
#include "gs_common.h"
#include "gs_block.h"

using namespace gs;

namespace {

using gs_detail::set_error;

constexpr int WAVE = 64;
constexpr int NP = GS_NPARAM;
constexpr double PI = 3.14159265358979323846;

inline int nstat_of(int F) { return F == 1 ? GS_NSTAT_1 : (F == 2 ? GS_NSTAT_2 : GS_NSTAT_3); }
inline int nspec_of(int F) { return F == 1 ? 1 : (F == 2 ? 2 : 4); }

}  // namespace

struct gs_plan {
    int device = 0;
    int L = 0, nside = 0, Npix = 0, F = 0, nchains = 0, chain0 = 0, quirks = 0, n_iter_mh = 1;
    int nspec = 0, nstat = 0, maxbins = 0;
    double kappa[3] = {0, 0, 0};
    int nbins[4] = {0, 0, 0, 0};
    int nblocks[4] = {0, 0, 0, 0};
    int acc_off[4] = {0, 0, 0, 0};   // offset of each spectrum's accept flags
    int nacc = 0;                    // accept flags per chain
    int mh_order[4] = {0, 1, 2, 3};
    bool has_mh = false;
    // the CR operator computed per lane inside the sweep (no block-parameter
    // launch) only for few chains: there a step is launch-bound; with many
    // chains the per-workgroup recomputation costs more than the table
    // (measured: 32 TEB chains at L 1024, sweep 271 -> 287 us)
    bool inkernel_params = false;
    // the latency form of the sweep (all loads first) may be used for short tasks;
    // GS_SWEEP_THROUGHPUT at plan creation forces the throughput form (A/B timing)
    bool sweep_latency = true;
    // MH phases: spectra whose blocks are mutually independent run in one launch
    int nphase = 0;
    int phase_n[4] = {0, 0, 0, 0};
    int phase_off[4] = {0, 0, 0, 0};
    int2* phase_tab = nullptr;       // (spectrum, block) pairs, phase-major
    int4* phase_rng = nullptr;       // per phase entry: (lo bin, hi bin, l0, l1); wide blocks first
    int phase_nwide[4] = {0, 0, 0, 0};
    // the MH split over two workgroups per chain (F >= 2; GS_MH_SPLIT=0|1, default 1):
    // BB shares no likelihood term with T / E, so its blocks are decided by a
    // workgroup of their own beside the T / E phases' one; tables of the split form
    bool mh_split = false;
    int sph_n[2] = {0, 0};                   // phases per workgroup kind
    int sph_sp[2][4][2], sph_off[2][4], sph_cnt[2][4], sph_nwide[2][4], sph_own[2] = {0, 0};
    int2* phase_tab_s = nullptr;
    int4* phase_rng_s = nullptr;
    int ntab_s = 0;
    int mh_lmin = 0;
    int phase_sp[4][2] = {{-1, -1}, {-1, -1}, {-1, -1}, {-1, -1}};
    int* ell2blk = nullptr;          // [nspec][L+1] MH block of each l (-1: none)
    double* gbuf = nullptr;          // [nchains][2][L+1] per-l likelihood differences
    // device constants
    double* bl = nullptr;            // [L+1]
    int* ell2bin = nullptr;          // [nspec][L+1]
    int* bins = nullptr;             // [nspec][maxbins+1]
    int* blocks = nullptr;           // [nspec][maxbins+1] (clipped edges)
    double* prop_sd = nullptr;       // [nspec][maxbins]
    int* meta = nullptr;             // [16]: nbins[4], nblocks[4], acc_off[4], mh_order[4]
    int2* tasks = nullptr;           // [npair] (tile group, row chunk) of the CR sweep
    int npair = 0, ntile = 0, nchunk = 0, rows_per_task = 64;
    int sweep_tw = 4, nchunkg = 0;   // tiles per sweep workgroup, chunks per tile
    int ntask = 0;                   // valid (tile, chunk) waves per chain
    // workspace
    double* partials = nullptr;      // [nchains][ntile][nchunkg][nstat][64]
    double* params = nullptr;        // [nchains][L+1][NP]
    double* stats = nullptr;         // [nchains][nstat][L+1]
    double* prop = nullptr;          // [nchains][nspec][maxbins]
    double* logr = nullptr;          // [nchains][nspec][maxbins]
    double* dl_tmp = nullptr;        // [nchains][nspec][maxbins]
    double* u_nat = nullptr;         // [nchains][nacc] native MH accept uniforms drawn by the prologue
    bool u_nat_ready = false;
    // device iteration counter (hipGraph replay of whole steps)
    uint32_t* iter_dev = nullptr;
    // few-chain centered steps: the C_l draw's random variates (Gamma / normal)
    // depend on the bins' degrees of freedom and the counters only, so extra
    // workgroups of the latency-form sweep draw them while the sweep runs, and
    // the draw after the statistics does the algebra alone.  (A side-stream
    // kernel as a parallel graph branch was measured first: 35.5 against 18.3
    // us per configs[1] step -- the branch's cross-queue synchronisation.)
    bool cls_pre = false;
    bool cls_pre_many = false;       // the same for many chains: front workgroups of the throughput sweep
    double* cls_var = nullptr;       // [nchains][nspec][maxbins][3]
    // many-chain NC steps: the MH proposals and native accept uniforms depend
    // only on the current D_l and the counters, so they are drawn by extra
    // workgroups at the front of the CR sweep's launch (or, when the sweep
    // cannot take them -- replayed normals -- of the statistics finish) instead
    // of in the prologue, which keeps the block parameters alone
    bool pro_pending = false;        // a prologue deferred its draws to the sweep / finish
    // the proposal launch of this step also wrote a snapshot of the chains'
    // D_l into dl_tmp: the split MH reads its start state from there (both
    // workgroups of a chain see the pre-MH D_l whatever their order)
    bool snap_ok = false;
    const double* pro_dl = nullptr;
    uint32_t pro_slo = 0, pro_shi = 0, pro_it = 0;
    bool iter_dev_on = false;
    const uint32_t* itp() const { return iter_dev_on ? iter_dev : nullptr; }
    // graph-captured steps (gs_graph_step): this step's offset from the device
    // base, and how far its last launch advances the base (0: not at all)
    uint32_t graph_off = 0, graph_adv = 1;
    IterArg ita(uint32_t host_it) const { return IterArg{iter_dev_on ? graph_off : host_it, itp()}; }
    uint32_t* adv_counter() const { return iter_dev_on && graph_adv ? iter_dev : nullptr; }
    // dominant-kernel timing
    bool timing = false;
    std::vector<hipEvent_t> ev;
    size_t ev_used = 0;
};

// ============================================================================
// stand-alone layout kernels
// ============================================================================
__device__ __forceinline__ void complex_index_to_lm(int L, long long i, int& ell, int& m) {
    // row m starts at S(m) = m(2L+3-m)/2 (ell = m)
    const double b = 2.0 * L + 3.0;
    int mm = (int)floor((b - sqrt(fmax(b * b - 8.0 * (double)i, 0.0))) * 0.5);
    mm = max(0, min(mm, L));
    while (mm < L && (long long)(mm + 1) * (2 * L + 2 - mm) / 2 <= i) ++mm;
    while (mm > 0 && (long long)mm * (2 * L + 3 - mm) / 2 > i) --mm;
    m = mm;
    ell = (int)(i - (long long)mm * (2 * L + 3 - mm) / 2) + mm;
}

__global__ void k_var_expand(int L, int n, const double* __restrict__ dl, double* __restrict__ var) {
    const long long nc = (long long)(L + 1) * (L + 2) / 2;
    const long long nr = (long long)(L + 1) * (L + 1);
    for (long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x; g < nc * n; g += (long long)gridDim.x * blockDim.x) {
        const int k = (int)(g / nc);
        const long long i = g % nc;
        int ell, m;
        complex_index_to_lm(L, i, ell, m);
        const double v = var_from_dl(dl[(long long)k * (L + 1) + ell], ell);
        double* o = var + k * nr;
        if (m == 0) o[ell] = v;
        else { const long long r = 2 * i - (L + 1); o[r] = v; o[r + 1] = v; }
    }
}

__global__ void k_real_to_complex(int L, int n, const double* __restrict__ re, double* __restrict__ cx) {
    const long long nc = (long long)(L + 1) * (L + 2) / 2;
    const long long nr = (long long)(L + 1) * (L + 1);
    const double isq2 = 1.0 / sqrt(2.0);
    for (long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x; g < nc * n; g += (long long)gridDim.x * blockDim.x) {
        const int k = (int)(g / nc);
        const long long i = g % nc;
        const double* a = re + k * nr;
        double* o = cx + 2 * (k * nc + i);
        if (i <= L) { o[0] = a[i]; o[1] = 0.0; }
        else { const long long r = 2 * i - (L + 1); o[0] = a[r] / sqrt(2.0); o[1] = a[r + 1] / sqrt(2.0); }
        (void)isq2;
    }
}

__global__ void k_complex_to_real(int L, int n, const double* __restrict__ cx, double* __restrict__ re) {
    const long long nc = (long long)(L + 1) * (L + 2) / 2;
    const long long nr = (long long)(L + 1) * (L + 1);
    const double sq2 = sqrt(2.0);
    for (long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x; g < nc * n; g += (long long)gridDim.x * blockDim.x) {
        const int k = (int)(g / nc);
        const long long i = g % nc;
        const double* c = cx + 2 * (k * nc + i);
        double* o = re + k * nr;
        if (i <= L) o[i] = c[0];
        else { const long long r = 2 * i - (L + 1); o[r] = c[0] * sq2; o[r + 1] = c[1] * sq2; }
    }
}

__global__ void k_remove_md(int L, int n, double* __restrict__ alm) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    double* a = alm + (long long)k * (L + 1) * (L + 1);
    a[0] = 0.0; a[1] = 0.0; a[L + 1] = 0.0; a[L + 2] = 0.0;
}

// generic alm2cl: one wave per (array, 64-l tile), lanes = l, loop over m
__global__ void k_alm2cl(int L, int n, const double* __restrict__ x, const double* __restrict__ y, double* __restrict__ cl) {
    const int ntile = (L + WAVE) / WAVE;
    const int w = blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE;
    const int lane = threadIdx.x & (WAVE - 1);
    if (w >= n * ntile) return;
    const int k = w / ntile, t = w % ntile;
    const int ell = t * WAVE + lane;
    if (ell > L) return;
    const long long nr = (long long)(L + 1) * (L + 1);
    const double* a = x + k * nr;
    const double* b = y + k * nr;
    double s = a[ell] * b[ell];
    for (int m = 1; m <= ell; ++m) {
        const long long i = (long long)m * (2 * L + 1 - m) / 2 + ell;
        const long long r = 2 * i - (L + 1);
        s += a[r] * b[r] + a[r + 1] * b[r + 1];
    }
    cl[(long long)k * (L + 1) + ell] = s / (2.0 * ell + 1.0);
}

__global__ void k_unfold(int n, const double* __restrict__ binned, const int* __restrict__ bins, int nbins,
                         double* __restrict__ out) {
    const int k = blockIdx.y;
    for (int b = blockIdx.x * blockDim.x + threadIdx.x; b < nbins; b += gridDim.x * blockDim.x) {
        const double v = binned[(long long)k * nbins + b];
        const int lo = bins[b], hi = bins[b + 1];
        const int base = bins[0];
        for (int l = lo; l < hi; ++l) out[(long long)k * (bins[nbins] - base) + (l - base)] = v;
    }
}

template <int F, int MODE>
__global__ __launch_bounds__(256) void k_block_params(int L, int nchains, int maxbins, const double* __restrict__ dl,
                                                      const int* __restrict__ ell2bin, const double* __restrict__ bl,
                                                      double k0, double k1, double k2, double* __restrict__ params) {
    block_params_at<F, MODE>(blockIdx.x * blockDim.x + threadIdx.x, L, nchains, maxbins, dl, ell2bin, bl, k0, k1, k2,
                             params);
}

// ============================================================================
// fused CR draw + per-l statistics (the dominant, HBM-bound kernel)
// ============================================================================
template <int F>
struct SweepAcc {
    static constexpr int NS = F == 1 ? GS_NSTAT_1 : (F == 2 ? GS_NSTAT_2 : GS_NSTAT_3);
    double v[NS];
};

// one (l, m) entry of every field: NV = 1 (m = 0, one real slot) or 2 (re, im)
template <int F, int NV>
__device__ __forceinline__ void load_d(const double* __restrict__ d, long long NR, long long r, double (&dv)[F][2]) {
#pragma unroll
    for (int f = 0; f < F; ++f)
#pragma unroll
        for (int c = 0; c < NV; ++c) dv[f][c] = d[f * NR + r + c];
}

// the same entry's loads with the field bases wave-uniform (SGPRs) and the
// row offset a 32-bit byte count (F (L+1)^2 doubles per chain < 4 GiB): the
// scalar-base + 32-bit vector-offset load form, no 64-bit address arithmetic
template <int F>
__device__ __forceinline__ void load_d2_off(const char* const (&db)[F], uint32_t rb, double (&dv)[F][2]) {
#pragma unroll
    for (int f = 0; f < F; ++f) {
        const double2 v = *reinterpret_cast<const double2*>(db[f] + rb);
        dv[f][0] = v.x;
        dv[f][1] = v.y;
    }
}

// ZM: 0 native RNG draw, 1 replay (z from memory), 2 statistics of a given s
template <int F, int ZM, bool STORE, int NV>
__device__ __forceinline__ void sweep_entry(const double (&dv)[F][2], const double* __restrict__ zc,
                                            double* __restrict__ sc, long long NR, long long r, uint32_t i,
                                            uint32_t tag, uint32_t iter, Key key, const double (&pm)[NP],
                                            double (&acc)[SweepAcc<F>::NS], const double* __restrict__ tab) {
    double zv[F][2], sv[F][NV];
    if constexpr (ZM == 2) {
#pragma unroll
        for (int f = 0; f < F; ++f)
#pragma unroll
            for (int c = 0; c < NV; ++c) sv[f][c] = sc[f * NR + r + c];
    } else {
#pragma unroll
    for (int f = 0; f < F; ++f) {
        if constexpr (ZM == 1) {
#pragma unroll
            for (int c = 0; c < NV; ++c) zv[f][c] = zc[f * NR + r + c];
        } else {
            box_muller_tab(philox<true>(i, (uint32_t)f, tag, iter, key), tab, zv[f][0], zv[f][1]);
        }
    }
#pragma unroll
    for (int c = 0; c < NV; ++c) {
        if constexpr (F == 3) {
            sv[0][c] = pm[0] * dv[0][c] + pm[1] * dv[1][c] + pm[5] * zv[0][c];
            sv[1][c] = pm[2] * dv[0][c] + pm[3] * dv[1][c] + pm[6] * zv[0][c] + pm[7] * zv[1][c];
            sv[2][c] = pm[4] * dv[2][c] + pm[8] * zv[2][c];
        } else {
#pragma unroll
            for (int f = 0; f < F; ++f) sv[f][c] = pm[f] * dv[f][c] + zv[f][c] * pm[F + f];
        }
    }
    }
    if constexpr (STORE) {
        // streaming output: non-temporal stores keep the data tiles in L2
#pragma unroll
        for (int f = 0; f < F; ++f)
#pragma unroll
            for (int c = 0; c < NV; ++c) {
                __builtin_nontemporal_store(sv[f][c], &sc[f * NR + r + c]);
            }
    }
#pragma unroll
    for (int c = 0; c < NV; ++c) {
        if constexpr (F == 3) {
            acc[0] += sv[0][c] * sv[0][c];
            acc[1] += sv[1][c] * sv[1][c];
            acc[2] += sv[2][c] * sv[2][c];
            acc[3] += sv[0][c] * sv[1][c];
            acc[4] += dv[0][c] * sv[0][c];
            acc[5] += dv[1][c] * sv[0][c];
            acc[6] += dv[1][c] * sv[1][c];
            acc[7] += dv[2][c] * sv[2][c];
        } else {
#pragma unroll
            for (int f = 0; f < F; ++f) {
                acc[f] += sv[f][c] * sv[f][c];
                acc[F + f] += dv[f][c] * sv[f][c];
            }
        }
    }
}

// where the sweep's per-l operator comes from: mode -1 the params table;
// GS_MODE_CENTERED / GS_MODE_NONCENTERED computed per lane from the chain's
// binned D_l (saves the block-parameter launch of a step)
struct SweepOp {
    int mode;
    int maxbins;
    const double* dl;
    const int* ell2bin;
    const double* bl;
    double k0, k1, k2;
};

// Tiling of the (l, m) triangle: 64-wide l tiles, descending from l = L
// (tile t holds l in [L-64t-63, L-64t]), rows m in chunks of TM.  A workgroup
// = 4 waves = 4 adjacent tiles (256 consecutive l) x one chunk (tw = 4), so
// every row of the workgroup is one contiguous 4 KiB run per field and chain;
// consecutive workgroups are consecutive chains of the same task and share the
// data reads in L2.  Each wave writes its 64 l's statistic partials of its
// chunk; k_stats_finish sums them in a fixed order.
// the operator of this lane's l: from the chain's D_l (op.mode >= 0) or the table
template <int F>
__device__ __forceinline__ void sweep_operator(bool ok, int chain, int ell, int L, const double* __restrict__ params,
                                               const SweepOp& op, double (&pm)[NP]) {
    if (ok && op.mode >= 0) {
        if (op.mode == GS_MODE_CENTERED)
            block_params_compute<F, GS_MODE_CENTERED>(chain, ell, L, op.maxbins, op.dl, op.ell2bin, op.bl, op.k0,
                                                      op.k1, op.k2, pm);
        else
            block_params_compute<F, GS_MODE_NONCENTERED>(chain, ell, L, op.maxbins, op.dl, op.ell2bin, op.bl, op.k0,
                                                         op.k1, op.k2, pm);
    } else if (ok) {
        const double* pp = params + ((long long)chain * (L + 1) + ell) * NP;
#pragma unroll
        for (int q = 0; q < NP; ++q) pm[q] = pp[q];
    } else {
#pragma unroll
        for (int q = 0; q < NP; ++q) pm[q] = 0.0;
    }
}

// The workgroup's statistic partials.  tw = 4 (4 tiles x 1 chunk): one store
// per wave.  tw = 2 / 1 (2 tiles x 2 chunks, 1 tile x 4 chunks): the cw = 4 / tw
// chunk-waves of a tile add their sums in LDS in chunk order ((c0 + c1) + c2) +
// c3, and the tile's first chunk-wave stores one partial per chunk group (every
// wave of the workgroup reaches the barrier; an inactive wave adds zeros).
template <int NS>
__device__ __forceinline__ void sweep_partials_store(const double (&acc)[NS], int tw, int w, int lane, bool store_ok,
                                                     double* __restrict__ po, double* red) {
    if (tw == 4) {
        if (store_ok)
#pragma unroll
            for (int q = 0; q < NS; ++q) po[q * WAVE + lane] = acc[q];
        return;
    }
    const int cw = 4 / tw, ci = w / tw, ti = w % tw;
    if (ci > 0)
#pragma unroll
        for (int q = 0; q < NS; ++q) red[(((ci - 1) * tw + ti) * NS + q) * WAVE + lane] = acc[q];
    __syncthreads();
    if (ci == 0 && store_ok) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            double v = acc[q];
            for (int k = 1; k < cw; ++k) v += red[(((k - 1) * tw + ti) * NS + q) * WAVE + lane];
            po[q * WAVE + lane] = v;
        }
    }
}

// Latency form of the sweep for few chains (PRE = the most rows a task holds):
// there the launch has ~one wave per SIMD and each wave's time is its chain of
// memory latencies, so every global load of the wave -- its PRE data rows, the
// Box-Muller tables, the operator's D_l -- is issued before any of them is
// used (one memory round trip instead of one per row plus two for the
// prologue).  Same arithmetic in the same order as the throughput form below.
template <int F, bool STORE, int PRE>
__device__ __forceinline__ void cr_sweep_latency(int L, int nchains, int ntile, int nchunkg, int tm, int tw,
                                                 const int2* __restrict__ tasks, const double* __restrict__ d,
                                                 double* __restrict__ s,
                                                 double* __restrict__ partials, uint32_t seed_lo, uint32_t seed_hi,
                                                 uint32_t iter, uint32_t substep, int chain0, const SweepOp& op,
                                                 double* tab, double* red, int bid = -1, int nwg = 0) {
    constexpr int NS = SweepAcc<F>::NS;
    if (bid < 0) { bid = blockIdx.x; nwg = gridDim.x; }
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int pair = wg / nchains;
    const int chain = wg % nchains;
    const int lane = threadIdx.x & 63;
    const int2 gc = tasks[pair];
    if (gc.x < 0) return;                       // padding pair (whole workgroup, before any barrier)
    const int w = threadIdx.x >> 6, cw = 4 / tw;
    const int t = tw * gc.x + w % tw;
    const int lhi = L - WAVE * t;
    const int m0 = (cw * gc.y + w / tw) * tm;
    const int m1 = min(m0 + tm, lhi + 1);
    const bool active = t < ntile && m0 < m1;
    GS_ASSERT(m1 - m0 <= PRE || !active);
    const int ell_lo = lhi - 63;
    const int ell = ell_lo + lane;
    const bool lane_ok = ell >= 0;
    const long long NR = (long long)(L + 1) * (L + 1);
    // 1. the data rows: lanes outside the triangle (l < m, l < 0) read the
    //    row's diagonal entry instead (in bounds, never used); row m = 0 is one
    //    slot per l (its second load, slot l + 1 <= L + 1, is never used).  No
    //    load sits behind a condition, so they all issue back to back.
    // 0. the l -> bin indices of the operator's D_l (first: the D_l loads that
    //    depend on them then wait for these alone, not for the rows below)
    constexpr int NSP = F == 1 ? 1 : (F == 2 ? 2 : 4);
    const int lc = max(ell, 0);
    int bidx[NSP];
#pragma unroll
    for (int q = 0; q < NSP; ++q) bidx[q] = op.ell2bin[q * (L + 1) + lc];
    double dq[PRE][F][2];
    {
        const int mlast = max(m1 - 1, m0);
#pragma unroll
        for (int k = 0; k < PRE; ++k) {
            const int mk = min(m0 + k, mlast);
            const int le = min(max(ell, mk), L);
            const long long i = (long long)mk * (2 * L + 1 - mk) / 2 + le;
            const long long r = mk == 0 ? (long long)le : 2 * i - (L + 1);
            load_d<F, 2>(d, NR, r, dq[k]);
        }
    }
    // 2. the Box-Muller tables into registers (staged in LDS below), the beam
    double tv[(BM_TAB_DOUBLES + 255) / 256];
#pragma unroll
    for (int k = 0; k < (BM_TAB_DOUBLES + 255) / 256; ++k) {
        const int j = threadIdx.x + 256 * k;
        tv[k] = j < BM_LOG_DOUBLES ? BM_LOG_TAB[j] : BM_TRIG_TAB[min(j - BM_LOG_DOUBLES, 511)];
    }
    const double bq = op.bl[lc];
    // 3. this l's D_l (the latency form always computes the operator in-kernel,
    //    op.mode >= 0; an unbinned l reads bin 0 and drops it)
    double dlq[NSP];
    {
        const double* dlc = op.dl + (long long)chain * NSP * op.maxbins;
#pragma unroll
        for (int q = 0; q < NSP; ++q) dlq[q] = dlc[q * op.maxbins + max(bidx[q], 0)];
#pragma unroll
        for (int q = 0; q < NSP; ++q) dlq[q] = bidx[q] < 0 ? 0.0 : dlq[q];
    }
    // 4. the operator
    double pm[NP];
    if (op.mode == GS_MODE_CENTERED)
        block_params_from<F, GS_MODE_CENTERED>(lc, bq, dlq, op.k0, op.k1, op.k2, pm);
    else
        block_params_from<F, GS_MODE_NONCENTERED>(lc, bq, dlq, op.k0, op.k1, op.k2, pm);
#pragma unroll
    for (int k = 0; k < (BM_TAB_DOUBLES + 255) / 256; ++k) {
        const int j = threadIdx.x + 256 * k;
        if (j < BM_TAB_DOUBLES) tab[j] = tv[k];
    }
    __syncthreads();
    const Key key = chain_key(seed_lo, seed_hi, (uint32_t)(chain0 + chain));
    const uint32_t tag = TAG_CR | (substep << 8);
    double acc[NS];
#pragma unroll
    for (int q = 0; q < NS; ++q) acc[q] = 0.0;
    double* sc = s + (long long)chain * F * NR;
#pragma unroll
    for (int k = 0; k < PRE; ++k) {
        const int m = m0 + k;
        if (active && m < m1 && lane_ok && ell >= m) {
            if (m == 0) {
                sweep_entry<F, 0, STORE, 1>(dq[k], nullptr, sc, NR, ell, (uint32_t)ell, tag, iter, key, pm, acc, tab);
            } else {
                const long long i = (long long)m * (2 * L + 1 - m) / 2 + ell;
                sweep_entry<F, 0, STORE, 2>(dq[k], nullptr, sc, NR, 2 * i - (L + 1), (uint32_t)i, tag, iter, key, pm,
                                            acc, tab);
            }
        }
    }
    double* po = partials + (((long long)chain * ntile + t) * nchunkg + gc.y) * NS * WAVE;
    sweep_partials_store<NS>(acc, tw, w, lane, t < ntile && (cw * gc.y) * tm <= lhi, po, red);
}

// the C_l draw's variates computed by extra workgroups of the latency-form
// sweep (few-chain centered steps): n workgroups ahead of the sweep's, 256
// items (chain, spectrum, bin) each; the draw after the statistics reads them
struct ClsPre {
    int n = 0;                       // extra workgroups (0: none)
    int nitem = 0;                   // nchains * nspec * maxbins
    int nspec = 0, maxbins = 0;
    const int* bins = nullptr;
    const int* nbins = nullptr;
    double* out = nullptr;           // [nchains][nspec][maxbins][3]
};
template <int F>
__device__ void cls_variates_item(const ClsPre& cp, int item, uint32_t seed_lo, uint32_t seed_hi, uint32_t iter,
                                  int chain0);

// many-chain NC steps: the MH proposals and native accept
// uniforms drawn by n extra workgroups at the FRONT of the throughput-form
// sweep's grid (they start first and their latency chains -- inverse normal
// CDFs, log-CDFs -- end long before the sweep does); n is a multiple of 8, so
// the sweep workgroups' XCD-aware remap keeps its placement
struct ProPre {
    int n = 0;                       // extra workgroups (0: none)
    int nbp = 0, nbu = 0;            // of which proposal / uniform workgroups
    int nspec = 0, nacc = 0, n_iter_mh = 0, maxbins = 0;
    const int* nbins = nullptr;      // plan meta (nbins per spectrum, blocks, accept offsets)
    const double* prop_sd = nullptr;
    const double* dl = nullptr;
    double* prop = nullptr;
    double* logr = nullptr;
    double* u_out = nullptr;
    double* snap = nullptr;          // nullable: the proposals' start D_l copied here (split MH)
    // many-chain centered / ASIS steps: the C_l draw's random variates (they need
    // only the bins' degrees of freedom and the counters) by nbv workgroups after
    // the proposal / uniform ones, as the latency form's ClsPre does for few chains
    int nbv = 0;
    ClsPre cp{};
};
template <int F>
__device__ void pro_pre_item(const ProPre& pp, int bx, int nchains, uint32_t seed_lo, uint32_t seed_hi, IterArg itarg,
                             int chain0);

// diagnostic timeline of the sweep's workgroups (-DGS_SWEEP_WGTIME, build
// variant "wgtime"; tools/sweep_timeline.py): per physical workgroup its first
// and last s_memrealtime, HW_ID and XCC_ID
#if defined(GS_SWEEP_WGTIME)
constexpr int SW_TL_MAX = 16384;
__device__ unsigned long long g_sw_tl[4 * SW_TL_MAX];
#endif

// one (tile group, row chunk) task of one chain: logical workgroup wg
template <int F, int ZM, bool STORE>
__device__ __forceinline__ void cr_sweep_task(int wg, int L, int nchains, int ntile, int nchunkg, int tm, int tw,
                                              const int2* __restrict__ tasks, const double* __restrict__ d,
                                              const double* __restrict__ params, const double* __restrict__ z,
                                              double* __restrict__ s, double* __restrict__ partials,
                                              uint32_t seed_lo, uint32_t seed_hi, uint32_t iter, uint32_t substep,
                                              int chain0, const SweepOp& op, const double* __restrict__ tab,
                                              double* red) {
    constexpr int NS = SweepAcc<F>::NS;
    const int pair = wg / nchains;
    const int chain = wg % nchains;
    const int lane = threadIdx.x & 63;
    const int2 gc = tasks[pair];
    if (gc.x < 0) return;                       // padding pair (whole workgroup)
    const int w = threadIdx.x >> 6, cw = 4 / tw;
    const int t = tw * gc.x + w % tw;
    const bool tile_ok = t < ntile;
    const int lhi = L - WAVE * t;
    const int m0 = (cw * gc.y + w / tw) * tm;
    const int m1 = min(m0 + tm, lhi + 1);
    const bool active = tile_ok && m0 < m1;
    GS_ASSERT(gc.y < nchunkg && gc.x * tw < ntile);
    const int ell_lo = lhi - 63;
    const int ell = ell_lo + lane;
    const bool lane_ok = ell >= 0;
    const long long NR = (long long)(L + 1) * (L + 1);
    const Key key = chain_key(seed_lo, seed_hi, (uint32_t)(chain0 + chain));
    const uint32_t tag = TAG_CR | (substep << 8);

    double pm[NP];
    sweep_operator<F>(ZM != 2 && lane_ok && active, chain, ell, L, params, op, pm);
    double acc[NS];
#pragma unroll
    for (int q = 0; q < NS; ++q) acc[q] = 0.0;

    const double* zc = ZM == 1 ? z + (long long)chain * F * NR : nullptr;
    double* sc = s + (long long)chain * F * NR;

    int m = active ? m0 : m1;
    double dv[F][2];
    if (active && m == 0) {
        if (lane_ok) {
            load_d<F, 1>(d, NR, ell, dv);
            sweep_entry<F, ZM, STORE, 1>(dv, zc, sc, NR, ell, (uint32_t)ell, tag, iter, key, pm, acc, tab);
        }
        m = 1;
    }
    // row m starts at complex index S(m) = m(2L+3-m)/2 (l = m); slot r = 2i-(L+1)
    long long i = (long long)m * (2 * L + 1 - m) / 2 + ell;
    if (m1 - 1 <= ell_lo && ell_lo >= 0) {
        // off-diagonal block: every lane active on every row
        if constexpr (ZM == 0 && !STORE) {
            // the headline form (native draws, no map written): 32-bit row offsets
            uint32_t i32 = (uint32_t)i;
            const char* db[F];
#pragma unroll
            for (int f = 0; f < F; ++f)
                db[f] = reinterpret_cast<const char*>(d + (size_t)f * (size_t)NR);   // wave-uniform bases
            GS_ASSERT(NR * 8 < (1ll << 32));
            for (; m < m1; ++m) {
                const uint32_t r = 2u * i32 - (uint32_t)(L + 1);
                load_d2_off<F>(db, r * 8u, dv);
                sweep_entry<F, ZM, STORE, 2>(dv, zc, sc, NR, (long long)r, i32, tag, iter, key, pm, acc, tab);
                GS_ASSERT((long long)r + 1 < NR && (long long)r > L);
                i32 += (uint32_t)(L - m);
            }
        } else {
        for (; m < m1; ++m) {
            load_d<F, 2>(d, NR, 2 * i - (L + 1), dv);
            sweep_entry<F, ZM, STORE, 2>(dv, zc, sc, NR, 2 * i - (L + 1), (uint32_t)i, tag, iter, key, pm, acc, tab);
            GS_ASSERT(2 * i - (L + 1) + 1 < NR && 2 * i - (L + 1) > L);
            i += L - m;
        }
        }
    } else if constexpr (ZM == 0 && !STORE) {
        // diagonal block of the headline form (lanes l < m idle): the same
        // 32-bit row offsets
        const char* db[F];
#pragma unroll
        for (int f = 0; f < F; ++f) db[f] = reinterpret_cast<const char*>(d + (size_t)f * (size_t)NR);
        uint32_t i32 = (uint32_t)i;
        for (; m < m1; ++m) {
            if (lane_ok && ell >= m) {
                const uint32_t r = 2u * i32 - (uint32_t)(L + 1);
                load_d2_off<F>(db, r * 8u, dv);
                sweep_entry<F, ZM, STORE, 2>(dv, zc, sc, NR, (long long)r, i32, tag, iter, key, pm, acc, tab);
            }
            i32 += (uint32_t)(L - m);
        }
    } else {
        for (; m < m1; ++m) {
            if (lane_ok && ell >= m) {
                load_d<F, 2>(d, NR, 2 * i - (L + 1), dv);
                sweep_entry<F, ZM, STORE, 2>(dv, zc, sc, NR, 2 * i - (L + 1), (uint32_t)i, tag, iter, key, pm,
                                                 acc, tab);
            }
            i += L - m;
        }
    }
    double* po = partials + (((long long)chain * ntile + t) * nchunkg + gc.y) * NS * WAVE;
    sweep_partials_store<NS>(acc, tw, w, lane, tile_ok && (cw * gc.y) * tm <= lhi, po, red);
}

// nlog: logical workgroups (chains x task pairs), one per sweep workgroup.
// r06 measured and not kept: fewer, persistent workgroups (4 per CU) taking the
// tasks in strides or from a global / per-XCD work queue -- occupancy 4.0 instead
// of ~3.1-3.3, but 200-289 against 191-195 us per configs[2] step: the loop-form
// kernel allocates more registers (and spills) and a global queue loses the
// XCD-local data reads (tools/sweep_timeline.py, tools/lib_ab.py)
#ifndef GS_SWEEP_MINW
#define GS_SWEEP_MINW 1
#endif
template <int F, int ZM, bool STORE, int PRE = 0>
__global__ __launch_bounds__(256, GS_SWEEP_MINW) void k_cr_sweep(int L, int nchains, int ntile, int nchunkg, int tm, int tw,
                                                  const int2* __restrict__ tasks, const double* __restrict__ d,
                                                  const double* __restrict__ params, const double* __restrict__ z,
                                                  double* __restrict__ s, double* __restrict__ partials,
                                                  uint32_t seed_lo, uint32_t seed_hi, IterArg itarg, uint32_t substep,
                                                  int chain0, SweepOp op, ClsPre cp, ProPre pp, int nlog) {
    if constexpr (PRE == 0 && ZM == 0) {
        if ((int)blockIdx.x < pp.n) {
            pro_pre_item<F>(pp, (int)blockIdx.x, nchains, seed_lo, seed_hi, itarg, chain0);
            return;
        }
    }
    const uint32_t iter = itarg.get();
    constexpr int NS = SweepAcc<F>::NS;
    __shared__ __attribute__((aligned(16))) double tab[ZM == 0 ? BM_TAB_DOUBLES : 2];
    __shared__ double red[3 * NS * WAVE];           // chunk-wave sums of tw < 4 shapes
    if constexpr (PRE > 0) {
        static_assert(ZM == 0, "latency form: native draws only");
        // the variate workgroups sit at the END of the grid, so the sweep's
        // workgroups keep physical ids 0.. and their XCD-aware remap (b % 8 =
        // the XCD) stays exact for any cp.n
        const int nsw = (int)gridDim.x - cp.n;
        if ((int)blockIdx.x >= nsw) {
            cls_variates_item<F>(cp, ((int)blockIdx.x - nsw) * blockDim.x + threadIdx.x, seed_lo, seed_hi, iter,
                                 chain0);
            return;
        }
        cr_sweep_latency<F, STORE, PRE>(L, nchains, ntile, nchunkg, tm, tw, tasks, d, s, partials, seed_lo,
                                        seed_hi, iter, substep, chain0, op, tab, red, (int)blockIdx.x, nsw);
        return;
    }
    if constexpr (ZM == 0) {
        bm_stage_tables(tab);
        __syncthreads();
    }
    // XCD-aware remap (bijective): workgroups are dealt round-robin over the 8
    // XCDs, so physical id b runs on XCD b % 8; give each XCD a contiguous range
    // of logical ids so that all chains of one (tiles, rows) block share one
    // XCD's L2 for the data reads (speed only -- any placement is correct)
    const int bid = (int)blockIdx.x - pp.n;     // (pp.n % 8 == 0: the same XCD as blockIdx.x)
    const int xcd = bid & 7, q8 = nlog >> 3, r8 = nlog & 7;
    const int base = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
#if defined(GS_SWEEP_WGTIME)
    const unsigned long long tl0 = wall_clock64();
#endif
    cr_sweep_task<F, ZM, STORE>(base + (bid >> 3), L, nchains, ntile, nchunkg, tm, tw, tasks, d, params, z, s,
                                partials, seed_lo, seed_hi, iter, substep, chain0, op, tab, red);
#if defined(GS_SWEEP_WGTIME)
    __syncthreads();
    if (threadIdx.x == 0 && bid < SW_TL_MAX) {
        unsigned long long* o = g_sw_tl + 4 * (size_t)bid;
        o[0] = tl0;
        o[1] = wall_clock64();
        o[2] = __builtin_amdgcn_s_getreg((31 << 11) | 4);     // HW_REG_HW_ID
        o[3] = __builtin_amdgcn_s_getreg((31 << 11) | 20);    // HW_REG_XCC_ID
    }
#endif
}

// one wave's share of a (chain, statistic, tile) finish: the sum of chunks w,
// w + 4, ... of the tile's 64 l (lanes; coalesced rows of the partials)
template <int G>
__device__ __forceinline__ double stats_finish_sum(int L, int ntile, int nchunkg, int tm, int nstat,
                                                   const double* partials, int chain, int q, int t,
                                                   int w, int lane) {
    const int cmax = (L - WAVE * t) / tm;               // last chunk of tile t
    GS_ASSERT(cmax < nchunkg);
    const double* pp = partials + ((long long)chain * ntile + t) * nchunkg * nstat * WAVE + q * WAVE + lane;
    const long long cs = (long long)nstat * WAVE;
    // groups of G of this wave's chunks, every load of a group issued before
    // the sums (the last group's loads clamped to a valid chunk, its extra
    // values dropped): with few chains the finish is a chain of memory
    // latencies, one per group (G = 16; 32 measured slower, 4.7 -> 5.4 us at
    // configs[1]); with many it is bound by the partials' bytes (32 chains at
    // L 1024: 73.5 MB in 13.2-13.3 us, ~5.6 TB/s, for either form), and the
    // unclamped four-in-flight form reads nothing twice.  The sums keep the
    // chunk order in both forms.
    double acc = 0.0;
    if constexpr (G <= 4) {
        // bandwidth-bound form (many chains): four loads in flight, no clamped extras
        int c = w;
        for (; c + 12 <= cmax; c += 16) {
            double v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = *(pp + (c + 4 * j) * cs);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc += v[j];
        }
        for (; c <= cmax; c += 4) acc += *(pp + c * cs);
    } else {
        for (int c = w; c <= cmax; c += 4 * G) {
            double v[G];
#pragma unroll
            for (int j = 0; j < G; ++j) v[j] = *(pp + min(c + 4 * j, cmax) * cs);
#pragma unroll
            for (int j = 0; j < G; ++j)
                if (c + 4 * j <= cmax) acc += v[j];
        }
    }
    return acc;
}

// fixed-order reduction of the sweep partials: stats[chain][q][l].  One
// workgroup per (chain, statistic, tile): wave w sums chunks w, w + 4, ... of
// the tile's 64 l, then the four wave sums in wave order -- the same order for
// any batch size, so every chain's trajectory is bit-identical for any chain
// count or GPU count
template <int G>
__global__ __launch_bounds__(256) void k_stats_finish(int L, int nchains, int ntile, int nchunkg, int tm, int nstat,
                                                      const double* __restrict__ partials,
                                                      double* __restrict__ stats) {
    const int t = blockIdx.x % ntile;
    const int q = (blockIdx.x / ntile) % nstat;
    const int chain = blockIdx.x / (ntile * nstat);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int Lp1 = L + 1;
    GS_ASSERT(chain < nchains);
    const double acc = stats_finish_sum<G>(L, ntile, nchunkg, tm, nstat, partials, chain, q, t, w, lane);
    __shared__ double red[4][WAVE];
    red[w][lane] = acc;
    __syncthreads();
    if (w == 0) {
        const int ell = L - WAVE * t - 63 + lane;
        if (ell >= 0)
            stats[((long long)chain * nstat + q) * Lp1 + ell] = ((red[0][lane] + red[1][lane]) + red[2][lane]) +
                                                                 red[3][lane];
    }
}

// ============================================================================
// centered C_l draw (CenteredGibbs.py:54-93) + TEB inverse-Wishart
// ============================================================================
// grid: (nchains, nspec, bin chunks of blockDim), one bin per thread (the
// gamma draws are latency chains: one per thread, not a loop per thread).
// Optional epilogue of graph-captured centered steps (as MhEpi): the trace
// record of every bin and the device counter advance by the last workgroup.
// device iteration counter advance by the last workgroup of a launch (ticket
// in counter[1]).  Every workgroup read counter[0] at its start and has used
// the value before the barrier, so the last ticket may advance it; no data is
// handed between workgroups here, so no release / acquire fence is needed
// (an agent-scope __threadfence costs ~3.5 us per workgroup,
// MI355X_MICROARCH.md visibility table); the next launch sees the counter.
__device__ __forceinline__ void ticket_advance(uint32_t* counter, uint32_t nblk, uint32_t adv) {
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t t = __hip_atomic_fetch_add(&counter[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t == nblk - 1) {
            __hip_atomic_store(&counter[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(&counter[0], adv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// the random variates of bin b's draw, which need only the bin's degrees of
// freedom and the counters (not the statistics): the TEB block's two Gamma
// variates and the Bartlett normal, or the inverse-Gamma draw 1 / Gamma.
// Computed here (in the draw, or ahead of it by k_cls_variates on a side
// stream while the sweep runs) by the same code, so either way gives the same bits.
template <int F>
__device__ __forceinline__ void cls_variates(int sp, int b, int l0, int l1, Key key, uint32_t iter, double (&v)[3]) {
    v[0] = v[1] = v[2] = 0.0;
    if ((F == 3) && (sp != 2)) {
        if (b >= 2) {
            const double nu = (double)(l1 * l1 - l0 * l0) - 3.0;
            gamma_mt_pair(0.5 * nu, 0.5 * (nu - 1.0), key, b, 16, 17, iter, 0, v[0], v[1]);
            v[2] = normal1(key, b, 0, TAG_IW_N, iter);
        }
    } else {
        const double expo = (double)(l1 * l1 - l0 * l0) / 2.0;
        const double alpha = b == 0 ? 1.0 : expo - 1.0;
        v[0] = b < 2 ? 0.0 : 1.0 / gamma_mt(alpha, key, b, sp, iter, 0);
    }
}

template <int F>
__device__ __forceinline__ void cls_draw_body(int chain, int sp, int b, int L, int maxbins, const int* __restrict__ bins,
                                              const int* __restrict__ nbins_arr, const double* stats,
                                              const double* __restrict__ variates, uint32_t seed_lo, uint32_t seed_hi,
                                              uint32_t iter, int chain0, double* __restrict__ dl_out,
                                              double* __restrict__ trace, int cap, int nchains,
                                              const double* __restrict__ pre = nullptr) {
    constexpr int NSP = F == 1 ? 1 : (F == 2 ? 2 : 4);
    constexpr int NS = SweepAcc<F>::NS;
    const int Lp1 = L + 1;
    const int nb = nbins_arr[sp];
    // trace slot of this iteration: trace[(iter - 1) % cap][chain][nspec][maxbins]
    double* tr = trace ? trace + ((long long)((iter + (uint32_t)cap - 1u) % (uint32_t)cap) * nchains + chain) * NSP * maxbins
                       : nullptr;
    const int* be = bins + sp * (maxbins + 1);
    const double* st = stats + (long long)chain * NS * Lp1;
    double* out = dl_out + ((long long)chain * NSP + sp) * maxbins;
    const Key key = chain_key(seed_lo, seed_hi, (uint32_t)(chain0 + chain));
    // which stat row holds ss of this spectrum
    int ssrow = sp;                 // F=1: ssTT=0; F=2: ssEE=0, ssBB=1; F=3: ssTT, ssEE, ssBB, ssTE = 0..3
    const bool iw = (F == 3) && (sp != 2);
    if (iw) {
        if (sp != 0) return;        // the TT block draws TT, EE and TE together
        if (b >= maxbins) return;
        if (b >= nb) {
            if (tr) { tr[0 * maxbins + b] = dl_out[((long long)chain * NSP + 0) * maxbins + b];
                      tr[1 * maxbins + b] = dl_out[((long long)chain * NSP + 1) * maxbins + b];
                      tr[3 * maxbins + b] = dl_out[((long long)chain * NSP + 3) * maxbins + b]; }
            return;
        }
        {
            // the bin's statistics in groups of 8 l with every load issued before
            // the sums (clamped indices, no load behind a condition); the first
            // group is issued before the Gamma draws, which need only the bin's
            // degrees of freedom, nu = sum (2l + 1) - 3 = l1^2 - l0^2 - 3 (exact,
            // as the reference's running sum is), so the loads and the draws
            // overlap.  The sums keep the l order.
            const int l0 = be[b], l1 = be[b + 1];
            double va[8], vd[8], vc[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int l = max(min(l0 + j, l1 - 1), 0);
                va[j] = *(st + 0 * Lp1 + l); vd[j] = *(st + 1 * Lp1 + l);
                vc[j] = *(st + 3 * Lp1 + l);
            }
            double vr[3];
            if (pre) {
                const double* q = pre + (((long long)chain * NSP + sp) * maxbins + b) * 3;
                vr[0] = q[0]; vr[1] = q[1]; vr[2] = q[2];
            } else {
                cls_variates<F>(sp, b, l0, l1, key, iter, vr);
            }
            const double g1 = vr[0], g2 = vr[1], n = vr[2];
            double a = 0.0, dd = 0.0, c = 0.0;
            for (int lg = l0; lg < l1; lg += 8) {
                if (lg > l0) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int l = min(lg + j, l1 - 1);
                        va[j] = *(st + 0 * Lp1 + l); vd[j] = *(st + 1 * Lp1 + l);
                        vc[j] = *(st + 3 * Lp1 + l);
                    }
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int l = lg + j;
                    if (l < l1) {
                        const double w = (double)l * (l + 1) / (2.0 * PI);
                        a += w * va[j];
                        dd += w * vd[j];
                        c += w * vc[j];
                    }
                }
            }
            double tt = 0.0, ee = 0.0, te = 0.0;
            if (b >= 2) {
                const double det = a * dd - c * c;
                const double s00 = dd / det, s11 = a / det, s01 = -c / det;
                const double l00 = sqrt(s00);
                const double l10 = s01 / l00;
                const double l11 = sqrt(s11 - l10 * l10);
                const double c1 = sqrt(2.0 * g1);
                const double c2 = sqrt(2.0 * g2);
                const double b00 = l00 * c1;
                const double b10 = l10 * c1 + l11 * n;
                const double b11 = l11 * c2;
                const double w00 = b00 * b00, w01 = b00 * b10, w11 = b10 * b10 + b11 * b11;
                const double wd = w00 * w11 - w01 * w01;
                tt = w11 / wd; ee = w00 / wd; te = -w01 / wd;
            }
            dl_out[((long long)chain * NSP + 0) * maxbins + b] = tt;
            dl_out[((long long)chain * NSP + 1) * maxbins + b] = ee;
            dl_out[((long long)chain * NSP + 3) * maxbins + b] = te;
            if (tr) { tr[0 * maxbins + b] = tt; tr[1 * maxbins + b] = ee; tr[3 * maxbins + b] = te; }
        }
        return;
    }
    if (b >= maxbins) return;
    if (b >= nb) {
        if (tr) tr[sp * maxbins + b] = out[b];
        return;
    }
    {
        // as the TEB block above: the first 24 statistics issued before the
        // Gamma draw, whose shape needs only sum (2l + 1) / 2 = (l1^2 - l0^2) / 2
        const int l0 = be[b], l1 = be[b + 1];
        constexpr int G = 24;
        double v[G];
#pragma unroll
        for (int j = 0; j < G; ++j) v[j] = *(st + ssrow * Lp1 + max(min(l0 + j, l1 - 1), 0));
        double X;
        if (variates) X = variates[((long long)chain * NSP + sp) * maxbins + b];
        else if (pre) X = pre[(((long long)chain * NSP + sp) * maxbins + b) * 3];
        else { double vr[3]; cls_variates<F>(sp, b, l0, l1, key, iter, vr); X = vr[0]; }
        double beta = 0.0;
        for (int lg = l0; lg < l1; lg += G) {
            if (lg > l0) {
#pragma unroll
                for (int j = 0; j < G; ++j) v[j] = *(st + ssrow * Lp1 + min(lg + j, l1 - 1));
            }
#pragma unroll
            for (int j = 0; j < G; ++j) {
                const int l = lg + j;
                if (l < l1) {
                    const double chat = v[j] / (2.0 * l + 1.0);
                    beta += (2.0 * l + 1.0) * l * (l + 1.0) * (chat / (4.0 * PI));
                }
            }
        }
        out[b] = b < 2 ? 0.0 : beta * X;
        if (tr) tr[sp * maxbins + b] = out[b];
    }
}

template <int F>
__global__ __launch_bounds__(64) void k_cls_draw(int L, int nchains, int maxbins, const int* __restrict__ bins,
                                                 const int* __restrict__ nbins_arr, const double* __restrict__ stats,
                                                 const double* __restrict__ variates, uint32_t seed_lo,
                                                 uint32_t seed_hi, IterArg itarg, int chain0,
                                                 double* __restrict__ dl_out, double* __restrict__ trace, int cap,
                                                 uint32_t* __restrict__ counter, uint32_t adv,
                                                 const double* __restrict__ pre) {
    const uint32_t iter = itarg.get();
    cls_draw_body<F>(blockIdx.x, blockIdx.y, blockIdx.z * blockDim.x + threadIdx.x, L, maxbins, bins, nbins_arr,
                     stats, variates, seed_lo, seed_hi, iter, chain0, dl_out, trace,
                     cap, nchains, pre);
    if (counter) ticket_advance(counter, gridDim.x * gridDim.y * gridDim.z, adv);
}

// one (chain, spectrum, bin) item of the draw's variates (the sweep's extra
// workgroups); bins past a spectrum's count are not drawn
template <int F>
__device__ void cls_variates_item(const ClsPre& cp, int item, uint32_t seed_lo, uint32_t seed_hi, uint32_t iter,
                                  int chain0) {
    if (item >= cp.nitem) return;                   // the last workgroup's tail
    const int b = item % cp.maxbins, sp = (item / cp.maxbins) % cp.nspec, chain = item / (cp.maxbins * cp.nspec);
    if (b >= cp.nbins[sp] || ((F == 3) && sp != 0 && sp != 2)) return;
    const int* be = cp.bins + sp * (cp.maxbins + 1);
    double v[3];
    cls_variates<F>(sp, b, be[b], be[b + 1], chain_key(seed_lo, seed_hi, (uint32_t)(chain0 + chain)), iter, v);
    double* q = cp.out + (long long)item * 3;
    q[0] = v[0]; q[1] = v[1]; q[2] = v[2];
}


// ============================================================================
// non-centered Metropolis-within-Gibbs (NonCenteredGibbs.py:292-445)
// ============================================================================
// standard normal truncated to [a, inf), a <= 0 (scipy truncnorm._ppf case_left)
__device__ __forceinline__ double tn_ppf(double q, double a) {
    const double pa = normcdf(a), pma = normcdf(-a);
    const double plo = pa + q * pma;
    const double phi = (1.0 - q) * pma;
    return plo < 0.5 ? normcdfinv(plo) : -normcdfinv(phi);
}

__device__ __forceinline__ double log_ndtr(double x) {
    if (x > -5.0) return log1p(-0.5 * erfc(x / sqrt(2.0)));
    const double t = -x / sqrt(2.0);
    return log(0.5 * erfcx(t)) - t * t;
}

// per-l log-likelihood term without the constant S_dd (NonCenteredGibbs.py:357-377),
// from this l's statistics sv[q] = stats[q][l]
template <int F>
__device__ __forceinline__ double f_ell_v(const double (&sv)[SweepAcc<F>::NS], double b, double k0, double k1,
                                          double k2, double v0, double v1, double v2, double v3) {
    if constexpr (F == 1) {
        const double a = sqrt(v0);
        return -0.5 * k0 * (-2.0 * b * (a * sv[1]) + b * b * (a * a * sv[0]));
    } else if constexpr (F == 2) {
        const double aE = sqrt(v0), aB = sqrt(v1);
        const double fE = -0.5 * k0 * (-2.0 * b * (aE * sv[2]) + b * b * (aE * aE * sv[0]));
        const double fB = -0.5 * k1 * (-2.0 * b * (aB * sv[3]) + b * b * (aB * aB * sv[1]));
        return fE + fB;
    } else {
        // v0..v3 = TT, EE, BB, TE
        const CovChol A = cov_chol_teb(v0, v1, v3, v2);
        const double ssTT = sv[0], ssEE = sv[1], ssBB = sv[2], ssTE = sv[3];
        const double dTsT = sv[4], dEsT = sv[5], dEsE = sv[6], dBsB = sv[7];
        const double fT = -0.5 * k0 * (-2.0 * b * (A.a00 * dTsT) + b * b * (A.a00 * A.a00 * ssTT));
        const double linE = A.a10 * dEsT + A.a11 * dEsE;
        const double quadE = A.a10 * A.a10 * ssTT + A.a10 * A.a11 * ssTE + A.a11 * A.a10 * ssTE + A.a11 * A.a11 * ssEE;
        const double fE = -0.5 * k1 * (-2.0 * b * linE + b * b * quadE);
        const double fB = -0.5 * k2 * (-2.0 * b * (A.aB * dBsB) + b * b * (A.aB * A.aB * ssBB));
        return fT + fE + fB;
    }
}

template <int F>
__device__ __forceinline__ double f_ell(const double* __restrict__ st, int Lp1, int l, double b, double k0, double k1,
                                        double k2, double v0, double v1, double v2, double v3) {
    double sv[SweepAcc<F>::NS];
#pragma unroll
    for (int q = 0; q < SweepAcc<F>::NS; ++q) sv[q] = st[q * Lp1 + l];
    return f_ell_v<F>(sv, b, k0, k1, k2, v0, v1, v2, v3);
}

__device__ __forceinline__ bool psd_ok(double tt, double ee, double te) {
    if (tt == 0.0 && te == 0.0) return ee >= 0.0;
    return tt > 0.0 && ee > 0.0 && tt * ee - te * te > 0.0;
}

// fixed-order wave reduction; the lane-0 total is broadcast so every lane
// takes the same accept decision
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    return __shfl(v, 0, 64);
}

// proposals (NonCenteredGibbs.py:292-309) and per-bin log proposal ratios
// (313-330, 410-413): one thread per (chain, spectrum, bin)
template <int F>
__device__ __forceinline__ void mh_propose_at(long long g, int nchains, int maxbins, const int* __restrict__ nbins_arr,
                                              const double* __restrict__ prop_sd, const double* __restrict__ dl,
                                              double* __restrict__ prop, double* __restrict__ logr,
                                              const double* __restrict__ u_prop, uint32_t seed_lo,
                                              uint32_t seed_hi, IterArg itarg, int chain0,
                                              double* __restrict__ snap = nullptr) {
    const uint32_t iter = itarg.get();
    constexpr int NSP = F == 1 ? 1 : (F == 2 ? 2 : 4);
    if (g >= (long long)nchains * NSP * maxbins) return;
    // (snap: a copy of the D_l the proposals start from, every item, for the split MH)
    if (snap) snap[g] = dl[g];
    const int b = (int)(g % maxbins);
    const int sp = (int)((g / maxbins) % NSP);
    const int chain = (int)(g / ((long long)maxbins * NSP));
    if (b < 2 || b >= nbins_arr[sp]) return;
    const Key key = chain_key(seed_lo, seed_hi, (uint32_t)(chain0 + chain));
    const double sd = prop_sd[sp * maxbins + b];
    const double old = dl[g];
    double p, lr;
    if (F == 3 && sp == 3) {
        // TE: symmetric normal proposal (build spec; no positivity constraint)
        const double y = u_prop ? normcdfinv(u_prop[g]) : normal1(key, b, sp, TAG_TN, iter);
        p = old + sd * y;
        lr = 0.0;
    } else {
        const double a = -old / sd;
        const double q = u_prop ? u_prop[g] : uniform1(key, b, sp, TAG_TN, iter);
        p = old + sd * tn_ppf(q, a);
        lr = log_ndtr(old / sd) - log_ndtr(p / sd);
    }
    prop[g] = p;
    logr[g] = lr;
}

template <int F>
__global__ __launch_bounds__(256) void k_mh_propose(int nchains, int maxbins, const int* __restrict__ nbins_arr,
                                                    const double* __restrict__ prop_sd, const double* __restrict__ dl,
                                                    double* __restrict__ prop, double* __restrict__ logr,
                                                    const double* __restrict__ u_prop, uint32_t seed_lo,
                                                    uint32_t seed_hi, IterArg itarg, int chain0,
                                                    double* __restrict__ snap) {
    mh_propose_at<F>(blockIdx.x * (long long)blockDim.x + threadIdx.x, nchains, maxbins, nbins_arr, prop_sd, dl, prop,
                     logr, u_prop, seed_lo, seed_hi, itarg, chain0, snap);
}

// flat accept order of the plan (same counters as k_mh_fused / k_mh_accept)
__device__ __forceinline__ void mh_uniform_at(long long g, int nchains, int nspec, const int* __restrict__ meta,
                                              int nacc, int n_iter_mh, uint32_t seed_lo, uint32_t seed_hi,
                                              uint32_t iter, int chain0, double* __restrict__ out) {
    if (g >= (long long)nchains * nacc) return;
    const int chain = (int)(g / nacc), flat = (int)(g % nacc);
    const int* nblocks = meta + 4;
    const int* acc_off = meta + 8;
    int sp = -1;
    for (int k = 0; k < nspec; ++k)
        if (flat >= acc_off[k] && flat < acc_off[k] + nblocks[k] * n_iter_mh) sp = k;
    if (sp < 0) return;
    const int r = flat - acc_off[sp];
    const int blk = r / n_iter_mh, att = r % n_iter_mh;
    const Key key = chain_key(seed_lo, seed_hi, (uint32_t)(chain0 + chain));
    out[g] = uniform1(key, blk, (uint32_t)sp | ((uint32_t)att << 8), TAG_MH_U, iter);
}

// k_stats_finish with nbp + nbu extra workgroups first (deferred draws the sweep could not take: replayed normals): the
// MH proposals and native accept uniforms of this step, the same items and
// code as k_nc_prologue's (bit-identical either way)
template <int F, int G>
__global__ __launch_bounds__(256) void k_stats_finish_pro(int L, int nchains, int ntile, int nchunkg, int tm,
                                                          int nstat, const double* __restrict__ partials,
                                                          double* __restrict__ stats, int nblk_prop, int nblk_u,
                                                          double* __restrict__ u_out, int nspec, int nacc,
                                                          int n_iter_mh, int maxbins,
                                                          const int* __restrict__ nbins_arr,
                                                          const double* __restrict__ prop_sd,
                                                          const double* __restrict__ dl, double* __restrict__ prop,
                                                          double* __restrict__ logr, uint32_t seed_lo,
                                                          uint32_t seed_hi, IterArg itarg, int chain0,
                                                          double* __restrict__ snap) {
    const int bx = (int)blockIdx.x;
    if (bx < nblk_prop) {
        mh_propose_at<F>(bx * (long long)blockDim.x + threadIdx.x, nchains, maxbins, nbins_arr, prop_sd, dl, prop,
                         logr, nullptr, seed_lo, seed_hi, itarg, chain0, snap);
        return;
    }
    if (bx < nblk_prop + nblk_u) {
        mh_uniform_at((bx - nblk_prop) * (long long)blockDim.x + threadIdx.x, nchains, nspec, nbins_arr, nacc,
                      n_iter_mh, seed_lo, seed_hi, itarg.get(), chain0, u_out);
        return;
    }
    const int b = bx - nblk_prop - nblk_u;
    const int t = b % ntile;
    const int q = (b / ntile) % nstat;
    const int chain = b / (ntile * nstat);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int Lp1 = L + 1;
    GS_ASSERT(chain < nchains);
    const double acc = stats_finish_sum<G>(L, ntile, nchunkg, tm, nstat, partials, chain, q, t, w, lane);
    __shared__ double red[4][WAVE];
    red[w][lane] = acc;
    __syncthreads();
    if (w == 0) {
        const int ell = L - WAVE * t - 63 + lane;
        if (ell >= 0)
            stats[((long long)chain * nstat + q) * Lp1 + ell] = ((red[0][lane] + red[1][lane]) + red[2][lane]) +
                                                                 red[3][lane];
    }
}

template <int F>
__device__ void pro_pre_item(const ProPre& pp, int bx, int nchains, uint32_t seed_lo, uint32_t seed_hi, IterArg itarg,
                             int chain0) {
    if (bx < pp.nbp)
        mh_propose_at<F>(bx * (long long)blockDim.x + threadIdx.x, nchains, pp.maxbins, pp.nbins, pp.prop_sd, pp.dl,
                         pp.prop, pp.logr, nullptr, seed_lo, seed_hi, itarg, chain0, pp.snap);
    else if (bx < pp.nbp + pp.nbu)
        mh_uniform_at((bx - pp.nbp) * (long long)blockDim.x + threadIdx.x, nchains, pp.nspec, pp.nbins, pp.nacc,
                      pp.n_iter_mh, seed_lo, seed_hi, itarg.get(), chain0, pp.u_out);
    else if (bx < pp.nbp + pp.nbu + pp.nbv)
        cls_variates_item<F>(pp.cp, (bx - pp.nbp - pp.nbu) * blockDim.x + threadIdx.x, seed_lo, seed_hi, itarg.get(),
                             chain0);
}

// non-centered prologue: the MH proposals depend only on the current D_l, not
// on the CR draw, so they are made in the same launch as the CR block
// parameters (proposal workgroups first; both halves are latency-bound).
template <int F>
__global__ __launch_bounds__(256) void k_nc_prologue(int nblk_prop, int nblk_par, double* __restrict__ u_out,
                                                     int nspec, int nacc, int n_iter_mh, int L, int nchains, int maxbins,
                                                     const int* __restrict__ ell2bin, const double* __restrict__ bl,
                                                     double k0, double k1, double k2, double* __restrict__ params,
                                                     const int* __restrict__ nbins_arr, const double* __restrict__ prop_sd,
                                                     const double* __restrict__ dl, double* __restrict__ prop,
                                                     double* __restrict__ logr, const double* __restrict__ u_prop,
                                                     uint32_t seed_lo, uint32_t seed_hi, IterArg itarg, int chain0,
                                                     double* __restrict__ snap) {
    if ((int)blockIdx.x >= nblk_prop + nblk_par) {
        // native accept uniforms of this step's MH (k_mh_fused reads them from LDS)
        mh_uniform_at(((int)blockIdx.x - nblk_prop - nblk_par) * (long long)blockDim.x + threadIdx.x, nchains, nspec,
                      nbins_arr, nacc, n_iter_mh, seed_lo, seed_hi, itarg.get(), chain0, u_out);
        return;
    }
    if ((int)blockIdx.x < nblk_prop)
        mh_propose_at<F>(blockIdx.x * (long long)blockDim.x + threadIdx.x, nchains, maxbins, nbins_arr, prop_sd, dl,
                         prop, logr, u_prop, seed_lo, seed_hi, itarg, chain0, snap);
    else
        block_params_at<F, 1>(((int)blockIdx.x - nblk_prop) * blockDim.x + threadIdx.x, L, nchains, maxbins, dl,
                              ell2bin, bl, k0, k1, k2, params);
}

// MH phase, step 1: per-(chain, l) likelihood difference of the phase's
// spectra, g = f_l(proposed) - f_l(current) (-inf when the proposed TE block
// is not positive definite).  One thread per (chain, l): the per-l
// decomposition of the all_sph likelihood makes this fully parallel.
template <int F>
__global__ __launch_bounds__(256) void k_mh_terms(int L, int nchains, int maxbins, int sp0, int sp1,
                                                  const int* __restrict__ ell2blk, const int* __restrict__ ell2bin,
                                                  const double* __restrict__ bl, double k0, double k1, double k2,
                                                  const double* __restrict__ stats, const double* __restrict__ dl,
                                                  const double* __restrict__ prop, double* __restrict__ gbuf) {
    constexpr int NSP = F == 1 ? 1 : (F == 2 ? 2 : 4);
    constexpr int NS = SweepAcc<F>::NS;
    const int Lp1 = L + 1;
    const long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (g >= (long long)nchains * Lp1) return;
    const int chain = (int)(g / Lp1), l = (int)(g % Lp1);
    const double* D = dl + (long long)chain * NSP * maxbins;
    const double* P = prop + (long long)chain * NSP * maxbins;
    const double* st = stats + (long long)chain * NS * Lp1;
    double vo[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < NSP; ++q) vo[q] = var_from_dl(dl_at(D, ell2bin, maxbins, Lp1, q, l), l);
    const double b = bl[l];
    const double fo = f_ell<F>(st, Lp1, l, b, k0, k1, k2, vo[0], vo[1], vo[2], vo[3]);
    const int sps[2] = {sp0, sp1};
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int sp = sps[k];
        if (sp < 0) continue;
        double out = 0.0;
        if (ell2blk[sp * Lp1 + l] >= 0) {
            double vn[4] = {vo[0], vo[1], vo[2], vo[3]};
            vn[sp] = var_from_dl(P[sp * maxbins + ell2bin[sp * Lp1 + l]], l);
            bool ok = true;
            if constexpr (F == 3) ok = psd_ok(vn[0], vn[1], vn[3]);
            out = ok ? f_ell<F>(st, Lp1, l, b, k0, k1, k2, vn[0], vn[1], vn[2], vn[3]) - fo : -INFINITY;
        }
        gbuf[((long long)chain * 2 + k) * Lp1 + l] = out;
    }
}

// MH phase, step 2: one wave per (chain, block): fixed-order sum of the
// block's g_l and proposal log ratios, accept with log u < delta + log r,
// n_iter_metropolis attempts (NonCenteredGibbs.py:427-442).
template <int F>
__global__ __launch_bounds__(256) void k_mh_accept(int L, int nchains, int maxbins, int sp0,
                                                   const int* __restrict__ bins, const int* __restrict__ blocks,
                                                   const int2* __restrict__ phase_blk, int nphase_blk,
                                                   const int* __restrict__ acc_off, int nacc, int n_iter_mh,
                                                   const double* __restrict__ gbuf, double* __restrict__ dl,
                                                   const double* __restrict__ prop, const double* __restrict__ logr,
                                                   const double* __restrict__ u_acc, uint32_t seed_lo,
                                                   uint32_t seed_hi, IterArg itarg, int chain0,
                                                   int32_t* __restrict__ accept_out) {
    const uint32_t iter = itarg.get();
    constexpr int NSP = F == 1 ? 1 : (F == 2 ? 2 : 4);
    const long long w = blockIdx.x * 4LL + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (w >= (long long)nchains * nphase_blk) return;
    const int chain = (int)(w / nphase_blk);
    const int2 sb = phase_blk[w % nphase_blk];
    const int sp = sb.x, blk = sb.y;
    const int k = sp == sp0 ? 0 : 1;
    const int Lp1 = L + 1;
    const Key key = chain_key(seed_lo, seed_hi, (uint32_t)(chain0 + chain));
    double* D = dl + (long long)chain * NSP * maxbins;
    const double* P = prop + (long long)chain * NSP * maxbins;
    const double* R = logr + (long long)chain * NSP * maxbins;
    const double* G = gbuf + ((long long)chain * 2 + k) * Lp1;
    const int* be = bins + sp * (maxbins + 1);
    const int* bk = blocks + sp * (maxbins + 1);
    const int lo = bk[blk], hi = bk[blk + 1];
    double lrs = 0.0, diff = 0.0;
    for (int q = lo + lane; q < hi; q += 64) lrs += R[sp * maxbins + q];
    if (hi > lo)
        for (int l = be[lo] + lane; l < be[hi]; l += 64) diff += G[l];
    lrs = wave_sum(lrs);
    diff = wave_sum(diff);
    bool taken = false;
    for (int att = 0; att < n_iter_mh; ++att) {
        const int flat = acc_off[sp] + blk * n_iter_mh + att;
        const double u = u_acc ? u_acc[(long long)chain * nacc + flat]
                               : uniform1(key, blk, (uint32_t)sp | ((uint32_t)att << 8), TAG_MH_U, iter);
        // after an acceptance the proposal IS the current state: delta = 0
        const double log_r = (taken ? 0.0 : diff) + lrs;
        const bool acc = log(u) < log_r;
        if (acc && !taken)
            for (int q = lo + lane; q < hi; q += 64) D[sp * maxbins + q] = P[sp * maxbins + q];
        taken = taken || acc;
        if (lane == 0 && accept_out) accept_out[(long long)chain * nacc + flat] = acc ? 1 : 0;
    }
}

// the native accept uniforms of every (chain, spectrum, block, attempt) in the
__global__ void k_mh_uniforms(int nchains, int nspec, int maxbins, const int* __restrict__ meta, int nacc,
                              int n_iter_mh, uint32_t seed_lo, uint32_t seed_hi, IterArg itarg, int chain0,
                              double* __restrict__ out) {
    mh_uniform_at(blockIdx.x * (long long)blockDim.x + threadIdx.x, nchains, nspec, meta, nacc, n_iter_mh, seed_lo,
                  seed_hi, itarg.get(), chain0, out);
}

// MH phases fused in one launch: one workgroup per chain walks the phases;
// per phase the per-l terms go to LDS, the per-(block, attempt) uniforms are
// drawn in parallel, blocks of <= 16 l are decided by one thread each and
// wider blocks by one wave each (fixed-order sums), then a barrier publishes
// the updated D_l to the next phase (same workgroup).
constexpr int MH_SMALL = 16;   // blocks of <= MH_SMALL multipoles are decided by one thread

struct MhPhases {
    int nphase;
    int sp0[4], sp1[4];     // the phase's two spectra
    int off[4];
    int n[4];
    int nwide[4];
    int lmin;     // smallest multipole any MH block covers (terms below it are never read)
    int own;      // spectra (bit per spectrum) whose D_l this workgroup decides and writes back
};

// a[q] for a wave-uniform q < 4 by constant indices (scalar selects)
__device__ __forceinline__ int mh_pick(const int (&a)[4], int q) {
    return q == 0 ? a[0] : (q == 1 ? a[1] : (q == 2 ? a[2] : a[3]));
}

// the kind-th workgroup's phases (k_mh_reg's split): a field-by-field select
// with constant indices, so neither by-value argument needs an address
__device__ __forceinline__ MhPhases mh_select(bool k1, const MhPhases& a, const MhPhases& b) {
    MhPhases r;
    r.nphase = k1 ? b.nphase : a.nphase;
    r.lmin = k1 ? b.lmin : a.lmin;
    r.own = k1 ? b.own : a.own;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        r.sp0[q] = k1 ? b.sp0[q] : a.sp0[q];
        r.sp1[q] = k1 ? b.sp1[q] : a.sp1[q];
        r.off[q] = k1 ? b.off[q] : a.off[q];
        r.n[q] = k1 ? b.n[q] : a.n[q];
        r.nwide[q] = k1 ? b.nwide[q] : a.nwide[q];
    }
    return r;
}

// optional tail of the fused MH kernel (graph-captured NC steps): record this
// chain's D_l in the trace and advance the device iteration counter once the
// last workgroup has finished (every workgroup read the counter at its start,
// so the ticket is race-free).  (Computing the next step's prologue here as
// well was measured slower: it puts that wide, latency-bound work on one
// workgroup per chain.)
struct MhEpi {
    double* trace;          // nullable: trace[(it-1) % cap][chain][nspec][maxbins]
    int cap;
    uint32_t* counter;      // nullable: [0] iteration base (advanced by adv), [1] finished-workgroup ticket
    int nchains;
    uint32_t adv;
    const double* dl_in;    // nullable (k_mh_reg): read the chains' D_l from here, write the decisions to dl
};

// SC: this chain's per-l statistics cached in LDS for the whole kernel (every
// phase evaluates f_l from them; LDS instead of three passes over L2) -- off
// by default (slower: the larger LDS fill costs more than the L2 reads save)
// workgroup copy global -> LDS with four independent loads per thread in flight
template <typename T>
__device__ __forceinline__ void lds_fill4(T* __restrict__ dst, const T* __restrict__ src, int n) {
    const int bd = blockDim.x;
    for (int k0 = threadIdx.x; k0 < n; k0 += 4 * bd) {
        T v[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] = k0 + t * bd < n ? src[k0 + t * bd] : T(0);
#pragma unroll
        for (int t = 0; t < 4; ++t)
            if (k0 + t * bd < n) dst[k0 + t * bd] = v[t];
    }
}

template <int F>
__global__ __launch_bounds__(1024) void k_mh_fused(int L, int maxbins, MhPhases ph, const int2* __restrict__ phase_tab,
                                                  const int4* __restrict__ phase_rng,
                                                  const int* __restrict__ bins, const int* __restrict__ blocks,
                                                  const int* __restrict__ acc_off, int nacc, int n_iter_mh,
                                                  const int* __restrict__ ell2blk, const int* __restrict__ ell2bin,
                                                  const double* __restrict__ bl, double k0, double k1, double k2,
                                                  const double* __restrict__ stats, double* __restrict__ dl,
                                                  const double* __restrict__ prop, const double* __restrict__ logr,
                                                  const double* __restrict__ u_acc, uint32_t seed_lo, uint32_t seed_hi,
                                                  IterArg itarg, int chain0, int32_t* __restrict__ accept_out,
                                                  MhEpi epi) {
    const uint32_t iter = itarg.get();
    constexpr int NSP = F == 1 ? 1 : (F == 2 ? 2 : 4);
    constexpr int NS = SweepAcc<F>::NS;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int Lp1 = L + 1;
    int maxnb = 0;
    for (int q = 0; q < ph.nphase; ++q) maxnb = max(maxnb, ph.n[q]);
    double* g = smem;                               // [2][L+1]
    double* ub = g + 2 * Lp1;                       // [phase blocks x n_iter]
    double* Ds = ub + maxnb * n_iter_mh;            // [NSP][maxbins] LDS copy of this chain's D_l
    double* ul = Ds + NSP * maxbins;                // [nacc] this chain's accept uniforms (u_acc given)
    int* e2b = reinterpret_cast<int*>(ul + (u_acc ? nacc : 0));   // [NSP][L+1]
    const int chain = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nwv = blockDim.x >> 6;
    const Key key = chain_key(seed_lo, seed_hi, (uint32_t)(chain0 + chain));
    constexpr int MAXW = 4;                         // wide blocks decided together
    __shared__ double wsum[MAXW][64];
    __shared__ int wflag[MAXW];
    double* D = dl + (long long)chain * NSP * maxbins;
    const double* P = prop + (long long)chain * NSP * maxbins;
    const double* R = logr + (long long)chain * NSP * maxbins;
    const double* stg = stats + (long long)chain * NS * Lp1;
    const double* st = stg;
    // LDS fill: the chain's D_l (kept in LDS for the whole sweep, written back at
    // the end), accept uniforms (u_acc) and the l -> bin map;
    // four loads in flight per thread and array
    lds_fill4(Ds, D, NSP * maxbins);
    if (u_acc) lds_fill4(ul, u_acc + (long long)chain * nacc, nacc);
    lds_fill4(e2b, ell2bin, NSP * Lp1);
    __syncthreads();
    for (int q = 0; q < ph.nphase; ++q) {
        const int nb = mh_pick(ph.n, q);
        if (nb == 0) continue;
        const int sp0 = mh_pick(ph.sp0, q), sp1 = mh_pick(ph.sp1, q);
        const int off = mh_pick(ph.off, q);
        const int2* tab = phase_tab + off;
        const int4* rng = phase_rng + off;
        const int nwide = mh_pick(ph.nwide, q);
        // per-l likelihood differences of the phase's spectra
        for (int l = ph.lmin + tid; l < Lp1; l += blockDim.x) {
            double vo[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int s = 0; s < NSP; ++s) vo[s] = var_from_dl(dl_at(Ds, e2b, maxbins, Lp1, s, l), l);
            const double b = bl[l];
            const double fo = f_ell<F>(st, Lp1, l, b, k0, k1, k2, vo[0], vo[1], vo[2], vo[3]);
            const int sps[2] = {sp0, sp1};
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int sp = sps[k];
                if (sp < 0) continue;
                double out = 0.0;
                if (ell2blk[sp * Lp1 + l] >= 0) {
                    double vn[4] = {vo[0], vo[1], vo[2], vo[3]};
                    vn[sp] = var_from_dl(P[sp * maxbins + e2b[sp * Lp1 + l]], l);
                    bool ok = true;
                    if constexpr (F == 3) ok = psd_ok(vn[0], vn[1], vn[3]);
                    out = ok ? f_ell<F>(st, Lp1, l, b, k0, k1, k2, vn[0], vn[1], vn[2], vn[3]) - fo : -INFINITY;
                }
                g[k * Lp1 + l] = out;
            }
        }
        // accept uniforms of every (block, attempt), in parallel
        for (int j = tid; j < nb * n_iter_mh; j += blockDim.x) {
            const int2 sb = tab[j / n_iter_mh];
            const int att = j % n_iter_mh;
            const int flat = acc_off[sb.x] + sb.y * n_iter_mh + att;
            ub[j] = u_acc ? ul[flat] : uniform1(key, sb.y, (uint32_t)sb.x | ((uint32_t)att << 8), TAG_MH_U, iter);
        }
        __syncthreads();
        // narrow blocks: one thread each
        for (int j = nwide + tid; j < nb; j += blockDim.x) {
            const int2 sb = tab[j];
            const int4 r = rng[j];
            const int sp = sb.x, blk = sb.y, k = sp == sp0 ? 0 : 1;
            const int lo = r.x, hi = r.y, l0 = r.z, l1 = r.w;
            GS_ASSERT(lo >= 0 && hi <= maxbins && l0 >= 0 && l1 <= Lp1);
            double diff = 0.0, lrs = 0.0;
            for (int l = l0; l < l1; ++l) diff += g[k * Lp1 + l];
            for (int b = lo; b < hi; ++b) lrs += R[sp * maxbins + b];
            bool taken = false;
            for (int att = 0; att < n_iter_mh; ++att) {
                const bool acc = log(ub[j * n_iter_mh + att]) < (taken ? 0.0 : diff) + lrs;
                if (acc && !taken)
                    for (int b = lo; b < hi; ++b) Ds[sp * maxbins + b] = P[sp * maxbins + b];
                taken = taken || acc;
                if (accept_out) accept_out[(long long)chain * nacc + acc_off[sp] + blk * n_iter_mh + att] = acc ? 1 : 0;
            }
        }
        // wide blocks: the whole workgroup, up to MAXW blocks together (fixed-order
        // sums per block: per-thread terms, wave sums, then the 16 wave sums in
        // wave order; the blocks of a phase are independent), so a phase's few
        // long blocks share one pair of barriers and do not serialise on one wave
        for (int j0 = 0; j0 < nwide; j0 += MAXW) {
            const int nw = min(MAXW, nwide - j0);
#pragma unroll
            for (int jj = 0; jj < MAXW; ++jj) {
                if (jj >= nw) break;
                const int2 sb = tab[j0 + jj];
                const int4 r = rng[j0 + jj];
                const int k = sb.x == sp0 ? 0 : 1;
                double diff = 0.0, lrs = 0.0;
                for (int l = r.z + tid; l < r.w; l += blockDim.x) diff += g[k * Lp1 + l];
                for (int b = r.x + tid; b < r.y; b += blockDim.x) lrs += R[sb.x * maxbins + b];
                diff = wave_sum(diff);
                lrs = wave_sum(lrs);
                if (lane == 0) { wsum[jj][wv] = diff; wsum[jj][32 + wv] = lrs; }
            }
            __syncthreads();
            if (tid < nw) {
                const int j = j0 + tid;
                const int2 sb = tab[j];
                const int sp = sb.x, blk = sb.y;
                double dsum = 0.0, lsum = 0.0;
                for (int w = 0; w < nwv; ++w) { dsum += wsum[tid][w]; lsum += wsum[tid][32 + w]; }
                bool taken = false;
                for (int att = 0; att < n_iter_mh; ++att) {
                    const bool acc = log(ub[j * n_iter_mh + att]) < (taken ? 0.0 : dsum) + lsum;
                    taken = taken || acc;
                    if (accept_out)
                        accept_out[(long long)chain * nacc + acc_off[sp] + blk * n_iter_mh + att] = acc ? 1 : 0;
                }
                wflag[tid] = taken ? 1 : 0;
            }
            __syncthreads();
            for (int jj = 0; jj < nw; ++jj) {
                if (!wflag[jj]) continue;
                const int2 sb = tab[j0 + jj];
                const int4 r = rng[j0 + jj];
                for (int b = r.x + tid; b < r.y; b += blockDim.x) Ds[sb.x * maxbins + b] = P[sb.x * maxbins + b];
            }
        }
        __syncthreads();
    }
    const int nrow = NSP * maxbins;
    for (int k = tid; k < nrow; k += blockDim.x) D[k] = Ds[k];
    // ---- epilogue (graph-captured NC steps) ----
    if (epi.trace) {
        const long long slot = (long long)((iter + (uint32_t)epi.cap - 1u) % (uint32_t)epi.cap);
        double* tr = epi.trace + (slot * epi.nchains + chain) * nrow;
        for (int k = tid; k < nrow; k += blockDim.x) tr[k] = Ds[k];
    }
    if (epi.counter) ticket_advance(epi.counter, gridDim.x, epi.adv);
}

// The MH phases with every global load issued once, at the start (r03): each
// thread owns one multipole l = lmin + tid and keeps that l's statistics, beam,
// l -> bin and l -> block indices in registers for the whole kernel; the
// chain's D_l, proposals, proposal log ratios and log accept uniforms are
// staged in LDS in the same round of loads (log u taken once, not per
// decision), and so is each thread's first narrow block per phase.  The phases
// then run on registers and LDS alone (no memory latency inside a phase):
//  * per-l terms: the likelihood is separable into the TE-block part
//    f_TE(TT, EE, TE) and the B part f_B(BB) (F = 3; F = 2: f_E + f_B), so a
//    proposal's difference is taken on its own part, g = f_part(new) -
//    f_part(old) (k_mh_fused differenced the whole per-l sum);
//  * wide blocks: one wave per block, lane-strided sums in l order and a
//    fixed-order butterfly (permlane swaps + DPP rotations) that leaves the
//    total on every lane -- no workgroup barrier inside a phase; narrow blocks
//    (one thread each) run beside them (disjoint bins).
// Decisions are the reference's (NonCenteredGibbs.py:427-442); the sums differ
// from k_mh_fused's only in rounding order.  k_mh_fused stays for plans whose
// l range exceeds one l per thread or whose arrays exceed the LDS.
//
// this thread's l -> bin / l -> block index of a spectrum (runtime sp): packed
// 16 bits per spectrum (value + 1) in one 64-bit word, so selecting by sp is a
// shift, not a dynamically indexed (scratch) register array
__device__ __forceinline__ int unpack16(uint64_t w, int sp) { return (int)((w >> (16 * sp)) & 0xFFFFu) - 1; }

constexpr int MH_REG_THREADS = 1024;

// the graph-step tail of an MH launch: this chain's D_l into the trace (each
// thread re-reads the D_l words it just wrote) and the device counter advance
// by the last of the nblk MH workgroups
// (own, maxbins: the spectra rows this workgroup wrote back -- the split MH)
__device__ __forceinline__ void mh_epilogue(const MhEpi& epi, uint32_t iter, int chain, int nrow,
                                            const double* __restrict__ dl, unsigned nblk, int maxbins = 1,
                                            int own = -1) {
    if (epi.trace) {
        const long long slot = (long long)((iter + (uint32_t)epi.cap - 1u) % (uint32_t)epi.cap);
        double* tr = epi.trace + (slot * epi.nchains + chain) * nrow;
        const double* D = dl + (long long)chain * nrow;
        for (int k = threadIdx.x; k < nrow; k += blockDim.x)
            if ((own >> (k / maxbins)) & 1) tr[k] = D[k];
    }
    if (epi.counter) ticket_advance(epi.counter, nblk, epi.adv);
}

// diagnostic timeline of the MH body (build variant "timeline", -DGS_MH_TIMELINE):
// thread 0 of chain 0's MH workgroup stamps s_memrealtime (100 MHz) at the
// stage boundaries
#if defined(GS_MH_TIMELINE)
__device__ unsigned long long g_mh_tl[32];
#define GS_TL(k) do { if (tl_on && threadIdx.x == 0) g_mh_tl[(k)] = wall_clock64(); } while (0)
#else
#define GS_TL(k) do { } while (0)
#endif

// fixed-order sum over the 64 lanes, the same bits on every lane: lane ^ 32
// (v_permlane32_swap), lane ^ 16 (v_permlane16_swap), then rotations by 8, 4,
// 2, 1 within each row of 16 (DPP row_ror); every step adds a symmetric pair,
// and fp addition is commutative, so both lanes of a pair hold the same value
__device__ __forceinline__ double wave_sum_bcast(double v) {
    {
        const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(v), __double2loint(v), false, false);
        const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(v), __double2hiint(v), false, false);
        v = __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
    }
    {
        const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(v), __double2loint(v), false, false);
        const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(v), __double2hiint(v), false, false);
        v = __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
    }
#define GS_ROR(CTRL)                                                                                     \
    {                                                                                                    \
        const int slo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xf, 0xf, false);        \
        const int shi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xf, 0xf, false);        \
        v = v + __hiloint2double(shi, slo);                                                              \
    }
    GS_ROR(0x128) GS_ROR(0x124) GS_ROR(0x122) GS_ROR(0x121)
#undef GS_ROR
    return v;
}

// the part of the per-l likelihood term (f_ell_v) that spectrum sp enters:
// F = 1: all; F = 2: f_E (sp 0) or f_B (sp 1); F = 3: f_B (sp 2) or the
// TE-block part f_T + f_E (TT, EE, TE).  v = (v0..v3) in the spectra order.
template <int F>
__device__ __forceinline__ double f_part(const double (&sv)[SweepAcc<F>::NS], double b, double k0, double k1,
                                         double k2, int sp, double v0, double v1, double v2, double v3) {
    if constexpr (F == 1) {
        const double a = sqrt(v0);
        return -0.5 * k0 * (-2.0 * b * (a * sv[1]) + b * b * (a * a * sv[0]));
    } else if constexpr (F == 2) {
        const bool e = sp == 0;
        const double a = sqrt(e ? v0 : v1);
        const double kk = e ? k0 : k1, ss = e ? sv[0] : sv[1], ds = e ? sv[2] : sv[3];
        return -0.5 * kk * (-2.0 * b * (a * ds) + b * b * (a * a * ss));
    } else {
        if (sp == 2) {
            const double aB = sqrt(v2);
            return -0.5 * k2 * (-2.0 * b * (aB * sv[7]) + b * b * (aB * aB * sv[2]));
        }
        double a00, a10, a11;
        if (v0 != 0.0) {
            a00 = sqrt(v0);
            a10 = v3 / a00;
            a11 = sqrt(fmax(v1 - a10 * a10, 0.0));
        } else {
            a00 = 0.0; a10 = 0.0; a11 = sqrt(v1);
        }
        const double fT = -0.5 * k0 * (-2.0 * b * (a00 * sv[4]) + b * b * (a00 * a00 * sv[0]));
        const double linE = a10 * sv[5] + a11 * sv[6];
        const double quadE = a10 * a10 * sv[0] + a10 * a11 * sv[3] + a11 * a10 * sv[3] + a11 * a11 * sv[1];
        const double fE = -0.5 * k1 * (-2.0 * b * linE + b * b * quadE);
        return fT + fE;
    }
}

// the f_part group of spectrum sp: F = 3: 0 = the TE block (TT, EE, TE), 1 = B;
// F = 2: 0 = E, 1 = B; F = 1: 0
template <int F>
__device__ __forceinline__ int f_group(int sp) { return F == 3 ? (sp == 2 ? 1 : 0) : (F == 2 ? sp : 0); }

// lane-strided sum a[lo + lane], a[lo + lane + 64], ... (< hi) in index order,
// U loads in flight per round
template <int U>
__device__ __forceinline__ double lane_strided_sum(const double* a, int lo, int hi, int lane) {
    double s = 0.0;
    for (int k0 = lo + lane; k0 < hi; k0 += 64 * U) {
        double v[U];
#pragma unroll
        for (int j = 0; j < U; ++j) v[j] = a[min(k0 + 64 * j, hi - 1)];
#pragma unroll
        for (int j = 0; j < U; ++j)
            if (k0 + 64 * j < hi) s += v[j];
    }
    return s;
}

// one phase-ordered MH sweep of one chain (workgroup = blockDim.x threads).
// Per thread, the current state of its l is kept across phases: the raw D_l
// and variance of every spectrum and the value of each f_part group; a phase
// evaluates only its proposals (one variance and one f_part each), and after
// the phase's decisions a thread whose D_l changed takes the proposal's values
// (identical bits to re-evaluating the new state).
template <int F>
__device__ __forceinline__ void mh_reg_body(int chain, bool tl_on, int L, int maxbins, const MhPhases& ph, int ntab,
                                            const int2* __restrict__ phase_tab, const int4* __restrict__ phase_rng,
                                            const int* __restrict__ meta, int nacc, int n_iter_mh,
                                            const int* __restrict__ ell2blk, const int* __restrict__ ell2bin,
                                            const double* __restrict__ bl, double k0, double k1, double k2,
                                            const double* __restrict__ stats, double* __restrict__ dl,
                                            const double* __restrict__ prop, const double* __restrict__ logr,
                                            const double* __restrict__ u_acc, uint32_t seed_lo, uint32_t seed_hi,
                                            uint32_t iter, int chain0, int32_t* __restrict__ accept_out,
                                            double* smem,
                                            const double* __restrict__ dl_in = nullptr) {
    (void)tl_on;
    GS_TL(0);
    constexpr int NSP = F == 1 ? 1 : (F == 2 ? 2 : 4);
    constexpr int NS = SweepAcc<F>::NS;
    constexpr int NG = F == 1 ? 1 : 2;
    const int Lp1 = L + 1;
    const int nrow = NSP * maxbins;
    double* g = smem;                    // [2][L+1] per-l likelihood differences of the phase
    double* lu = g + 2 * Lp1;            // [nacc] log accept uniforms, flat accept order
    double* Ds = lu + nacc;              // [NSP][maxbins] this chain's D_l
    double* Ps = Ds + nrow;              // [NSP][maxbins] proposals
    double* Rs = Ps + nrow;              // [NSP][maxbins] proposal log ratios
    // [ntab] phase entries (lo bin, hi bin, l0, l1), 16-B aligned, then (spectrum, block)
    int4* rngs = reinterpret_cast<int4*>(Rs + nrow + ((2 * Lp1 + nacc + 3 * nrow) & 1));
    int2* tabs = reinterpret_cast<int2*>(rngs + ntab); // [ntab] phase entries: (spectrum, block)
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nwv = blockDim.x >> 6;
    const Key key = chain_key(seed_lo, seed_hi, (uint32_t)(chain0 + chain));
    __shared__ int s_ao[4];
    double* D = dl + (long long)chain * nrow;
    // dl_in (ASIS): the draw's D_l are read from there and the decisions land in dl
    const double* Din = dl_in ? dl_in + (long long)chain * nrow : D;
    const double* P = prop + (long long)chain * nrow;
    const double* R = logr + (long long)chain * nrow;
    const double* stg = stats + (long long)chain * NS * Lp1;
    const int* acc_off = meta + 8;
    // ---- one round of loads: this thread's l ...
    const int l = ph.lmin + tid;
    const bool lok = l < Lp1;
    const int lc = lok ? l : L;
    int eb[NSP], ek[NSP];
    double sv[NS];
#pragma unroll
    for (int q = 0; q < NSP; ++q) { eb[q] = ell2bin[q * Lp1 + lc]; ek[q] = ell2blk[q * Lp1 + lc]; }
#pragma unroll
    for (int q = 0; q < NS; ++q) sv[q] = stg[q * Lp1 + lc];
    if (tid < NSP) s_ao[tid] = acc_off[tid];
    const double b = bl[lc];
    // ... and the LDS arrays: up to MH_FILL rows of D / P / R per thread with
    // every load issued before the stores (one memory round trip; a loop over
    // rows would make one per row), the phase tables likewise
    constexpr int MH_FILL = 8;
    if (nrow <= MH_FILL * MH_REG_THREADS) {
        double dv[MH_FILL], pv[MH_FILL], rv[MH_FILL];
#pragma unroll
        for (int j = 0; j < MH_FILL; ++j) {
            const int k = min(tid + j * MH_REG_THREADS, nrow - 1);
            dv[j] = Din[k]; pv[j] = P[k]; rv[j] = R[k];
        }
        int4 rr[2];
        int2 tt[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int k = min(tid + j * MH_REG_THREADS, max(ntab - 1, 0));
            rr[j] = phase_rng[k]; tt[j] = phase_tab[k];
        }
#pragma unroll
        for (int j = 0; j < MH_FILL; ++j) {
            const int k = tid + j * MH_REG_THREADS;
            if (k < nrow) { Ds[k] = dv[j]; Ps[k] = pv[j]; Rs[k] = rv[j]; }
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int k = tid + j * MH_REG_THREADS;
            if (k < ntab) { rngs[k] = rr[j]; tabs[k] = tt[j]; }
        }
        for (int k = tid + 2 * MH_REG_THREADS; k < ntab; k += MH_REG_THREADS) {
            rngs[k] = phase_rng[k];
            tabs[k] = phase_tab[k];
        }
    } else {
        for (int k = tid; k < nrow; k += MH_REG_THREADS) { Ds[k] = Din[k]; Ps[k] = P[k]; Rs[k] = R[k]; }
        for (int k = tid; k < ntab; k += MH_REG_THREADS) { rngs[k] = phase_rng[k]; tabs[k] = phase_tab[k]; }
    }
    if (u_acc) {
        for (int k = tid; k < nacc; k += MH_REG_THREADS) lu[k] = log(u_acc[(long long)chain * nacc + k]);
    } else {
        // in-kernel uniforms (the flat order's (spectrum, block, attempt) counters)
        for (int k = tid; k < nacc; k += MH_REG_THREADS) {
            int sp = 0, base = 0;
#pragma unroll
            for (int q = 0; q < NSP; ++q) {
                const int a = acc_off[q];
                if (k >= a && k < a + meta[4 + q] * n_iter_mh) { sp = q; base = a; }
            }
            const int r = k - base;
            lu[k] = log(uniform1(key, r / n_iter_mh, (uint32_t)sp | ((uint32_t)(r % n_iter_mh) << 8), TAG_MH_U, iter));
        }
    }
    uint64_t ebp = 0, ekp = 0;
#pragma unroll
    for (int q = 0; q < NSP; ++q) {
        ebp |= (uint64_t)(uint32_t)(eb[q] + 1) << (16 * q);
        ekp |= (uint64_t)(uint32_t)(ek[q] + 1) << (16 * q);
    }
    __syncthreads();
    GS_TL(1);
    // ---- the current state of this l
    double dcur[NSP], vcur[4] = {0.0, 0.0, 0.0, 0.0}, fcur[NG];
#pragma unroll
    for (int s = 0; s < NSP; ++s) {
        dcur[s] = eb[s] < 0 ? 0.0 : Ds[s * maxbins + eb[s]];
        vcur[s] = var_from_dl(dcur[s], l);
    }
    fcur[0] = f_part<F>(sv, b, k0, k1, k2, 0, vcur[0], vcur[1], vcur[2], vcur[3]);
    if constexpr (NG > 1) fcur[NG - 1] = f_part<F>(sv, b, k0, k1, k2, F == 3 ? 2 : 1, vcur[0], vcur[1], vcur[2], vcur[3]);
    bool okcur = true;
    if constexpr (F == 3) okcur = psd_ok(vcur[0], vcur[1], vcur[3]);
    for (int q = 0; q < ph.nphase; ++q) {
        // the phase's scalars picked with constant indices (a runtime index into
        // the by-value kernel argument would copy it to scratch in every thread)
        const int nb = mh_pick(ph.n, q);
        if (nb == 0) continue;
        const int sp0 = mh_pick(ph.sp0, q), sp1 = mh_pick(ph.sp1, q);
        const int off = mh_pick(ph.off, q);
        const int2* tab = tabs + off;
        const int4* rng = rngs + off;
        const int nwide = mh_pick(ph.nwide, q);
        // per-l likelihood differences of the phase's proposals on their own parts
        double pvk[2] = {0.0, 0.0}, fnk[2] = {0.0, 0.0};
        bool okk[2] = {false, false};
        if (lok) {
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int sp = k == 0 ? sp0 : sp1;
                if (sp < 0) continue;
                double out = 0.0;
                if (unpack16(ekp, sp) >= 0) {
                    const double pv = var_from_dl(Ps[sp * maxbins + unpack16(ebp, sp)], l);
                    double vn[4] = {vcur[0], vcur[1], vcur[2], vcur[3]};
#pragma unroll
                    for (int s = 0; s < NSP; ++s) vn[s] = s == sp ? pv : vn[s];
                    bool ok = true;
                    if constexpr (F == 3) ok = sp == 2 ? okcur : psd_ok(vn[0], vn[1], vn[3]);
                    const double fn = ok ? f_part<F>(sv, b, k0, k1, k2, sp, vn[0], vn[1], vn[2], vn[3]) : 0.0;
                    const double fo = NG > 1 && f_group<F>(sp) == 1 ? fcur[NG - 1] : fcur[0];
                    out = ok ? fn - fo : -INFINITY;
                    pvk[k] = pv; fnk[k] = fn; okk[k] = ok;
                }
                g[k * Lp1 + l] = out;
            }
        }
        __syncthreads();
        GS_TL(2 + 4 * q);
        // narrow blocks: one thread each
        for (int j = nwide + tid; j < nb; j += blockDim.x) {
            const int2 sb = tab[j];
            const int4 r = rng[j];
            const int sp = sb.x, blk = sb.y, k = sp == sp0 ? 0 : 1;
            const int lo = r.x, hi = r.y, l0 = r.z, l1 = r.w;
            GS_ASSERT(lo >= 0 && hi <= maxbins && l0 >= 0 && l1 <= Lp1);
            double diff = 0.0, lrs = 0.0;
            for (int ll = l0; ll < l1; ++ll) diff += g[k * Lp1 + ll];
            for (int bb = lo; bb < hi; ++bb) lrs += Rs[sp * maxbins + bb];
            bool taken = false;
            const int flat0 = s_ao[sp] + blk * n_iter_mh;
            for (int att = 0; att < n_iter_mh; ++att) {
                const bool acc = lu[flat0 + att] < (taken ? 0.0 : diff) + lrs;
                if (acc && !taken)
                    for (int bb = lo; bb < hi; ++bb) Ds[sp * maxbins + bb] = Ps[sp * maxbins + bb];
                taken = taken || acc;
                if (accept_out) accept_out[(long long)chain * nacc + flat0 + att] = acc ? 1 : 0;
            }
        }
        GS_TL(3 + 4 * q);
        // wide blocks: one wave each (lane-strided sums in l / bin order with
        // eight loads in flight, then the fixed-order butterfly), decided and
        // applied by that wave
        for (int j = wv; j < nwide; j += nwv) {
            const int2 sb = tab[j];
            const int4 r = rng[j];
            const int sp = sb.x, blk = sb.y, k = sp == sp0 ? 0 : 1;
            double diff = lane_strided_sum<8>(g + k * Lp1, r.z, r.w, lane);
            double lrs = lane_strided_sum<8>(Rs + sp * maxbins, r.x, r.y, lane);
            diff = wave_sum_bcast(diff);
            lrs = wave_sum_bcast(lrs);
            bool taken = false;
            const int flat0 = s_ao[sp] + blk * n_iter_mh;
            for (int att = 0; att < n_iter_mh; ++att) {
                const bool acc = lu[flat0 + att] < (taken ? 0.0 : diff) + lrs;
                taken = taken || acc;
                if (accept_out && lane == 0) accept_out[(long long)chain * nacc + flat0 + att] = acc ? 1 : 0;
            }
            if (taken)
                for (int bb = r.x + lane; bb < r.y; bb += 64) Ds[sp * maxbins + bb] = Ps[sp * maxbins + bb];
        }
        GS_TL(4 + 4 * q);
        __syncthreads();
        GS_TL(5 + 4 * q);
        // take the accepted proposals into this l's state
        if (lok) {
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int sp = k == 0 ? sp0 : sp1;
                if (sp < 0 || !okk[k]) continue;
                const double d = Ds[sp * maxbins + unpack16(ebp, sp)];
                bool changed = false;
#pragma unroll
                for (int s = 0; s < NSP; ++s)
                    if (s == sp && d != dcur[s]) { dcur[s] = d; vcur[s] = pvk[k]; changed = true; }
                if (changed) {
                    if (NG > 1 && f_group<F>(sp) == 1) fcur[NG - 1] = fnk[k]; else fcur[0] = fnk[k];
                    if constexpr (F == 3) okcur = psd_ok(vcur[0], vcur[1], vcur[3]);
                }
            }
        }
    }
    for (int k = tid; k < nrow; k += blockDim.x)
        if ((ph.own >> (k / maxbins)) & 1) D[k] = Ds[k];
    GS_TL(20);
}

template <int F>
__global__ __launch_bounds__(MH_REG_THREADS) void k_mh_reg(int L, int maxbins, MhPhases ph, int ntab,
                                                           const int2* __restrict__ phase_tab,
                                                           const int4* __restrict__ phase_rng,
                                                           const int* __restrict__ meta, int nacc, int n_iter_mh,
                                                           const int* __restrict__ ell2blk,
                                                           const int* __restrict__ ell2bin,
                                                           const double* __restrict__ bl, double k0, double k1,
                                                           double k2, const double* __restrict__ stats,
                                                           double* __restrict__ dl, const double* __restrict__ prop,
                                                           const double* __restrict__ logr,
                                                           const double* __restrict__ u_acc, uint32_t seed_lo,
                                                           uint32_t seed_hi, IterArg itarg, int chain0,
                                                           int32_t* __restrict__ accept_out, MhEpi epi,
                                                           MhPhases ph1, int nsplit) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const uint32_t iter = itarg.get();
    // nsplit 2: workgroup 2c decides chain c's T / E phases, 2c + 1 its BB blocks
    const int chain = (int)blockIdx.x / nsplit, kind = (int)blockIdx.x % nsplit;
    const MhPhases phk = mh_select(kind != 0, ph, ph1);
    mh_reg_body<F>(chain, blockIdx.x == 0, L, maxbins, phk, ntab, phase_tab, phase_rng, meta, nacc, n_iter_mh, ell2blk,
                   ell2bin, bl, k0, k1, k2, stats, dl, prop, logr, u_acc, seed_lo, seed_hi, iter, chain0, accept_out,
                   smem, epi.dl_in);
    mh_epilogue(epi, iter, chain, (F == 1 ? 1 : (F == 2 ? 2 : 4)) * maxbins, dl, gridDim.x, maxbins, phk.own);
}

// stats of s_nc = A^+ s, A = chol(C(dl)) (ASIS.py:185-189)
// (pp.n front workgroups: the ASIS MH proposals from the same dl, ProPre)
template <int F>
__global__ void k_stats_to_nc(int L, int nchains, int maxbins, const double* __restrict__ dl,
                              const int* __restrict__ ell2bin, double* __restrict__ stats, ProPre pp,
                              uint32_t seed_lo, uint32_t seed_hi, IterArg itarg, int chain0) {
    if ((int)blockIdx.x < pp.n) {
        pro_pre_item<F>(pp, (int)blockIdx.x, nchains, seed_lo, seed_hi, itarg, chain0);
        return;
    }
    constexpr int NSP = F == 1 ? 1 : (F == 2 ? 2 : 4);
    constexpr int NS = SweepAcc<F>::NS;
    const int Lp1 = L + 1;
    const int g = ((int)blockIdx.x - pp.n) * blockDim.x + threadIdx.x;
    if (g >= nchains * Lp1) return;
    const int chain = g / Lp1, l = g % Lp1;
    const double* D = dl + (long long)chain * NSP * maxbins;
    double* st = stats + (long long)chain * NS * Lp1;
    if constexpr (F != 3) {
#pragma unroll
        for (int f = 0; f < F; ++f) {
            const double v = var_from_dl(dl_at(D, ell2bin, maxbins, Lp1, f, l), l);
            const double T = v != 0.0 ? sqrt(1.0 / v) : 0.0;
            st[f * Lp1 + l] *= T * T;
            st[(F + f) * Lp1 + l] *= T;
        }
    } else {
        const double tt = var_from_dl(dl_at(D, ell2bin, maxbins, Lp1, 0, l), l);
        const double ee = var_from_dl(dl_at(D, ell2bin, maxbins, Lp1, 1, l), l);
        const double bb = var_from_dl(dl_at(D, ell2bin, maxbins, Lp1, 2, l), l);
        const double te = var_from_dl(dl_at(D, ell2bin, maxbins, Lp1, 3, l), l);
        const CovChol A = cov_chol_teb(tt, ee, te, bb);
        const double i00 = A.a00 != 0.0 ? 1.0 / A.a00 : 0.0;
        const double i11 = A.a11 != 0.0 ? 1.0 / A.a11 : 0.0;
        const double t10 = -A.a10 * i00 * i11;
        const double iB = A.aB != 0.0 ? 1.0 / A.aB : 0.0;
        const double ssTT = st[0 * Lp1 + l], ssEE = st[1 * Lp1 + l], ssBB = st[2 * Lp1 + l], ssTE = st[3 * Lp1 + l];
        const double dTsT = st[4 * Lp1 + l], dEsT = st[5 * Lp1 + l], dEsE = st[6 * Lp1 + l], dBsB = st[7 * Lp1 + l];
        st[0 * Lp1 + l] = i00 * i00 * ssTT;
        st[1 * Lp1 + l] = t10 * t10 * ssTT + 2.0 * t10 * i11 * ssTE + i11 * i11 * ssEE;
        st[2 * Lp1 + l] = iB * iB * ssBB;
        st[3 * Lp1 + l] = i00 * t10 * ssTT + i00 * i11 * ssTE;
        st[4 * Lp1 + l] = dTsT * i00;
        st[5 * Lp1 + l] = dEsT * i00;
        st[6 * Lp1 + l] = dEsT * t10 + dEsE * i11;
        st[7 * Lp1 + l] = dBsB * iB;
    }
}

// s <- R_l s, R = A(C_new) [A(C_old)^+]
template <int F>
__global__ void k_recentre(int L, int nchains, int maxbins, const double* __restrict__ dl_new,
                           const double* __restrict__ dl_old, const int* __restrict__ ell2bin, double* __restrict__ s) {
    constexpr int NSP = F == 1 ? 1 : (F == 2 ? 2 : 4);
    const int Lp1 = L + 1;
    const long long nc = (long long)(L + 1) * (L + 2) / 2;
    const long long NR = (long long)(L + 1) * (L + 1);
    for (long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x; g < nc * nchains;
         g += (long long)gridDim.x * blockDim.x) {
        const int chain = (int)(g / nc);
        const long long i = g % nc;
        int l, m;
        complex_index_to_lm(L, i, l, m);
        const long long r = m == 0 ? (long long)l : 2 * i - (L + 1);
        const int nv = m == 0 ? 1 : 2;
        const double* Dn = dl_new + (long long)chain * NSP * maxbins;
        const double* Do = dl_old ? dl_old + (long long)chain * NSP * maxbins : nullptr;
        double* sc = s + (long long)chain * F * NR;
        if constexpr (F != 3) {
            for (int f = 0; f < F; ++f) {
                double R = sqrt(var_from_dl(dl_at(Dn, ell2bin, maxbins, Lp1, f, l), l));
                if (Do) {
                    const double v = var_from_dl(dl_at(Do, ell2bin, maxbins, Lp1, f, l), l);
                    R *= v != 0.0 ? sqrt(1.0 / v) : 0.0;
                }
                for (int c = 0; c < nv; ++c) sc[f * NR + r + c] *= R;
            }
        } else {
            const CovChol An = cov_chol_teb(var_from_dl(dl_at(Dn, ell2bin, maxbins, Lp1, 0, l), l),
                                            var_from_dl(dl_at(Dn, ell2bin, maxbins, Lp1, 1, l), l),
                                            var_from_dl(dl_at(Dn, ell2bin, maxbins, Lp1, 3, l), l),
                                            var_from_dl(dl_at(Dn, ell2bin, maxbins, Lp1, 2, l), l));
            double t00 = 1.0, t10 = 0.0, t11 = 1.0, tB = 1.0;
            if (Do) {
                const CovChol Ao = cov_chol_teb(var_from_dl(dl_at(Do, ell2bin, maxbins, Lp1, 0, l), l),
                                                var_from_dl(dl_at(Do, ell2bin, maxbins, Lp1, 1, l), l),
                                                var_from_dl(dl_at(Do, ell2bin, maxbins, Lp1, 3, l), l),
                                                var_from_dl(dl_at(Do, ell2bin, maxbins, Lp1, 2, l), l));
                t00 = Ao.a00 != 0.0 ? 1.0 / Ao.a00 : 0.0;
                t11 = Ao.a11 != 0.0 ? 1.0 / Ao.a11 : 0.0;
                t10 = -Ao.a10 * t00 * t11;
                tB = Ao.aB != 0.0 ? 1.0 / Ao.aB : 0.0;
            }
            const double r00 = An.a00 * t00;
            const double r10 = An.a10 * t00 + An.a11 * t10;
            const double r11 = An.a11 * t11;
            const double rB = An.aB * tB;
            for (int c = 0; c < nv; ++c) {
                const double sT = sc[0 * NR + r + c], sE = sc[1 * NR + r + c];
                sc[0 * NR + r + c] = r00 * sT;
                sc[1 * NR + r + c] = r10 * sT + r11 * sE;
                sc[2 * NR + r + c] *= rB;
            }
        }
    }
}

__global__ void k_iter_advance(uint32_t* it) { *it += 1u; }

// trace[(it - 1) % capacity] <- dl, it from the device counter (or host value)
__global__ void k_record_trace(long long n, const double* __restrict__ dl, double* __restrict__ trace, int capacity,
                               IterArg itarg) {
    const uint32_t it = itarg.get();
    const long long slot = (long long)((it + capacity - 1u) % (uint32_t)capacity);
    for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < n; k += (long long)gridDim.x * blockDim.x)
        trace[slot * n + k] = dl[k];
}

// ============================================================================
// host side
// ============================================================================
// the library options (gs_option_set): a fixed set of names
static const char* const k_options[] = {
    "GS_SWEEP_TW", "GS_SWEEP_THROUGHPUT", "GS_MH_SPLIT", "GS_CLS_PRE", "GS_CLS_PRE_MANY", "GS_F2_GROUP_BYTES",
    "GS_F2_BATCH_BYTES", "GS_SHT_LDS_FFT_MAX", "GS_SHT_SEG", "GS_SHT_SYN", "GS_SHT_ANA", "GS_SHT_MERGE_RINGS",
    "GS_SHT_CONST_RINGS", "GS_SHT_BLOCKS_MFMA", "GS_SHT_BLK_STAGE", "GS_SHT_FUSED_AUX", "GS_SHT_MFMA_MAX_GB",
    "GS_SHT_RING_TW2"};
static bool opt_known(const char* name) {
    for (const char* k : k_options)
        if (std::strcmp(k, name) == 0) return true;
    return false;
}
static std::mutex& opt_mu() { static std::mutex m; return m; }
static std::map<std::string, std::string>& opt_tab() { static std::map<std::string, std::string> t; return t; }

const char* gs_detail::option(const char* name) {
    std::lock_guard<std::mutex> g(opt_mu());
    const auto it = opt_tab().find(name);
    // the map's nodes are stable: the pointer stays valid until the option is reset
    return it == opt_tab().end() ? nullptr : it->second.c_str();
}

namespace {

template <typename T>
int dev_upload(T** dst, const std::vector<T>& src) {
    if (src.empty()) { *dst = nullptr; return 0; }
    GS_CHECK(hipMalloc((void**)dst, src.size() * sizeof(T)));
    GS_CHECK(hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
    return 0;
}

template <typename T>
int dev_alloc(T** dst, size_t n) {
    GS_CHECK(hipMalloc((void**)dst, std::max<size_t>(n, 1) * sizeof(T)));
    GS_CHECK(hipMemset(*dst, 0, std::max<size_t>(n, 1) * sizeof(T)));
    return 0;
}

inline hipStream_t S(void* s) { return (hipStream_t)s; }
inline unsigned nblk(long long n, int bs) { return (unsigned)std::max<long long>(1, std::min<long long>((n + bs - 1) / bs, 1 << 20)); }

void build_tasks(gs_plan* p) {
    const int L = p->L;
    p->ntile = (L + 1 + WAVE - 1) / WAVE;
    auto waves = [&](int tm) {
        long long n = 0;
        for (int t = 0; t < p->ntile; ++t) n += (L - WAVE * t) / tm + 1;
        return n;
    };
    // rows per chunk: fixed (independent of the chain count), so the fixed-order
    // statistic sums -- and therefore every chain's trajectory -- are bit-identical
    // whatever the batch size or GPU count; a function of L only.  Measured with
    // tools/step_ab.py (whole graph-captured steps, interleaved in one process),
    // r02 with the workgroup-per-tile statistics finish: NC TEB 32 chains at
    // L 1024: 12 / 16 / 20 / 24 rows 308.5 / 308.5 / 312.0 / 319.3 us per step;
    // centered 1 chain at L 512: 2 / 4 / 8 rows 25.7 / 22.4 / 26.0 us
    const int tm = L > 512 ? 16 : (L > 256 ? 4 : 8);
    p->rows_per_task = tm;
    p->nchunk = L / tm + 1;
    p->ntask = (int)waves(tm);
    // workgroup shape: 2 tiles x 2 chunks (r03; each row one 2 KiB run per
    // field, the two chunks' statistic sums added in LDS: half the partial
    // bytes of 4 tiles x 1 chunk): NC TEB 32 chains at L 1024, whole steps
    // interleaved in one process (tools/step_ab.py), 289.6-291.4 against
    // 294.3 us.  1 tile x 4 chunks (a quarter of the partials, 1 KiB runs)
    // measured slower there in r02 (sweep 282-294 vs 261-281 us), but short
    // tasks (the latency form, few chains) take it: their finish is a chain of
    // memory latencies, one per group of chunk partials it reads.
    // r05, after the sweep's per-row instruction count fell (406 -> 379) and the
    // MH lost its scratch copies, 1 x 4 is the faster shape for many chains too:
    // NC TEB 32 chains at L 1024 212.2-212.7 against 215.2-215.8 us per step,
    // ASIS 225.5 against 231.4 (tools/step_ab.py; 16 rows per task stays best
    // with either shape: 12 / 20 / 24 / 32 rows 220.1 / 220.3 / 221.9 / 221.1).
    // option GS_SWEEP_TW = 1 | 2 | 4 overrides (the stored-map line: 2).
    int tw = 1;
    if (const char* env = gs_detail::option("GS_SWEEP_TW")) {
        const int v = atoi(env);
        if (v == 1 || v == 2 || v == 4) tw = v;
    }
    const int cw = 4 / tw;
    p->sweep_tw = tw;
    p->nchunkg = (p->nchunk + cw - 1) / cw;
    // (tile group, chunk group) pairs, with their work in active lane-rows
    std::vector<std::pair<long long, int2>> work;
    for (int g = 0; tw * g < p->ntile; ++g)
        for (int c = 0; c * cw * tm <= L - WAVE * tw * g; ++c) {
            long long wl = 0;
            for (int t = tw * g; t < std::min(tw * g + tw, p->ntile); ++t) {
                const int lhi = L - WAVE * t, lo = std::max(lhi - 63, 0);
                for (int m = c * cw * tm; m < std::min((c + 1) * cw * tm, lhi + 1); ++m)
                    wl += lhi - std::max(lo, m) + 1;
            }
            work.push_back({wl, make_int2(g, c)});
        }
    // the sweep gives XCD x a contiguous range of pairs (all chains of a pair on
    // one XCD); deal the pairs heaviest-first over 8 buckets so every XCD gets
    // the same work, padding with empty pairs (g = -1) to a multiple of 8
    std::stable_sort(work.begin(), work.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
    const int per = (int)((work.size() + 7) / 8);
    std::vector<std::vector<int2>> bucket(8);
    std::vector<long long> load(8, 0);
    for (const auto& w : work) {
        int best = -1;
        for (int x = 0; x < 8; ++x)
            if ((int)bucket[x].size() < per && (best < 0 || load[x] < load[best])) best = x;
        bucket[best].push_back(w.second);
        load[best] += w.first;
    }
    std::vector<int2> tasks;
    for (int x = 0; x < 8; ++x) {
        for (const int2& t : bucket[x]) tasks.push_back(t);
        for (int k = (int)bucket[x].size(); k < per; ++k) tasks.push_back(make_int2(-1, 0));
    }
    p->npair = (int)tasks.size();
    dev_upload(&p->tasks, tasks);
}

int check_plan(const gs_plan* p) {
    if (!p) return set_error("null plan");
    return 0;
}

}  // namespace

extern "C" {

int gs_abi_version(void) { return GS_ABI_VERSION; }
const char* gs_last_error(void) { return gs_detail::g_last_error.c_str(); }

int gs_option_set(const char* name, const char* value) {
    if (!name || !opt_known(name)) return set_error(std::string("gs_option_set: unknown option ") + (name ? name : "(null)"));
    std::lock_guard<std::mutex> g(opt_mu());
    if (value) opt_tab()[name] = value; else opt_tab().erase(name);
    return 0;
}

const char* gs_option_get(const char* name) { return name ? gs_detail::option(name) : nullptr; }

int gs_plan_create(const gs_model_desc* desc, gs_plan** out) {
    if (!desc || !out) return set_error("gs_plan_create: null argument");
    const int L = desc->lmax, F = desc->nfields;
    if (L < 2 || L > 16384) return set_error("gs_plan_create: lmax out of range");
    if (F < 1 || F > 3) return set_error("gs_plan_create: nfields must be 1, 2 or 3");
    if (desc->nchains < 1) return set_error("gs_plan_create: nchains < 1");
    if (!desc->bl || !desc->noise_var) return set_error("gs_plan_create: bl / noise_var required");
    gs_plan* p = new gs_plan();
    GS_CHECK(hipGetDevice(&p->device));
    p->L = L; p->F = F; p->nside = desc->nside; p->Npix = 12 * desc->nside * desc->nside;
    p->nchains = desc->nchains; p->chain0 = desc->chain0; p->quirks = desc->quirks;
    p->n_iter_mh = std::max(1, desc->n_iter_metropolis);
    p->nspec = nspec_of(F); p->nstat = nstat_of(F);
    for (int f = 0; f < F; ++f) {
        if (!(desc->noise_var[f] > 0)) { delete p; return set_error("noise_var must be > 0"); }
        p->kappa[f] = (double)p->Npix / (4.0 * PI * desc->noise_var[f]);
    }
    int maxbins = 0;
    for (int sp = 0; sp < p->nspec; ++sp) {
        if (!desc->bins[sp] || desc->nbin_edges[sp] < 2) { delete p; return set_error("bins required for every spectrum"); }
        p->nbins[sp] = desc->nbin_edges[sp] - 1;
        maxbins = std::max(maxbins, p->nbins[sp]);
        const int* e = desc->bins[sp];
        for (int i = 0; i + 1 < desc->nbin_edges[sp]; ++i)
            if (e[i] < 0 || e[i + 1] < e[i] || e[i + 1] > L + 1) { delete p; return set_error("invalid bin edges"); }
    }
    p->maxbins = maxbins;
    if (F == 3) {
        for (int sp : {1, 3}) {
            if (p->nbins[sp] != p->nbins[0] ||
                !std::equal(desc->bins[sp], desc->bins[sp] + desc->nbin_edges[sp], desc->bins[0])) {
                delete p;
                return set_error("TEB: TT, EE and TE must share bins (inverse-Wishart draw)");
            }
        }
    }
    std::vector<double> bl(desc->bl, desc->bl + L + 1);
    std::vector<int> ell2bin((size_t)p->nspec * (L + 1), -1), bins((size_t)p->nspec * (maxbins + 1), 0),
        blocks((size_t)p->nspec * (maxbins + 1), 0);
    std::vector<double> psd((size_t)p->nspec * maxbins, 0.0);
    p->has_mh = true;
    int off = 0;
    if (F == 3) { p->mh_order[0] = 1; p->mh_order[1] = 2; p->mh_order[2] = 0; p->mh_order[3] = 3; }
    for (int sp = 0; sp < p->nspec; ++sp) {
        const int* e = desc->bins[sp];
        for (int i = 0; i <= p->nbins[sp]; ++i) bins[sp * (maxbins + 1) + i] = e[i];
        for (int i = 0; i < p->nbins[sp]; ++i)
            for (int l = e[i]; l < e[i + 1]; ++l) ell2bin[sp * (L + 1) + l] = i;
        if (desc->blocks[sp] && desc->nblock_edges[sp] >= 2) {
            p->nblocks[sp] = desc->nblock_edges[sp] - 1;
            for (int i = 0; i <= p->nblocks[sp]; ++i)
                blocks[sp * (maxbins + 1) + i] = std::min(std::max(desc->blocks[sp][i], 0), p->nbins[sp]);
        } else {
            p->has_mh = false;
        }
        if (desc->prop_var[sp]) {
            for (int b = 2; b < p->nbins[sp]; ++b) psd[sp * maxbins + b] = std::sqrt(desc->prop_var[sp][b - 2]);
        } else {
            p->has_mh = false;
        }
    }
    for (int oi = 0; oi < p->nspec; ++oi) {
        const int sp = p->mh_order[oi];
        p->acc_off[sp] = off;
        off += p->nblocks[sp] * p->n_iter_mh;
    }
    p->nacc = off;
    // phases: F=1 [TT]; F=2 [EE, BB]; F=3 [EE, BB], [TT], [TE] (BB shares no
    // likelihood term with T/E; EE, TT, TE all enter the TE block)
    std::vector<std::vector<int>> phases;
    if (F == 1) phases = {{0}};
    else if (F == 2) phases = {{0, 1}};
    else phases = {{1, 2}, {0}, {3}};
    std::vector<int2> ptab;
    std::vector<int4> prng;
    int lmin = L + 1;
    p->nphase = (int)phases.size();
    for (int ph = 0; ph < p->nphase; ++ph) {
        p->phase_off[ph] = (int)ptab.size();
        for (size_t q = 0; q < phases[ph].size(); ++q) p->phase_sp[ph][q] = phases[ph][q];
        // wide blocks (> MH_SMALL multipoles, one wave each in k_mh_fused) first
        for (int pass = 0; pass < 2; ++pass)
            for (int sp : phases[ph])
                for (int b = 0; b < p->nblocks[sp]; ++b) {
                    const int lo = blocks[sp * (maxbins + 1) + b], hi = blocks[sp * (maxbins + 1) + b + 1];
                    const int l0 = hi > lo ? bins[sp * (maxbins + 1) + lo] : 0;
                    const int l1 = hi > lo ? bins[sp * (maxbins + 1) + hi] : 0;
                    if ((l1 - l0 > MH_SMALL) != (pass == 0)) continue;
                    ptab.push_back(make_int2(sp, b));
                    prng.push_back(make_int4(lo, hi, l0, l1));
                    if (pass == 0) p->phase_nwide[ph]++;
                    if (hi > lo) lmin = std::min(lmin, l0);
                }
        p->phase_n[ph] = (int)ptab.size() - p->phase_off[ph];
    }
    p->mh_lmin = std::min(lmin, L);
    // the split form's tables: kind 0 the T / E phases ([EE] [TT] [TE] or [EE]),
    // kind 1 [BB]; the same entries in the same order per spectrum
    std::vector<int2> stab;
    std::vector<int4> srng;
    if (F >= 2) {
        const std::vector<std::vector<std::vector<int>>> kinds =
            F == 2 ? std::vector<std::vector<std::vector<int>>>{{{0}}, {{1}}}
                   : std::vector<std::vector<std::vector<int>>>{{{1}, {0}, {3}}, {{2}}};
        for (int k = 0; k < 2; ++k) {
            p->sph_n[k] = (int)kinds[k].size();
            for (int ph = 0; ph < p->sph_n[k]; ++ph) {
                p->sph_off[k][ph] = (int)stab.size();
                p->sph_nwide[k][ph] = 0;
                p->sph_sp[k][ph][0] = kinds[k][ph][0];
                p->sph_sp[k][ph][1] = -1;
                const int sp = kinds[k][ph][0];
                p->sph_own[k] |= 1 << sp;
                for (int pass = 0; pass < 2; ++pass)
                    for (int b = 0; b < p->nblocks[sp]; ++b) {
                        const int lo = blocks[sp * (maxbins + 1) + b], hi = blocks[sp * (maxbins + 1) + b + 1];
                        const int l0 = hi > lo ? bins[sp * (maxbins + 1) + lo] : 0;
                        const int l1 = hi > lo ? bins[sp * (maxbins + 1) + hi] : 0;
                        if ((l1 - l0 > MH_SMALL) != (pass == 0)) continue;
                        stab.push_back(make_int2(sp, b));
                        srng.push_back(make_int4(lo, hi, l0, l1));
                        if (pass == 0) p->sph_nwide[k][ph]++;
                    }
                p->sph_cnt[k][ph] = (int)stab.size() - p->sph_off[k][ph];
            }
        }
        // the T / E workgroup also owns the rows of no MH spectrum (none for F >= 2)
        p->ntab_s = (int)stab.size();
        const char* e = gs_detail::option("GS_MH_SPLIT");
        p->mh_split = e ? std::atoi(e) != 0 : true;
    }
    int rc = 0;
    if (!stab.empty()) { rc |= dev_upload(&p->phase_tab_s, stab); rc |= dev_upload(&p->phase_rng_s, srng); }
    rc |= dev_upload(&p->bl, bl);
    rc |= dev_upload(&p->ell2bin, ell2bin);
    rc |= dev_upload(&p->bins, bins);
    rc |= dev_upload(&p->blocks, blocks);
    rc |= dev_upload(&p->prop_sd, psd);
    std::vector<int> meta(16, 0);
    for (int k = 0; k < 4; ++k) {
        meta[k] = p->nbins[k]; meta[4 + k] = p->nblocks[k]; meta[8 + k] = p->acc_off[k]; meta[12 + k] = p->mh_order[k];
    }
    rc |= dev_upload(&p->meta, meta);
    rc |= dev_upload(&p->phase_tab, ptab);
    rc |= dev_upload(&p->phase_rng, prng);
    std::vector<int> e2k((size_t)p->nspec * (L + 1), -1);
    for (int sp = 0; sp < p->nspec; ++sp)
        for (int b = 0; b < p->nblocks[sp]; ++b) {
            const int lo = blocks[sp * (maxbins + 1) + b], hi = blocks[sp * (maxbins + 1) + b + 1];
            if (hi <= lo) continue;
            for (int l = desc->bins[sp][lo]; l < desc->bins[sp][hi]; ++l) e2k[sp * (L + 1) + l] = b;
        }
    rc |= dev_upload(&p->ell2blk, e2k);
    rc |= dev_alloc(&p->gbuf, (size_t)p->nchains * 2 * (L + 1));
    build_tasks(p);
    // many chains: the parameter table by the prologue (r05: every sweep lane
    // computing its operator measured 231.8 against 223.8 us per NC step at
    // configs[2]); few chains: in the sweep, no parameter launch
    p->inkernel_params = p->nchains <= 4;
    p->sweep_latency = gs_detail::option("GS_SWEEP_THROUGHPUT") == nullptr;
    const size_t nc = (size_t)p->nchains;
    rc |= dev_alloc(&p->partials, nc * p->ntile * p->nchunkg * p->nstat * WAVE);
    rc |= dev_alloc(&p->params, nc * (L + 1) * NP);
    rc |= dev_alloc(&p->stats, nc * p->nstat * (L + 1));
    rc |= dev_alloc(&p->prop, nc * p->nspec * maxbins);
    rc |= dev_alloc(&p->logr, nc * p->nspec * maxbins);
    rc |= dev_alloc(&p->dl_tmp, nc * p->nspec * maxbins);
    rc |= dev_alloc(&p->u_nat, nc * std::max(p->nacc, 1));
    rc |= dev_alloc(&p->iter_dev, 4);
    {
        const char* e = gs_detail::option("GS_CLS_PRE");
        p->cls_pre = e ? std::atoi(e) != 0 : p->nchains <= 4;
    }
    {
        const char* e = gs_detail::option("GS_CLS_PRE_MANY");
        p->cls_pre_many = !p->cls_pre && (e ? std::atoi(e) != 0 : true);
    }
    if (p->cls_pre || p->cls_pre_many) rc |= dev_alloc(&p->cls_var, nc * p->nspec * maxbins * 3);
    if (rc) { gs_plan_destroy(p); return -1; }
    *out = p;
    return 0;
}

int gs_plan_destroy(gs_plan* p) {
    if (!p) return 0;
    void* bufs[] = {p->iter_dev, p->ell2blk, p->gbuf, p->phase_tab, p->phase_rng, p->meta, p->bl, p->ell2bin, p->bins, p->blocks, p->prop_sd, p->tasks, p->partials, p->u_nat,
                    p->params, p->stats, p->prop, p->logr, p->dl_tmp, p->cls_var, p->phase_tab_s, p->phase_rng_s};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    for (hipEvent_t e : p->ev) (void)hipEventDestroy(e);
    delete p;
    return 0;
}

int gs_plan_info(const gs_plan* p, int* maxbins, int* nstat, int* nblocks_total, int* nspec) {
    if (check_plan(p)) return -1;
    if (maxbins) *maxbins = p->maxbins;
    if (nstat) *nstat = p->nstat;
    if (nblocks_total) *nblocks_total = p->nacc;
    if (nspec) *nspec = p->nspec;
    return 0;
}

int gs_plan_sweep_info(const gs_plan* p, int* ntask, int* rows_per_task) {
    if (check_plan(p)) return -1;
    if (ntask) *ntask = p->ntask;
    if (rows_per_task) *rows_per_task = p->rows_per_task;
    return 0;
}

// ---- stand-alone helpers ----------------------------------------------------
// stateless helpers: lmax >= 0, n >= 0 (n == 0: nothing to do), non-null buffers
static int check_lmax_n(const char* fn, int lmax, int n, const void* a, const void* b) {
    if (lmax < 0 || n < 0) return set_error(std::string(fn) + ": lmax / n out of range");
    if (n > 0 && (!a || !b)) return set_error(std::string(fn) + ": null argument");
    return 0;
}

int gs_var_expand(int lmax, int n, const double* dl, double* var, void* stream) {
    if (check_lmax_n("gs_var_expand", lmax, n, dl, var)) return -1;
    if (n == 0) return 0;
    const long long nc = (long long)(lmax + 1) * (lmax + 2) / 2 * n;
    hipLaunchKernelGGL(k_var_expand, dim3(nblk(nc, 256)), dim3(256), 0, S(stream), lmax, n, dl, var);
    GS_LAUNCH_CHECK("k_var_expand");
    return 0;
}

int gs_real_to_complex(int lmax, int n, const double* re, double* cx, void* stream) {
    if (check_lmax_n("gs_real_to_complex", lmax, n, re, cx)) return -1;
    if (n == 0) return 0;
    const long long nc = (long long)(lmax + 1) * (lmax + 2) / 2 * n;
    hipLaunchKernelGGL(k_real_to_complex, dim3(nblk(nc, 256)), dim3(256), 0, S(stream), lmax, n, re, cx);
    GS_LAUNCH_CHECK("k_real_to_complex");
    return 0;
}

int gs_complex_to_real(int lmax, int n, const double* cx, double* re, void* stream) {
    if (check_lmax_n("gs_complex_to_real", lmax, n, cx, re)) return -1;
    if (n == 0) return 0;
    const long long nc = (long long)(lmax + 1) * (lmax + 2) / 2 * n;
    hipLaunchKernelGGL(k_complex_to_real, dim3(nblk(nc, 256)), dim3(256), 0, S(stream), lmax, n, cx, re);
    GS_LAUNCH_CHECK("k_complex_to_real");
    return 0;
}

int gs_remove_monopole_dipole(int lmax, int n, double* alm, void* stream) {
    if (check_lmax_n("gs_remove_monopole_dipole", lmax, n, alm, alm)) return -1;
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_remove_md, dim3(nblk(n, 64)), dim3(64), 0, S(stream), lmax, n, alm);
    GS_LAUNCH_CHECK("k_remove_md");
    return 0;
}

int gs_alm2cl(int lmax, int n, const double* x, const double* y, double* cl, void* stream) {
    if (check_lmax_n("gs_alm2cl", lmax, n, x, cl)) return -1;
    if (n == 0) return 0;
    const int ntile = (lmax + WAVE) / WAVE;
    const long long waves = (long long)n * ntile;
    hipLaunchKernelGGL(k_alm2cl, dim3(nblk(waves, 4)), dim3(256), 0, S(stream), lmax, n, x, y ? y : x, cl);
    GS_LAUNCH_CHECK("k_alm2cl");
    return 0;
}

int gs_unfold_bins(int n, const double* binned, const int* bins, int nbins, double* out, void* stream) {
    if (n < 0 || nbins < 0) return set_error("gs_unfold_bins: n / nbins out of range");
    if (n == 0 || nbins == 0) return 0;
    if (!binned || !bins || !out) return set_error("gs_unfold_bins: null argument");
    hipLaunchKernelGGL(k_unfold, dim3(nblk(nbins, 256), n), dim3(256), 0, S(stream), n, binned, bins, nbins, out);
    GS_LAUNCH_CHECK("k_unfold");
    return 0;
}

// ---- plan stages -----------------------------------------------------------------
int gs_block_params(gs_plan* p, int mode, const double* dl, double* params, void* stream) {
    if (check_plan(p)) return -1;
    if (!dl || !params) return set_error("gs_block_params: null argument");
    const long long n = (long long)p->nchains * (p->L + 1);
    const dim3 g(nblk(n, 256)), b(256);
#define GS_BP(FF, MM) hipLaunchKernelGGL((k_block_params<FF, MM>), g, b, 0, S(stream), p->L, p->nchains, p->maxbins, dl, \
                                         p->ell2bin, p->bl, p->kappa[0], p->kappa[1], p->kappa[2], params)
    if (mode == GS_MODE_CENTERED) {
        if (p->F == 1) GS_BP(1, 0); else if (p->F == 2) GS_BP(2, 0); else GS_BP(3, 0);
    } else if (mode == GS_MODE_NONCENTERED) {
        if (p->F == 1) GS_BP(1, 1); else if (p->F == 2) GS_BP(2, 1); else GS_BP(3, 1);
    } else {
        return set_error("gs_block_params: bad mode");
    }
#undef GS_BP
    GS_LAUNCH_CHECK("k_block_params");
    return 0;
}

// an event record that also works while the stream is being captured into a
// hipGraph (then it becomes an external event-record node, timed at replay)
static int record_ev(hipEvent_t e, hipStream_t s) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    hipGraph_t graph = nullptr;
    const hipGraphNode_t* deps = nullptr;
    size_t ndeps = 0;
    GS_CHECK(hipStreamGetCaptureInfo_v2(s, &cs, &id, &graph, &deps, &ndeps));
    if (cs != hipStreamCaptureStatusActive) {
        GS_CHECK(hipEventRecord(e, s));
        return 0;
    }
    // capturing: add an event-record node after the stream's current frontier
    hipGraphNode_t node = nullptr;
    GS_CHECK(hipGraphAddEventRecordNode(&node, graph, deps, ndeps, e));
    GS_CHECK(hipStreamUpdateCaptureDependencies(s, &node, 1, hipStreamSetCaptureDependencies));
    return 0;
}

static int timing_begin(gs_plan* p, hipStream_t s, hipEvent_t* e0, hipEvent_t* e1) {
    if (!p->timing) return 0;
    if (p->ev_used + 2 > p->ev.size()) {
        // timing-only events: no system-scope fence at record (a fence per
        // record writes back and invalidates the caches -- ~6 us between the
        // graph's kernels and a slower next kernel); read after a device sync
        for (int k = 0; k < 64; ++k) {
            hipEvent_t e;
            GS_CHECK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
            p->ev.push_back(e);
        }
    }
    *e0 = p->ev[p->ev_used];
    *e1 = p->ev[p->ev_used + 1];
    p->ev_used += 2;
    return record_ev(*e0, s);
}

static int stats_finish(gs_plan* p, double* stats, void* stream) {
    const long long n = (long long)p->nchains * p->nstat * p->ntile;
    if (p->pro_pending) {
        // the prologue's deferred draws in front of the partial sums
        p->pro_pending = false;
        const int nbp = nblk((long long)p->nchains * p->nspec * p->maxbins, 256);
        const int nbu = p->u_nat_ready ? nblk((long long)p->nchains * p->nacc, 256) : 0;
        const int tmf = p->rows_per_task * (4 / p->sweep_tw);
#define GS_FP(FF, GG) hipLaunchKernelGGL((k_stats_finish_pro<FF, GG>), dim3((unsigned)(n + nbp + nbu)), dim3(256), 0,   \
                                         S(stream), p->L, p->nchains, p->ntile, p->nchunkg, tmf, p->nstat, p->partials, \
                                         stats, nbp, nbu, p->u_nat, p->nspec, p->nacc, p->n_iter_mh, p->maxbins,        \
                                         p->meta, p->prop_sd, p->pro_dl, p->prop, p->logr, p->pro_slo, p->pro_shi,      \
                                         p->ita(p->pro_it), p->chain0, p->dl_tmp)
#define GS_FPG(FF) do { if (p->nchains <= 4) GS_FP(FF, 16); else GS_FP(FF, 4); } while (0)
        if (p->F == 1) GS_FPG(1); else if (p->F == 2) GS_FPG(2); else GS_FPG(3);
#undef GS_FPG
#undef GS_FP
        GS_LAUNCH_CHECK("k_stats_finish_pro");
        p->snap_ok = true;
        return 0;
    }
    if (p->nchains <= 4)
        hipLaunchKernelGGL(k_stats_finish<16>, dim3((unsigned)n), dim3(256), 0, S(stream), p->L, p->nchains, p->ntile,
                           p->nchunkg, p->rows_per_task * (4 / p->sweep_tw), p->nstat, p->partials, stats);
    else
        hipLaunchKernelGGL(k_stats_finish<4>, dim3((unsigned)n), dim3(256), 0, S(stream), p->L, p->nchains, p->ntile,
                           p->nchunkg, p->rows_per_task * (4 / p->sweep_tw), p->nstat, p->partials, stats);
    GS_LAUNCH_CHECK("k_stats_finish");
    return 0;
}

static int sweep_launch(gs_plan* p,const double* d_alm, const double* params, const double* z, uint64_t seed,
                        uint32_t iteration, uint32_t substep, double* s_out, double* stats, bool given,
                        void* stream, bool finish = true, int pmode = -1, const double* dl = nullptr,
                        bool* cls_pre_done = nullptr) {
    if (check_plan(p)) return -1;
    if (!d_alm || !stats || (!given && !params && pmode < 0) || (given && !s_out) || (pmode >= 0 && !dl))
        return set_error("gs_cr_sweep: null argument");
    const SweepOp op{pmode, p->maxbins, dl, p->ell2bin, p->bl, p->kappa[0], p->kappa[1], p->kappa[2]};
    const uint32_t slo = (uint32_t)(seed & 0xFFFFFFFFu), shi = (uint32_t)(seed >> 32);
    const int nlog = (int)((long long)p->nchains * p->npair);
    dim3 g((unsigned)nlog), b(256);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (timing_begin(p, S(stream), &e0, &e1)) return -1;
    const bool rep = z != nullptr, st = s_out != nullptr;
    // latency form (all loads first) for few chains with short tasks; the
    // throughput form otherwise (more chains: its registers buy occupancy)
    const bool lat = pmode >= 0 && p->rows_per_task <= 4 && !given && !rep && p->sweep_latency;
    const ClsPre none{};
    if (cls_pre_done) *cls_pre_done = false;
    if (lat) {
        ClsPre cp{};
        if (cls_pre_done && p->cls_pre) {
            cp.nspec = p->nspec; cp.maxbins = p->maxbins; cp.bins = p->bins; cp.nbins = p->meta; cp.out = p->cls_var;
            cp.nitem = p->nchains * p->nspec * p->maxbins;
            cp.n = (cp.nitem + 255) / 256;
            g.x += cp.n;
            *cls_pre_done = true;
        }
#define GS_SWL(FF, SS) hipLaunchKernelGGL((k_cr_sweep<FF, 0, SS, 4>), g, b, 0, S(stream), p->L, p->nchains, p->ntile, \
                                          p->nchunkg, p->rows_per_task, p->sweep_tw, p->tasks, d_alm, params, z,    \
                                          s_out, p->partials, slo, shi, p->ita(iteration), substep, p->chain0, op, cp, \
                                          ProPre{}, nlog)
#define GS_SWL2(FF) do { if (st) GS_SWL(FF, true); else GS_SWL(FF, false); } while (0)
        if (p->F == 1) GS_SWL2(1); else if (p->F == 2) GS_SWL2(2); else GS_SWL2(3);
#undef GS_SWL2
#undef GS_SWL
        GS_LAUNCH_CHECK("k_cr_sweep");
        if (p->timing && record_ev(e1, S(stream))) return -1;
        return finish ? stats_finish(p, stats, stream) : 0;
    }
    // the prologue's deferred MH draws in front of this sweep (native, same step)
    ProPre pp{};
    if (cls_pre_done && p->cls_pre_many && !rep && !given && p->cls_var) {
        // the C_l draw's variates in front workgroups (many chains, centered CR)
        pp.cp.nspec = p->nspec; pp.cp.maxbins = p->maxbins; pp.cp.bins = p->bins; pp.cp.nbins = p->meta;
        pp.cp.out = p->cls_var;
        pp.cp.nitem = p->nchains * p->nspec * p->maxbins;
        pp.nbv = (pp.cp.nitem + 255) / 256;
        *cls_pre_done = true;
    }
    if (p->pro_pending && !rep && !given && iteration == p->pro_it) {
        p->pro_pending = false;
        p->snap_ok = true;
        pp.nbp = nblk((long long)p->nchains * p->nspec * p->maxbins, 256);
        pp.nbu = p->u_nat_ready ? nblk((long long)p->nchains * p->nacc, 256) : 0;
        pp.nspec = p->nspec; pp.nacc = p->nacc; pp.n_iter_mh = p->n_iter_mh; pp.maxbins = p->maxbins;
        pp.nbins = p->meta; pp.prop_sd = p->prop_sd; pp.dl = p->pro_dl;
        pp.prop = p->prop; pp.logr = p->logr; pp.u_out = p->u_nat; pp.snap = p->dl_tmp;
    }
    pp.n = (pp.nbp + pp.nbu + pp.nbv + 7) / 8 * 8;
    g.x += pp.n;
#define GS_SW(FF, RR, SS) hipLaunchKernelGGL((k_cr_sweep<FF, RR, SS>), g, b, 0, S(stream), p->L, p->nchains, p->ntile, \
                                             p->nchunkg, p->rows_per_task, p->sweep_tw, p->tasks, d_alm, params, z,   \
                                             s_out,                                                                   \
                                             p->partials, slo, shi, p->ita(iteration), substep, p->chain0, \
                                             op, none, pp, nlog)
#define GS_SWF(FF) do { if (given) GS_SW(FF, 2, false); else if (rep && st) GS_SW(FF, 1, true); \
                        else if (rep) GS_SW(FF, 1, false); else if (st) GS_SW(FF, 0, true);            \
                        else GS_SW(FF, 0, false); } while (0)
    if (p->F == 1) GS_SWF(1); else if (p->F == 2) GS_SWF(2); else GS_SWF(3);
#undef GS_SWF
#undef GS_SW
    GS_LAUNCH_CHECK("k_cr_sweep");
    if (p->timing && record_ev(e1, S(stream))) return -1;
    return finish ? stats_finish(p, stats, stream) : 0;
}

int gs_cr_sweep(gs_plan* p, const double* d_alm, const double* params, const double* z, uint64_t seed,
                uint32_t iteration, uint32_t substep, double* s_out, double* stats, void* stream) {
    return sweep_launch(p, d_alm, params, z, seed, iteration, substep, s_out, stats, false, stream);
}

int gs_sweep_stats(gs_plan* p, const double* d_alm, const double* s, double* stats, void* stream) {
    return sweep_launch(p, d_alm, nullptr, nullptr, 0, 0, 0, const_cast<double*>(s), stats, true, stream);
}

static int cls_draw_launch(gs_plan* p, const double* stats, const double* variates, uint64_t seed,
                           uint32_t iteration, double* dl_out, double* trace, int cap, uint32_t* counter,
                           void* stream, const double* pre = nullptr) {
    if (check_plan(p)) return -1;
    if (!stats || !dl_out) return set_error("gs_cls_draw: null argument");
    const uint32_t slo = (uint32_t)(seed & 0xFFFFFFFFu), shi = (uint32_t)(seed >> 32);
    const dim3 g(p->nchains, p->nspec, (p->maxbins + 63) / 64), b(64);
#define GS_CD(FF) hipLaunchKernelGGL((k_cls_draw<FF>), g, b, 0, S(stream), p->L, p->nchains, p->maxbins, p->bins, p->meta, \
                                     stats, variates, slo, shi, p->ita(iteration), p->chain0, dl_out, trace, \
                                     cap, counter, p->graph_adv, pre)
    if (p->F == 1) GS_CD(1); else if (p->F == 2) GS_CD(2); else GS_CD(3);
#undef GS_CD
    GS_LAUNCH_CHECK("k_cls_draw");
    return 0;
}


int gs_cls_draw(gs_plan* p, const double* stats, const double* variates, uint64_t seed, uint32_t iteration,
                double* dl_out, void* stream) {
    return cls_draw_launch(p, stats, variates, seed, iteration, dl_out, nullptr, 1, nullptr, stream);
}

static int mh_decide(gs_plan* p, const double* stats, double* dl, const double* u_acc, uint32_t slo, uint32_t shi,
                     uint32_t iteration, int32_t* accept_out, void* stream, const MhEpi* epi = nullptr);

int gs_mh_propose(gs_plan* p, const double* dl, const double* u_prop, uint64_t seed, uint32_t iteration,
                  double* prop_out, double* logr_out, double* u_acc_out, void* stream) {
    if (check_plan(p)) return -1;
    if (!p->has_mh) return set_error("gs_mh_propose: plan has no MH blocks / proposal variances");
    if (!dl || !prop_out || !logr_out) return set_error("gs_mh_propose: null argument");
    const uint32_t slo = (uint32_t)(seed & 0xFFFFFFFFu), shi = (uint32_t)(seed >> 32);
    const long long nprop = (long long)p->nchains * p->nspec * p->maxbins;
    GS_CHECK(hipMemsetAsync(prop_out, 0, nprop * sizeof(double), S(stream)));
    GS_CHECK(hipMemsetAsync(logr_out, 0, nprop * sizeof(double), S(stream)));
#define GS_MP(FF) hipLaunchKernelGGL((k_mh_propose<FF>), dim3(nblk(nprop, 256)), dim3(256), 0, S(stream), p->nchains, \
                                     p->maxbins, p->meta, p->prop_sd, dl, prop_out, logr_out, u_prop, slo, shi,     \
                                     p->ita(iteration), p->chain0, nullptr)
    if (p->F == 1) GS_MP(1); else if (p->F == 2) GS_MP(2); else GS_MP(3);
#undef GS_MP
    GS_LAUNCH_CHECK("k_mh_propose");
    if (u_acc_out) {
        const long long n = (long long)p->nchains * p->nacc;
        hipLaunchKernelGGL(k_mh_uniforms, dim3(nblk(n, 256)), dim3(256), 0, S(stream), p->nchains, p->nspec,
                           p->maxbins, p->meta, p->nacc, p->n_iter_mh, slo, shi, p->ita(iteration),
                           p->chain0, u_acc_out);
        GS_LAUNCH_CHECK("k_mh_uniforms");
    }
    return 0;
}

int gs_nc_mh(gs_plan* p, const double* stats, double* dl, const double* u_prop, const double* u_acc, uint64_t seed,
             uint32_t iteration, int32_t* accept_out, void* stream) {
    if (check_plan(p)) return -1;
    if (!p->has_mh) return set_error("gs_nc_mh: plan has no MH blocks / proposal variances");
    if (!stats || !dl) return set_error("gs_nc_mh: null argument");
    const uint32_t slo = (uint32_t)(seed & 0xFFFFFFFFu), shi = (uint32_t)(seed >> 32);
    const long long nprop = (long long)p->nchains * p->nspec * p->maxbins;
#define GS_MP(FF) hipLaunchKernelGGL((k_mh_propose<FF>), dim3(nblk(nprop, 256)), dim3(256), 0, S(stream), p->nchains, \
                                     p->maxbins, p->meta, p->prop_sd, dl, p->prop, p->logr, u_prop, slo, shi, p->ita(iteration), \
                                     p->chain0, p->dl_tmp)
    if (p->F == 1) GS_MP(1); else if (p->F == 2) GS_MP(2); else GS_MP(3);
#undef GS_MP
    GS_LAUNCH_CHECK("k_mh_propose");
    p->snap_ok = true;
    return mh_decide(p, stats, dl, u_acc, slo, shi, iteration, accept_out, stream);
}

// the MH phases proper (proposals already in p->prop / p->logr)
static int mh_decide(gs_plan* p, const double* stats, double* dl, const double* u_acc, uint32_t slo, uint32_t shi,
                     uint32_t iteration, int32_t* accept_out, void* stream, const MhEpi* epi) {
    int maxnb = 0;
    const MhEpi none{nullptr, 1, nullptr, p->nchains, 0, nullptr};
    MhEpi E = epi ? *epi : none;
    // the proposal launch's D_l snapshot belongs to this decision only
    const bool snap = p->snap_ok;
    p->snap_ok = false;
    MhPhases ph{};
    ph.nphase = p->nphase;
    ph.lmin = p->mh_lmin;
    ph.own = -1;
    for (int q = 0; q < 4; ++q) {
        ph.sp0[q] = p->phase_sp[q][0]; ph.sp1[q] = p->phase_sp[q][1];
        ph.off[q] = p->phase_off[q]; ph.n[q] = p->phase_n[q]; ph.nwide[q] = p->phase_nwide[q];
        maxnb = std::max(maxnb, p->phase_n[q]);
    }
    const size_t lds = (2 * (size_t)(p->L + 1) + (size_t)maxnb * p->n_iter_mh + (size_t)p->nspec * p->maxbins) *
                           sizeof(double) + (size_t)p->nspec * (p->L + 1) * sizeof(int);
    const size_t lds_u = u_acc ? (size_t)p->nacc * sizeof(double) : 0;
    // r03: the register / LDS-resident form when the phase l range is at most
    // one l per thread and its arrays fit the LDS (k_mh_fused otherwise)
    int ntab = 0;
    for (int q = 0; q < p->nphase; ++q) ntab += p->phase_n[q];
    const size_t lds_reg = (2 * (size_t)(p->L + 1) + (size_t)p->nacc + 3 * (size_t)p->nspec * p->maxbins) *
                           sizeof(double) + 16 + (size_t)ntab * (sizeof(int4) + sizeof(int2));
    const bool reg = p->L + 1 - p->mh_lmin <= MH_REG_THREADS && lds_reg <= 150 * 1024;
    if (!reg && E.dl_in) {
        // the older MH forms read and write dl in place: copy the input first
        const size_t bytes = (size_t)p->nchains * p->nspec * p->maxbins * sizeof(double);
        GS_CHECK(hipMemcpyAsync(dl, E.dl_in, bytes, hipMemcpyDeviceToDevice, S(stream)));
        E.dl_in = nullptr;
    }
    // the split form (two workgroups per chain): both workgroups of a chain read
    // its start D_l, the T / E one writes its rows of dl at its end, so neither
    // may read dl itself -- the BB workgroup's PSD test of the T / E state would
    // depend on the order the two run in.  They read a stable copy:
    // the caller's dl_in (ASIS: the drawn D_l) or the snapshot the proposal
    // launch wrote (dl_tmp); without either the chain runs in one workgroup.
    bool split = reg && p->mh_split && p->ntab_s > 0;
    if (split && !E.dl_in) {
        if (snap) E.dl_in = p->dl_tmp;
        else split = false;
    }
    MhPhases ph1{};
    if (split) {
        MhPhases* k2[2] = {&ph, &ph1};
        for (int k = 0; k < 2; ++k) {
            MhPhases& h = *k2[k];
            h = MhPhases{};
            h.nphase = p->sph_n[k];
            h.lmin = p->mh_lmin;
            h.own = k == 0 ? ~p->sph_own[1] : p->sph_own[1];
            for (int q = 0; q < 4; ++q) {
                const bool on = q < h.nphase;
                h.sp0[q] = on ? p->sph_sp[k][q][0] : -1; h.sp1[q] = -1;
                h.off[q] = on ? p->sph_off[k][q] : 0; h.n[q] = on ? p->sph_cnt[k][q] : 0;
                h.nwide[q] = on ? p->sph_nwide[k][q] : 0;
            }
        }
    }
    if (reg) {
        static bool attr_set[4] = {false, false, false, false};
#define GS_MR(FF) do {                                                                                                 \
        if (!attr_set[FF])                                                                                             \
            GS_CHECK(hipFuncSetAttribute((const void*)k_mh_reg<FF>, hipFuncAttributeMaxDynamicSharedMemorySize,       \
                                         150 * 1024));                                                                 \
        attr_set[FF] = true;                                                                                           \
        hipLaunchKernelGGL((k_mh_reg<FF>), dim3(p->nchains * (split ? 2 : 1)), dim3(MH_REG_THREADS), lds_reg, S(stream), \
                           p->L, p->maxbins, ph, split ? p->ntab_s : ntab, split ? p->phase_tab_s : p->phase_tab,          \
                           split ? p->phase_rng_s : p->phase_rng, p->meta, p->nacc, p->n_iter_mh, p->ell2blk,           \
                           p->ell2bin, p->bl, p->kappa[0], p->kappa[1], p->kappa[2], stats, dl, p->prop, p->logr,      \
                           u_acc, slo, shi, p->ita(iteration), p->chain0, accept_out, E, ph1, split ? 2 : 1); } while (0)
        if (p->F == 1) GS_MR(1); else if (p->F == 2) GS_MR(2); else GS_MR(3);
#undef GS_MR
        GS_LAUNCH_CHECK("k_mh_reg");
        return 0;
    }
    if (lds <= 128 * 1024) {
#define GS_MF(FF) hipLaunchKernelGGL((k_mh_fused<FF>), dim3(p->nchains), dim3(1024), lds + lds_u, S(stream), p->L, p->maxbins, ph, \
                                     p->phase_tab, p->phase_rng, p->bins, p->blocks, p->meta + 8, p->nacc, p->n_iter_mh, p->ell2blk,    \
                                     p->ell2bin, p->bl, p->kappa[0], p->kappa[1], p->kappa[2], stats, dl, p->prop,       \
                                     p->logr, u_acc, slo, shi, p->ita(iteration), p->chain0, accept_out, E)
        if (p->F == 1) { GS_MF(1); } else if (p->F == 2) { GS_MF(2); } else { GS_MF(3); }
#undef GS_MF
        GS_LAUNCH_CHECK("k_mh_fused");
        return 0;
    }
    if (epi) return set_error("mh_decide: the fused epilogue needs the single-launch MH (l_max too large)");
    // very large l_max: two launches per phase (terms in HBM, one wave per block)
    const long long nl = (long long)p->nchains * (p->L + 1);
    for (int ph = 0; ph < p->nphase; ++ph) {
        const int nb = p->phase_n[ph];
        if (nb == 0) continue;
        const int sp0 = p->phase_sp[ph][0], sp1 = p->phase_sp[ph][1];
#define GS_MT(FF) hipLaunchKernelGGL((k_mh_terms<FF>), dim3(nblk(nl, 256)), dim3(256), 0, S(stream), p->L, p->nchains, \
                                     p->maxbins, sp0, sp1, p->ell2blk, p->ell2bin, p->bl, p->kappa[0], p->kappa[1],  \
                                     p->kappa[2], stats, dl, p->prop, p->gbuf)
        if (p->F == 1) GS_MT(1); else if (p->F == 2) GS_MT(2); else GS_MT(3);
#undef GS_MT
        GS_LAUNCH_CHECK("k_mh_terms");
        const long long waves = (long long)p->nchains * nb;
        const int2* tab = p->phase_tab + p->phase_off[ph];
#define GS_MA(FF) hipLaunchKernelGGL((k_mh_accept<FF>), dim3(nblk(waves, 4)), dim3(256), 0, S(stream), p->L, p->nchains, \
                                     p->maxbins, sp0, p->bins, p->blocks, tab, nb, p->meta + 8, p->nacc, p->n_iter_mh, \
                                     p->gbuf, dl, p->prop, p->logr, u_acc, slo, shi, p->ita(iteration), p->chain0, accept_out)
        if (p->F == 1) GS_MA(1); else if (p->F == 2) GS_MA(2); else GS_MA(3);
#undef GS_MA
        GS_LAUNCH_CHECK("k_mh_accept");
    }
    return 0;
}

// pro: also the MH proposals from dl (native draws) in front workgroups
static int stats_to_nc_launch(gs_plan* p, const double* dl, double* stats, void* stream, bool pro = false,
                              uint64_t seed = 0, uint32_t it = 0) {
    const long long n = (long long)p->nchains * (p->L + 1);
    ProPre pp{};
    if (pro) {
        pp.nbp = nblk((long long)p->nchains * p->nspec * p->maxbins, 256);
        pp.n = pp.nbp;
        pp.nspec = p->nspec; pp.nacc = p->nacc; pp.n_iter_mh = p->n_iter_mh; pp.maxbins = p->maxbins;
        pp.nbins = p->meta; pp.prop_sd = p->prop_sd; pp.dl = dl; pp.prop = p->prop; pp.logr = p->logr;
    }
    const uint32_t slo = (uint32_t)(seed & 0xFFFFFFFFu), shi = (uint32_t)(seed >> 32);
#define GS_TN(FF) hipLaunchKernelGGL((k_stats_to_nc<FF>), dim3(nblk(n, 256) + (unsigned)pp.n), dim3(256), 0, S(stream), \
                                     p->L, p->nchains, p->maxbins, dl, p->ell2bin, stats, pp, slo, shi, p->ita(it),     \
                                     p->chain0)
    if (p->F == 1) GS_TN(1); else if (p->F == 2) GS_TN(2); else GS_TN(3);
#undef GS_TN
    GS_LAUNCH_CHECK("k_stats_to_nc");
    return 0;
}

int gs_stats_to_noncentered(gs_plan* p, const double* dl, double* stats, void* stream) {
    if (check_plan(p)) return -1;
    if (!dl || !stats) return set_error("gs_stats_to_noncentered: null argument");
    return stats_to_nc_launch(p, dl, stats, stream);
}

int gs_recentre(gs_plan* p, const double* dl_new, const double* dl_old, double* s, void* stream) {
    if (check_plan(p)) return -1;
    if (!dl_new || !s) return set_error("gs_recentre: null argument");
    const long long n = (long long)p->nchains * (p->L + 1) * (p->L + 2) / 2;
#define GS_RC(FF) hipLaunchKernelGGL((k_recentre<FF>), dim3(nblk(n, 256)), dim3(256), 0, S(stream), p->L, p->nchains, \
                                     p->maxbins, dl_new, dl_old, p->ell2bin, s)
    if (p->F == 1) GS_RC(1); else if (p->F == 2) GS_RC(2); else GS_RC(3);
#undef GS_RC
    GS_LAUNCH_CHECK("k_recentre");
    return 0;
}

// the CR of a step: block parameters of dl (mode) + the sweep, the operator
// either from the parameter table (many chains) or computed inside the sweep
static int step_sweep(gs_plan* p, int mode, const double* d_alm, const double* dl, const double* z, uint64_t seed,
                      uint32_t it, double* s_out, void* stream, bool finish = true, bool* cls_pre_done = nullptr) {
    if (cls_pre_done) *cls_pre_done = false;
    if (p->inkernel_params)
        return sweep_launch(p, d_alm, nullptr, z, seed, it, 0, s_out, p->stats, false, stream, finish, mode, dl,
                            cls_pre_done);
    if (gs_block_params(p, mode, dl, p->params, stream)) return -1;
    return sweep_launch(p, d_alm, p->params, z, seed, it, 0, s_out, p->stats, false, stream, finish, -1, nullptr,
                        mode == GS_MODE_CENTERED ? cls_pre_done : nullptr);
}

// ---- fused iterations ------------------------------------------------------

int gs_step_centered(gs_plan* p, const double* d_alm, double* dl, double* s_out, const double* z,
                     const double* igvar, uint64_t seed, uint32_t it, void* stream) {
    if (check_plan(p)) return -1;
    if (!d_alm || !dl) return set_error("gs_step_centered: null argument");
    bool pre = false;
    if (step_sweep(p, GS_MODE_CENTERED, d_alm, dl, z, seed, it, s_out, stream, true, igvar ? nullptr : &pre))
        return -1;
    return cls_draw_launch(p, p->stats, igvar, seed, it, dl, nullptr, 1, nullptr, stream, pre ? p->cls_var : nullptr);
}

int gs_step_centered_fused(gs_plan* p, const double* d_alm, double* dl, double* s_out, uint64_t seed, uint32_t it,
                           double* trace, int capacity, void* stream) {
    if (check_plan(p)) return -1;
    if (!p->iter_dev_on) return set_error("gs_step_centered_fused: device iteration counter not enabled");
    if (trace && capacity < 1) return set_error("gs_step_centered_fused: capacity < 1");
    if (!d_alm || !dl) return set_error("gs_step_centered_fused: null argument");
    bool pre = false;
    if (step_sweep(p, GS_MODE_CENTERED, d_alm, dl, nullptr, seed, it, s_out, stream, true, &pre)) return -1;
    return cls_draw_launch(p, p->stats, nullptr, seed, it, dl, trace, trace ? capacity : 1, p->adv_counter(), stream,
                           pre ? p->cls_var : nullptr);
}

int gs_nc_prologue(gs_plan* p, const double* dl, const double* u_prop, uint64_t seed, uint32_t it, void* stream) {
    if (check_plan(p)) return -1;
    if (!p->has_mh) return set_error("gs_nc_prologue: plan has no MH blocks / proposal variances");
    if (!dl) return set_error("gs_nc_prologue: null argument");
    const uint32_t slo = (uint32_t)(seed & 0xFFFFFFFFu), shi = (uint32_t)(seed >> 32);
    const int nbp = nblk((long long)p->nchains * p->nspec * p->maxbins, 256);
    // block parameters here (table) unless the sweep computes them per lane
    const int nbq = p->inkernel_params ? 0 : nblk((long long)p->nchains * (p->L + 1), 256);
    // native mode: the MH accept uniforms are drawn here too (replay draws them on the host)
    p->u_nat_ready = u_prop == nullptr && p->nacc > 0;
    const int nbu = p->u_nat_ready ? nblk((long long)p->nchains * p->nacc, 256) : 0;
    p->snap_ok = false;
    if (u_prop == nullptr && (nbq > 0 || p->nchains > 4)) {
        // native draws: to the front of this step's sweep (or statistics finish)
        p->pro_pending = true;
        p->pro_dl = dl; p->pro_slo = slo; p->pro_shi = shi; p->pro_it = it;
        if (nbq == 0) return 0;                   // the sweep computes the operator: no launch
#define GS_PRQ(FF) hipLaunchKernelGGL((k_nc_prologue<FF>), dim3(nbq), dim3(256), 0, S(stream), 0, nbq, p->u_nat,     \
                                      p->nspec, p->nacc, p->n_iter_mh, p->L, p->nchains, p->maxbins, p->ell2bin, p->bl, \
                                      p->kappa[0], p->kappa[1], p->kappa[2], p->params, p->meta, p->prop_sd, dl,        \
                                      p->prop, p->logr, u_prop, slo, shi, p->ita(it), p->chain0, nullptr)
        if (p->F == 1) GS_PRQ(1); else if (p->F == 2) GS_PRQ(2); else GS_PRQ(3);
#undef GS_PRQ
        GS_LAUNCH_CHECK("k_nc_prologue");
        return 0;
    }
    p->pro_pending = false;
#define GS_PRO(FF) hipLaunchKernelGGL((k_nc_prologue<FF>), dim3(nbp + nbq + nbu), dim3(256), 0, S(stream), nbp, nbq,   \
                                      p->u_nat, p->nspec, p->nacc, p->n_iter_mh, p->L,                                  \
                                      p->nchains, p->maxbins, p->ell2bin, p->bl, p->kappa[0], p->kappa[1], p->kappa[2], \
                                      p->params, p->meta, p->prop_sd, dl, p->prop, p->logr, u_prop, slo, shi,            \
                                      p->ita(it), p->chain0, p->dl_tmp)
    if (p->F == 1) GS_PRO(1); else if (p->F == 2) GS_PRO(2); else GS_PRO(3);
#undef GS_PRO
    GS_LAUNCH_CHECK("k_nc_prologue");
    p->snap_ok = true;
    return 0;
}

int gs_nc_sweep(gs_plan* p, const double* d_alm, const double* dl, double* s_out, const double* z, uint64_t seed,
                uint32_t it, int finish, void* stream) {
    if (check_plan(p)) return -1;
    if (!dl) return set_error("gs_nc_sweep: null argument");
    if (p->inkernel_params)
        return sweep_launch(p, d_alm, nullptr, z, seed, it, 0, s_out, p->stats, false, stream, finish != 0,
                            GS_MODE_NONCENTERED, dl);
    return sweep_launch(p, d_alm, p->params, z, seed, it, 0, s_out, p->stats, false, stream, finish != 0);
}

int gs_nc_finish(gs_plan* p, void* stream) {
    if (check_plan(p)) return -1;
    return stats_finish(p, p->stats, stream);
}

int gs_nc_decide(gs_plan* p, double* dl, const double* u_acc, uint64_t seed, uint32_t it, int32_t* accept_out,
                 void* stream) {
    if (check_plan(p)) return -1;
    if (!p->has_mh) return set_error("gs_nc_decide: plan has no MH blocks / proposal variances");
    if (!dl) return set_error("gs_nc_decide: null argument");
    if (p->pro_pending) return set_error("gs_nc_decide: the prologue's draws wait for gs_nc_finish");
    const uint32_t slo = (uint32_t)(seed & 0xFFFFFFFFu), shi = (uint32_t)(seed >> 32);
    return mh_decide(p, p->stats, dl, u_acc, slo, shi, it, accept_out, stream);
}

int gs_nc_decide_fused(gs_plan* p, double* dl, uint64_t seed, uint32_t it, int32_t* accept_out, double* trace,
                       int capacity, void* stream) {
    if (check_plan(p)) return -1;
    if (!p->has_mh) return set_error("gs_nc_decide_fused: plan has no MH blocks / proposal variances");
    if (!dl) return set_error("gs_nc_decide_fused: null argument");
    if (trace && capacity < 1) return set_error("gs_nc_decide_fused: capacity < 1");
    if (p->pro_pending) return set_error("gs_nc_decide_fused: the prologue's draws wait for gs_nc_finish");
    const uint32_t slo = (uint32_t)(seed & 0xFFFFFFFFu), shi = (uint32_t)(seed >> 32);
    const MhEpi epi{trace, std::max(capacity, 1), p->adv_counter(), p->nchains, p->graph_adv, nullptr};
    return mh_decide(p, p->stats, dl, p->u_nat_ready ? p->u_nat : nullptr, slo, shi, it, accept_out, stream, &epi);
}

int gs_step_noncentered(gs_plan* p, const double* d_alm, double* dl, double* s_out, const double* z,
                        const double* u_prop, const double* u_acc, uint64_t seed, uint32_t it, int32_t* accept_out,
                        void* stream) {
    if (check_plan(p)) return -1;
    if (!p->has_mh) return set_error("gs_step_noncentered: plan has no MH blocks / proposal variances");
    if (!d_alm || !dl) return set_error("gs_step_noncentered: null argument");
    if (gs_nc_prologue(p, dl, u_prop, seed, it, stream)) return -1;
    if (gs_nc_sweep(p, d_alm, dl, s_out, z, seed, it, 1, stream)) return -1;
    return gs_nc_decide(p, dl, u_acc, seed, it, accept_out, stream);
}

int gs_step_asis(gs_plan* p, const double* d_alm, double* dl, double* s_out, const double* z, const double* igvar,
                 const double* u_prop, const double* u_acc, uint64_t seed, uint32_t it, int32_t* accept_out,
                 double* dl_tmp_out, int recentre, void* stream) {
    if (check_plan(p)) return -1;
    // validated before anything is launched (dl is overwritten mid-step)
    if (!p->has_mh) return set_error("gs_step_asis: plan has no MH blocks / proposal variances");
    if (!d_alm || !dl) return set_error("gs_step_asis: null argument");
    double* tmp = dl_tmp_out ? dl_tmp_out : p->dl_tmp;
    if (step_sweep(p, GS_MODE_CENTERED, d_alm, dl, z, seed, it, s_out, stream)) return -1;
    if (gs_cls_draw(p, p->stats, igvar, seed, it, tmp, stream)) return -1;
    if (gs_stats_to_noncentered(p, tmp, p->stats, stream)) return -1;
    const size_t bytes = (size_t)p->nchains * p->nspec * p->maxbins * sizeof(double);
    GS_CHECK(hipMemcpyAsync(dl, tmp, bytes, hipMemcpyDeviceToDevice, S(stream)));
    if (gs_nc_mh(p, p->stats, dl, u_prop, u_acc, seed, it, accept_out, stream)) return -1;
    if (recentre && s_out) {
        // ASIS.py:203 (quirk) re-centres the centered map: s <- A(C_new) s;
        // the corrected form is s <- A(C_new) A(C_tmp)^+ s
        const bool quirk = (p->quirks & GS_QUIRK_ASIS_RECENTRE_CENTERED) != 0;
        if (gs_recentre(p, dl, quirk ? nullptr : tmp, s_out, stream)) return -1;
    }
    return 0;
}

int gs_step_asis_fused(gs_plan* p, const double* d_alm, double* dl, double* s_out, uint64_t seed, uint32_t it,
                       int32_t* accept_out, double* dl_tmp_out, int recentre, double* trace, int capacity,
                       void* stream) {
    if (check_plan(p)) return -1;
    if (!p->iter_dev_on) return set_error("gs_step_asis_fused: device iteration counter not enabled");
    if (!p->has_mh) return set_error("gs_step_asis_fused: plan has no MH blocks / proposal variances");
    if (trace && capacity < 1) return set_error("gs_step_asis_fused: capacity < 1");
    if (!d_alm || !dl) return set_error("gs_step_asis_fused: null argument");
    double* tmp = dl_tmp_out ? dl_tmp_out : p->dl_tmp;
    const uint32_t slo = (uint32_t)(seed & 0xFFFFFFFFu), shi = (uint32_t)(seed >> 32);
    bool pre = false;
    if (step_sweep(p, GS_MODE_CENTERED, d_alm, dl, nullptr, seed, it, s_out, stream, true, &pre)) return -1;
    if (cls_draw_launch(p, p->stats, nullptr, seed, it, tmp, nullptr, 1, nullptr, stream, pre ? p->cls_var : nullptr))
        return -1;
    // the non-centred statistics and, in front workgroups of the same launch,
    // the MH proposals from the drawn D_l (tmp); the MH reads tmp and writes dl
    // (no copy: the same values as copying tmp to dl first)
    if (stats_to_nc_launch(p, tmp, p->stats, stream, true, seed, it)) return -1;
    // the trace record and the counter advance ride in the MH launch (no kernel
    // after it reads the counter: the re-centring uses D_l only)
    const MhEpi epi{trace, trace ? capacity : 1, p->adv_counter(), p->nchains, p->graph_adv, tmp};
    if (mh_decide(p, p->stats, dl, nullptr, slo, shi, it, accept_out, stream, &epi)) return -1;
    if (recentre && s_out) {
        const bool quirk = (p->quirks & GS_QUIRK_ASIS_RECENTRE_CENTERED) != 0;
        if (gs_recentre(p, dl, quirk ? nullptr : tmp, s_out, stream)) return -1;
    }
    return 0;
}

#if defined(GS_SWEEP_WGTIME)
int gs_debug_sweep_timeline(unsigned long long* out, int n) {
    GS_CHECK(hipDeviceSynchronize());
    GS_CHECK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sw_tl), sizeof(unsigned long long) * 4 * std::min(n, SW_TL_MAX)));
    return 0;
}
#endif

#if defined(GS_MH_TIMELINE)
int gs_debug_mh_timeline(unsigned long long* out) {
    GS_CHECK(hipDeviceSynchronize());
    GS_CHECK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mh_tl), sizeof(unsigned long long) * 32));
    return 0;
}
#endif

int gs_iteration_counter(gs_plan* p, int enable, uint32_t start) {
    if (check_plan(p)) return -1;
    p->iter_dev_on = enable != 0;
    p->graph_off = 0;
    p->graph_adv = 1;
    if (enable) GS_CHECK(hipMemcpy(p->iter_dev, &start, sizeof(uint32_t), hipMemcpyHostToDevice));
    return 0;
}

int gs_graph_step(gs_plan* p, uint32_t offset, uint32_t advance) {
    if (check_plan(p)) return -1;
    if (!p->iter_dev_on) return set_error("gs_graph_step: device counter not enabled");
    p->graph_off = offset;
    p->graph_adv = advance;
    return 0;
}

int gs_advance_iteration(gs_plan* p, void* stream) {
    if (check_plan(p)) return -1;
    if (!p->iter_dev_on) return set_error("gs_advance_iteration: device counter not enabled");
    hipLaunchKernelGGL(k_iter_advance, dim3(1), dim3(1), 0, S(stream), p->iter_dev);
    GS_LAUNCH_CHECK("k_iter_advance");
    return 0;
}

int gs_record_trace(gs_plan* p, const double* dl, double* trace, int capacity, uint32_t iteration, void* stream) {
    if (check_plan(p)) return -1;
    if (capacity < 1) return set_error("gs_record_trace: capacity < 1");
    if (!dl || !trace) return set_error("gs_record_trace: null argument");
    const long long n = (long long)p->nchains * p->nspec * p->maxbins;
    hipLaunchKernelGGL(k_record_trace, dim3(nblk(n, 256)), dim3(256), 0, S(stream), n, dl, trace, capacity,
                       p->ita(iteration));
    GS_LAUNCH_CHECK("k_record_trace");
    return 0;
}

int gs_sweep_timing(gs_plan* p, int enable, double* total_ms, int* count) {
    if (check_plan(p)) return -1;
    if (enable == 2 || enable == 3) {           // pause / resume, keeping the launches timed so far
        p->timing = enable == 3;
        return 0;
    }
    if (enable) {
        p->timing = true;
        p->ev_used = 0;
        return 0;
    }
    double tot = 0.0;
    int n = 0;
    for (size_t k = 0; k + 1 < p->ev_used; k += 2) {
        GS_CHECK(hipEventSynchronize(p->ev[k + 1]));
        float ms = 0.f;
        GS_CHECK(hipEventElapsedTime(&ms, p->ev[k], p->ev[k + 1]));
        tot += ms;
        ++n;
    }
    p->timing = false;
    p->ev_used = 0;
    if (total_ms) *total_ms = tot;
    if (count) *count = n;
    return 0;
}

}  // extern "C"
