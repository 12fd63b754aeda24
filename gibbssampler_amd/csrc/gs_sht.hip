// gs_sht.hip -- HEALPix RING spherical-harmonic transforms on gfx950 (fp64).
//
// Replaces the healpy calls of the reference's masked CR variants
// (hp.alm2map: CenteredGibbs.py:204,505,698,751,791, NonCenteredGibbs.py:350;
// hp.map2alm: CenteredGibbs.py:298,513,717,773,812, utils.py:89,104,
// NonCenteredGibbs.py:155).  Conventions: SURVEY.md Appendix A.4 and
// oracle/sht.py (Condon-Shortley lambda_lm, Zaldarriaga-Seljak F1/F2 spin-2
// functions, Q + iU = -sum (a_E + i a_B) 2Y_lm, map2alm = (4pi/Npix) x adjoint).
//
// Structure (per transform, one chain):
//   synthesis  k_sht_synth_leg : per (m, ring pair) Legendre sums
//                  Phi_m(ring) = sum_l a_lm G_lm(theta)      [compute bound, fp64 VALU]
//              k_sht_synth_ring: per ring pair: alias-fold Phi_m into nphi bins,
//                  one complex FFT for the north+south rings (Hermitian packing)
//   analysis   k_sht_anal_ring : per ring pair: one complex FFT of north + i south,
//                  split, un-alias into Phi_m
//              k_sht_anal_leg  : per (m, l) sums over rings (4 ring pairs per lane,
//                  fixed-order LDS reduction per 4-l chunk) -> per-tile partials
//              k_sht_anal_finish: fixed-order tile sum, weight, output layout
//
// Legendre functions run the normalised three-term recurrence in l with a
// scale exponent (lambda = v * 2^(768 k), k <= 0), so the sin^m theta start
// values of high m near the poles do not underflow.  A plan-time pass finds,
// per (m, 64-ring-pair group), the first l where any ring of the group is
// representable (k = 0) and stores the recurrence state there: the
// transforms skip the exponentially small part of the (l, ring) plane
// exactly instead of iterating through it.
//
// Ring FFTs: nphi = 4i (caps) or 4 N_side (equator).  Power-of-two lengths
// use an in-place radix-2 Stockham FFT in LDS; other lengths use Bluestein's
// chirp-z with a power-of-two length M >= 2 nphi - 1 and a plan-time FFT of
// the chirp kernel per ring.  Launches are split by M so each uses exactly
// the LDS it needs (M <= 8192 in LDS; larger M in a global scratch).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include <string>
#include <vector>
#include <algorithm>
#include <cstdlib>
#include <cstdio>

#include "gibbs_capi.h"
#include "gs_common.h"
#include "gs_aux.h"

using gs_detail::set_error;

namespace {

constexpr double PI = 3.14159265358979323846;
constexpr int LEG_BLOCK = 256;
#ifndef GS_ANA_C
#define GS_ANA_C 4
#endif
constexpr int ANA_C = GS_ANA_C;             // l per reduction chunk (even)
// Legendre stages: the per-l coefficient (and synthesis a_lm) lines are read
// by wave-uniform scalar loads, one wait per chunk; a vector load GS_*_PF l
// ahead pulls those lines into L2 first, so the scalar loads hit there instead
// of HBM (N_side 2048: TEB map2alm 33.5 -> 32.0 ms, alm2map 26.1 -> 25.6 ms;
// 0 turns it off)
#ifndef GS_ANA_PF
#define GS_ANA_PF 16
#endif
#ifndef GS_SYN_PF
#define GS_SYN_PF 16
#endif
constexpr int LDS_FFT_MAX = 8192;           // complex points held in LDS
constexpr int RING_MC_LDS_MAX = 160 * 1024;   // LDS of a multi-component ring workgroup
constexpr double SC_UP = 0x1p768;
constexpr double SC_DN = 0x1p-768;
constexpr double SC_HI = 0x1p384;
constexpr double SC_LO = 0x1p-384;

struct PairGeom {
    double x;            // cos theta of the north ring
    double s;            // sin theta
    double is2;          // 1 / sin^2 theta
    long long startN;    // first pixel of the north ring
    long long startS;    // first pixel of the south ring, -1 for the equator
    int nphi;
    int phi_half;        // phi0 = phi_half * pi / nphi
    int M;               // FFT length
    int logM;
    long long bs_off;    // Bluestein kernel offset (complex entries), -1 if nphi = M
    int split;           // 1: DFT_nphi = two DFT_(nphi/2) (even / odd samples), each a
                         //    Bluestein of length M held in LDS (instead of one M > LDS)
    int sslot;           // index of the ring pair among the split ones (global scratch slot)
};

// per (l, m) recurrence + spin-2 coefficients (64 B, one scalar load)
struct LegCoef {
    double a, b;   // lambda_l = a (x lambda_{l-1} - b lambda_{l-2})
    double P, Q;   // F1 = -(P is2 + Q) lambda_l + R (x is2) lambda_{l-1}
    double R, T;   // F2 = -T (x is2) lambda_l + Rm is2 lambda_{l-1}
    double Rm, pad;
};

// The analysis' form of (l, m): the recurrence step l -> l + 1 (a, b of l + 1)
// and the spin-2 terms of l divided by Q_l, which the ring reduction's output
// multiplies back (acq[l] = Q_l; 0 for l < 2):
//   F1 / (is2 Q) = R' (x lambda_{l-1}) - (P' + sin^2) lambda_l
//   F2 / (is2 Q) = Rm' lambda_{l-1} - T' (x lambda_l)
// 12 scalar registers per l (LegCoef's walk reads 16: its l and the a, b of
// l + 1), and every fp64 operation takes at most one of them (the VALU reads
// one scalar operand per instruction).
struct AnaCoef {
    double a1, b1;   // lambda_{l+1} = a1 (x lambda_l - b1 lambda_{l-1})
    double P, R;     // P / Q, R / Q
    double T, Rm;    // T / Q, Rm / Q
};

struct ShtDev {
    int L, npair, ngroup, nlm;
    const PairGeom* geom;
    const LegCoef* coef;
    const int* lstart;       // [L+1][ngroup]
    const double2* st;       // [L+1][npair] (lambda_{ls-1}, lambda_ls), scaled
    const int* stk;          // [L+1][npair] scale exponent at ls
    // l-segmented analysis (small maps): segment s of m covers l in
    // [m + s seg, m + (s + 1) seg); the recurrence state at each segment start
    // s >= 1 is a plan-time table (0: no segments, one walk from m to L)
    int seg;
    int segmul;              // table rows per segment of this launch (seg / the table's)
    const int* segoff;       // [L+1] first table row of m's segments s >= 1
    const double2* sst;      // [rows][npair] (lambda_{lA-1}, lambda_lA), scaled
    const int* sstk;         // [rows][npair] scale exponent at lA
};

__device__ __forceinline__ long long cidx(int L, int l, int m) { return (long long)m * (2 * L + 1 - m) / 2 + l; }

// Ring phases Phi_m(pair), one plane per (comp, north/south): blocks of PHI_MB
// consecutive m of one ring pair are contiguous ([m / MB][pair][m % MB]), so
// the ring stage (threads = consecutive m of one pair) moves whole 128-B lines
// while the Legendre stage (lanes = pairs at fixed m) keeps one element per
// lane.  PHI_MB = 1 is the plain m-major layout.
#ifndef GS_PHI_MB
#define GS_PHI_MB 4
#endif
constexpr int PHI_MB = GS_PHI_MB;
__host__ __device__ __forceinline__ long long phi_plane(int L, int npair) {
    return (long long)((L + PHI_MB) / PHI_MB) * PHI_MB * npair;
}
__device__ __forceinline__ long long phi_at(int m, int p, int npair) {
    return ((long long)(m / PHI_MB) * npair + p) * PHI_MB + (m % PHI_MB);
}

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 conj2(double2 a) { return make_double2(a.x, -a.y); }

// e^{i pi t / n} for integer t (reduced mod 2n exactly)
__device__ __forceinline__ double2 expi_pi_frac(long long t, long long n) {
    long long r = t % (2 * n);
    if (r < 0) r += 2 * n;
    double sn, cs;
    sincospi((double)r / (double)n, &sn, &cs);
    return make_double2(cs, sn);
}
// the same values for the ring stage's small arguments (0 <= t < 2^32, n < 2^30)
// with a 32-bit reduction instead of a 64-bit division: e^{i pi t / n} ...
__device__ __forceinline__ double2 expi_pi_u32(unsigned t, unsigned n) {
    const unsigned r = t % (2u * n);
    double sn, cs;
    sincospi((double)r / (double)n, &sn, &cs);
    return make_double2(cs, sn);
}
// ... and e^{-i pi t / n} (bit for bit expi_pi_frac(-t, n))
__device__ __forceinline__ double2 expi_pi_neg_u32(unsigned t, unsigned n) {
    unsigned r = t % (2u * n);
    r = r ? 2u * n - r : 0u;
    double sn, cs;
    sincospi((double)r / (double)n, &sn, &cs);
    return make_double2(cs, sn);
}

// ---------------------------------------------------------------------------
// a_lm access in the caller's layout: 0 = real m-major (utils.py:49-76),
// 1 = healpy complex m-major interleaved
// ---------------------------------------------------------------------------
__device__ __forceinline__ double2 alm_get(const double* __restrict__ a, int layout, int L, int l, int m) {
    if (layout == GS_ALM_COMPLEX) {
        const long long i = cidx(L, l, m);
        return make_double2(a[2 * i], a[2 * i + 1]);
    }
    if (m == 0) return make_double2(a[l], 0.0);
    const long long r = 2 * cidx(L, l, m) - (L + 1);
    constexpr double IS2 = 0.70710678118654752440;
    return make_double2(a[r] * IS2, a[r + 1] * IS2);
}

__host__ __device__ __forceinline__ long long alm_comp_stride(int layout, int L) {
    return layout == GS_ALM_COMPLEX ? (long long)(L + 1) * (L + 2) : (long long)(L + 1) * (L + 1);
}

// ---------------------------------------------------------------------------
// plan-time Legendre start tables
// ---------------------------------------------------------------------------
// lambda_mm per (m, pair), scaled: v * 2^(768 k)
__global__ void k_sht_lmm(int L, int npair, const PairGeom* __restrict__ geom, double* __restrict__ lmm,
                          int* __restrict__ lmk) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npair) return;
    const double s = geom[p].s;
    double v = 0.28209479177387814347;   // 1/sqrt(4 pi)
    int k = 0;
    for (int m = 0; m <= L; ++m) {
        if (m > 0) {
            v *= -sqrt((2.0 * m + 1.0) / (2.0 * m)) * s;
            if (fabs(v) < SC_LO) { v *= SC_UP; --k; }
        }
        lmm[(long long)m * npair + p] = v;
        lmk[(long long)m * npair + p] = k;
    }
}

// per (m, pair): run the scaled recurrence to find where the group of 64 ring
// pairs becomes representable, then store the state there
__global__ __launch_bounds__(256) void k_sht_onset(ShtDev D, const double* __restrict__ lmm, const int* __restrict__ lmk,
                                                   int* __restrict__ lstart, double2* __restrict__ st,
                                                   int* __restrict__ stk) {
    const int L = D.L, npair = D.npair;
    const int m = blockIdx.y;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    const bool act = p < npair;
    const double x = act ? D.geom[p].x : 0.0;
    const long long base = cidx(L, m, m);
    const double v0i = act ? lmm[(long long)m * npair + p] : 0.0;
    const int k0 = act ? lmk[(long long)m * npair + p] : 0;
    // pass 1: onset
    int lon = L + 1;
    {
        double v1 = 0.0, v0 = v0i;
        int k = k0;
        if (act) {
            for (int l = m; l <= L; ++l) {
                if (k == 0) { lon = l; break; }
                if (l == L) break;
                const LegCoef c = D.coef[base + (l + 1 - m)];
                const double vn = c.a * (x * v0 - c.b * v1);
                v1 = v0; v0 = vn;
                if (fabs(v0) > SC_HI) { v0 *= SC_DN; v1 *= SC_DN; ++k; }
            }
        }
    }
    // wave minimum (64 consecutive pairs = one group)
    int ls = lon;
    for (int o = 32; o > 0; o >>= 1) ls = min(ls, __shfl_xor(ls, o, 64));
    const int group = p >> 6;
    if ((threadIdx.x & 63) == 0 && group < D.ngroup) lstart[(long long)m * D.ngroup + group] = ls;
    // pass 2: state at ls
    double v1 = 0.0, v0 = v0i;
    int k = k0;
    if (act && ls <= L) {
        for (int l = m; l < ls; ++l) {
            const LegCoef c = D.coef[base + (l + 1 - m)];
            const double vn = c.a * (x * v0 - c.b * v1);
            v1 = v0; v0 = vn;
            if (k < 0 && fabs(v0) > SC_HI) { v0 *= SC_DN; v1 *= SC_DN; ++k; }
        }
    }
    if (act) {
        st[(long long)m * npair + p] = make_double2(v1, v0);
        stk[(long long)m * npair + p] = k;
    }
}

// per (m, pair): the analysis recurrence's state at every segment start
// lA = m + s seg (s >= 1) past the group's onset, walked from the onset state
// with exactly the transform's step and rescaling (rec_step below), so a
// segment entered at lA continues the same sequence a single walk would hold
__device__ __forceinline__ void rec_step(const LegCoef& c, double x, double& v0, double& v1);

// x lambda as its own rounded product (never contracted into a neighbouring
// add): the recurrence and the spin-2 terms share it (rec_from below)
__device__ __forceinline__ double mul_nc(double a, double b) {
#pragma clang fp contract(off)
    return a * b;
}
__global__ __launch_bounds__(256) void k_sht_segstate(ShtDev D) {
    const int L = D.L, npair = D.npair, S = D.seg;
    const int m = blockIdx.y;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npair || S <= 0) return;
    const int ls = D.lstart[(long long)m * D.ngroup + (p >> 6)];
    const long long row0 = D.segoff[m];
    const double x = D.geom[p].x;
    const LegCoef* cf = D.coef + (cidx(L, m, m) - m);
    double v1 = 0.0, v0 = 0.0;
    int k = 0;
    if (ls <= L) {
        const double2 s0 = D.st[(long long)m * npair + p];
        v1 = s0.x; v0 = s0.y;
        k = D.stk[(long long)m * npair + p];
    }
    int l = ls;                                   // the state holds lambda_l
    for (int s = 1; m + s * S <= L; ++s) {
        const int lA = m + s * S;
        if (ls <= L && lA > ls) {
            for (; l < lA; ++l) {
                rec_step(cf[l + 1], x, v0, v1);
                if (k < 0 && fabs(v0) > SC_HI) { v0 *= SC_DN; v1 *= SC_DN; ++k; }
            }
        }
        const long long o = (row0 + s - 1) * npair + p;
        const bool live = ls <= L && lA > ls;
        const_cast<double2*>(D.sst)[o] = live ? make_double2(v1, v0) : make_double2(0.0, 0.0);
        const_cast<int*>(D.sstk)[o] = live ? k : 0;
    }
}

// ---------------------------------------------------------------------------
// Legendre stages: shared layout
// ---------------------------------------------------------------------------
// A workgroup covers 4 SR consecutive 64-ring-pair groups for one m pair
// (m, L - m: balanced work) or one m (paired = 0: small maps, where the m
// pairs alone do not give ~4 waves per SIMD); lane `lane` of wave `w` owns the SR ring
// pairs tile*1024 + w*256 + r*64 + lane, so (wave, slot r) is exactly one
// 64-pair onset group and every per-l coefficient / a_lm value is a
// wave-uniform scalar load.  Each slot enters at its group's onset l with the
// plan-time recurrence state; while any lane of a slot is still below the
// representable range (k < 0) the slow path masks and rescales, afterwards
// the parity-unrolled fast path runs the plain recurrence.
// NC = 1: T (spin 0); 2: E,B <-> Q,U; 3: T,E,B <-> T,Q,U.
// phi layout: [comp][ns][m][pair] (double2), ns 0 = north, 1 = south

// a_lm in the caller's layout -> ain[comp][nlm] (healpy-ordered complex)
// l of healpy m-major complex index i (m > 0 part of the real layout)
__device__ __forceinline__ int l_of_cidx(int L, long long i) {
    const double b = 2.0 * L + 3.0;
    int m = (int)floor((b - sqrt(fmax(b * b - 8.0 * (double)i, 0.0))) / 2.0);
    m = max(0, min(m, L));
    while (m > 0 && (long long)m * (2 * L + 3 - m) / 2 > i) --m;
    while (m < L && (long long)(m + 1) * (2 * L + 2 - m) / 2 <= i) ++m;
    return (int)(i - (long long)m * (2 * L + 1 - m) / 2);
}

// a_lm -> the Legendre stage's complex layout; bl != nullptr (real layout only)
// applies the per-l beam on the way in: (b_l s) rounded, then the 1/sqrt 2 --
// the same two roundings as a separate beam pass (the masked CR's b s, whose
// k_mc_beam launch and scratch write this replaces)
// acq != nullptr (the on-the-fly synthesis: its AnaCoef terms are F / Q_l):
// the spin-2 comps of each map (nc comps: 2 = E, B; 3 = T, E, B) leave scaled by Q_l
__global__ void k_sht_alm_in(int L, int nlm, int ncomp, const double* __restrict__ alm, int layout,
                             double2* __restrict__ ain, const double* __restrict__ bl, int nc = 1,
                             const double* __restrict__ acq = nullptr) {
    const long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (g >= (long long)ncomp * nlm) return;
    const int comp = (int)(g / nlm);
    const long long i = g % nlm;
    const double* a = alm + comp * alm_comp_stride(layout, L);
    double2 v;
    if (layout == GS_ALM_COMPLEX) {
        v = make_double2(a[2 * i], a[2 * i + 1]);
    } else if (i <= L) {
        v = make_double2(bl ? bl[i] * a[i] : a[i], 0.0);
    } else {
        constexpr double IS2 = 0.70710678118654752440;
        const long long r = 2 * i - (L + 1);
        if (bl) {
            const double b = bl[l_of_cidx(L, i)];
            v = make_double2((b * a[r]) * IS2, (b * a[r + 1]) * IS2);
        } else {
            v = make_double2(a[r] * IS2, a[r + 1] * IS2);
        }
    }
    if (acq && !(nc == 1 || (nc == 3 && comp % 3 == 0))) {
        const double q = acq[i <= L ? (int)i : l_of_cidx(L, i)];
        v = make_double2(v.x * q, v.y * q);
    }
    ain[g] = v;
}

struct SynAcc {
    double tp[2], tn[2];        // T: parity + / -
    double sp[4], sn[4];        // Q re, Q im, U re, U im: parity + / -
};

// The spin-2 terms of one (l, ring pair) in the on-the-fly kernels, without
// their common factors 1/sin^2 and Q_l:
//   F1 / (is2 Q) = R' (x lambda_{l-1}) - (P' + sin^2) lambda_l
//   F2 / (is2 Q) = Rm' lambda_{l-1} - T' (x lambda_l)
// (AnaCoef).  x lambda_l is the recurrence's own product and x lambda_{l-1}
// the previous step's, so a unit costs 5 fp64 ops instead of 8; is2 goes onto
// the ring's phases (analysis) or its output sums (synthesis) once per m, Q_l
// onto the a_lm (synthesis) or the reduced outputs (analysis).

// v0 = lambda_l, v1 = lambda_{l-1}, xv0 = x v0, xv1 = x v1 (mul_nc products);
// c in the AnaCoef form (spin-2 terms / Q_l: aE, aB arrive scaled by Q_l,
// k_sht_alm_in), the factor is2 applied at the output (syn_store)
template <int NC, bool EVEN>
__device__ __forceinline__ void syn_accumulate(SynAcc& A, const AnaCoef& c, double v0, double v1, double xv0,
                                               double xv1, double s2, double2 aT, double2 aE, double2 aB) {
    if constexpr (NC != 2) {
        if (EVEN) { A.tp[0] = fma(aT.x, v0, A.tp[0]); A.tp[1] = fma(aT.y, v0, A.tp[1]); }
        else      { A.tn[0] = fma(aT.x, v0, A.tn[0]); A.tn[1] = fma(aT.y, v0, A.tn[1]); }
    }
    if constexpr (NC != 1) {
        const double F1 = fma(c.R, xv1, -((c.P + s2) * v0));
        const double F2 = fma(c.Rm, v1, -(c.T * xv0));
        double* a1 = EVEN ? A.sp : A.sn;   // F1 carries lambda's parity
        double* a2 = EVEN ? A.sn : A.sp;   // F2 the opposite one
        a1[0] = fma(aE.x, F1, a1[0]); a2[0] = fma(-aB.y, F2, a2[0]);
        a1[1] = fma(aE.y, F1, a1[1]); a2[1] = fma(aB.x, F2, a2[1]);
        a1[2] = fma(aB.x, F1, a1[2]); a2[2] = fma(aE.y, F2, a2[2]);
        a1[3] = fma(aB.y, F1, a1[3]); a2[3] = fma(-aE.x, F2, a2[3]);
    }
}

// a ring pair's phases from its sums: T from the parity sums; Q, U = -(...)
// times the spin-2 terms' common factor is2
template <int NC>
__device__ __forceinline__ void syn_store(const SynAcc& A, double2* __restrict__ phi, long long plane, long long o,
                                          double is2) {
    int comp = 0;
    if constexpr (NC != 2) {
        phi[(2 * comp + 0) * plane + o] = make_double2(A.tp[0] + A.tn[0], A.tp[1] + A.tn[1]);
        phi[(2 * comp + 1) * plane + o] = make_double2(A.tp[0] - A.tn[0], A.tp[1] - A.tn[1]);
        ++comp;
    }
    if constexpr (NC != 1) {
        const double w = -is2;
        phi[(2 * comp + 0) * plane + o] = make_double2(w * (A.sp[0] + A.sn[0]), w * (A.sp[1] + A.sn[1]));
        phi[(2 * comp + 1) * plane + o] = make_double2(w * (A.sp[0] - A.sn[0]), w * (A.sp[1] - A.sn[1]));
        ++comp;
        phi[(2 * comp + 0) * plane + o] = make_double2(w * (A.sp[2] + A.sn[2]), w * (A.sp[3] + A.sn[3]));
        phi[(2 * comp + 1) * plane + o] = make_double2(w * (A.sp[2] - A.sn[2]), w * (A.sp[3] - A.sn[3]));
    }
}

// one recurrence step from the product xv0 = mul_nc(x, v0)
__device__ __forceinline__ void rec_from(const LegCoef& c, double xv0, double& v0, double& v1) {
    const double vn = c.a * fma(-c.b, v1, xv0);
    v1 = v0;
    v0 = vn;
}
__device__ __forceinline__ void rec_step(const LegCoef& c, double x, double& v0, double& v1) {
    rec_from(c, mul_nc(x, v0), v0, v1);
}
// the on-the-fly kernels' step from an AnaCoef (a, b of l + 1 stored at l):
// the same arithmetic as rec_from
__device__ __forceinline__ void rec_ana(const AnaCoef& c, double xv0, double& v0, double& v1) {
    const double vn = c.a1 * fma(-c.b1, v1, xv0);
    v1 = v0;
    v0 = vn;
}
// ring constants of the spin-2 terms: sin^2 = 1 / is2 (0 on an idle lane)
__device__ __forceinline__ double ring_s2(bool act, double is2) { return act ? 1.0 / is2 : 0.0; }

template <int NC, int SR>
__global__ __launch_bounds__(LEG_BLOCK) void k_sht_synth_leg(ShtDev D, const AnaCoef* __restrict__ coef,
                                                             const double2* __restrict__ ain,
                                                             double2* __restrict__ phi, int paired) {
    const int L = D.L, npair = D.npair, nlm = D.nlm;
    const int q = blockIdx.x, tile = blockIdx.y;
    // map b of a batch (chains): its a_lm and phase planes
    ain += (long long)blockIdx.z * NC * nlm;
    phi += (long long)blockIdx.z * NC * 2 * phi_plane(L, npair);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g0 = tile * (LEG_BLOCK / 64) * SR + wave * SR;   // onset group of slot 0
    double x[SR], s2[SR];
    int pr[SR];
    bool act[SR];
#pragma unroll
    for (int r = 0; r < SR; ++r) {
        pr[r] = (g0 + r) * 64 + lane;
        act[r] = pr[r] < npair;
        x[r] = act[r] ? D.geom[pr[r]].x : 0.0;
        s2[r] = ring_s2(act[r], act[r] ? D.geom[pr[r]].is2 : 0.0);
    }
    const double2 z2 = make_double2(0.0, 0.0);
    for (int h = 0; h < 2; ++h) {
        const int m = h == 0 ? q : L - q;
        if (h == 1 && (!paired || m <= q)) break;
        int ls[SR];
        int lmin = L + 1;
#pragma unroll
        for (int r = 0; r < SR; ++r) {
            ls[r] = __builtin_amdgcn_readfirstlane(g0 + r < D.ngroup ? D.lstart[(long long)m * D.ngroup + g0 + r]
                                                                     : L + 1);
            lmin = min(lmin, ls[r]);
        }
        SynAcc A[SR];
        double v0[SR], v1[SR], xv1[SR];
        int kk[SR];
#pragma unroll
        for (int r = 0; r < SR; ++r) {
#pragma unroll
            for (int i = 0; i < 2; ++i) { A[r].tp[i] = 0.0; A[r].tn[i] = 0.0; }
#pragma unroll
            for (int i = 0; i < 4; ++i) { A[r].sp[i] = 0.0; A[r].sn[i] = 0.0; }
            v0[r] = 0.0; v1[r] = 0.0; kk[r] = 0;
        }
        const long long base = cidx(L, m, m) - m;              // + l = complex index of (l, m)
        const AnaCoef* cf = coef + base;
        const double2* aT = ain + base;
        const double2* aE = ain + (NC == 3 ? nlm : 0) + base;
        const double2* aB = aE + nlm;
        int l = lmin;
        // ---- slow path: slot activation and scaled lanes ----
        while (l <= L) {
            bool live = true;
#pragma unroll
            for (int r = 0; r < SR; ++r) {
                if (l == ls[r] && act[r]) {
                    const double2 s0 = D.st[(long long)m * npair + pr[r]];
                    v1[r] = s0.x; v0[r] = s0.y;
                    kk[r] = D.stk[(long long)m * npair + pr[r]];
                }
                if (ls[r] <= L && (l < ls[r] || __any(kk[r] < 0))) live = false;
            }
            if (live) break;
            const AnaCoef c = cf[l];
            const double2 t = NC != 2 ? aT[l] : z2;
            const double2 e = NC != 1 ? aE[l] : z2;
            const double2 b = NC != 1 ? aB[l] : z2;
            const bool even = ((l - m) & 1) == 0;
#pragma unroll
            for (int r = 0; r < SR; ++r) {
                if (l < ls[r]) continue;
                const double w0 = kk[r] == 0 ? v0[r] : 0.0, w1 = kk[r] == 0 ? v1[r] : 0.0;
                const double xw0 = mul_nc(x[r], w0), xw1 = mul_nc(x[r], w1);
                if (even) syn_accumulate<NC, true>(A[r], c, w0, w1, xw0, xw1, s2[r], t, e, b);
                else syn_accumulate<NC, false>(A[r], c, w0, w1, xw0, xw1, s2[r], t, e, b);
                if (l < L) {
                    rec_ana(c, mul_nc(x[r], v0[r]), v0[r], v1[r]);
                    if (kk[r] < 0 && fabs(v0[r]) > SC_HI) { v0[r] *= SC_DN; v1[r] *= SC_DN; ++kk[r]; }
                }
            }
            ++l;
        }
        // ---- fast path: every live slot active and representable; x lambda_{l-1}
        // carried from the previous step (the same rounded product) ----
#pragma unroll
        for (int r = 0; r < SR; ++r) xv1[r] = mul_nc(x[r], v1[r]);
        if (l <= L && ((l - m) & 1)) {
            const AnaCoef c = cf[l];
            const double2 t = NC != 2 ? aT[l] : z2, e = NC != 1 ? aE[l] : z2, b = NC != 1 ? aB[l] : z2;
#pragma unroll
            for (int r = 0; r < SR; ++r) {
                if (ls[r] > L) continue;
                const double xv0 = mul_nc(x[r], v0[r]);
                syn_accumulate<NC, false>(A[r], c, v0[r], v1[r], xv0, xv1[r], s2[r], t, e, b);
                rec_ana(c, xv0, v0[r], v1[r]);       // past L: unused
                xv1[r] = xv0;
            }
            ++l;
        }
#if defined(GS_ASM_MARKERS)
        asm volatile("; SYN_FAST_BEGIN");
#endif
#if GS_SYN_PF > 0
        // the coefficient and a_lm lines GS_SYN_PF l ahead pulled into L2 by one
        // vector load (lanes 4k + j: stream j), consumed one step later
        double pfv = 0.0;
        const double* pfs = (lane & 3) == 0 ? reinterpret_cast<const double*>(cf)
                          : reinterpret_cast<const double*>(NC == 1 ? aT : ((lane & 3) == 1 ? aT : ((lane & 3) == 2 ? aE : aB)));
        const int pfw = (lane & 3) == 0 ? 6 : 2;            // doubles per l of the stream
#endif
        for (; l + 1 <= L; l += 2) {
#if GS_SYN_PF > 0
            if (pfv == 7.0e300) { if constexpr (NC == 1) A[0].tp[0] += 1.0; else A[0].sp[0] += 1.0; }
            pfv = pfs[(long long)min(l + GS_SYN_PF, L) * pfw];
#endif
            const AnaCoef c0 = cf[l], c1 = cf[l + 1];
            const double2 t0 = NC != 2 ? aT[l] : z2, e0 = NC != 1 ? aE[l] : z2, b0 = NC != 1 ? aB[l] : z2;
            const double2 t1 = NC != 2 ? aT[l + 1] : z2, e1 = NC != 1 ? aE[l + 1] : z2, b1 = NC != 1 ? aB[l + 1] : z2;
#pragma unroll
            for (int r = 0; r < SR; ++r) {
                if (ls[r] > L) continue;
                const double xa = mul_nc(x[r], v0[r]);
                syn_accumulate<NC, true>(A[r], c0, v0[r], v1[r], xa, xv1[r], s2[r], t0, e0, b0);
                rec_ana(c0, xa, v0[r], v1[r]);
                const double xb = mul_nc(x[r], v0[r]);
                syn_accumulate<NC, false>(A[r], c1, v0[r], v1[r], xb, xa, s2[r], t1, e1, b1);
                rec_ana(c1, xb, v0[r], v1[r]);
                xv1[r] = xb;
            }
        }
        if (l <= L) {
            const AnaCoef c = cf[l];
            const double2 t = NC != 2 ? aT[l] : z2, e = NC != 1 ? aE[l] : z2, b = NC != 1 ? aB[l] : z2;
#pragma unroll
            for (int r = 0; r < SR; ++r) {
                if (ls[r] > L) continue;
                syn_accumulate<NC, true>(A[r], c, v0[r], v1[r], mul_nc(x[r], v0[r]), xv1[r], s2[r], t, e, b);
            }
        }
        // ---- outputs ----
        const long long plane = phi_plane(L, npair);
#pragma unroll
        for (int r = 0; r < SR; ++r) {
            if (!act[r]) continue;
            syn_store<NC>(A[r], phi, plane, phi_at(m, pr[r], npair), D.geom[pr[r]].is2);
        }
    }
}

// l-segmented synthesis for small maps (D.seg > 0, one ring group per lane):
// workgroup = (m, 64-pair group), wave w = segment w of m's l range, entered
// at lA = m + w seg with the plan-time recurrence state (or at the group's
// onset, if later); the segments' partial sums meet in LDS and wave 0 adds
// them in segment order.  The chain of one wave is <= seg l steps instead of
// L + 1 - m.  Waves whose segment starts past L end at once (before the
// barrier; an ended wave no longer counts at it).
template <int NC>
__global__ __launch_bounds__(1024) void k_sht_synth_leg_seg(ShtDev D, const AnaCoef* __restrict__ coef,
                                                           const double2* __restrict__ ain,
                                                           double2* __restrict__ phi) {
    // per wave a slice of SEG_SLICE doubles: the segment's recurrence / spin-2
    // coefficients (66 l: the loop reads up to l + 2) and a_lm (64 l per comp),
    // staged once with coalesced vector loads (the single-walk kernel reads them
    // as scalar loads per l, a memory latency per step); after the walk the
    // slice holds the wave's 12 x 64 partial sums
    constexpr int SEG_SLICE = 66 * 8 + 3 * 64 * 2;
    extern __shared__ __attribute__((aligned(16))) double sred[];   // [waves][SEG_SLICE]
    const int L = D.L, npair = D.npair, nlm = D.nlm;
    const int m = blockIdx.x, grp = blockIdx.y;
    ain += (long long)blockIdx.z * NC * nlm;                       // map b of a batch
    phi += (long long)blockIdx.z * NC * 2 * phi_plane(L, npair);
    const int lane = threadIdx.x & 63;
    const int sg = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lA = m + sg * D.seg;
    if (lA > L) return;
    const int nact = (L - m) / D.seg + 1;                 // segments of this m
    const int lend = min(lA + D.seg - 1, L);
    const int pr = grp * 64 + lane;
    const bool act = pr < npair;
    const double x = act ? D.geom[pr].x : 0.0;
    const double is2 = act ? D.geom[pr].is2 : 0.0;
    const double s2 = ring_s2(act, is2);
    int ls = __builtin_amdgcn_readfirstlane(D.lstart[(long long)m * D.ngroup + grp]);
    const bool tab = ls <= L && ls < lA;
    if (tab) ls = lA;
    if (ls > lend) ls = L + 1;
    const double2 z2 = make_double2(0.0, 0.0);
    SynAcc A;
#pragma unroll
    for (int i = 0; i < 2; ++i) { A.tp[i] = 0.0; A.tn[i] = 0.0; }
#pragma unroll
    for (int i = 0; i < 4; ++i) { A.sp[i] = 0.0; A.sn[i] = 0.0; }
    double v0 = 0.0, v1 = 0.0;
    int kk = 0;
    if (tab && ls <= L && act) {
        const long long o = (long long)(D.segoff[m] + sg * D.segmul - 1) * npair + pr;
        const double2 s0 = D.sst[o];
        v1 = s0.x; v0 = s0.y;
        kk = D.sstk[o];
    }
    const long long base = cidx(L, m, m) - m;
    double* slice = sred + (long long)sg * SEG_SLICE;
    {
        const AnaCoef* cfg = coef + base;
        auto put = [&](int slot, int l) {
            const double2* src = reinterpret_cast<const double2*>(cfg + l);
            double2* dst = reinterpret_cast<double2*>(slice + slot * 6);
            const double2 q0 = src[0], q1 = src[1], q2 = src[2];
            dst[0] = q0; dst[1] = q1; dst[2] = q2;
        };
        put(lane, min(lA + lane, L));
        if (lane < 2) put(64 + lane, min(lA + 64 + lane, L));
        const int la = min(lA + lane, L);
        double2* as = reinterpret_cast<double2*>(slice + 66 * 8);
        if constexpr (NC != 2) as[lane] = ain[base + la];
        if constexpr (NC != 1) {
            const double2* aEg = ain + (NC == 3 ? nlm : 0) + base;
            as[(NC == 3 ? 64 : 0) + lane] = aEg[la];
            as[(NC == 3 ? 128 : 64) + lane] = aEg[nlm + la];
        }
    }
    __syncthreads();            // every wave still running reaches it (ended waves do not count)
    const AnaCoef* cfs = reinterpret_cast<const AnaCoef*>(slice);
    const double2* as = reinterpret_cast<const double2*>(slice + 66 * 8);
    auto cf = [&](int l) { return cfs[l - lA]; };
    auto aT = [&](int l) { return as[l - lA]; };
    auto aE = [&](int l) { return as[(NC == 3 ? 64 : 0) + l - lA]; };
    auto aB = [&](int l) { return as[(NC == 3 ? 128 : 64) + l - lA]; };
    if (ls <= L) {
        int l = ls;
        // slow path: activation at the onset, scaled lanes
        while (l <= lend) {
            if (l == ls && act && !tab) {
                const double2 s0 = D.st[(long long)m * npair + pr];
                v1 = s0.x; v0 = s0.y;
                kk = D.stk[(long long)m * npair + pr];
            }
            if (!__any(kk < 0)) break;
            const AnaCoef c = cf(l);
            const double2 t = NC != 2 ? aT(l) : z2;
            const double2 e = NC != 1 ? aE(l) : z2;
            const double2 b = NC != 1 ? aB(l) : z2;
            const double w0 = kk == 0 ? v0 : 0.0, w1 = kk == 0 ? v1 : 0.0;
            const double xw0 = mul_nc(x, w0), xw1 = mul_nc(x, w1);
            if (((l - m) & 1) == 0) syn_accumulate<NC, true>(A, c, w0, w1, xw0, xw1, s2, t, e, b);
            else syn_accumulate<NC, false>(A, c, w0, w1, xw0, xw1, s2, t, e, b);
            if (l < L) {
                rec_ana(c, mul_nc(x, v0), v0, v1);
                if (kk < 0 && fabs(v0) > SC_HI) { v0 *= SC_DN; v1 *= SC_DN; ++kk; }
            }
            ++l;
        }
        // fast path (onset state loaded above when the onset is the first l)
        double xv1 = mul_nc(x, v1);
        if (l <= lend && ((l - m) & 1)) {
            const AnaCoef c = cf(l);
            const double2 t = NC != 2 ? aT(l) : z2, e = NC != 1 ? aE(l) : z2, b = NC != 1 ? aB(l) : z2;
            const double xv0 = mul_nc(x, v0);
            syn_accumulate<NC, false>(A, c, v0, v1, xv0, xv1, s2, t, e, b);
            rec_ana(c, xv0, v0, v1);                 // past L: unused
            xv1 = xv0;
            ++l;
        }
        for (; l + 1 <= lend; l += 2) {
            const AnaCoef c0 = cf(l), c1 = cf(l + 1);
            const double2 t0 = NC != 2 ? aT(l) : z2, e0 = NC != 1 ? aE(l) : z2, b0 = NC != 1 ? aB(l) : z2;
            const double2 t1 = NC != 2 ? aT(l + 1) : z2, e1 = NC != 1 ? aE(l + 1) : z2, b1 = NC != 1 ? aB(l + 1) : z2;
            const double xa = mul_nc(x, v0);
            syn_accumulate<NC, true>(A, c0, v0, v1, xa, xv1, s2, t0, e0, b0);
            rec_ana(c0, xa, v0, v1);
            const double xb = mul_nc(x, v0);
            syn_accumulate<NC, false>(A, c1, v0, v1, xb, xa, s2, t1, e1, b1);
            rec_ana(c1, xb, v0, v1);
            xv1 = xb;
        }
        if (l <= lend) {
            const AnaCoef c = cf(l);
            const double2 t = NC != 2 ? aT(l) : z2, e = NC != 1 ? aE(l) : z2, b = NC != 1 ? aB(l) : z2;
            syn_accumulate<NC, true>(A, c, v0, v1, mul_nc(x, v0), xv1, s2, t, e, b);
        }
    }
    // segment partial sums -> LDS; wave 0 adds them in segment order
    double* my = slice + lane;      // this wave's own slice (its staging is no longer read)
#pragma unroll
    for (int i = 0; i < 2; ++i) { my[i * 64] = A.tp[i]; my[(2 + i) * 64] = A.tn[i]; }
#pragma unroll
    for (int i = 0; i < 4; ++i) { my[(4 + i) * 64] = A.sp[i]; my[(8 + i) * 64] = A.sn[i]; }
    __syncthreads();
    if (sg != 0 || !act) return;
    for (int w = 1; w < nact; ++w) {
        const double* o = sred + (long long)w * SEG_SLICE + lane;
#pragma unroll
        for (int i = 0; i < 2; ++i) { A.tp[i] += o[i * 64]; A.tn[i] += o[(2 + i) * 64]; }
#pragma unroll
        for (int i = 0; i < 4; ++i) { A.sp[i] += o[(4 + i) * 64]; A.sn[i] += o[(8 + i) * 64]; }
    }
    syn_store<NC>(A, phi, phi_plane(L, npair), phi_at(m, pr, npair), is2);
}

// ---------------------------------------------------------------------------
// f2 block synthesis (pixel-domain NC likelihood, NonCenteredGibbs.py:333-355):
// the maps y_k = A(delta a_k) of K Metropolis blocks at once.  Every (l, field)
// belongs to at most one block (blk[f][l], -1: none), so one pass of the
// Legendre recurrence per (m, ring pair) serves every block: the field's
// accumulator is flushed to block k's phase plane when l leaves block k and
// reset, i.e. the recurrence is shared and only the outputs multiply.
// NC = 1: T (spin 0, one output comp per block); 2: E, B -> Q, U (two comps).
// phib: [K * NCO comps][ns][phi plane]; block k's comps hold only m <= its
// largest l (the ring stage reads no further, comp_lmax).
// ---------------------------------------------------------------------------
struct BlkAcc { double p[4], n[4]; };

template <int NC, bool EVEN>
__device__ __forceinline__ void blk_accumulate(BlkAcc& A, int f, const LegCoef& c, double v0, double v1, double is2,
                                               double xis2, double2 a) {
    if constexpr (NC == 1) {
        double* t = EVEN ? A.p : A.n;
        t[0] = fma(a.x, v0, t[0]);
        t[1] = fma(a.y, v0, t[1]);
    } else {
        const double F1 = fma(c.R * xis2, v1, -fma(c.P, is2, c.Q) * v0);
        const double F2 = fma(c.Rm * is2, v1, -(c.T * xis2) * v0);
        double* a1 = EVEN ? A.p : A.n;   // F1 carries lambda's parity
        double* a2 = EVEN ? A.n : A.p;   // F2 the opposite one
        if (f == 0) {                    // E
            a1[0] = fma(a.x, F1, a1[0]); a1[1] = fma(a.y, F1, a1[1]);
            a2[2] = fma(a.y, F2, a2[2]); a2[3] = fma(-a.x, F2, a2[3]);
        } else {                         // B
            a2[0] = fma(-a.y, F2, a2[0]); a2[1] = fma(a.x, F2, a2[1]);
            a1[2] = fma(a.x, F1, a1[2]); a1[3] = fma(a.y, F1, a1[3]);
        }
    }
}

// STG: the m's recurrence coefficients, a_lm and block indices (l = m..L) are
// staged in LDS by coalesced loads once per m (small l_max: <= 64 KB), instead
// of wave-uniform scalar loads -- one memory latency -- per l step
// A batch of chains (blockIdx.z = chain): chain z's inputs at ain + z NF nlm, its
// planes at phib + z chain_stride (the block table is shared: every chain of a
// batch sweeps the same blocks); each chain's arithmetic is the one-chain one.
template <int NC, int SR, bool STG>
__global__ __launch_bounds__(LEG_BLOCK) void k_sht_synth_blocks(ShtDev D, const LegCoef* __restrict__ coef,
                                                                const double2* __restrict__ ain,
                                                                const int* __restrict__ blk,
                                                                double2* __restrict__ phib, int paired,
                                                                long long chain_stride) {
    extern __shared__ __attribute__((aligned(16))) double2 bstage[];
    constexpr int NF = NC;                      // input fields
    constexpr int NCO = NC == 1 ? 1 : 2;        // output comps per block
    const int L = D.L, npair = D.npair, nlm = D.nlm;
    ain += (long long)blockIdx.z * NF * nlm;
    phib += (long long)blockIdx.z * chain_stride;
    // XCD-aware remap (bijective): workgroups are dealt round-robin over the 8
    // XCDs; give each XCD a contiguous range of (tile, m) items, m fastest, so
    // the four m of one [m/4] group of the phase planes are written by
    // neighbouring workgroups of one XCD and their 16-B pieces of each 64-B run
    // meet in that XCD's L2 before write-back (the planes are written 16 B per
    // lane at a 64-B stride)
    const int gx = gridDim.x, nwg = gx * gridDim.y;
    const int bl = blockIdx.x + blockIdx.y * gx;
    const int xcd = bl & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int wgl = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bl >> 3);
    const int q = wgl % gx, tile = wgl / gx;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g0 = tile * (LEG_BLOCK / 64) * SR + wave * SR;
    double x[SR], is2[SR], xis2[SR];
    int pr[SR];
    bool act[SR];
#pragma unroll
    for (int r = 0; r < SR; ++r) {
        pr[r] = (g0 + r) * 64 + lane;
        act[r] = pr[r] < npair;
        x[r] = act[r] ? D.geom[pr[r]].x : 0.0;
        is2[r] = act[r] ? D.geom[pr[r]].is2 : 0.0;
        xis2[r] = x[r] * is2[r];
    }
    const long long plane = phi_plane(L, npair);
    for (int h = 0; h < 2; ++h) {
        const int m = h == 0 ? q : L - q;
        if (h == 1 && (!paired || m <= q)) break;
        int ls[SR];
        int lmin = L + 1;
#pragma unroll
        for (int r = 0; r < SR; ++r) {
            ls[r] = __builtin_amdgcn_readfirstlane(g0 + r < D.ngroup ? D.lstart[(long long)m * D.ngroup + g0 + r]
                                                                     : L + 1);
            lmin = min(lmin, ls[r]);
        }
        BlkAcc A[NF][SR];
        double v0[SR], v1[SR];
        int kk[SR];
#pragma unroll
        for (int f = 0; f < NF; ++f)
#pragma unroll
            for (int r = 0; r < SR; ++r)
#pragma unroll
                for (int i = 0; i < 4; ++i) { A[f][r].p[i] = 0.0; A[f][r].n[i] = 0.0; }
#pragma unroll
        for (int r = 0; r < SR; ++r) { v0[r] = 0.0; v1[r] = 0.0; kk[r] = 0; }
        int cur[NF];
#pragma unroll
        for (int f = 0; f < NF; ++f) cur[f] = -1;
        const long long base = cidx(L, m, m) - m;
        const LegCoef* cf = coef + base;
        const double2* a0 = ain + base;
        const int nl = L + 1 - m;                  // l = m .. L
        const LegCoef* cfs = nullptr;
        const double2* as = nullptr;
        const int* bs = nullptr;
        if constexpr (STG) {
            __syncthreads();                       // the previous m's readers are done
            double2* c2 = bstage;                                  // [nl][4] (LegCoef)
            double2* a2 = bstage + 4 * nl;                         // [NF][nl]
            int* b2 = reinterpret_cast<int*>(a2 + NF * nl);        // [NF][nl]
            const double2* src = reinterpret_cast<const double2*>(coef + base + m);
            for (int i = threadIdx.x; i < 4 * nl; i += LEG_BLOCK) c2[i] = src[i];
            for (int i = threadIdx.x; i < NF * nl; i += LEG_BLOCK) {
                const int f = i / nl, j = i - f * nl;
                a2[i] = a0[(long long)f * nlm + m + j];
                b2[i] = blk[f * (L + 1) + m + j];
            }
            __syncthreads();
            cfs = reinterpret_cast<const LegCoef*>(c2);
            as = a2;
            bs = b2;
        }
        auto CF = [&](int l) -> LegCoef { if constexpr (STG) return cfs[l - m]; else return cf[l]; };
        auto AL = [&](int f, int l) -> double2 {
            if constexpr (STG) return as[f * nl + l - m]; else return a0[(long long)f * nlm + l];
        };
        auto BK = [&](int f, int l) -> int { if constexpr (STG) return bs[f * nl + l - m]; else return blk[f * (L + 1) + l]; };
        // write field f's accumulators to its current block's planes (if any), reset
        auto flush = [&](int f) {
            const int k = cur[f];
            GS_ASSERT(k < 0 || m <= L);
#pragma unroll
            for (int r = 0; r < SR; ++r) {
                BlkAcc& B = A[f][r];
                if (k >= 0 && act[r]) {
                    const long long o = phi_at(m, pr[r], npair);
                    double2* P = phib + (long long)(k * NCO) * 2 * plane;
                    if constexpr (NC == 1) {
                        P[o] = make_double2(B.p[0] + B.n[0], B.p[1] + B.n[1]);
                        P[plane + o] = make_double2(B.p[0] - B.n[0], B.p[1] - B.n[1]);
                    } else {
                        P[o] = make_double2(-(B.p[0] + B.n[0]), -(B.p[1] + B.n[1]));
                        P[plane + o] = make_double2(-(B.p[0] - B.n[0]), -(B.p[1] - B.n[1]));
                        P[2 * plane + o] = make_double2(-(B.p[2] + B.n[2]), -(B.p[3] + B.n[3]));
                        P[3 * plane + o] = make_double2(-(B.p[2] - B.n[2]), -(B.p[3] - B.n[3]));
                    }
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) { B.p[i] = 0.0; B.n[i] = 0.0; }
            }
        };
        auto track = [&](int l) {
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const int b = BK(f, l);
                if (b != cur[f]) { flush(f); cur[f] = b; }
            }
        };
        // blocks wholly below every slot's onset: zero planes (their terms underflow)
        for (int l = m; l < lmin && l <= L; ++l) track(l);
        int l = lmin;
        // ---- slow path: slot activation and scaled lanes ----
        while (l <= L) {
            bool live = true;
#pragma unroll
            for (int r = 0; r < SR; ++r) {
                if (l == ls[r] && act[r]) {
                    const double2 s0 = D.st[(long long)m * npair + pr[r]];
                    v1[r] = s0.x; v0[r] = s0.y;
                    kk[r] = D.stk[(long long)m * npair + pr[r]];
                }
                if (ls[r] <= L && (l < ls[r] || __any(kk[r] < 0))) live = false;
            }
            if (live) break;
            track(l);
            const LegCoef c = CF(l);
            const LegCoef cn = CF(min(l + 1, L));
            const bool even = ((l - m) & 1) == 0;
#pragma unroll
            for (int r = 0; r < SR; ++r) {
                if (l < ls[r]) continue;
                const double w0 = kk[r] == 0 ? v0[r] : 0.0, w1 = kk[r] == 0 ? v1[r] : 0.0;
#pragma unroll
                for (int f = 0; f < NF; ++f) {
                    const double2 a = AL(f, l);
                    if (even) blk_accumulate<NC, true>(A[f][r], f, c, w0, w1, is2[r], xis2[r], a);
                    else blk_accumulate<NC, false>(A[f][r], f, c, w0, w1, is2[r], xis2[r], a);
                }
                if (l < L) {
                    rec_step(cn, x[r], v0[r], v1[r]);
                    if (kk[r] < 0 && fabs(v0[r]) > SC_HI) { v0[r] *= SC_DN; v1[r] *= SC_DN; ++kk[r]; }
                }
            }
            ++l;
        }
        // ---- every live slot active and representable ----
        for (; l <= L; ++l) {
            track(l);
            const LegCoef c = CF(l);
            const LegCoef cn = CF(min(l + 1, L));
            const bool even = ((l - m) & 1) == 0;
            double2 a[NF];
#pragma unroll
            for (int f = 0; f < NF; ++f) a[f] = AL(f, l);
#pragma unroll
            for (int r = 0; r < SR; ++r) {
                if (ls[r] > L) continue;
#pragma unroll
                for (int f = 0; f < NF; ++f) {
                    if (even) blk_accumulate<NC, true>(A[f][r], f, c, v0[r], v1[r], is2[r], xis2[r], a[f]);
                    else blk_accumulate<NC, false>(A[f][r], f, c, v0[r], v1[r], is2[r], xis2[r], a[f]);
                }
                if (l < L) rec_step(cn, x[r], v0[r], v1[r]);
            }
        }
#pragma unroll
        for (int f = 0; f < NF; ++f) flush(f);
    }
}

// ---------------------------------------------------------------------------
// ring FFTs (block-wide, in place, buffer in LDS or global scratch)
// ---------------------------------------------------------------------------
// forward (dir = -1): X_k = sum_j x_j e^{-2 pi i jk/M};  dir = +1: conjugate
// twiddles; tw[k] = e^{-2 pi i k / Mmax}, k < Mmax/2.  Each thread owns at most
// NB butterflies per stage (M / 2 <= NB * blockDim).
// e^{dir 2 pi i t / Mmax} for 0 <= t < Mmax from the half-circle table, or
// (Mmax < 0: a ring workgroup whose full table does not fit its LDS) from the
// two-level LDS tables hi[a] = e^{-2 pi i 64 a / |Mmax|}, lo[b] = e^{-2 pi i b /
// |Mmax|} (b < 64) at tw, tw + |Mmax| / 64: one complex product, no global load
__device__ __forceinline__ double2 twid(int t, int dir, const double2* __restrict__ tw, int Mmax) {
    if (Mmax < 0) {
        double2 w = cmul(tw[t >> 6], tw[(-Mmax >> 6) + (t & 63)]);
        if (dir > 0) w.y = -w.y;
        return w;
    }
    const int h = Mmax >> 1;
    double2 w = tw[t < h ? t : t - h];
    if (t >= h) { w.x = -w.x; w.y = -w.y; }
    if (dir > 0) w.y = -w.y;
    return w;
}

// v <- DFT_R(v) in registers, natural order: v_k = sum_n v_n e^{dir 2 pi i nk/R}
// (R = 8: three radix-2 decimation-in-frequency levels, then the bit reversal)
template <int R>
__device__ __forceinline__ void dft_reg(double2* v, int dir) {
    const double sg = dir > 0 ? 1.0 : -1.0;
    auto bfly = [](double2& a, double2& b) {
        const double2 t = make_double2(a.x - b.x, a.y - b.y);
        a = make_double2(a.x + b.x, a.y + b.y);
        b = t;
    };
    // multiply by e^{sg i pi / 2} = sg i
    auto rot4 = [&](double2 a) { return make_double2(-sg * a.y, sg * a.x); };
    if constexpr (R == 2) {
        bfly(v[0], v[1]);
    } else if constexpr (R == 4) {
        bfly(v[0], v[2]); bfly(v[1], v[3]);
        v[3] = rot4(v[3]);
        bfly(v[0], v[1]); bfly(v[2], v[3]);
        const double2 t = v[1]; v[1] = v[2]; v[2] = t;          // bit reversal
    } else if constexpr (R == 16) {
        // 16 = 4 x 4: DFT_4 over a of v[4a + b], the twiddles e^{dir 2 pi i b k1 / 16},
        // DFT_4 over b; X[k1 + 4 k2]
        constexpr double W[10][2] = {{1.0, 0.0},
                                     {0.92387953251128675613, 0.38268343236508977173},
                                     {0.70710678118654752440, 0.70710678118654752440},
                                     {0.38268343236508977173, 0.92387953251128675613},
                                     {0.0, 1.0},
                                     {-0.38268343236508977173, 0.92387953251128675613},
                                     {-0.70710678118654752440, 0.70710678118654752440},
                                     {-0.92387953251128675613, 0.38268343236508977173},
                                     {-1.0, 0.0},
                                     {-0.92387953251128675613, -0.38268343236508977173}};
        double2 t[4][4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            double2 q[4] = {v[b], v[4 + b], v[8 + b], v[12 + b]};
            dft_reg<4>(q, dir);
#pragma unroll
            for (int k = 0; k < 4; ++k) t[b][k] = q[k];
        }
#pragma unroll
        for (int b = 1; b < 4; ++b)
#pragma unroll
            for (int k = 1; k < 4; ++k) t[b][k] = cmul(t[b][k], make_double2(W[b * k][0], sg * W[b * k][1]));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            double2 q[4] = {t[0][k], t[1][k], t[2][k], t[3][k]};
            dft_reg<4>(q, dir);
#pragma unroll
            for (int k2 = 0; k2 < 4; ++k2) v[k + 4 * k2] = q[k2];
        }
    } else {
        constexpr double C = 0.70710678118654752440;
        bfly(v[0], v[4]); bfly(v[1], v[5]); bfly(v[2], v[6]); bfly(v[3], v[7]);
        // v5 *= W8, v6 *= W8^2, v7 *= W8^3 (W8 = e^{sg i pi/4})
        v[5] = make_double2(C * (v[5].x - sg * v[5].y), C * (v[5].y + sg * v[5].x));
        v[6] = rot4(v[6]);
        v[7] = make_double2(C * (-v[7].x - sg * v[7].y), C * (-v[7].y + sg * v[7].x));
        bfly(v[0], v[2]); bfly(v[1], v[3]); bfly(v[4], v[6]); bfly(v[5], v[7]);
        v[3] = rot4(v[3]); v[7] = rot4(v[7]);
        bfly(v[0], v[1]); bfly(v[2], v[3]); bfly(v[4], v[5]); bfly(v[6], v[7]);
        double2 t = v[1]; v[1] = v[4]; v[4] = t;                 // bit reversal (1 4)(3 6)
        t = v[3]; v[3] = v[6]; v[6] = t;
    }
}

// elementwise operations an FFT applies to its input as the first pass reads it
// and to its output before the last pass writes it (index in natural order)
struct FftId {
    __device__ __forceinline__ double2 operator()(int, double2 v) const { return v; }
};

// one Stockham stage of radix R at span Ns (Ns = product of the earlier
// radices): butterfly j reads x[j + k M/R], twiddles by e^{dir 2 pi i (j mod Ns) k
// / (Ns R)}, and writes y[(j - j mod Ns) R + j mod Ns + k Ns] (in place: all
// reads, barrier, all writes).  NV complex values per thread at most.  The first
// stage (Ns = 1) applies in to what it reads, the last (Ns R = M) out to what
// it writes -- the Bluestein chirp / kernel products without passes of their own
template <int R, int NV, class In = FftId, class Out = FftId>
__device__ __forceinline__ void stockham_stage(double2* buf, int M, int Ns, int dir, const double2* __restrict__ tw,
                                               int Mmax, const In& in = In{}, const Out& out = Out{}) {
    constexpr int NBF = NV / R > 0 ? NV / R : 1;   // radix 16 at 8 values per thread: half the threads
    const int nb = M / R;
    const int step = (Mmax < 0 ? -Mmax : Mmax) / (Ns * R);
    double2 v[NBF][R];
#pragma unroll
    for (int b = 0; b < NBF; ++b) {
        const int j = threadIdx.x + b * blockDim.x;
        if (j < nb) {
#pragma unroll
            for (int k = 0; k < R; ++k) v[b][k] = buf[j + k * nb];
            if (Ns == 1) {
#pragma unroll
                for (int k = 0; k < R; ++k) v[b][k] = in(j + k * nb, v[b][k]);
            }
            if (Ns > 1) {
                const int jm = j & (Ns - 1);
                if (R == 8 && Mmax < 0) {
                    // two-level tables: w^k from one lookup of w (depth <= 3
                    // products) -- 2 LDS reads per butterfly instead of 14
                    const double2 w1 = twid(jm * step, dir, tw, Mmax);
                    const double2 w2 = cmul(w1, w1), w4 = cmul(w2, w2);
                    const double2 w[8] = {w1, w1, w2, cmul(w1, w2), w4, cmul(w1, w4), cmul(w2, w4),
                                          cmul(cmul(w1, w2), w4)};
#pragma unroll
                    for (int k = 1; k < R; ++k) v[b][k] = cmul(v[b][k], w[k]);
                } else {
#pragma unroll
                    for (int k = 1; k < R; ++k) v[b][k] = cmul(v[b][k], twid(jm * k * step, dir, tw, Mmax));
                }
            }
            dft_reg<R>(v[b], dir);
            if (Ns * R == M) {
                const int jm = j & (Ns - 1);
                const int base = (j - jm) * R + jm;
#pragma unroll
                for (int k = 0; k < R; ++k) v[b][k] = out(base + k * Ns, v[b][k]);
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < NBF; ++b) {
        const int j = threadIdx.x + b * blockDim.x;
        if (j < nb) {
            const int jm = j & (Ns - 1);
            const int base = (j - jm) * R + jm;
#pragma unroll
            for (int k = 0; k < R; ++k) buf[base + k * Ns] = v[b][k];
        }
    }
    __syncthreads();
}

// in-place power-of-two FFT in buf (LDS or global scratch), M <= 2 NB blockDim:
// mixed-radix Stockham, one radix-16 or radix-4 stage first (M = 2^(3q+1), or
// 2^(3q+2); radix 2 at M = 2), then radix-8 stages -- 4 block-wide passes at M =
// 8192 instead of 13
template <int NB, class In = FftId, class Out = FftId>
__device__ __forceinline__ void fft_pow2(double2* buf, int M, int dir, const double2* __restrict__ tw, int Mmax,
                                         const In& in = In{}, const Out& out = Out{}) {
    constexpr int NV = 2 * NB;
    const int p = 31 - __clz(M);
    int Ns = 1;
    if (p % 3 == 1 && p >= 4) { stockham_stage<16, NV>(buf, M, 1, dir, tw, Mmax, in, out); Ns = 16; }
    else if (p % 3 == 1) { stockham_stage<2, NV>(buf, M, 1, dir, tw, Mmax, in, out); Ns = 2; }
    else if (p % 3 == 2) { stockham_stage<4, NV>(buf, M, 1, dir, tw, Mmax, in, out); Ns = 4; }
    for (; Ns < M; Ns *= 8) stockham_stage<8, NV>(buf, M, Ns, dir, tw, Mmax, in, out);
}

// an elementwise pass over j < n in batches of U per thread (j = j0 + u
// blockDim): every load of a batch is issued before its first use -- one
// memory round trip per batch instead of one per element (a large ring
// workgroup has its CU to itself, nothing else hides the latency); the uses
// run in the same order on the same values
// (U capped at 8: the 16-per-thread passes of the global-scratch classes
// would spill)
constexpr int ew_u(int u) { return u > 8 ? 8 : u; }
template <int U, class Ld, class Use>
__device__ __forceinline__ void ew_pass(int n, Ld ld, Use use) {
    using T = decltype(ld(0));
    for (int j0 = threadIdx.x; j0 < n; j0 += U * blockDim.x) {
        T v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = j0 + u * blockDim.x;
            if (j < n) v[u] = ld(j);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = j0 + u * blockDim.x;
            if (j < n) use(j, v[u]);
        }
    }
}

// forward DFT of length n held in buf[0..n) (Bluestein when n is not a power
// of two: M = g.M, kernel V = FFT of the chirp, followed in the plan's table by
// the chirp c_j = e^{-i pi j^2 / n}, j < n, itself -- tabulated at plan time
// with the same function, so the ring kernels load it instead of two fp64
// sincospi per element); result in buf[0..n)
// (cj: conj(DFT(conj x)) -- the conjugations ride in the first and last products)
// The products with the chirp (x_j c_j, j < n; 0 past n), the kernel V and the
// chirp again (with 1 / M) are applied by the FFTs' first / last passes as they
// read / write (FftId hooks): the same operations as separate passes, 3 LDS
// round trips and 3 barriers fewer
template <int NB>
__device__ __forceinline__ void bluestein_forward(double2* buf, int n, int M, const double2* __restrict__ V,
                                  const double2* __restrict__ tw, int Mmax, bool cj = false) {
    const double2* __restrict__ C = V + M;
    const double2 z = make_double2(0.0, 0.0);
    const double inv = 1.0 / M;
    // c_j = e^{-i pi j^2/n}
    auto chirp_in = [&](int j, double2 x) {
        if (j >= n) return z;
        if (cj) x.y = -x.y;
        return cmul(x, C[j]);
    };
    auto kern = [&](int j, double2 y) { return cmul(y, V[j]); };
    auto chirp_out = [&](int j, double2 y) {
        if (j >= n) return y;
        const double2 v = cmul(y, C[j]);
        double2 r = make_double2(v.x * inv, v.y * inv);
        if (cj) r.y = -r.y;
        return r;
    };
    fft_pow2<NB>(buf, M, -1, tw, Mmax, chirp_in, kern);
    fft_pow2<NB>(buf, M, +1, tw, Mmax, FftId{}, chirp_out);
}

// conj(DFT(conj x)) = unnormalised inverse DFT, Bluestein of length n
template <int NB>
__device__ __forceinline__ void bluestein_inverse(double2* buf, int n, int M, const double2* __restrict__ V,
                                  const double2* __restrict__ tw, int Mmax) {
    bluestein_forward<NB>(buf, n, M, V, tw, Mmax, true);
}

template <int NB>
__device__ __forceinline__ void dft_forward(double2* buf, const PairGeom& g, const double2* __restrict__ tw, int Mmax,
                            const double2* __restrict__ bsk) {
    if (g.bs_off < 0) { fft_pow2<NB>(buf, g.M, -1, tw, Mmax); return; }
    bluestein_forward<NB>(buf, g.nphi, g.M, bsk + g.bs_off, tw, Mmax);
}

// inverse (unnormalised) DFT: y_j = sum_k Z_k e^{+2 pi i jk/n}
template <int NB>
__device__ __forceinline__ void dft_inverse(double2* buf, const PairGeom& g, const double2* __restrict__ tw, int Mmax,
                            const double2* __restrict__ bsk) {
    if (g.bs_off < 0) { fft_pow2<NB>(buf, g.M, +1, tw, Mmax); return; }
    bluestein_inverse<NB>(buf, g.nphi, g.M, bsk + g.bs_off, tw, Mmax);
}

// plan time: V = FFT_M(w), w_t = e^{+i pi t^2/n} for |t| < n (cyclic), then the
// chirp e^{-i pi j^2/n}, j < n, at V + M
__global__ __launch_bounds__(1024) void k_sht_bluestein_setup(const int* __restrict__ pairs,
                                                              const PairGeom* __restrict__ geom,
                                                              const double2* __restrict__ tw, int Mmax,
                                                              double2* __restrict__ bsk) {
    const PairGeom g = geom[pairs[blockIdx.x]];
    double2* buf = bsk + g.bs_off;
    const int n = g.split ? g.nphi / 2 : g.nphi, M = g.M;
    for (int t = threadIdx.x; t < M; t += blockDim.x) {
        long long tt = -1;
        if (t < n) tt = t;
        else if (t > M - n) tt = M - t;
        buf[t] = tt >= 0 ? expi_pi_frac(tt * tt, n) : make_double2(0.0, 0.0);
    }
    for (int j = threadIdx.x; j < n; j += blockDim.x) buf[M + j] = expi_pi_neg_u32((unsigned)j * (unsigned)j, n);
    __syncthreads();
    fft_pow2<8>(buf, M, -1, tw, Mmax);
}

__global__ void k_sht_twiddles(int Mmax, double2* __restrict__ tw) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= Mmax / 2) return;
    double sn, cs;
    sincospi(-2.0 * (double)k / (double)Mmax, &sn, &cs);
    tw[k] = make_double2(cs, sn);
}

// threads per FFT workgroup for a class of length M, and butterflies per thread
inline int ring_block(int M) { return std::min(1024, std::max(64, M / 8)); }

// the ring's twiddle table e^{-2 pi i t / M}, t < M / 2, copied into LDS at the
// kernel start (its loads overlap the fold / map loads): the FFT stages then
// read twiddles from LDS instead of one global-memory round trip per stage.
// Visible to the FFT after the barrier that precedes it.
__device__ __forceinline__ const double2* ring_twiddles_lds(double2* twl, int M, const double2* __restrict__ tw,
                                                            int Mmax, int& twM) {
    const int st = Mmax / M;
    for (int t = threadIdx.x; t < M / 2; t += blockDim.x) twl[t] = tw[t * st];
    twM = M;
    return twl;
}
// the two-level tables of twid (Mmax < 0) at twl: Mmax / 64 + 64 entries, read
// from the half-circle table (twM = -Mmax)
__device__ __forceinline__ const double2* ring_twiddles_two(double2* twl, const double2* __restrict__ tw, int Mmax,
                                                            int& twM) {
    const int nh = Mmax >> 6;
    for (int t = threadIdx.x; t < nh + 64; t += blockDim.x)
        twl[t] = twid(t < nh ? 64 * t : t - nh, -1, tw, Mmax);
    twM = -Mmax;
    return twl;
}
// a ring's phase factors e^{i pi t / n}, t < 2n, from two LDS tables (a per-ring
// two-level table built at the kernel start: 2n / 64 + 64 sincospi instead of
// one per use -- the fold's, the split combine's and the phase stores'
// half-pixel and odd-sample factors); tables at tab, visible after a barrier.
// tab == nullptr (the merged one-component launch, whose results the
// multi-component kernels reproduce bit for bit): the direct sincospi
struct RingPh {
    const double2* A;
    const double2* B;
    unsigned n;
    __device__ __forceinline__ double2 pos(unsigned t) const {
        return A ? cmul(A[t >> 6], B[t & 63]) : expi_pi_u32(t, n);
    }
    __device__ __forceinline__ double2 neg(unsigned t) const {
        if (!A) return expi_pi_neg_u32(t, n);
        const double2 e = pos(t);
        return make_double2(e.x, -e.y);
    }
};
__device__ __forceinline__ RingPh ring_phases(double2* tab, unsigned n) {
    if (!tab) return RingPh{nullptr, nullptr, n};
    const int na = (int)((2 * n + 63) / 64);
    for (int i = threadIdx.x; i < na + 64; i += blockDim.x)
        tab[i] = i < na ? expi_pi_u32(64u * (unsigned)i, n) : expi_pi_u32((unsigned)(i - na), n);
    return RingPh{tab, tab + na, n};
}
// LDS entries of ring_phases for rings of a class of length M (n <= M + 1)
inline int ring_ph_entries(int M) { return (2 * M + 2 + 63) / 64 + 64; }

// the same with the loads of a thread issued together (M / 2 <= U blockDim)
template <int U>
__device__ __forceinline__ const double2* ring_twiddles_lds_u(double2* twl, int M, const double2* __restrict__ tw,
                                                              int Mmax, int& twM) {
    const int st = Mmax / M;
    ew_pass<U>(M / 2, [&](int t) { return tw[t * st]; }, [&](int t, double2 v) { twl[t] = v; });
    twM = M;
    return twl;
}

// ---------------------------------------------------------------------------
// synthesis: ring stage.  grid (pairs of this M class, ncomp)
// ---------------------------------------------------------------------------
// Fold: G_k = sum_{m = k mod n, m <= L} c_m Phi_m e^{i m phi0} (c_0 = 1, else 2),
// for north and south; the Hermitian parts of both go into one complex FFT:
// Z_k = (G^N_k + conj G^N_-k)/2 + i (G^S_k + conj G^S_-k)/2.  Thread slot s owns
// the bin pair (k, n-k), k = s mod K (K = n/2 + 1) and the aliases j = s / K
// (mod J); J > 1 only for short rings, reduced in LDS in a fixed order.
struct Fold4 { double2 nk, nmk, sk, smk; };

// the pixel operations a ring stage applies before its pixels leave it: y ->
// the value stored for comp c at the ring pair's pixels iN (north) / iS (south)
// pre / fin: the same operation with the pixel's loads issued first (fin(pre(..),
// y) == operator()(.., y)), so the per-class ring stage batches them
struct PixNone {
    static constexpr bool kConst = false;
    struct Pre {};
    __device__ __forceinline__ double2 operator()(int, long long, long long, bool, double2 y) const { return y; }
    __device__ __forceinline__ Pre pre(int, long long, long long, bool) const { return Pre{}; }
    __device__ __forceinline__ double2 fin(int, long long, long long, bool, const Pre&, double2 y) const { return y; }
};
struct PixAux {                     // the aux-variable v | s update (gs_aux.h), comps (chain, field)
    gs::GsAuxPix a;
    static constexpr bool kConst = false;
    struct Pre { gs::GsAuxPre n, s; };
    __device__ __forceinline__ Pre pre(int c, long long iN, long long iS, bool eq) const {
        const int b = c / a.F, k = c - b * a.F;
        Pre q;
        q.n = gs::mc_aux_load(a, b, k, iN);
        q.s = eq ? gs::GsAuxPre{0.0, 0.0, 0.0, 0.0} : gs::mc_aux_load(a, b, k, iS);
        return q;
    }
    __device__ __forceinline__ double2 fin(int c, long long iN, long long iS, bool eq, const Pre& q, double2 y) const {
        const int b = c / a.F, k = c - b * a.F;
        const double yn = gs::mc_aux_apply(a, b, k, iN, q.n, y.x);
        return make_double2(yn, eq ? 0.0 : gs::mc_aux_apply(a, b, k, iS, q.s, y.y));
    }
    __device__ __forceinline__ double2 operator()(int c, long long iN, long long iS, bool eq, double2 y) const {
        const int b = c / a.F, k = c - b * a.F;
        const double yn = gs::mc_aux_pixel(a, b, k, iN, y.x);
        return make_double2(yn, eq ? 0.0 : gs::mc_aux_pixel(a, b, k, iS, y.y));
    }
};

// Op (PixAux): the aux-variable step applied to the synthesised pixels A b s
// on their way out -- the map stored is y = v + N^-1 d (and v), the pixel
// kernel k_mc_v's arithmetic on the same values (bit-identical)
template <int NB, class Op = PixNone>
__global__ __launch_bounds__(1024) void k_sht_synth_ring(int L, int npair, long long npix,
                                                         const int* __restrict__ pairs,
                                                         const PairGeom* __restrict__ geom,
                                                         const double2* __restrict__ phi,
                                                         const double2* __restrict__ tw, int Mmax,
                                                         const double2* __restrict__ bsk,
                                                         double2* __restrict__ gscratch, double* __restrict__ maps,
                                                         double2* __restrict__ sscr, int nsplit, int sstride,
                                                         const int* __restrict__ comp_lmax, int comp_div, int twoff,
                                                         int phoff, Op op = Op{}) {
    extern __shared__ double2 lbuf[];
    const int p = pairs[blockIdx.x];
    const int comp = blockIdx.y;
    // block syntheses (f2): comp c holds only m <= comp_lmax[c / comp_div]
    const int Lc = comp_lmax ? comp_lmax[comp / comp_div] : L;
    GS_ASSERT(Lc <= L && p < npair);
    const PairGeom g = geom[p];
    const int BD = blockDim.x;
    double2* buf = gscratch ? gscratch + ((long long)comp * gridDim.x + blockIdx.x) * Mmax : lbuf;
    // fold reduction slots (J > 1 only, short rings) alias the FFT buffer: with
    // J > 1 the fold is one pass whose reduction ends before buf is written
    Fold4* red = reinterpret_cast<Fold4*>(lbuf);
    const int n = g.nphi;
    const double2* twx = tw;
    int twM = Mmax;
    if (twoff >= 0) twx = ring_twiddles_lds_u<ew_u(NB)>(lbuf + twoff, g.M, tw, Mmax, twM);
    else if (twoff <= -2) twx = ring_twiddles_two(lbuf + (-2 - twoff), tw, Mmax, twM);
    const RingPh ph = ring_phases(phoff >= 0 ? lbuf + phoff : nullptr, (unsigned)g.nphi);
    __syncthreads();                                // the phase tables before the fold
    const long long plane = phi_plane(L, npair);
    const double2* PN = phi + (2LL * comp + 0) * plane;
    const double2* PS = phi + (2LL * comp + 1) * plane;
    const bool eq = g.startS < 0;
    const int K = n / 2 + 1;
    const int J = K >= BD ? 1 : BD / K;          // threads per bin pair
    // c_m Phi_m; the half-pixel phase e^{i pi m / n} of phi_half rings is
    // e^{i pi k / n} (-1)^q for m = k + q n: the fold sums (-1)^q c_m Phi_m and
    // the bin's one phase factor is applied after the fold (one sincospi per bin
    // pair instead of one per m)
    auto H = [&](const double2* P, int m, bool neg) {
        const double2 v = P[phi_at(m, p, npair)];
        const double cm = (m == 0 ? 1.0 : 2.0) * (neg ? -1.0 : 1.0);
        return make_double2(cm * v.x, cm * v.y);
    };
    // a folded bin pair (k, n - k) -> the FFT input
    auto emit = [&](int k, int nk, Fold4 f) {
        if (g.phi_half) {
            // e^{i pi k / n}; for nk = n - k: e^{i pi (n - k) / n} = -conj(e^{i pi k / n})
            const double2 ek = ph.pos((unsigned)k);
            const double2 enk = make_double2(-ek.x, ek.y);
            f.nk = cmul(f.nk, ek);
            f.sk = cmul(f.sk, ek);
            f.nmk = cmul(f.nmk, enk);
            f.smk = cmul(f.smk, enk);
        }
        if (nk == k) { f.nmk = f.nk; f.smk = f.sk; }
        // Z_k = hN_k + i hS_k, hX_k = (G_k + conj G_-k)/2
        const double2 hn = make_double2(0.5 * (f.nk.x + f.nmk.x), 0.5 * (f.nk.y - f.nmk.y));
        const double2 hs = make_double2(0.5 * (f.sk.x + f.smk.x), 0.5 * (f.sk.y - f.smk.y));
        buf[k] = make_double2(hn.x - hs.y, hn.y + hs.x);
        if (nk != k) {
            const double2 hn2 = make_double2(hn.x, -hn.y), hs2 = make_double2(hs.x, -hs.y);
            buf[nk] = make_double2(hn2.x - hs2.y, hn2.y + hs2.x);
        }
    };
    const double2 z2 = make_double2(0.0, 0.0);
    if (J == 1 && n > Lc) {
        // long rings: each side of a bin pair holds at most one m (k or n - k,
        // both below n), so the fold is a gather -- the loads of a batch of
        // bin pairs issued together (ew_pass); the same sums as the loop below
        struct G4 { double2 nk, sk, nmk, smk; };
        ew_pass<2>(K, [&](int k) {
            const int nk = (n - k) % n;
            G4 r = {z2, z2, z2, z2};
            if (k <= Lc) { r.nk = H(PN, k, false); if (!eq) r.sk = H(PS, k, false); }
            if (nk != k && nk <= Lc) { r.nmk = H(PN, nk, false); if (!eq) r.smk = H(PS, nk, false); }
            return r;
        }, [&](int k, const G4& r) {
            Fold4 f = {z2, z2, z2, z2};
            f.nk.x += r.nk.x; f.nk.y += r.nk.y; f.sk.x += r.sk.x; f.sk.y += r.sk.y;
            f.nmk.x += r.nmk.x; f.nmk.y += r.nmk.y; f.smk.x += r.smk.x; f.smk.y += r.smk.y;
            emit(k, (n - k) % n, f);
        });
    } else
    for (int s0 = 0; s0 < K * J; s0 += BD) {
        const int sl = s0 + threadIdx.x;
        Fold4 f = {make_double2(0, 0), make_double2(0, 0), make_double2(0, 0), make_double2(0, 0)};
        const int k = sl % K, j0 = sl / K;
        const int nk = (n - k) % n;
        if (sl < K * J) {
            for (int m = k + j0 * n, q = j0; m <= Lc; m += J * n, q += J) {
                const bool neg = g.phi_half && (q & 1);
                const double2 a = H(PN, m, neg);
                f.nk.x += a.x; f.nk.y += a.y;
                if (!eq) { const double2 b = H(PS, m, neg); f.sk.x += b.x; f.sk.y += b.y; }
            }
            if (nk != k)
                for (int m = nk + j0 * n, q = j0; m <= Lc; m += J * n, q += J) {
                    const bool neg = g.phi_half && (q & 1);
                    const double2 a = H(PN, m, neg);
                    f.nmk.x += a.x; f.nmk.y += a.y;
                    if (!eq) { const double2 b = H(PS, m, neg); f.smk.x += b.x; f.smk.y += b.y; }
                }
        }
        if (J > 1) {
            red[threadIdx.x] = f;
            __syncthreads();
            if (sl < K * J && j0 == 0) {
                for (int jj = 1; jj < J; ++jj) {
                    const Fold4 o = red[threadIdx.x + jj * K];
                    f.nk.x += o.nk.x; f.nk.y += o.nk.y; f.nmk.x += o.nmk.x; f.nmk.y += o.nmk.y;
                    f.sk.x += o.sk.x; f.sk.y += o.sk.y; f.smk.x += o.smk.x; f.smk.y += o.smk.y;
                }
            }
            __syncthreads();
        }
        if (sl < K * J && j0 == 0) emit(k, nk, f);
    }
    __syncthreads();
    double* mc = maps + (long long)comp * npix;
    if (g.split) {
        // y_j = A_(j mod h) + e^{2 pi i j / n} B_(j mod h), A / B = IDFT_h of the even /
        // odd bins (each a Bluestein of length h in LDS; A and the odd bins wait in
        // global scratch)
        const int h = n / 2;
        double2* A = sscr + ((long long)comp * nsplit + g.sslot) * sstride;
        double2* Zo = A + h;
        for (int k = threadIdx.x; k < h; k += BD) Zo[k] = buf[2 * k + 1];
        double2 ev[NB];
#pragma unroll
        for (int t = 0; t < NB; ++t) {
            const int k = threadIdx.x + t * BD;
            ev[t] = k < h ? buf[2 * k] : make_double2(0.0, 0.0);
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < NB; ++t) {
            const int k = threadIdx.x + t * BD;
            if (k < h) buf[k] = ev[t];
        }
        __syncthreads();
        const double2* V = bsk + g.bs_off;
        bluestein_inverse<NB>(buf, h, g.M, V, twx, twM);
        for (int k = threadIdx.x; k < h; k += BD) A[k] = buf[k];
        __syncthreads();
        ew_pass<ew_u(NB)>(h, [&](int k) { return Zo[k]; }, [&](int k, double2 v) { buf[k] = v; });
        __syncthreads();
        bluestein_inverse<NB>(buf, h, g.M, V, twx, twM);
        struct Ld { double2 a; typename Op::Pre q0, q1; };
        ew_pass<1>(h, [&](int k) {
            return Ld{A[k], op.pre(comp, g.startN + k, g.startS + k, eq), op.pre(comp, g.startN + k + h, g.startS + k + h, eq)};
        }, [&](int k, const Ld& ld) {
            const double2 a = ld.a;
            const double2 b = cmul(buf[k], ph.pos(2u * k));
            const double2 y0 = op.fin(comp, g.startN + k, g.startS + k, eq, ld.q0, make_double2(a.x + b.x, a.y + b.y));
            const double2 y1 = op.fin(comp, g.startN + k + h, g.startS + k + h, eq, ld.q1, make_double2(a.x - b.x, a.y - b.y));
            mc[g.startN + k] = y0.x;
            mc[g.startN + k + h] = y1.x;
            if (!eq) { mc[g.startS + k] = y0.y; mc[g.startS + k + h] = y1.y; }
        });
        return;
    }
    dft_inverse<NB>(buf, g, twx, twM, bsk);
    // the pixel operation's loads of UO pixels issued before the first use (more spill)
    constexpr int UO = 2;
    for (int j0 = threadIdx.x; j0 < n; j0 += UO * BD) {
        typename Op::Pre q[UO];
#pragma unroll
        for (int u = 0; u < UO; ++u) {
            const int j = j0 + u * BD;
            if (j < n) q[u] = op.pre(comp, g.startN + j, g.startS + j, eq);
        }
#pragma unroll
        for (int u = 0; u < UO; ++u) {
            const int j = j0 + u * BD;
            if (j < n) {
                const double2 y = op.fin(comp, g.startN + j, g.startS + j, eq, q[u], buf[j]);
                mc[g.startN + j] = y.x;
                if (!eq) mc[g.startS + j] = y.y;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// analysis: ring stage.  grid (pairs of this M class, ncomp)
// ---------------------------------------------------------------------------
template <int NB>
__global__ __launch_bounds__(1024) void k_sht_anal_ring(int L, int npair, long long npix,
                                                        const int* __restrict__ pairs,
                                                        const PairGeom* __restrict__ geom,
                                                        const double* __restrict__ maps,
                                                        const double2* __restrict__ tw, int Mmax,
                                                        const double2* __restrict__ bsk,
                                                        double2* __restrict__ gscratch, double2* __restrict__ phi,
                                                        double2* __restrict__ sscr, int nsplit, int sstride, int twoff,
                                                        int phoff, const double* __restrict__ wts, int wnc) {
    extern __shared__ double2 lbuf[];
    const int p = pairs[blockIdx.x];
    const int comp = blockIdx.y;
    const PairGeom g = geom[p];
    double2* buf = gscratch ? gscratch + ((long long)comp * gridDim.x + blockIdx.x) * Mmax : lbuf;
    const double2* twx = tw;
    int twM = Mmax;
    if (twoff >= 0) twx = ring_twiddles_lds_u<ew_u(NB)>(lbuf + twoff, g.M, tw, Mmax, twM);
    else if (twoff <= -2) twx = ring_twiddles_two(lbuf + (-2 - twoff), tw, Mmax, twM);
    // (visible to the combine and the stores below: the FFTs' barriers come first)
    const RingPh ph = ring_phases(phoff >= 0 ? lbuf + phoff : nullptr, (unsigned)g.nphi);
    const int n = g.nphi;
    const bool eq = g.startS < 0;
    const double* mc = maps + (long long)comp * npix;
    // wts != nullptr: the transform of the pixel product wts * maps (the masked
    // CR's N^-1 A b s, one rounding as in a separate multiply pass)
    // (a batch of maps shares one set of wnc weight maps: comp = b * wnc + c)
    const double* wc = wts ? wts + (long long)(comp % wnc) * npix : nullptr;
    auto mv = [&](long long i) { return wc ? wc[i] * mc[i] : mc[i]; };
    if (g.split) {
        // X_k = E_k + e^{-2 pi i k / n} O_k, X_(k+h) = E_k - (...) O_k with E / O the
        // length-h DFTs of the even / odd samples (Bluestein in LDS; O waits in scratch)
        const int h = n / 2;
        double2* O = sscr + ((long long)comp * nsplit + g.sslot) * sstride;
        const double2* V = bsk + g.bs_off;
        // (h <= M / 2 <= NB blockDim)
        ew_pass<ew_u(NB)>(h, [&](int k) { return make_double2(mv(g.startN + 2 * k + 1), eq ? 0.0 : mv(g.startS + 2 * k + 1)); },
                    [&](int k, double2 v) { buf[k] = v; });
        __syncthreads();
        bluestein_forward<NB>(buf, h, g.M, V, twx, twM);
        for (int k = threadIdx.x; k < h; k += blockDim.x) O[k] = buf[k];
        __syncthreads();
        ew_pass<ew_u(NB)>(h, [&](int k) { return make_double2(mv(g.startN + 2 * k), eq ? 0.0 : mv(g.startS + 2 * k)); },
                    [&](int k, double2 v) { buf[k] = v; });
        __syncthreads();
        bluestein_forward<NB>(buf, h, g.M, V, twx, twM);
        ew_pass<ew_u(NB)>(h, [&](int k) { return O[k]; }, [&](int k, double2 ok) {
            const double2 e = buf[k];
            const double2 o = cmul(ok, ph.neg(2u * k));
            buf[k] = make_double2(e.x + o.x, e.y + o.y);
            buf[k + h] = make_double2(e.x - o.x, e.y - o.y);
        });
        __syncthreads();
    } else {
        // (n <= M <= 2 NB blockDim)
        ew_pass<ew_u(2 * NB)>(n, [&](int j) { return make_double2(mv(g.startN + j), eq ? 0.0 : mv(g.startS + j)); },
                        [&](int j, double2 v) { buf[j] = v; });
        __syncthreads();
        dft_forward<NB>(buf, g, twx, twM, bsk);
    }
    const long long plane = phi_plane(L, npair);
    double2* oN = phi + (2LL * comp + 0) * plane;
    double2* oS = phi + (2LL * comp + 1) * plane;
    for (int m = threadIdx.x; m <= L; m += blockDim.x) {
        const int k = m % n;
        const int nk = k == 0 ? 0 : n - k;
        const double2 a = buf[k], b = buf[nk];
        // north: (Z_k + conj Z_-k)/2 ; south: (Z_k - conj Z_-k)/(2i)
        double2 xn = make_double2(0.5 * (a.x + b.x), 0.5 * (a.y - b.y));
        double2 xs = make_double2(0.5 * (a.y + b.y), -0.5 * (a.x - b.x));
        if (g.phi_half) {
            const double2 e = ph.neg((unsigned)m % (2u * (unsigned)n));
            xn = cmul(xn, e);
            xs = cmul(xs, e);
        }
        if (m == 0) { xn.y = 0.0; xs.y = 0.0; }
        oN[phi_at(m, p, npair)] = xn;
        oS[phi_at(m, p, npair)] = eq ? make_double2(0.0, 0.0) : xs;
    }
}

// ---------------------------------------------------------------------------
// ring stage, NCB components per workgroup (batched small maps: the merged
// launch, every ring's FFT in LDS, no split rings).  The components of one
// ring pair share the workgroup's barriers, its LDS twiddle table and the
// ring's Bluestein chirp / kernel loads; each FFT stage runs over all their
// buffers (stride SB).  Per component the arithmetic is that of
// k_sht_synth_ring / k_sht_anal_ring, so the results are bit-identical.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int ilog2d(int x) { return 31 - __clz(x); }

template <int R, int NV>
__device__ __forceinline__ void stockham_stage_mc(double2* buf, int SB, int nc, int lgM, int Ns, int dir,
                                                  const double2* __restrict__ tw, int Mmax) {
    constexpr int NBF = NV / R > 0 ? NV / R : 1;
    constexpr int LGR = R == 2 ? 1 : (R == 4 ? 2 : (R == 8 ? 3 : 4));
    const int lgnb = lgM - LGR;
    const int nb = 1 << lgnb;
    const int nbt = nb * nc;
    const int step = Mmax / (Ns * R);
    double2 v[NBF][R];
#pragma unroll
    for (int b = 0; b < NBF; ++b) {
        const int jj = threadIdx.x + b * blockDim.x;
        if (jj < nbt) {
            const int j = jj & (nb - 1);
            const double2* B = buf + (jj >> lgnb) * SB;
#pragma unroll
            for (int k = 0; k < R; ++k) v[b][k] = B[j + k * nb];
            if (Ns > 1) {
                const int jm = j & (Ns - 1);
#pragma unroll
                for (int k = 1; k < R; ++k) v[b][k] = cmul(v[b][k], twid(jm * k * step, dir, tw, Mmax));
            }
            dft_reg<R>(v[b], dir);
        }
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < NBF; ++b) {
        const int jj = threadIdx.x + b * blockDim.x;
        if (jj < nbt) {
            const int j = jj & (nb - 1);
            double2* B = buf + (jj >> lgnb) * SB;
            const int jm = j & (Ns - 1);
            const int base = (j - jm) * R + jm;
#pragma unroll
            for (int k = 0; k < R; ++k) B[base + k * Ns] = v[b][k];
        }
    }
    __syncthreads();
}

template <int NV>
__device__ __forceinline__ void fft_pow2_mc(double2* buf, int SB, int nc, int M, int dir,
                                            const double2* __restrict__ tw, int Mmax) {
    const int p = ilog2d(M);
    int Ns = 1;
    if (p % 3 == 1 && p >= 4) { stockham_stage_mc<16, NV>(buf, SB, nc, p, 1, dir, tw, Mmax); Ns = 16; }
    else if (p % 3 == 1) { stockham_stage_mc<2, NV>(buf, SB, nc, p, 1, dir, tw, Mmax); Ns = 2; }
    else if (p % 3 == 2) { stockham_stage_mc<4, NV>(buf, SB, nc, p, 1, dir, tw, Mmax); Ns = 4; }
    for (; Ns < M; Ns *= 8) stockham_stage_mc<8, NV>(buf, SB, nc, p, Ns, dir, tw, Mmax);
}

template <int NV>
__device__ __forceinline__ void bluestein_forward_mc(double2* buf, int SB, int nc, int n, int M,
                                                     const double2* __restrict__ V, const double2* __restrict__ tw,
                                                     int Mmax) {
    const double2* __restrict__ C = V + M;
    const int lgM = ilog2d(M);
    for (int jj = threadIdx.x; jj < nc * M; jj += blockDim.x) {
        const int j = jj & (M - 1);
        double2* b = buf + (jj >> lgM) * SB + j;
        *b = j < n ? cmul(*b, C[j]) : make_double2(0.0, 0.0);
    }
    __syncthreads();
    fft_pow2_mc<NV>(buf, SB, nc, M, -1, tw, Mmax);
    for (int jj = threadIdx.x; jj < nc * M; jj += blockDim.x) {
        const int j = jj & (M - 1);
        double2* b = buf + (jj >> lgM) * SB + j;
        *b = cmul(*b, V[j]);
    }
    __syncthreads();
    fft_pow2_mc<NV>(buf, SB, nc, M, +1, tw, Mmax);
    const double inv = 1.0 / M;
    for (int jj = threadIdx.x; jj < nc * n; jj += blockDim.x) {
        const int c = jj / n, j = jj - c * n;
        double2* b = buf + c * SB + j;
        const double2 v = cmul(*b, C[j]);
        *b = make_double2(v.x * inv, v.y * inv);
    }
    __syncthreads();
}

template <int NV>
__device__ __forceinline__ void dft_mc(double2* buf, int SB, int nc, const PairGeom& g, int dir,
                                       const double2* __restrict__ tw, int Mmax, const double2* __restrict__ bsk) {
    if (g.bs_off < 0) { fft_pow2_mc<NV>(buf, SB, nc, g.M, dir, tw, Mmax); return; }
    const int n = g.nphi;
    if (dir > 0) {                                // conj(DFT(conj x))
        for (int jj = threadIdx.x; jj < nc * n; jj += blockDim.x) { const int c = jj / n; buf[c * SB + jj - c * n].y *= -1.0; }
        __syncthreads();
    }
    bluestein_forward_mc<NV>(buf, SB, nc, n, g.M, bsk + g.bs_off, tw, Mmax);
    if (dir > 0) {
        for (int jj = threadIdx.x; jj < nc * n; jj += blockDim.x) { const int c = jj / n; buf[c * SB + jj - c * n].y *= -1.0; }
        __syncthreads();
    }
}

// XCD-aware 1-D order of the multi-component ring launches: blocks lin, lin +
// 8, ... run on one XCD, which takes two consecutive ring entries (pairs p, p +
// 1 share every 128-B line of the phase planes) with all their component
// groups back to back (the ring's Bluestein tables then come from HBM into
// that XCD's L2 once).  Returns false past the last ring.
// measured: the XCD order 332 / 350 us against 318 / 340 us ring-major
// (synthesis / analysis ring stage, 16 spin-2 maps, same box): off
#ifndef GS_RING_XCD
#define GS_RING_XCD 0
#endif
__device__ __forceinline__ bool ring_mc_slot(int nring, int ncg, int& idx, int& cg) {
    if (!GS_RING_XCD) {                            // A/B: ring-major, ring fastest
        idx = blockIdx.x % nring;
        cg = blockIdx.x / nring;
        return cg < ncg;
    }
    const int lin = blockIdx.x, xcd = lin & 7, slot = lin >> 3;
    const int j = slot / (2 * ncg), rem = slot - j * 2 * ncg;
    idx = 2 * (8 * j + xcd) + rem / ncg;
    cg = rem % ncg;
    return idx < nring;
}

// a ring pair without weight (pflag 0): its analysis phases are exact zeros
// (0 x pixel, transformed) and are written as such, no ring work
__device__ __forceinline__ void ring_zero_phases(int L, int npair, int p, double2* phi, int c0, int nc) {
    const long long plane = phi_plane(L, npair);
    for (int jj = threadIdx.x; jj < nc * (L + 1); jj += blockDim.x) {
        const int c = jj / (L + 1), m = jj - c * (L + 1);
        double2* oN = phi + (2LL * (c0 + c) + 0) * plane;
        oN[phi_at(m, p, npair)] = make_double2(0.0, 0.0);
        oN[plane + phi_at(m, p, npair)] = make_double2(0.0, 0.0);
    }
}

// the support of a weighted analysis: pflag[p] = 1 when a pixel of either ring
// of pair p has a nonzero weight in some component (one workgroup per pair).
// A pair without weight contributes exact zeros to the analysis (0 x pixel),
// so the ring stage writes its phases as zeros and the matrix-core Legendre
// stages skip 16-pair tiles without weight -- the same bits, less work (a
// galactic cut in galactic coordinates removes whole equatorial rings; the
// bench's |cos theta| > 0.2 band 15 % of the pairs, 4 of 32 tiles)
__global__ __launch_bounds__(256) void k_pair_support(long long npix, const PairGeom* __restrict__ geom,
                                                      const double* __restrict__ wts, int wnc, int* __restrict__ pflag) {
    const int p = blockIdx.x;
    const PairGeom g = geom[p];
    const int n = g.nphi;
    const bool eq = g.startS < 0;
    // chunk by chunk until a nonzero weight is seen (a live pair: usually the
    // first chunk; a pair without weight: every pixel)
    int any = 0;
    for (int i0 = 0; i0 < wnc * n && !any; i0 += blockDim.x) {
        const int i = i0 + threadIdx.x;
        int f = 0;
        if (i < wnc * n) {
            const int c = i / n, j = i - c * n;
            const double* wc = wts + (long long)c * npix;
            f = wc[g.startN + j] != 0.0 || (!eq && wc[g.startS + j] != 0.0);
        }
        any = __syncthreads_or(f);
    }
    if (threadIdx.x == 0) pflag[p] = any;
}

// the registered weights' ring classes (gs_sht_register_weights), one workgroup
// per pair: pflag[p] = 0 (no weight on either ring), 1 (weighted), 3 (weighted
// and every weight row constant on each ring of the pair -- e.g. isotropic noise
// on rings the mask leaves whole); wconst[p][c] = (north, south) constants of row c
// (south 0 for the equatorial ring).  A constant ring's inverse DFT, pixel
// weight and forward DFT collapse to n w (the unnormalised round trip times the
// constant), and its pixel vector's weighted inner products are those of its
// Fourier coordinates (Parseval): the ring stages use both (k_sht_apply_ring_mc,
// k_sht_synth_ring_mc's Parseval mode).
__global__ __launch_bounds__(256) void k_ring_classes(long long npix, const PairGeom* __restrict__ geom,
                                                      const double* __restrict__ wts, int wnc,
                                                      int* __restrict__ pflag, double2* __restrict__ wconst) {
    const int p = blockIdx.x;
    const PairGeom g = geom[p];
    const int n = g.nphi;
    const bool eq = g.startS < 0;
    int any = 0, cst = 1;
    for (int c = 0; c < wnc; ++c) {
        const double* wc = wts + (long long)c * npix;
        const double vn = wc[g.startN], vs = eq ? 0.0 : wc[g.startS];
        int a = 0, d = 0;
        for (int j = threadIdx.x; j < n; j += blockDim.x) {
            const double xn = wc[g.startN + j], xs = eq ? 0.0 : wc[g.startS + j];
            a |= xn != 0.0 || xs != 0.0;
            d |= xn != vn || xs != vs;
        }
        any |= __syncthreads_or(a);
        cst &= !__syncthreads_or(d);
        if (threadIdx.x == 0) wconst[(long long)p * wnc + c] = make_double2(vn, vs);
    }
    if (threadIdx.x == 0) pflag[p] = any ? (1 | (cst << 1)) : 0;
}

// tile t (pairs 16 t ..) has weight: any of its pair flags
__device__ __forceinline__ bool tile_support(const int* __restrict__ pflag, int t, int npair) {
    bool any = false;
#pragma unroll
    for (int k = 0; k < 16; ++k) any |= 16 * t + k < npair && pflag[min(16 * t + k, npair - 1)] != 0;
    return any;
}

// Parseval coordinates of a constant-weight ring pair (k_ring_classes): from the
// packed spectrum a_q = s (Z^N_q + i Z^S_q) of the pair (Z the coefficients of
// y_j = sum_q Z_q e^{2 pi i q j / n}, both rings real) the n real coordinates u
// of each ring with sum_j y_j^2 = sum_j u_j^2: u_0 = sqrt(n) Z_0, (u_{2q-1}, u_{2q})
// = sqrt(2n) (Re, Im) Z_q for 0 < q < n / 2, u_{n-1} = sqrt(n) Z_{n/2} (n even,
// as every HEALPix ring).  Written over the rings' pixel slots: on such a ring
// the weight is one number, so the f2 Gram pass's weighted sums over these
// coordinates equal those over the pixels (its rows of block maps, residual).
__device__ __forceinline__ void parseval_store(const double2* buf, int SB, int nc, int n, double s,
                                               const PairGeom& g, double* maps, long long npix, int c0) {
    const bool eq = g.startS < 0;
    const double r1 = sqrt((double)n) * s, r2 = sqrt(2.0 * n) * s;
    for (int jj = threadIdx.x; jj < nc * n; jj += blockDim.x) {
        const int c = jj / n, j = jj - c * n;
        const double2* b = buf + c * SB;
        const int q = (j + 1) >> 1;
        const double2 a = b[q], bb = b[(n - q) % n];
        const double2 zn = make_double2(0.5 * (a.x + bb.x), 0.5 * (a.y - bb.y));
        const double2 zs = make_double2(0.5 * (a.y + bb.y), -0.5 * (a.x - bb.x));
        double un, us;
        if (j == 0 || 2 * q == n) { un = r1 * zn.x; us = r1 * zs.x; }
        else if (j & 1) { un = r2 * zn.x; us = r2 * zs.x; }
        else { un = r2 * zn.y; us = r2 * zs.y; }
        double* mc = maps + (long long)(c0 + c) * npix;
        mc[g.startN + j] = un;
        if (!eq) mc[g.startS + j] = us;
    }
}

// synthesis: 1-D grid over (ring pair, component group of NCB) (ring_mc_slot);
// LDS NCB x SB + twiddles.  pconst (f2 block maps only; nullptr otherwise): a
// pair of class 0 (no weight) is skipped (its pixels keep the caller's finite
// values), one of class 3 (constant weights) writes its Parseval coordinates
// instead of its pixels (parseval_store)
template <int NV>
__global__ __launch_bounds__(1024) void k_sht_synth_ring_mc(int L, int npair, long long npix,
                                                            const int* __restrict__ pairs,
                                                            const PairGeom* __restrict__ geom,
                                                            const double2* __restrict__ phi,
                                                            const double2* __restrict__ tw, int Mmax,
                                                            const double2* __restrict__ bsk, double* __restrict__ maps,
                                                            int ncomp, int NCB, int SB, int twoff,
                                                            const int* __restrict__ comp_lmax, int comp_div,
                                                            int nring, const int* __restrict__ pconst) {
    extern __shared__ double2 lbuf[];
    int idx, cg;
    if (!ring_mc_slot(nring, (ncomp + NCB - 1) / NCB, idx, cg)) return;
    const int p = pairs[idx];
    const int c0 = cg * NCB;
    const int nc = min(NCB, ncomp - c0);
    const PairGeom g = geom[p];
    const int cls = pconst ? pconst[p] : 1;
    // no weight: the Gram pass multiplies these pixels by 0 (the caller's maps
    // hold finite values there -- gs_masked's block maps stay at their
    // allocation's zeros), so nothing is computed or written
    if (cls == 0) return;
    const int TC = blockDim.x / NCB;               // fold threads per component
    const int cl = threadIdx.x / TC, tl = threadIdx.x - cl * TC;
    const bool live = cl < nc;
    int twM = Mmax;
    const double2* twx = ring_twiddles_lds(lbuf + twoff, g.M, tw, Mmax, twM);
    double2* buf = lbuf + cl * SB;
    // fold reduction slots (J > 1: one pass) alias the component's own buffer
    Fold4* red = reinterpret_cast<Fold4*>(buf);
    const int n = g.nphi;
    const long long plane = phi_plane(L, npair);
    const double2* PN = phi + (2LL * (live ? c0 + cl : 0) + 0) * plane;
    const double2* PS = PN + plane;
    const bool eq = g.startS < 0;
    const int K = n / 2 + 1;
    const int J = K >= TC ? 1 : TC / K;
    // block syntheses (f2): comp c holds only m <= comp_lmax[c / comp_div]
    const int Lc = comp_lmax && live ? comp_lmax[(c0 + cl) / comp_div] : L;
    auto H = [&](const double2* P, int m, bool neg) {
        const double2 v = P[phi_at(m, p, npair)];
        const double cm = (m == 0 ? 1.0 : 2.0) * (neg ? -1.0 : 1.0);
        return make_double2(cm * v.x, cm * v.y);
    };
    for (int s0 = 0; s0 < K * J; s0 += TC) {
        const int sl = s0 + tl;
        Fold4 f = {make_double2(0, 0), make_double2(0, 0), make_double2(0, 0), make_double2(0, 0)};
        const int k = sl % K, j0 = sl / K;
        const int nk = (n - k) % n;
        const bool on = live && sl < K * J;
        if (on) {
            for (int m = k + j0 * n, q = j0; m <= Lc; m += J * n, q += J) {
                const bool neg = g.phi_half && (q & 1);
                const double2 a = H(PN, m, neg);
                f.nk.x += a.x; f.nk.y += a.y;
                if (!eq) { const double2 b = H(PS, m, neg); f.sk.x += b.x; f.sk.y += b.y; }
            }
            if (nk != k)
                for (int m = nk + j0 * n, q = j0; m <= Lc; m += J * n, q += J) {
                    const bool neg = g.phi_half && (q & 1);
                    const double2 a = H(PN, m, neg);
                    f.nmk.x += a.x; f.nmk.y += a.y;
                    if (!eq) { const double2 b = H(PS, m, neg); f.smk.x += b.x; f.smk.y += b.y; }
                }
        }
        if (J > 1) {
            if (live) red[tl] = f;
            __syncthreads();
            if (on && j0 == 0) {
                for (int jj = 1; jj < J; ++jj) {
                    const Fold4 o = red[tl + jj * K];
                    f.nk.x += o.nk.x; f.nk.y += o.nk.y; f.nmk.x += o.nmk.x; f.nmk.y += o.nmk.y;
                    f.sk.x += o.sk.x; f.sk.y += o.sk.y; f.smk.x += o.smk.x; f.smk.y += o.smk.y;
                }
            }
            __syncthreads();
        }
        if (on && j0 == 0) {
            if (g.phi_half) {
                const double2 ek = expi_pi_u32(k, n);
                const double2 enk = make_double2(-ek.x, ek.y);
                f.nk = cmul(f.nk, ek);
                f.sk = cmul(f.sk, ek);
                f.nmk = cmul(f.nmk, enk);
                f.smk = cmul(f.smk, enk);
            }
            if (nk == k) { f.nmk = f.nk; f.smk = f.sk; }
            const double2 hn = make_double2(0.5 * (f.nk.x + f.nmk.x), 0.5 * (f.nk.y - f.nmk.y));
            const double2 hs = make_double2(0.5 * (f.sk.x + f.smk.x), 0.5 * (f.sk.y - f.smk.y));
            buf[k] = make_double2(hn.x - hs.y, hn.y + hs.x);
            if (nk != k) {
                const double2 hn2 = make_double2(hn.x, -hn.y), hs2 = make_double2(hs.x, -hs.y);
                buf[nk] = make_double2(hn2.x - hs2.y, hn2.y + hs2.x);
            }
        }
    }
    __syncthreads();
    if (cls & 2) {                                 // constant weights: Parseval coordinates
        parseval_store(lbuf, SB, nc, n, 1.0, g, maps, npix, c0);
        return;
    }
    dft_mc<NV>(lbuf, SB, nc, g, +1, twx, twM, bsk);
    for (int jj = threadIdx.x; jj < nc * n; jj += blockDim.x) {
        const int c = jj / n, j = jj - c * n;
        const double2 y = lbuf[c * SB + j];
        double* mc = maps + (long long)(c0 + c) * npix;
        mc[g.startN + j] = y.x;
        if (!eq) mc[g.startS + j] = y.y;
    }
}

// the Parseval coordinates of maps on the constant-weight pairs (class 3 of
// pconst), in place: forward DFT of each such pair's two rings, Z = DFT / n,
// parseval_store; other pairs keep their pixels.  1-D grid as the ring stages.
template <int NV>
__global__ __launch_bounds__(1024) void k_sht_parseval_ring_mc(long long npix, const int* __restrict__ pairs,
                                                               const PairGeom* __restrict__ geom,
                                                               const double2* __restrict__ tw, int Mmax,
                                                               const double2* __restrict__ bsk, double* maps,
                                                               int ncomp, int NCB, int SB, int twoff, int nring,
                                                               const int* __restrict__ pconst) {
    extern __shared__ double2 lbuf[];
    int idx, cg;
    if (!ring_mc_slot(nring, (ncomp + NCB - 1) / NCB, idx, cg)) return;
    const int p = pairs[idx];
    if (!(pconst[p] & 2)) return;
    const int c0 = cg * NCB;
    const int nc = min(NCB, ncomp - c0);
    const PairGeom g = geom[p];
    int twM = Mmax;
    const double2* twx = ring_twiddles_lds(lbuf + twoff, g.M, tw, Mmax, twM);
    const int n = g.nphi;
    const bool eq = g.startS < 0;
    for (int jj = threadIdx.x; jj < nc * n; jj += blockDim.x) {
        const int c = jj / n, j = jj - c * n;
        const double* mc = maps + (long long)(c0 + c) * npix;
        lbuf[c * SB + j] = make_double2(mc[g.startN + j], eq ? 0.0 : mc[g.startS + j]);
    }
    __syncthreads();
    dft_mc<NV>(lbuf, SB, nc, g, -1, twx, twM, bsk);
    parseval_store(lbuf, SB, nc, n, 1.0 / n, g, maps, npix, c0);
}

// analysis: 1-D grid over (ring pair, component group of NCB) (ring_mc_slot)
template <int NV>
__global__ __launch_bounds__(1024) void k_sht_anal_ring_mc(int L, int npair, long long npix,
                                                           const int* __restrict__ pairs,
                                                           const PairGeom* __restrict__ geom,
                                                           const double* __restrict__ maps,
                                                           const double2* __restrict__ tw, int Mmax,
                                                           const double2* __restrict__ bsk, double2* __restrict__ phi,
                                                           int ncomp, int NCB, int SB, int twoff,
                                                           const double* __restrict__ wts, int wnc, int nring,
                                                           const int* __restrict__ pflag) {
    extern __shared__ double2 lbuf[];
    int idx, cg;
    if (!ring_mc_slot(nring, (ncomp + NCB - 1) / NCB, idx, cg)) return;
    const int p = pairs[idx];
    const int c0 = cg * NCB;
    const int nc = min(NCB, ncomp - c0);
    if (pflag && !pflag[p]) { ring_zero_phases(L, npair, p, phi, c0, nc); return; }
    const PairGeom g = geom[p];
    int twM = Mmax;
    const double2* twx = ring_twiddles_lds(lbuf + twoff, g.M, tw, Mmax, twM);
    const int n = g.nphi;
    const bool eq = g.startS < 0;
    for (int jj = threadIdx.x; jj < nc * n; jj += blockDim.x) {
        const int c = jj / n, j = jj - c * n;
        const int comp = c0 + c;
        const double* mc = maps + (long long)comp * npix;
        const double* wc = wts ? wts + (long long)(comp % wnc) * npix : nullptr;
        const long long iN = g.startN + j, iS = g.startS + j;
        const double vn = wc ? wc[iN] * mc[iN] : mc[iN];
        const double vs = eq ? 0.0 : (wc ? wc[iS] * mc[iS] : mc[iS]);
        lbuf[c * SB + j] = make_double2(vn, vs);
    }
    __syncthreads();
    dft_mc<NV>(lbuf, SB, nc, g, -1, twx, twM, bsk);
    const long long plane = phi_plane(L, npair);
    for (int jj = threadIdx.x; jj < nc * (L + 1); jj += blockDim.x) {
        const int c = jj / (L + 1), m = jj - c * (L + 1);
        const double2* buf = lbuf + c * SB;
        double2* oN = phi + (2LL * (c0 + c) + 0) * plane;
        double2* oS = oN + plane;
        const int k = m % n;
        const int nk = k == 0 ? 0 : n - k;
        const double2 a = buf[k], b = buf[nk];
        double2 xn = make_double2(0.5 * (a.x + b.x), 0.5 * (a.y - b.y));
        double2 xs = make_double2(0.5 * (a.y + b.y), -0.5 * (a.x - b.x));
        if (g.phi_half) {
            const double2 e = expi_pi_neg_u32(m, n);
            xn = cmul(xn, e);
            xs = cmul(xs, e);
        }
        if (m == 0) { xn.y = 0.0; xs.y = 0.0; }
        oN[phi_at(m, p, npair)] = xn;
        oS[phi_at(m, p, npair)] = eq ? make_double2(0.0, 0.0) : xs;
    }
}

// the pixel operations of the fused ring stage (k_sht_apply_ring_mc): y -> the
// analysis input of comp c at the ring pair's pixels iN (north) / iS (south)
struct PixWeights {                 // the masked PCG's N^-1 (weights [wnc][Npix] shared by the batch)
    const double* wts;
    int wnc;
    long long npix;
    const double2* wconst;          // registered constant-ring values (nullptr: none)
    static constexpr bool kConst = true;
    __device__ __forceinline__ double2 operator()(int c, long long iN, long long iS, bool eq, double2 y) const {
        const double* wc = wts + (long long)(c % wnc) * npix;
        return make_double2(wc[iN] * y.x, eq ? 0.0 : wc[iS] * y.y);
    }
};
// (PixAux: above, with k_sht_synth_ring)

// fused ring stage: per ring pair the synthesis ring work (fold, inverse DFT),
// a pixel operation (the masked PCG's N^-1 weights: the operator A^T N^-1 A; or
// the aux-variable v | s update that turns A b s into y = v + N^-1 d), and the
// analysis ring work (forward DFT, unfold) in one workgroup, the pixels never
// leaving LDS: the same arithmetic as k_sht_synth_ring_mc, a map stored, the
// pixel kernel and k_sht_anal_ring_mc (bit-identical), phases updated in place
// (each pair's phases are read and written by its own workgroup only)
template <int NV, class Op>
__global__ __launch_bounds__(1024) void k_sht_apply_ring_mc(int L, int npair, long long npix,
                                                            const int* __restrict__ pairs,
                                                            const PairGeom* __restrict__ geom, double2* phi,
                                                            const double2* __restrict__ tw, int Mmax,
                                                            const double2* __restrict__ bsk, int ncomp, int NCB, int SB,
                                                            int twoff, Op op, int nring,
                                                            const int* __restrict__ pflag) {
    extern __shared__ double2 lbuf[];
    int idx, cg;
    if (!ring_mc_slot(nring, (ncomp + NCB - 1) / NCB, idx, cg)) return;
    const int p = pairs[idx];
    const int c0 = cg * NCB;
    const int nc = min(NCB, ncomp - c0);
    if (pflag && !pflag[p]) { ring_zero_phases(L, npair, p, phi, c0, nc); return; }
    // registered constant-weight pair (k_ring_classes): no DFTs, see below
    bool cring = false;
    if constexpr (Op::kConst) cring = op.wconst && (pflag[p] & 2);
    const PairGeom g = geom[p];
    const int TC = blockDim.x / NCB;
    const int cl = threadIdx.x / TC, tl = threadIdx.x - cl * TC;
    const bool live = cl < nc;
    int twM = Mmax;
    const double2* twx = ring_twiddles_lds(lbuf + twoff, g.M, tw, Mmax, twM);
    double2* buf = lbuf + cl * SB;
    Fold4* red = reinterpret_cast<Fold4*>(buf);
    const int n = g.nphi;
    const long long plane = phi_plane(L, npair);
    const double2* PN = phi + (2LL * (live ? c0 + cl : 0) + 0) * plane;
    const double2* PS = PN + plane;
    const bool eq = g.startS < 0;
    const int K = n / 2 + 1;
    const int J = K >= TC ? 1 : TC / K;
    auto H = [&](const double2* P, int m, bool neg) {
        const double2 v = P[phi_at(m, p, npair)];
        const double cm = (m == 0 ? 1.0 : 2.0) * (neg ? -1.0 : 1.0);
        return make_double2(cm * v.x, cm * v.y);
    };
    for (int s0 = 0; s0 < K * J; s0 += TC) {
        const int sl = s0 + tl;
        Fold4 f = {make_double2(0, 0), make_double2(0, 0), make_double2(0, 0), make_double2(0, 0)};
        const int k = sl % K, j0 = sl / K;
        const int nk = (n - k) % n;
        const bool on = live && sl < K * J;
        if (on) {
            for (int m = k + j0 * n, q = j0; m <= L; m += J * n, q += J) {
                const bool neg = g.phi_half && (q & 1);
                const double2 a = H(PN, m, neg);
                f.nk.x += a.x; f.nk.y += a.y;
                if (!eq) { const double2 b = H(PS, m, neg); f.sk.x += b.x; f.sk.y += b.y; }
            }
            if (nk != k)
                for (int m = nk + j0 * n, q = j0; m <= L; m += J * n, q += J) {
                    const bool neg = g.phi_half && (q & 1);
                    const double2 a = H(PN, m, neg);
                    f.nmk.x += a.x; f.nmk.y += a.y;
                    if (!eq) { const double2 b = H(PS, m, neg); f.smk.x += b.x; f.smk.y += b.y; }
                }
        }
        if (J > 1) {
            if (live) red[tl] = f;
            __syncthreads();
            if (on && j0 == 0) {
                for (int jj = 1; jj < J; ++jj) {
                    const Fold4 o = red[tl + jj * K];
                    f.nk.x += o.nk.x; f.nk.y += o.nk.y; f.nmk.x += o.nmk.x; f.nmk.y += o.nmk.y;
                    f.sk.x += o.sk.x; f.sk.y += o.sk.y; f.smk.x += o.smk.x; f.smk.y += o.smk.y;
                }
            }
            __syncthreads();
        }
        if (on && j0 == 0) {
            if (g.phi_half) {
                const double2 ek = expi_pi_u32(k, n);
                const double2 enk = make_double2(-ek.x, ek.y);
                f.nk = cmul(f.nk, ek);
                f.sk = cmul(f.sk, ek);
                f.nmk = cmul(f.nmk, enk);
                f.smk = cmul(f.smk, enk);
            }
            if (nk == k) { f.nmk = f.nk; f.smk = f.sk; }
            const double2 hn = make_double2(0.5 * (f.nk.x + f.nmk.x), 0.5 * (f.nk.y - f.nmk.y));
            const double2 hs = make_double2(0.5 * (f.sk.x + f.smk.x), 0.5 * (f.sk.y - f.smk.y));
            buf[k] = make_double2(hn.x - hs.y, hn.y + hs.x);
            if (nk != k) {
                const double2 hn2 = make_double2(hn.x, -hn.y), hs2 = make_double2(hs.x, -hs.y);
                buf[nk] = make_double2(hn2.x - hs2.y, hn2.y + hs2.x);
            }
        }
    }
    __syncthreads();
    if (cring) {
        // weights c_N / c_S constant on the rings: inverse DFT (unnormalised),
        // weight, forward DFT = n (c_N Z^N_k + i c_S Z^S_k) per bin of the packed
        // spectrum a_k = Z^N_k + i Z^S_k, i.e. n ((c_N + c_S) / 2 a_k + (c_N - c_S) / 2
        // conj a_{n-k}) -- the two DFTs skipped (the same sums up to rounding)
        const int nh = n / 2 + 1;
        for (int jj = threadIdx.x; jj < nc * nh; jj += blockDim.x) {
            const int c = jj / nh, k = jj - c * nh, nk = (n - k) % n;
            double2 wcv = make_double2(0.0, 0.0);
            if constexpr (Op::kConst) wcv = op.wconst[(long long)p * op.wnc + (c0 + c) % op.wnc];
            const double hp = 0.5 * (wcv.x + wcv.y) * n, hm = 0.5 * (wcv.x - wcv.y) * n;
            double2* bb = lbuf + c * SB;
            const double2 a = bb[k], b = bb[nk];
            bb[k] = make_double2(hp * a.x + hm * b.x, hp * a.y - hm * b.y);
            if (nk != k) bb[nk] = make_double2(hp * b.x + hm * a.x, hp * b.y - hm * a.y);
        }
        __syncthreads();
    } else {
        dft_mc<NV>(lbuf, SB, nc, g, +1, twx, twM, bsk);
        // the pixel operation on the ring's pixels (north .x, south .y): the analysis input
        for (int jj = threadIdx.x; jj < nc * n; jj += blockDim.x) {
            const int c = jj / n, j = jj - c * n;
            lbuf[c * SB + j] = op(c0 + c, g.startN + j, g.startS + j, eq, lbuf[c * SB + j]);
        }
        __syncthreads();
        dft_mc<NV>(lbuf, SB, nc, g, -1, twx, twM, bsk);
    }
    for (int jj = threadIdx.x; jj < nc * (L + 1); jj += blockDim.x) {
        const int c = jj / (L + 1), m = jj - c * (L + 1);
        const double2* b2 = lbuf + c * SB;
        double2* oN = phi + (2LL * (c0 + c) + 0) * plane;
        double2* oS = oN + plane;
        const int k = m % n;
        const int nk = k == 0 ? 0 : n - k;
        const double2 a = b2[k], b = b2[nk];
        double2 xn = make_double2(0.5 * (a.x + b.x), 0.5 * (a.y - b.y));
        double2 xs = make_double2(0.5 * (a.y + b.y), -0.5 * (a.x - b.x));
        if (g.phi_half) {
            const double2 e = expi_pi_neg_u32(m, n);
            xn = cmul(xn, e);
            xs = cmul(xs, e);
        }
        if (m == 0) { xn.y = 0.0; xs.y = 0.0; }
        oN[phi_at(m, p, npair)] = xn;
        oS[phi_at(m, p, npair)] = eq ? make_double2(0.0, 0.0) : xs;
    }
}

// ---------------------------------------------------------------------------
// analysis: Legendre stage.  grid (m pairs or m, tiles of 4 ASR groups of 64 ring pairs)
// out: part[tile][comp][nlm] (double2), unweighted sums
//   T: sum lambda Phi_T ;  E: sum (Q F1 + i U F2) ;  B: sum (U F1 - i Q F2)
// Per chunk of ANA_C l (aligned to m's parity) every lane sums its 4 ring
// pairs in registers; the workgroup then reduces the chunk's NO x ANA_C
// partial sums over its 256 lanes in LDS in a fixed order.
// ---------------------------------------------------------------------------
// v0 = lambda_l, v1 = lambda_{l-1}, xv0 / xv1 = their mul_nc products with x;
// the spin-2 phases fp / fn [cq..] carry the factor is2 and the outputs the
// factor Q_l (AnaCoef)
template <int NC, bool EVEN, bool SLOW>
__device__ __forceinline__ void ana_term(double* a, const AnaCoef& c, double v0, double v1, double xv0, double xv1,
                                         int k, double s2, const double2* fp, const double2* fn) {
    const double lam = SLOW ? (k == 0 ? v0 : 0.0) : v0;
    const double lam1 = SLOW ? (k == 0 ? v1 : 0.0) : v1;
    const double xl = SLOW ? (k == 0 ? xv0 : 0.0) : xv0;
    const double xl1 = SLOW ? (k == 0 ? xv1 : 0.0) : xv1;
    int o = 0;
    if constexpr (NC != 2) {
        const double2 t = EVEN ? fp[0] : fn[0];
        a[0] = fma(lam, t.x, a[0]);
        a[1] = fma(lam, t.y, a[1]);
        o = 2;
    }
    if constexpr (NC != 1) {
        constexpr int cq = NC == 3 ? 1 : 0;
        const double F1 = fma(c.R, xl1, -((c.P + s2) * lam));
        const double F2 = fma(c.Rm, lam1, -(c.T * xl));
        const double2 Q1 = EVEN ? fp[cq] : fn[cq];          // F1 parity
        const double2 U1 = EVEN ? fp[cq + 1] : fn[cq + 1];
        const double2 Q2 = EVEN ? fn[cq] : fp[cq];          // F2 parity
        const double2 U2 = EVEN ? fn[cq + 1] : fp[cq + 1];
        a[o + 0] = fma(F1, Q1.x, fma(-F2, U2.y, a[o + 0]));
        a[o + 1] = fma(F1, Q1.y, fma(F2, U2.x, a[o + 1]));
        a[o + 2] = fma(F1, U1.x, fma(F2, Q2.y, a[o + 2]));
        a[o + 3] = fma(F1, U1.y, fma(-F2, Q2.x, a[o + 3]));
    }
}

template <int NC, int ASR, bool SEGL>
__global__ __launch_bounds__(LEG_BLOCK, 2) void k_sht_anal_leg(ShtDev D, const AnaCoef* __restrict__ coef,
                                                            const double2* __restrict__ phi,
                                                            double2* __restrict__ part, int paired) {
    // SEGL (l-segmented launches): the segment's coefficients (<= seg + 2 l) are
    // staged once per workgroup in LDS with coalesced loads instead of one
    // scalar load (a memory latency) per l step and wave
    __shared__ __attribute__((aligned(16))) AnaCoef cstage[SEGL ? 68 : 1];
    constexpr int NO = NC == 1 ? 2 : (NC == 2 ? 4 : 6);   // real outputs per l
    constexpr int NV = NO * ANA_C;
    static_assert(NV <= 32, "chunk too large for the wave reduction");
    __shared__ double red_all[4][2 * 16 * (NV + 2)];   // per wave: two chunk buffers
    const int L = D.L, npair = D.npair;
    const int q = blockIdx.x, tile = blockIdx.y;
    // grid z = map b of a batch x the l-segments of one map
    const int nsegz = D.seg > 0 ? (L + D.seg) / D.seg : 1;
    const int sg = (int)blockIdx.z % nsegz, bmap = (int)blockIdx.z / nsegz;
    const int ncb = (int)gridDim.z / nsegz * NC;              // comps of the whole batch
    // l-segmented launch: segments starting past L (about half of the grid at
    // small maps) leave before any load
    if (D.seg > 0 && !paired && q + sg * D.seg > D.L) return;
    phi += (long long)bmap * NC * 2 * phi_plane(L, npair);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g0 = tile * (LEG_BLOCK / 64) * ASR + wave * ASR;
    const long long plane = phi_plane(L, npair);
    double x[ASR], s2[ASR];
    int pr[ASR];
    bool act[ASR];
#pragma unroll
    for (int r = 0; r < ASR; ++r) {
        pr[r] = (g0 + r) * 64 + lane;
        act[r] = pr[r] < npair;
        x[r] = act[r] ? D.geom[pr[r]].x : 0.0;
        s2[r] = ring_s2(act[r], act[r] ? D.geom[pr[r]].is2 : 0.0);
    }
    for (int h = 0; h < 2; ++h) {
        const int m = h == 0 ? q : L - q;
        if (h == 1 && (!paired || m <= q)) break;
        // l-segment of this launch (D.seg > 0, unpaired m): [lA, lend]; else m..L
        const int lA = D.seg > 0 ? m + sg * D.seg : m;
        if (lA > L) break;
        const int lend = D.seg > 0 ? min(lA + D.seg - 1, L) : L;
        int ls[ASR];
        bool tab[ASR];
#pragma unroll
        for (int r = 0; r < ASR; ++r) {
            ls[r] = __builtin_amdgcn_readfirstlane(g0 + r < D.ngroup ? D.lstart[(long long)m * D.ngroup + g0 + r]
                                                                     : L + 1);
            // a slot already past its onset at the segment start enters at lA with
            // the tabulated state (loaded below); otherwise at its onset, as before
            tab[r] = ls[r] <= L && ls[r] < lA;
            if (tab[r]) ls[r] = lA;
            if (ls[r] > lend) ls[r] = L + 1;          // nothing of this slot in the segment
        }
        // each wave walks l from its own slots' first onset (no workgroup sync)
        int lmin = L + 1;
#pragma unroll
        for (int r = 0; r < ASR; ++r) lmin = min(lmin, ls[r]);
        // parity-combined ring phases: [+]: N + S, [-]: N - S
        double2 fp[ASR][NC], fn[ASR][NC];
        double v0[ASR], v1[ASR];
        int kk[ASR];
#pragma unroll
        for (int r = 0; r < ASR; ++r) {
            v0[r] = 0.0; v1[r] = 0.0; kk[r] = 0;
            if (tab[r] && ls[r] <= L && act[r]) {
                const long long o = (long long)(D.segoff[m] + sg * D.segmul - 1) * npair + pr[r];
                const double2 s0 = D.sst[o];
                v1[r] = s0.x; v0[r] = s0.y;
                kk[r] = D.sstk[o];
            }
            const double is2 = act[r] && ls[r] <= L ? D.geom[pr[r]].is2 : 0.0;
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                double2 a = make_double2(0.0, 0.0), b = a;
                if (act[r] && ls[r] <= L) {
                    a = phi[(2LL * c + 0) * plane + phi_at(m, pr[r], npair)];
                    b = phi[(2LL * c + 1) * plane + phi_at(m, pr[r], npair)];
                }
                // spin-2 components carry the factor is2 of their terms
                const double w = (NC == 3 && c == 0) || NC == 1 ? 1.0 : is2;
                fp[r][c] = make_double2(w * (a.x + b.x), w * (a.y + b.y));
                fn[r][c] = make_double2(w * (a.x - b.x), w * (a.y - b.y));
            }
        }
        const long long obase = cidx(L, m, m) - m;
        const AnaCoef* cf = coef + obase;
        if constexpr (SEGL) {
            __syncthreads();                        // the previous m's readers are done
            const double2* src = reinterpret_cast<const double2*>(coef);
            double2* dst = reinterpret_cast<double2*>(cstage);
            for (int i = tid; i < (D.seg + 2) * 3; i += LEG_BLOCK)
                dst[i] = src[(obase + min(lA + i / 3, L)) * 3 + i % 3];
            __syncthreads();
            cf = cstage - lA;                       // cf[l], lA <= l <= lA + seg + 1
        }
        // chunks start on m's parity so positions 0, 2 of a chunk are even
        const int lstart0 = lmin - ((lmin - m) & 1);
        double* red = red_all[wave];
        // ---- fixed-order wave reduction of a chunk's NV partial sums ----
        // Two butterfly levels across the wave halves (v_permlane32_swap: lane ^ 32)
        // and rows (v_permlane16_swap: lane ^ 16) leave each lane NV/4 sums of 4
        // lanes (outputs block B = lane >> 4); the 16 lanes of a row then meet in
        // wave-private LDS (one row of NV per lane, two buffers): two lanes per
        // output sum 8 rows each and combine.  put_chunk writes a chunk, get_chunk
        // issues its reads, fin_chunk sums and stores; the fast loop reads chunk
        // k - 1 before computing chunk k, so the LDS latency hides under the
        // Legendre work (LDS ops of one wave complete in order: no fences).
        constexpr int H1 = NV / 2, H2 = NV / 4, RS2 = NV + 2, RBUF = 16 * RS2;
        auto put_chunk = [&](const double (&acc)[NV], int bsel) {
            double w1[H1], w2[H2];
#pragma unroll
            for (int t = 0; t < H1; ++t) {
                const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(acc[t]), __double2loint(acc[t + H1]),
                                                                 false, false);
                const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(acc[t]), __double2hiint(acc[t + H1]),
                                                                 false, false);
                w1[t] = __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
            }
#pragma unroll
            for (int t = 0; t < H2; ++t) {
                const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(w1[t]), __double2loint(w1[t + H2]),
                                                                 false, false);
                const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(w1[t]), __double2hiint(w1[t + H2]),
                                                                 false, false);
                w2[t] = __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
            }
            double* rowp = red + bsel * RBUF + (lane & 15) * RS2 + (lane >> 4) * H2;
#pragma unroll
            for (int t = 0; t < H2; t += 2)
                *reinterpret_cast<double2*>(rowp + t) = make_double2(w2[t], w2[t + 1]);
        };
        auto get_chunk = [&](int bsel, double (&rv)[8]) {
            const int o = min(lane >> 1, NV - 1), hh = lane & 1;
            const double* col = red + bsel * RBUF + (hh * 8) * RS2 + o;
#pragma unroll
            for (int i = 0; i < 8; ++i) rv[i] = col[i * RS2];
        };
        auto fin_chunk = [&](const double (&rv)[8], int l0) {
            const int o = lane >> 1, hh = lane & 1;
            double sum = rv[0];
#pragma unroll
            for (int i = 1; i < 8; ++i) sum += rv[i];
            const int slo = __builtin_amdgcn_update_dpp(0, __double2loint(sum), 0xB1, 0xf, 0xf, false);
            const int shi = __builtin_amdgcn_update_dpp(0, __double2hiint(sum), 0xB1, 0xf, 0xf, false);
            const double other = __hiloint2double(shi, slo);
            sum = hh ? other + sum : sum + other;   // rows 0-7 then 8-15 on both lanes
            if (hh == 0 && o < NV) {
                const int cc = o / NO, oo = o % NO;
                const int l = l0 + cc;
                if (l >= lA && l <= lend) {
                    const int comp = oo >> 1;
                    double* dst = reinterpret_cast<double*>(
                        part + (((long long)tile * 4 + wave) * ncb + bmap * NC + comp) * D.nlm + obase + l);
                    dst[oo & 1] = sum;          // spin 2: without the factor Q_l (the finish applies it)
                }
            }
        };
        auto reduce_store = [&](const double (&acc)[NV], int l0) {
            double rv[8];
            put_chunk(acc, 0);
            get_chunk(0, rv);
            fin_chunk(rv, l0);
        };
        // guarded chunk: slot activation at its onset, scaled lanes masked and
        // rescaled, l beyond L skipped
        auto slow_chunk = [&](double (&acc)[NV], int l0) {
#pragma unroll
            for (int cc = 0; cc < ANA_C; ++cc) {
                const int l = l0 + cc;
                if (l > lend) break;
                const AnaCoef c = cf[l];
#pragma unroll
                for (int r = 0; r < ASR; ++r) {
                    if (l < ls[r]) continue;                 // uniform per wave
                    if (l == ls[r] && act[r] && !tab[r]) {
                        const double2 s0 = D.st[(long long)m * npair + pr[r]];
                        v1[r] = s0.x; v0[r] = s0.y;
                        kk[r] = D.stk[(long long)m * npair + pr[r]];
                    }
                    const double xw0 = mul_nc(x[r], v0[r]), xw1 = mul_nc(x[r], v1[r]);
                    if ((cc & 1) == 0) ana_term<NC, true, true>(acc + cc * NO, c, v0[r], v1[r], xw0, xw1, kk[r], s2[r], fp[r], fn[r]);
                    else ana_term<NC, false, true>(acc + cc * NO, c, v0[r], v1[r], xw0, xw1, kk[r], s2[r], fp[r], fn[r]);
                    if (l < L) {
                        rec_ana(c, xw0, v0[r], v1[r]);
                        if (kk[r] < 0 && fabs(v0[r]) > SC_HI) { v0[r] *= SC_DN; v1[r] *= SC_DN; ++kk[r]; }
                    }
                }
            }
        };
        int l0 = lstart0;
        // phase 1: guarded chunks until every live slot is active and representable
        for (; l0 <= lend; l0 += ANA_C) {
            double acc[NV];
#pragma unroll
            for (int i = 0; i < NV; ++i) acc[i] = 0.0;
            slow_chunk(acc, l0);
            reduce_store(acc, l0);
            bool live = true;
#pragma unroll
            for (int r = 0; r < ASR; ++r)
                if (ls[r] <= L && (l0 + ANA_C <= ls[r] || __any(kk[r] < 0))) live = false;
            if (live) { l0 += ANA_C; break; }
        }
        // phase 2: full chunks, no guards (a dead slot, ls > L, has zero phases
        // and zero state and adds exact zeros)
#if defined(GS_ASM_MARKERS)
        asm volatile("; ANA_FAST_BEGIN");
#endif
        {
            bool pend = false;
            int pl0 = 0, cur = 0;
#if GS_ANA_PF > 0
            double pfv = 0.0;
#endif
            for (; l0 + ANA_C - 1 <= lend; l0 += ANA_C) {
                double rv[8];
                if (pend) get_chunk(cur ^ 1, rv);
                double acc[NV];
#pragma unroll
                for (int i = 0; i < NV; ++i) acc[i] = 0.0;
#if GS_ANA_PF > 0
                // coefficient lines GS_ANA_PF l ahead pulled into L2 by a vector load
                // (lanes 0-2: the chunk's 192 B from three 64-B steps; the table is
                // padded by 4 entries); consumed one chunk later
                acc[0] = pfv == 7.0e300 ? 1.0 : 0.0;
                pfv = reinterpret_cast<const double*>(reinterpret_cast<const char*>(cf + min(l0 + GS_ANA_PF, L + 1))
                                                      + (lane % 3) * 64)[0];
#endif
                // x lambda_{l-1}: carried from the previous step inside the chunk
                // (the same rounded product), recomputed at its start (a carry
                // across chunks costs the 4-slot TEB kernel its second wave)
                double xv1[ASR];
#pragma unroll
                for (int r = 0; r < ASR; ++r) xv1[r] = mul_nc(x[r], v1[r]);
#pragma unroll
                for (int cc = 0; cc < ANA_C; ++cc) {
                    const int l = l0 + cc;
                    const AnaCoef c = cf[l];
#pragma unroll
                    for (int r = 0; r < ASR; ++r) {
                        const double xv0 = mul_nc(x[r], v0[r]);
                        if ((cc & 1) == 0) ana_term<NC, true, false>(acc + cc * NO, c, v0[r], v1[r], xv0, xv1[r], 0, s2[r], fp[r], fn[r]);
                        else ana_term<NC, false, false>(acc + cc * NO, c, v0[r], v1[r], xv0, xv1[r], 0, s2[r], fp[r], fn[r]);
                        rec_ana(c, xv0, v0[r], v1[r]);
                        xv1[r] = xv0;
                    }
                }
                if (pend) fin_chunk(rv, pl0);
                put_chunk(acc, cur);
                pend = true;
                pl0 = l0;
                cur ^= 1;
            }
            if (pend) {
                double rv[8];
                get_chunk(cur ^ 1, rv);
                fin_chunk(rv, pl0);
            }
        }
#if defined(GS_ASM_MARKERS)
        asm volatile("; ANA_CHUNK_END");
#endif
        // phase 3: the partial last chunk
        if (l0 <= lend) {
            double acc[NV];
#pragma unroll
            for (int i = 0; i < NV; ++i) acc[i] = 0.0;
            slow_chunk(acc, l0);
            reduce_store(acc, l0);
        }
        // l below the wave's first chunk: exact zeros
        for (int l = lA + lane; l < min(lstart0, lend + 1); l += 64)
            for (int c = 0; c < NC; ++c)
                part[(((long long)tile * 4 + wave) * ncb + bmap * NC + c) * D.nlm + obase + l] = make_double2(0.0, 0.0);
    }
}

// sum tiles in fixed order, weight, sign (spin 2: and the factor Q_l the
// Legendre stage left out, AnaCoef), write the caller's layout (accumulate
// into it when acc != 0: the Jacobi steps of map2alm(iter > 0))
template <int NC>
__global__ void k_sht_anal_finish(int L, int nlm, int ntile, const double2* __restrict__ part, double w, int layout,
                                  int acc, double* __restrict__ alm, int nmap, const double* __restrict__ acq) {
    const long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    const int ncb = NC * nmap;                     // comps of the batch: comp = b * NC + c
    if (g >= (long long)ncb * nlm) return;
    const int comp = (int)(g / nlm);
    const long long i = g % nlm;
    double2 s = make_double2(0.0, 0.0);
    for (int t = 0; t < ntile; ++t) {
        const double2 v = part[((long long)t * ncb + comp) * nlm + i];
        s.x += v.x; s.y += v.y;
    }
    // (l, m) of complex index i
    // m = largest with cidx(L, m, m) = m(2L+3-m)/2 <= i
    const double b = 2.0 * L + 3.0;
    int m = (int)floor((b - sqrt(fmax(b * b - 8.0 * (double)i, 0.0))) / 2.0);
    m = max(0, min(m, L));
    while (m > 0 && (long long)m * (2 * L + 3 - m) / 2 > i) --m;
    while (m < L && (long long)(m + 1) * (2 * L + 2 - m) / 2 <= i) ++m;
    const int l = (int)(i - (long long)m * (2 * L + 1 - m) / 2);
    const bool spin0 = NC == 1 || (NC == 3 && comp % NC == 0);
    const double f = spin0 ? w : -w;
    s.x *= f; s.y *= f;
    if (!spin0) { s.x *= acq[l]; s.y *= acq[l]; }
    double* out = alm + comp * alm_comp_stride(layout, L);
    if (layout == GS_ALM_COMPLEX) {
        if (acc) { out[2 * i] += s.x; out[2 * i + 1] += s.y; }
        else { out[2 * i] = s.x; out[2 * i + 1] = s.y; }
    } else if (m == 0) {
        if (acc) out[l] += s.x; else out[l] = s.x;
    } else {
        constexpr double SQ2 = 1.41421356237309504880;
        const long long r = 2 * i - (L + 1);
        if (acc) { out[r] += SQ2 * s.x; out[r + 1] += SQ2 * s.y; }
        else { out[r] = SQ2 * s.x; out[r + 1] = SQ2 * s.y; }
    }
}

__global__ void k_sub_maps(long long n, const double* __restrict__ a, double* __restrict__ b) {
    const long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (g < n) b[g] = a[g] - b[g];
}

// ===========================================================================
// Batched small maps: the Legendre stage as dense fp64 matrix-core contractions
// ===========================================================================
// For a batch of B maps the Legendre stage of one m is a matrix product whose
// inner dimension is shared by every map:
//   synthesis  Phi[ring][col] = sum_{l, F} G_F(l, ring) a_F(l, col)   (K = l)
//   analysis   a[l][col]      = sum_{ring, F} G_F(l, ring) Phi_F(ring, col)  (K = rings)
// with col = (map, output part) and G = lambda (spin 0) or the spin-2 F1 / F2,
// the north / south parity folded as in the VALU kernels (output rows of one
// l parity).  lambda comes from a plan-time table (MfTab) filled by the same
// scaled recurrence the VALU kernels run -- a value the recurrence holds below
// the representable range (k < 0) is stored as 0, exactly what they multiply --
// and the spin-2 F1 / F2 are formed in the kernels from the table's lambda_l,
// lambda_{l-1} and the per-l coefficients (the VALU kernels' expressions, a few
// fp64 operations shared by every column group), so both transform kernels are
// v_mfma_f64_16x16x4_f64 streams whose K loop reads the table once per
// transform for every map of the batch.  The table costs 8 B x N_ringpair x
// N_lm (0.54 GB at N_side 256 / l_max 512; r04 first stored lambda, F1 and F2:
// three times the bytes, and the kernels ran at 3-4 TB/s of HBM reading it),
// so it is built for small maps only (large maps keep the on-the-fly
// recurrence).  Blocks of 16 l x 16 ring pairs; blocks wholly below the
// representable range of a (m, 16-pair tile) are not stored (b0, chosen so the
// stored blocks also hold the row above the first representable l).  At that
// first l the recurrence's lambda_{l-1} is already rescaled while its own row
// (k < 0) multiplies 0: the table keeps the rescaled value there (it enters the
// sums at l - 1 with weight ~2^-384, far below the fp64 rounding of the sums).
constexpr int MF_TILE = 16;
constexpr int MF_BLK = 256;                      // doubles per block (16 l x 16 pairs of lambda)

struct MfTab {
    const double* tab;       // blocks
    const long long* off;    // [L+1][ntile] first stored block of (m, tile)
    const int* b0;           // [L+1][ntile] first stored block index (l = m + 16 b)
    int ntile;
    long long nblk;          // stored blocks (the GS_DEBUG bounds check of every table read)
};

// GS_DEBUG tripwire: every table address the matrix-core
// kernels load lies inside the table (a read before its start faulted an r04
// experiment build); compiled out otherwise
__device__ __forceinline__ const double* mf_chk(const MfTab& T, const double* a) {
    GS_ASSERT(a >= T.tab && a < T.tab + T.nblk * MF_BLK);
    return a;
}

// pass 1: first representable l of every (m, ring pair) -> per (m, 16-pair tile) b0
__global__ __launch_bounds__(256) void k_mf_onset(ShtDev D, const double* __restrict__ lmm, const int* __restrict__ lmk,
                                                  int* __restrict__ b0) {
    const int L = D.L, npair = D.npair;
    const int m = blockIdx.y;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    int lon = L + 1;
    if (p < npair) {
        const double x = D.geom[p].x;
        const LegCoef* cf = D.coef + (cidx(L, m, m) - m);
        double v1 = 0.0, v0 = lmm[(long long)m * npair + p];
        int k = lmk[(long long)m * npair + p];
        for (int l = m; l <= L; ++l) {
            if (k == 0) { lon = l; break; }
            if (l == L) break;
            rec_step(cf[l + 1], x, v0, v1);
            if (k < 0 && fabs(v0) > SC_HI) { v0 *= SC_DN; v1 *= SC_DN; ++k; }
        }
    }
    // min over the 16 pairs of the tile (lanes 16 t .. 16 t + 15 of the wave)
    for (int o = 8; o > 0; o >>= 1) lon = min(lon, __shfl_xor(lon, o, 16));
    if ((threadIdx.x & 15) == 0 && p < npair) {
        const int nb = (L - m + MF_TILE) / MF_TILE;
        // the stored blocks start at the one holding lon - 1 (the kernels read
        // lambda_{lon-1} for F1 / F2 at lon)
        b0[(long long)m * ((npair + MF_TILE - 1) / MF_TILE) + p / MF_TILE] =
            lon > L ? nb : (max(lon - 1, m) - m) / MF_TILE;
    }
}

// pass 2: every (m, ring pair) walks its recurrence from m and writes lambda of
// the stored blocks (the VALU kernels' values: k < 0 -> 0; at the first
// representable l the row above takes the recurrence's rescaled lambda_{l-1})
__global__ __launch_bounds__(256) void k_mf_fill(ShtDev D, const double* __restrict__ lmm, const int* __restrict__ lmk,
                                                 MfTab T) {
    const int L = D.L, npair = D.npair;
    const int m = blockIdx.y;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npair) return;
    const int t = p / MF_TILE, j = p % MF_TILE;
    const long long ti = (long long)m * T.ntile + t;
    const int b0 = T.b0[ti], nb = (L - m + MF_TILE) / MF_TILE;
    if (b0 >= nb) return;
    double* out = const_cast<double*>(T.tab) + T.off[ti] * MF_BLK;
    const double x = D.geom[p].x;
    const LegCoef* cf = D.coef + (cidx(L, m, m) - m);
    double v1 = 0.0, v0 = lmm[(long long)m * npair + p];
    int k = lmk[(long long)m * npair + p];
    bool was_on = false;
    for (int l = m; l < m + nb * MF_TILE; ++l) {
        const int b = (l - m) / MF_TILE, r = (l - m) % MF_TILE;
        double lam = 0.0;
        if (l <= L) {
            const bool on = k == 0;
            lam = on ? v0 : 0.0;
            if (on && !was_on && l > m && (l - 1 - m) / MF_TILE >= b0)   // the onset's lambda_{l-1}
                out[(long long)((l - 1 - m) / MF_TILE - b0) * MF_BLK + ((l - 1 - m) % MF_TILE) * MF_TILE + j] = v1;
            was_on = on;
            if (l < L) {
                rec_step(cf[l + 1], x, v0, v1);
                if (k < 0 && fabs(v0) > SC_HI) { v0 *= SC_DN; v1 *= SC_DN; ++k; }
            }
        }
        if (b >= b0) out[(long long)(b - b0) * MF_BLK + r * MF_TILE + j] = lam;
    }
}

typedef double f64x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f64x4 mfma64(double a, double b, f64x4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// ---- synthesis: one wave per 16-pair tile, 4 tiles per workgroup ----------------
// Spin 2 (E, B -> Q, U): per quad of l (l0 = m + 16 b + 4 q, l0 - m even) the
// "+" product takes G+ (F1 at even l - m, F2 at odd) and the "-" product G-,
// so lane (g = lane / 16, j = lane % 16) holds A = G+-(l0 + g, pair 16 t + j)
// and B = the matching a_lm row of (l0 + g, col j); col = (map 4 cg + j / 4,
// part o = j % 4 = Q re, Q im, U re, U im):
//   F1 row: (aE.x, aE.y, aB.x, aB.y)     F2 row: (-aB.y, aB.x, aE.y, -aE.x)
// N = -(C+ + C-), S = -(C+ - C-).  The rows are staged in LDS already permuted
// ("+" row, "-" row per (l, map)), so the K loop is two LDS reads and two
// MFMAs per quad and column group.  Spin 0 (T): per octet the "+" K entries
// are the even l (l0, l0+2, l0+4, l0+6) and the "-" the odd ones, lambda rows,
// col = (map 8 cg + j / 2, re / im).  The a_lm of the workgroup's maps for
// MF_CH l are staged in LDS (every tile of the m reads them); the next chunk's
// are loaded into registers while this chunk's MFMAs run, and each block's
// table values are loaded one block ahead of their MFMAs.
// optional occupancy targets (build-time A/B only: the default lets the
// compiler keep every prefetched value in registers)
#ifdef GS_MF_SYN_WPE
#define GS_MF_SYN_ATTR __attribute__((amdgpu_waves_per_eu(GS_MF_SYN_WPE)))
#else
#define GS_MF_SYN_ATTR
#endif
#ifdef GS_MF_ANA_WPE
#define GS_MF_ANA_ATTR __attribute__((amdgpu_waves_per_eu(GS_MF_ANA_WPE)))
#else
#define GS_MF_ANA_ATTR
#endif
// (measured, 16 spin-2 maps, same box: 0 = 563 us, 1 = 544 us)
#ifndef GS_MF_SYN_XCD
#define GS_MF_SYN_XCD 1
#endif
// synthesis staging item order: 1 = consecutive threads take consecutive maps
// at one l (LDS rows written contiguously; each quarter-wave's global reads
// touch 16 lines), 0 = consecutive l of one map (coalesced global reads; the
// LDS writes then step a row per thread, 16-way bank conflicts)
#ifndef GS_MF_SMAP
#define GS_MF_SMAP 1
#endif
// analysis staging item order: 1 = consecutive threads take consecutive maps
// of one ring pair (LDS rows written contiguously), 0 = consecutive pairs of
// one map (phase reads in 64-B runs; LDS writes a row apart per thread).
// Measured (16 spin-2 maps, same box): 0 = 651 us, 1 = 805 us; the synthesis'
// GS_MF_SMAP 1 / 0 = 567 / 591 us
#ifndef GS_MF_AMAP
#define GS_MF_AMAP 0
#endif
// LDS row padding (doubles) of the synthesis / analysis staging (A/B: 0)
#ifndef GS_MF_SPAD
#define GS_MF_SPAD 8
#endif
#ifndef GS_MF_APAD
#define GS_MF_APAD 16
#endif
#ifndef GS_MF_ADB
#define GS_MF_ADB 1
#endif
#ifndef GS_MF_SDB
#define GS_MF_SDB 0
#endif
// table prefetch distance of the synthesis in blocks (1: the block after the
// one being multiplied; 2: two blocks ahead, a second register set)
#ifndef GS_MF_TPF
#define GS_MF_TPF 2
#endif
// synthesis: a quad's A operands computed during the previous quad's MFMAs (1)
// or at its own start (0, r04)
#ifndef GS_MF_SPIPE
#define GS_MF_SPIPE 1
#endif
// wave priority while a wave issues its MFMA burst (s_setprio; 0 = off): a
// wave with matrix work ready is picked before the staging waves of the SIMD
#ifndef GS_MF_PRIO
#define GS_MF_PRIO 0
#endif
__device__ __forceinline__ void mf_prio_hi() { if (GS_MF_PRIO) __builtin_amdgcn_s_setprio(GS_MF_PRIO); }
__device__ __forceinline__ void mf_prio_lo() { if (GS_MF_PRIO) __builtin_amdgcn_s_setprio(0); }
constexpr int MF_CH = 32;                          // l staged per chunk (two blocks)
constexpr int MF_TL_MAX = 256;                     // tiles of a support-skipping analysis (N_side <= 2048)
// RIN: the input is the caller's real-layout a_lm (areal, comp stride
// (L + 1)^2) with the optional beam bl, read and scaled while staging exactly as
// k_sht_alm_in would have (no separate input pass); otherwise the plan's
// complex-layout ain
template <int SPIN, int CGW, int CPW, bool RIN>
__global__ __launch_bounds__(256 * (CGW / CPW)) GS_MF_SYN_ATTR void k_sht_synth_mfma(ShtDev D, MfTab T, const double2* __restrict__ ain,
                                                        double2* __restrict__ phi, int nmap, int ncm, int cbase,
                                                        const int* __restrict__ pflag, const double* __restrict__ areal,
                                                        const double* __restrict__ bl) {
    constexpr int CPG = SPIN == 2 ? 4 : 8;         // maps per 16-column group
    constexpr int MPW = CGW * CPG;                 // maps per workgroup
    constexpr int NIT = MF_CH * MPW;               // staged (l, map) items per chunk
    constexpr int H = CGW / CPW;                   // waves per tile (column-group slices)
    constexpr int NT = 256 * H;                    // 4 tiles per workgroup
    constexpr int PER = (NIT + NT - 1) / NT;       // staged items per thread
    // staged rows (spin 2: per l a "+" and a "-" row of MPW x 4 doubles; spin 0
    // per l one row of MPW x 2), padded by 64 B: the four 16-lane groups of a
    // wave read four consecutive l, and rows 128 B apart mod 256 B put the two
    // groups of each half-wave on disjoint banks
    constexpr int SR = SPIN == 2 ? MPW * 4 + GS_MF_SPAD : MPW * 2 + GS_MF_SPAD;
    constexpr int NROW = SPIN == 2 ? 2 * MF_CH : MF_CH;
    // GS_MF_SDB: two staging buffers (the next chunk staged while this one is
    // multiplied: one barrier per chunk instead of two)
    constexpr int NBUF = GS_MF_SDB ? 2 : 1;
    __shared__ __attribute__((aligned(16))) double sb[NBUF * NROW * SR];
    // spin 2: the chunk's per-l coefficients (P, Q, R, T, Rm, 0) of F1 / F2
    __shared__ __attribute__((aligned(16))) double sc[NBUF * (SPIN == 2 ? MF_CH * 6 : 2)];
    constexpr int SCN = SPIN == 2 ? MF_CH * 6 : 2;
    int bsel = 0;                                  // the buffer the chunk's MFMAs read
    const int L = D.L, nlm = D.nlm, npair = D.npair;
    // GS_MF_SYN_XCD 0: grid (tile group, m, map group): the tile groups of one
    // m are consecutive blocks -- one per XCD, at the same time, so m's a_lm
    // come from HBM once (the other XCDs hit the infinity cache) -- and the 4 m
    // of a phase block written by one tile group land on that tile group's XCD.
    // 1: a 1-D grid in which each XCD takes whole phase blocks (4 m x every
    // tile group) back to back: a_lm and phase lines both stay in one L2.
    int m, tg;
    if (GS_MF_SYN_XCD) {
        const int ty = (T.ntile + 3) / 4, lin = blockIdx.x, slot = lin >> 3, per = PHI_MB * ty;
        m = ((slot / per) * 8 + (lin & 7)) * PHI_MB + (slot % per) / ty;
        tg = (slot % per) % ty;
        if (m > L) return;
    } else {
        m = blockIdx.y;
        tg = blockIdx.x;
    }
    // pflag (the fused weighted operator): tiles without weight need no phases
    // (the ring stage writes zeros there); a tile group without any leaves
    if (pflag) {
        bool any = false;
        for (int k = 0; k < 4; ++k) any |= tg * 4 + k < T.ntile && tile_support(pflag, tg * 4 + k, D.npair);
        if (!any) return;
    }
    const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int t = tg * 4 + wave / H;
    const bool tlive = t < T.ntile && (!pflag || tile_support(pflag, t, D.npair));
    const int cg0 = (wave % H) * CPW;             // this wave's first column group
    const int c0 = blockIdx.z * MPW;
    // the wave's column groups holding maps (wave-uniform; a batch of fewer maps
    // than the workgroup's columns -- the batched CG's unconverged chains)
    const int ncl = min(CPW, (nmap - c0 - cg0 * CPG + CPG - 1) / CPG);
    const int nb = (L - m + MF_TILE) / MF_TILE;
    const long long ti = (long long)m * T.ntile + min(t, T.ntile - 1);
    const int b0 = tlive ? T.b0[ti] : nb;
    const double* tab = T.tab + (t < T.ntile ? T.off[ti] : 0) * MF_BLK;
    const long long base = cidx(L, m, m) - m;
    // the lane's ring pair (F1 / F2 geometry)
    const int pj = min(MF_TILE * min(t, T.ntile - 1) + j, npair - 1);
    const double is2 = D.geom[pj].is2, xis2 = D.geom[pj].x * is2;
    // per-l coefficients of the chunk (threads < MF_CH; spin 2)
    const double2* cfb = reinterpret_cast<const double2*>(D.coef + base);
    double2 pc[3];
    auto fetchc = [&](int cb) __attribute__((always_inline)) {
        if constexpr (SPIN == 2) {
            // every thread loads (thread i the row i mod MF_CH: no branch around
            // the loads, see tblk); threads < MF_CH stage them
            const int l = min(m + cb * MF_TILE + (int)(threadIdx.x & (MF_CH - 1)), L);
            pc[0] = cfb[4 * l + 1]; pc[1] = cfb[4 * l + 2]; pc[2] = cfb[4 * l + 3];   // (P, Q), (R, T), (Rm, -)
        }
    };
    auto stagec = [&](int cb, int bf) __attribute__((always_inline)) {
        if constexpr (SPIN == 2) {
            if (threadIdx.x < MF_CH) {
                const bool ok = m + cb * MF_TILE + (int)threadIdx.x <= L;
                double2* d = reinterpret_cast<double2*>(sc + bf * SCN + threadIdx.x * 6);
                // (component selects: a select of double2 values goes through scratch)
                d[0] = make_double2(ok ? pc[0].x : 0.0, ok ? pc[0].y : 0.0);
                d[1] = make_double2(ok ? pc[1].x : 0.0, ok ? pc[1].y : 0.0);
                d[2] = make_double2(ok ? pc[2].x : 0.0, 0.0);
            }
        }
    };
    // item i: (l, map) in the GS_MF_SMAP order
    const long long NR = (long long)(L + 1) * (L + 1);
    double pb[PER];                                // RIN: the items' beam factors
    auto fetch = [&](int cb, double2 (&pf)[PER][SPIN == 2 ? 2 : 1]) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int i = threadIdx.x + NT * k;
            const int lr = GS_MF_SMAP ? i / MPW : i % MF_CH, mp = GS_MF_SMAP ? i % MPW : i / MF_CH;
            const int l = m + cb * MF_TILE + lr, c = c0 + mp;
            const bool ok = i < NIT && l <= L && c < nmap;
            // clamped address: the load is unconditional, the value selected when
            // staged (a select here would wait for the load)
            if constexpr (RIN) {
                // real layout: m = 0 at [l] (the next double is read and dropped),
                // m > 0 (re, im) at 2 cidx(l, m) - (L + 1)
                const int lq = ok ? l : m;
                const long long r = m == 0 ? lq : 2 * (base + lq) - (L + 1);
                const double* a = areal + ((long long)(ok ? c : 0) * ncm + cbase) * NR + r;
                pf[k][0] = make_double2(a[0], a[1]);
                if constexpr (SPIN == 2) pf[k][1] = make_double2(a[NR], a[NR + 1]);
                pb[k] = bl ? bl[lq] : 1.0;
            } else {
                const double2* src = ain + ((long long)(ok ? c : 0) * ncm + cbase) * nlm + base + (ok ? l : m);
                pf[k][0] = src[0];
                if constexpr (SPIN == 2) pf[k][1] = src[nlm];
            }
        }
    };
    // RIN: k_sht_alm_in's scaling of an item (m = 0: b a; m > 0: (b a) / sqrt 2)
    auto rin = [&](double2 v, double b) __attribute__((always_inline)) -> double2 {
        constexpr double IS2 = 0.70710678118654752440;
        if (m == 0) return make_double2(b * v.x, 0.0);
        return make_double2((b * v.x) * IS2, (b * v.y) * IS2);
    };
    auto stage = [&](int cb, const double2 (&pf)[PER][SPIN == 2 ? 2 : 1], int bf) __attribute__((always_inline)) {
        double* sbf = sb + bf * (NROW * SR);
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int i = threadIdx.x + NT * k;
            if (i >= NIT) continue;
            const int lr = GS_MF_SMAP ? i / MPW : i % MF_CH, mp = GS_MF_SMAP ? i % MPW : i / MF_CH;
            const bool ok = m + cb * MF_TILE + lr <= L && c0 + mp < nmap;
            double2 v0 = pf[k][0];
            double2 v1 = SPIN == 2 ? pf[k][SPIN == 2 ? 1 : 0] : v0;
            if constexpr (RIN) { v0 = rin(v0, pb[k]); v1 = rin(v1, pb[k]); }
            if constexpr (SPIN == 2) {
                const double ex = ok ? v0.x : 0.0, ey = ok ? v0.y : 0.0;
                const double bx = ok ? v1.x : 0.0, by = ok ? v1.y : 0.0;
                // F1 row (ex, ey, bx, by), F2 row (-by, bx, ey, -ex); "+" = F1 at even l - m
                const bool ev = (lr & 1) == 0;     // l - m parity (chunks start at even l - m)
                double2* P = reinterpret_cast<double2*>(sbf + (lr * 2 + 0) * SR + mp * 4);
                double2* M = reinterpret_cast<double2*>(sbf + (lr * 2 + 1) * SR + mp * 4);
                P[0] = make_double2(ev ? ex : -by, ev ? ey : bx);
                P[1] = make_double2(ev ? bx : ey, ev ? by : -ex);
                M[0] = make_double2(ev ? -by : ex, ev ? bx : ey);
                M[1] = make_double2(ev ? ey : bx, ev ? -ex : by);
            } else {
                reinterpret_cast<double2*>(sbf + lr * SR)[mp] = make_double2(ok ? v0.x : 0.0, ok ? v0.y : 0.0);
            }
        }
    };
    // block b's table (a block outside [b0, nb) reads the table's first block
    // instead -- always valid, never multiplied: mma skips it), so the loads
    // carry no condition (a conditional load would make the compiler wait on
    // the older loads at the join, the a_lm prefetch among them)
    auto tblk = [&](int b) __attribute__((always_inline)) -> const double* {
        const bool ok = b >= b0 && b < nb;
        return ok ? tab + (long long)(b - b0) * MF_BLK : T.tab;
    };
    // the table values of quad / octet-half q of a block: spin 2 lambda_l and
    // lambda_{l-1} (row 4 q + g and the row above; for the first row the
    // previous block's last one, read only when that block is stored: mma
    // zeroes it otherwise), spin 0 lambda
    auto tload = [&](const double* blk, bool prev, int q, double (&gv)[8]) __attribute__((always_inline)) {
        if constexpr (SPIN == 2) {
            const int row = 4 * q + g;
            gv[2 * q + 0] = *mf_chk(T, blk + row * MF_TILE + j);
            gv[2 * q + 1] = *mf_chk(T, row > 0 ? blk + (row - 1) * MF_TILE + j
                                               : (prev ? blk - MF_BLK + 15 * MF_TILE + j : T.tab));
        } else {
            // q = 2 h + e: octet half h, even (e = 0) / odd row of lambda
            const int row = 8 * (q >> 1) + 2 * g + (q & 1);
            gv[q] = *mf_chk(T, blk + row * MF_TILE + j);
        }
    };
    f64x4 Cp[CPW], Cm[CPW];
#pragma unroll
    for (int c = 0; c < CPW; ++c) { Cp[c] = f64x4{0, 0, 0, 0}; Cm[c] = f64x4{0, 0, 0, 0}; }
    const int o = j & 3;
    // the staged B operands of quad / octet-half q (rows lr0 + ..): "+" and "-"
    // per column group
    // the lane's base in the staged rows; everything else is a compile-time
    // offset (the ds_read immediate), so no per-read address registers
    const double* sbl0 = SPIN == 2 ? sb + (g * 2) * SR + (cg0 * 4 + (j >> 2)) * 4 + o
                                   : sb + (2 * g) * SR + (cg0 * 8 + (j >> 1)) * 2 + (j & 1);
    auto lds = [&](int lr0, int q, double (&bq)[2 * CPW]) __attribute__((always_inline)) {
        const double* sbl = sbl0 + bsel * (NROW * SR);
#pragma unroll
        for (int c = 0; c < CPW; ++c) {
            if constexpr (SPIN == 2) {
                const int r0 = lr0 + 4 * q;         // row = r0 + g
                bq[2 * c + 0] = sbl[(r0 * 2 + 0) * SR + c * 16];
                bq[2 * c + 1] = sbl[(r0 * 2 + 1) * SR + c * 16];
            } else {
                const int r0 = lr0 + 8 * q;         // even row = r0 + 2 g
                bq[2 * c + 0] = sbl[r0 * SR + c * 16];
                bq[2 * c + 1] = sbl[(r0 + 1) * SR + c * 16];
            }
        }
    };
    // block b's MFMAs (staged rows lr0 ..): each quad's B operands read one quad
    // ahead, its table registers refilled with block b + 1's values as soon as
    // they are consumed (a block of MFMAs ahead of their use)
    auto mma = [&](int b, int lr0, double (&gv)[8]) __attribute__((always_inline)) {
        // refill with block b + GS_MF_TPF (its row above: block b + GS_MF_TPF - 1's
        // last row, read when both blocks are stored)
        const double* nblk = tblk(b + GS_MF_TPF);
        const bool nprev = b + GS_MF_TPF - 1 >= b0 && b + GS_MF_TPF < nb;
        const bool prev = b - 1 >= b0;               // block b's
        // every load unconditional (a load in one arm of a branch makes the
        // compiler's wait at the join cover the other arm's registers too); only
        // the MFMAs sit under the wave-uniform block test
        const bool on = b >= b0 && b < nb;
        constexpr int NQ = SPIN == 2 ? 4 : 2;
        double bq[2][2 * CPW];                      // two rolling buffers
        double cv[2][5];                            // spin 2: (P, Q, R, T, Rm) of the lane's row
        auto ldc = [&](int q, double (&c)[5]) __attribute__((always_inline)) {
            if constexpr (SPIN == 2) {
                const double* cq = sc + bsel * SCN + (lr0 + 4 * q + g) * 6;
#pragma unroll
                for (int k = 0; k < 5; ++k) c[k] = cq[k];
            }
        };
        // the A operands of quad q: spin 2 F1 / F2 at l = m + 16 b + 4 q + g (the
        // VALU kernels' expressions; G+ = the one with lambda's parity: F1 at
        // even l - m), spin 0 lambda
        auto opnd = [&](int q, double& ap, double& am) __attribute__((always_inline)) {
            if constexpr (SPIN == 2) {
                const double w0 = gv[2 * q];
                const double w1 = (q > 0 || g > 0 || prev) ? gv[2 * q + 1] : 0.0;
                const int u = q & 1;
                const double f1 = fma(cv[u][2] * xis2, w1, -fma(cv[u][0], is2, cv[u][1]) * w0);
                const double f2 = fma(cv[u][4] * is2, w1, -(cv[u][3] * xis2) * w0);
                const bool ev = (g & 1) == 0;
                ap = ev ? f1 : f2;
                am = ev ? f2 : f1;
            } else {
                ap = gv[2 * q];
                am = gv[2 * q + 1];
            }
        };
        lds(lr0, 0, bq[0]);
        ldc(0, cv[0]);
        double apc = 0.0, amc = 0.0;
        if (GS_MF_SPIPE) opnd(0, apc, amc);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            if (q + 1 < NQ) { lds(lr0, q + 1, bq[(q + 1) & 1]); ldc(q + 1, cv[(q + 1) & 1]); }
            // keep the order as written: the scheduler would sink the next
            // quad's reads and the table refills behind the MFMAs
            __builtin_amdgcn_sched_barrier(0);
            if (!GS_MF_SPIPE) opnd(q, apc, amc);
            if (on) {
                mf_prio_hi();
#pragma unroll
                for (int c = 0; c < CPW; ++c) {
                    if (c < ncl) {                  // (a column group without maps: no MFMAs)
                        Cp[c] = mfma64(apc, bq[q & 1][2 * c + 0], Cp[c]);
                        Cm[c] = mfma64(amc, bq[q & 1][2 * c + 1], Cm[c]);
                    }
                }
                mf_prio_lo();
            }
            __builtin_amdgcn_sched_barrier(0);
            // the next quad's operands while these MFMAs run (their fp64 chain
            // no longer sits between a quad's loads and its MFMAs; GS_MF_SPIPE 0:
            // computed at the quad's start, the r04 order, A/B only)
            double apn = 0.0, amn = 0.0;
            if (GS_MF_SPIPE && q + 1 < NQ) opnd(q + 1, apn, amn);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (SPIN == 2) tload(nblk, nprev, q, gv);
            else { tload(nblk, false, 2 * q, gv); tload(nblk, false, 2 * q + 1, gv); }
            __builtin_amdgcn_sched_barrier(0);
            apc = apn;
            amc = amn;
        }
    };
    double2 pf[PER][SPIN == 2 ? 2 : 1];
    double gv[8], gw[8];
    auto tload4 = [&](int b, double (&g)[8]) __attribute__((always_inline)) {
        const bool pv = b - 1 >= b0 && b < nb;
        if constexpr (SPIN == 2) {
#pragma unroll
            for (int q = 0; q < 4; ++q) tload(tblk(b), pv, q, g);
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) tload(tblk(b), false, q, g);
        }
    };
    tload4(0, gv);
    if (GS_MF_TPF == 2) tload4(1, gw);
    fetch(0, pf);
    fetchc(0);
    constexpr int CS = MF_CH / MF_TILE;              // blocks per chunk
    if (GS_MF_SDB) {
        // chunk 0 staged up front, chunk 1 in registers
        stage(0, pf, 0);
        stagec(0, 0);
        if (CS < nb) { fetch(CS, pf); fetchc(CS); }
        __syncthreads();
    }
    for (int cb = 0; cb < nb; cb += CS) {
        if (GS_MF_SDB) {
            // this chunk was staged during the last one (buffer bsel); the next is
            // staged now into the other buffer and the one after loaded; one
            // barrier ends the chunk (the staging visible, this buffer read by
            // every wave before it is written again)
            bsel = (cb / CS) & 1;
            if (cb + CS < nb) { stage(cb + CS, pf, bsel ^ 1); stagec(cb + CS, bsel ^ 1); }
            if (cb + 2 * CS < nb) { fetch(cb + 2 * CS, pf); fetchc(cb + 2 * CS); }
        } else {
            __syncthreads();                        // the previous chunk's readers are done
            stage(cb, pf, 0);
            stagec(cb, 0);
            __syncthreads();
            if (cb + CS < nb) { fetch(cb + CS, pf); fetchc(cb + CS); }
        }
        mma(cb, 0, gv);
        mma(cb + 1, MF_TILE, GS_MF_TPF == 2 ? gw : gv);
        if (GS_MF_SDB) __syncthreads();
    }
    if (!tlive) return;
    // D layout: lane (g, j) holds rows g + 4 r (pairs 16 t + g + 4 r), col j
    const long long plane = phi_plane(L, npair);
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        const int mp = SPIN == 2 ? (cg0 + c) * 4 + (j >> 2) : (cg0 + c) * 8 + (j >> 1);
        const int map = c0 + mp;
        if (map >= nmap) continue;
        const int comp = SPIN == 2 ? cbase + ((j & 3) >> 1) : cbase;
        const int part = j & 1;
        double* PN = reinterpret_cast<double*>(phi + (((long long)map * ncm + comp) * 2 + 0) * plane);
        double* PS = reinterpret_cast<double*>(phi + (((long long)map * ncm + comp) * 2 + 1) * plane);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int pr = MF_TILE * t + g + 4 * r;
            if (pr >= npair) continue;
            const double sp = Cp[c][r], sn = Cm[c][r];
            const long long off = 2 * phi_at(m, pr, npair) + part;
            if constexpr (SPIN == 2) { PN[off] = -(sp + sn); PS[off] = -(sp - sn); }
            else { PN[off] = sp + sn; PS[off] = sp - sn; }
        }
    }
}

// ---- f2 block synthesis on the matrix cores (tables; spin 2: E, B -> Q, U) -------
// The maps y_k = A(delta a_k) of a group's Metropolis blocks for a batch of
// chains (NonCenteredGibbs.py:333-355 scores every block with one of them):
// per (m, ring pair) the sums of k_sht_synth_mfma restricted to each block's l
// range.  Every (field, l) belongs to at most one block, so the columns carry
// one source field at a time (blockIdx.z = 2 chain group + field; a pass stages
// only its field's delta a: F1 row (ex, ey, 0, 0) / F2 row (0, 0, ey, -ex) for E,
// (0, 0, bx, by) / (-by, bx, 0, 0) for B).
// The planes are the cost (1.1 GB per chain at N_side 256, l_max 512 against
// ~2 GFLOP of MFMA), so a workgroup owns one 16-pair tile and the 4 m of one
// phase block (wave w: m = 4 mq + w): the blocks are walked in l order, each
// wave adds the block's rows of its m (a quad that straddles a block edge runs
// with the other rows' B operands zeroed), and at the block's end the four
// waves' sums go through LDS and out as whole 64-B runs (4 m x one pair), 1 KB
// contiguous per (chain, component, N / S).  Writing 16 B per lane at the
// planes' 64-B stride instead ran at 0.7 TB/s (27.7 ms for 16 chains against
// 2.7 ms with the stores removed).  Blocks below a tile's representable onset
// get zero planes.  da: [nmap][2][(L+1)^2] real layout (the beam folded in by
// k_f2_delta); blk: [2][L+1] local block ids (-1: none); phib [nmap][K][2
// comps][N, S][plane].
template <int CGW>
__global__ __launch_bounds__(256) void k_sht_blocks_mfma(ShtDev D, MfTab T, const double* __restrict__ da, int nmap,
                                                         const int* __restrict__ blk, int K,
                                                         double2* __restrict__ phib) {
    constexpr int CPG = 4;                          // chains per 16-column group
    constexpr int MPW = CGW * CPG;                  // chains per workgroup
    constexpr int CH = MF_TILE;                     // l staged per chunk (one table block)
    constexpr int NIT = CH * MPW;                   // staged (l, chain) items per wave and chunk
    constexpr int PER = (NIT + 63) / 64;
    constexpr int SR = MPW * 4 + GS_MF_SPAD;
    constexpr int NROW = 2 * CH;
    constexpr int NCOL = MPW * 4;                   // columns: chain x (Q re, Q im, U re, U im)
    __shared__ __attribute__((aligned(16))) double sb[4 * NROW * SR];      // per wave
    __shared__ __attribute__((aligned(16))) double sc[4 * CH * 6];         // per wave
    __shared__ __attribute__((aligned(16))) double fb[4 * MF_TILE * NCOL * 2];
    extern __shared__ int sblk[];                   // the field's block ids, l = 0 .. L
    const int L = D.L, npair = D.npair;
    const int fld = blockIdx.z & 1;
    const int c0 = (blockIdx.z >> 1) * MPW;
    const int t = blockIdx.x;
    const int m0 = 4 * blockIdx.y;
    const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int m = m0 + w;                           // this wave's m
    const bool mlive = m <= L;
    for (int l = threadIdx.x; l <= L; l += blockDim.x) sblk[l] = blk[fld * (L + 1) + l];
    const int mc = min(m, L);
    const int nb = (L - mc + MF_TILE) / MF_TILE;
    const long long ti = (long long)mc * T.ntile + t;
    const int b0 = mlive ? T.b0[ti] : nb;
    const double* tab = T.tab + T.off[ti] * MF_BLK;
    const long long base = cidx(L, mc, mc) - mc;
    const int pj = min(MF_TILE * t + j, npair - 1);
    const double is2 = D.geom[pj].is2, xis2 = D.geom[pj].x * is2;
    const double2* cfb = reinterpret_cast<const double2*>(D.coef + base);
    const long long NR = (long long)(L + 1) * (L + 1);
    double* sbw = sb + w * NROW * SR;
    double* scw = sc + w * CH * 6;
    // stage table block / chunk ch of this wave's m (wave-local LDS; rows past L zero)
    int staged = -1;
    auto stage = [&](int ch) __attribute__((always_inline)) {
        constexpr double IS2 = 0.70710678118654752440;
        double2 v[PER];
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int i = lane + 64 * k;
            const int lr = i / MPW, mp = i % MPW;
            const int l = mc + ch * CH + lr, c = c0 + mp;
            const bool ok = i < NIT && l <= L && c < nmap && mlive;
            const int lq = ok ? l : mc;
            const long long r = mc == 0 ? lq : 2 * (base + lq) - (L + 1);
            const double* a = da + ((long long)(ok ? c : 0) * 2 + fld) * NR + r;
            const double2 x = make_double2(a[0], a[1]);
            v[k] = !ok ? make_double2(0.0, 0.0)
                       : (mc == 0 ? make_double2(x.x, 0.0) : make_double2(x.x * IS2, x.y * IS2));
        }
        double2 pc[3];
        {
            const int lr = lane & (CH - 1);
            const int l = min(mc + ch * CH + lr, L);
            pc[0] = cfb[4 * l + 1]; pc[1] = cfb[4 * l + 2]; pc[2] = cfb[4 * l + 3];
        }
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int i = lane + 64 * k;
            if (i >= NIT) continue;
            const int lr = i / MPW, mp = i % MPW;
            const double ex = fld == 0 ? v[k].x : 0.0, ey = fld == 0 ? v[k].y : 0.0;
            const double bx = fld == 1 ? v[k].x : 0.0, by = fld == 1 ? v[k].y : 0.0;
            const bool ev = (lr & 1) == 0;
            double2* P = reinterpret_cast<double2*>(sbw + (lr * 2 + 0) * SR + mp * 4);
            double2* M = reinterpret_cast<double2*>(sbw + (lr * 2 + 1) * SR + mp * 4);
            P[0] = make_double2(ev ? ex : -by, ev ? ey : bx);
            P[1] = make_double2(ev ? bx : ey, ev ? by : -ex);
            M[0] = make_double2(ev ? -by : ex, ev ? bx : ey);
            M[1] = make_double2(ev ? ey : bx, ev ? -ex : by);
        }
        if (lane < CH) {
            const bool ok = mc + ch * CH + lane <= L;
            double2* d = reinterpret_cast<double2*>(scw + lane * 6);
            d[0] = make_double2(ok ? pc[0].x : 0.0, ok ? pc[0].y : 0.0);
            d[1] = make_double2(ok ? pc[1].x : 0.0, ok ? pc[1].y : 0.0);
            d[2] = make_double2(ok ? pc[2].x : 0.0, 0.0);
        }
        // the wave's own LDS writes complete before its lanes read them
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        staged = ch;
    };
    f64x4 Cp[CGW], Cm[CGW];
#pragma unroll
    for (int c = 0; c < CGW; ++c) { Cp[c] = f64x4{0, 0, 0, 0}; Cm[c] = f64x4{0, 0, 0, 0}; }
    const int o = j & 3;
    // rows [lo, hi) of this wave's m (block k's part of it)
    auto accumulate = [&](int lo, int hi) __attribute__((always_inline)) {
        lo = max(lo, m);
        if (!mlive || hi <= lo) return;
        for (int i0 = (lo - m) & ~3; m + i0 < hi; i0 += 4) {
            const int ch = i0 / CH, rr0 = i0 % CH;
            if (ch != staged) stage(ch);
            if (ch < b0 || ch >= nb) continue;          // below the onset: lambda = 0 (wave-uniform)
            const double* bp = tab + (long long)(ch - b0) * MF_BLK;
            const int rr = rr0 + g;
            const double w0 = *mf_chk(T, bp + rr * MF_TILE + j);
            double w1 = 0.0;
            if (rr > 0) w1 = *mf_chk(T, bp + (rr - 1) * MF_TILE + j);
            else if (ch - 1 >= b0) w1 = *mf_chk(T, bp - MF_BLK + 15 * MF_TILE + j);
            const double* cq = scw + rr * 6;
            const double f1 = fma(cq[2] * xis2, w1, -fma(cq[0], is2, cq[1]) * w0);
            const double f2 = fma(cq[4] * is2, w1, -(cq[3] * xis2) * w0);
            const bool ev = (g & 1) == 0;
            const double ap = ev ? f1 : f2, am = ev ? f2 : f1;
            const int l = m + i0 + g;
            const bool mine = l >= lo && l < hi;
            const double* sbl = sbw + (rr * 2) * SR + (j >> 2) * 4 + o;
#pragma unroll
            for (int c = 0; c < CGW; ++c) {
                const double bqp = mine ? sbl[c * 16] : 0.0;
                const double bqm = mine ? sbl[SR + c * 16] : 0.0;
                Cp[c] = mfma64(ap, bqp, Cp[c]);
                Cm[c] = mfma64(am, bqm, Cm[c]);
            }
        }
    };
    const long long plane = phi_plane(L, npair);
    __syncthreads();                                // sblk visible
    for (int l = m0; l <= L;) {
        const int k = sblk[l];
        int le = l + 1;
        while (le <= L && sblk[le] == k) ++le;
        if (k >= 0) {
            accumulate(l, le);
            // block k's sums of the 4 m -> LDS -> whole 64-B runs of the planes
            __syncthreads();                        // (the previous flush's readers are done)
#pragma unroll
            for (int c = 0; c < CGW; ++c)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int pl = g + 4 * r, col = c * 16 + j;
                    const double sp = Cp[c][r], sn = Cm[c][r];
                    double* f = fb + ((w * MF_TILE + pl) * NCOL + col) * 2;
                    f[0] = -(sp + sn);
                    f[1] = -(sp - sn);
                }
#pragma unroll
            for (int c = 0; c < CGW; ++c) { Cp[c] = f64x4{0, 0, 0, 0}; Cm[c] = f64x4{0, 0, 0, 0}; }
            __syncthreads();
            constexpr int NPC = MPW * 2 * 2 * MF_TILE * 4;     // 16-B pieces: chain, comp, N/S, pair, m
            for (int pc = threadIdx.x; pc < NPC; pc += blockDim.x) {
                const int wm = pc & 3, pl = (pc >> 2) & (MF_TILE - 1), rest = pc >> 6;
                const int h = rest & 1, q = (rest >> 1) & 1, cc = rest >> 2;
                const int pr = MF_TILE * t + pl, mm = m0 + wm;
                if (c0 + cc >= nmap || pr >= npair || mm > L) continue;
                const double* f = fb + ((wm * MF_TILE + pl) * NCOL + cc * 4 + q * 2) * 2 + h;
                phib[((((long long)(c0 + cc) * K + k) * 2 + q) * 2 + h) * plane + phi_at(mm, pr, npair)] =
                    make_double2(f[0], f[2]);
            }
        }
        l = le;
    }
}

// ---- analysis: one wave per 32-l window (16 even + 16 odd l), all pair tiles ----
// a^T[col][l] = sum_K Phi^T[col][K] G[K][l], K = 4 ring pairs of one function
// per MFMA: A = Phi^T (lane: row = col j, k = pair 4 s + g), B = G (lane: k =
// pair, col = l index j of the window's parity-p rows, l = lw + 2 j + p).  The
// ring phases of each 16-pair tile are staged once per workgroup in LDS as the
// parity-combined (N + S, N - S) of Q, U (spin 2) or T (spin 0), the next
// tile's loaded into registers while this tile's MFMAs run.  Spin 2, even l
// (p = 0; p = 1 swaps + and -), output parts o = (E re, E im, B re, B im):
//   F1 coefficients (+Q.x, +Q.y, +U.x, +U.y)[o]
//   F2 coefficients sign(o) (-)[3 - o] of (-Q.x, -Q.y, -U.x, -U.y), sign - for o = 0, 3
// where + = N + S, - = N - S (ana_term of the recurrence kernels).  The tiles
// are summed inside the accumulator in tile order (no cross-workgroup
// reduction); the weight (spin 0: w, spin 2: -w) and the caller's layout are
// applied on the store.
template <int SPIN, int CGW, int CPW, int NT>
__global__ __launch_bounds__(NT) GS_MF_ANA_ATTR void k_sht_anal_mfma(ShtDev D, MfTab T, const double2* __restrict__ phi, int nmap,
                                                       int ncm, int cbase, double w, int layout, int acc,
                                                       double* __restrict__ alm, const int* __restrict__ pflag) {
    constexpr int CPG = SPIN == 2 ? 4 : 8;
    constexpr int MPW = CGW * CPG;
    constexpr int NV = SPIN == 2 ? 8 : 4;          // staged doubles per (pair, map)
    constexpr int NIT = MF_TILE * MPW;             // staged (pair, map) items per tile
    constexpr int PER = (NIT + NT - 1) / NT;
    // per ring pair jp a row [N + S | N - S] x [map] x [component] (HV = NV / 2
    // components: Q.x Q.y U.x U.y or T.x T.y), so the 16 lanes of a group read
    // 16 consecutive doubles; rows padded to 128 B mod 256 B, so the two groups
    // of a half-wave (pairs 4 s + g, g = 0 / 1 and 2 / 3) use disjoint banks
    constexpr int HV = NV / 2;
    constexpr int RW = 2 * MPW * HV + GS_MF_APAD;
    // GS_MF_ADB: two staging buffers (the next tile staged while this one is
    // multiplied: one barrier per tile instead of two)
    __shared__ __attribute__((aligned(16))) double sp_[(GS_MF_ADB ? 2 : 1) * MF_TILE * RW];
    __shared__ int tl_[MF_TL_MAX];                 // pflag: the tiles with weight, in order
    __shared__ int ntl_;
    const int L = D.L, npair = D.npair;
    // XCD-aware order (1-D grid over (m, window group)): blocks lin, lin + 8,
    // ... run on one XCD, and each XCD takes whole phase blocks -- the 4 m x
    // WGY window groups that read the same 128-B phase lines -- back to back,
    // so those lines come from HBM once into that XCD's L2
    constexpr int H = CGW / CPW;                   // waves per window (column-group slices)
    constexpr int WPG = NT / 64 / H;               // windows per workgroup
    const int WGY = ((L + 1 + 31) / 32 + WPG - 1) / WPG;   // window groups of m = 0
    const int lin = blockIdx.x, slot = lin >> 3, per = PHI_MB * WGY;
    const int m = ((slot / per) * 8 + (lin & 7)) * PHI_MB + (slot % per) / WGY;
    const int wgy = (slot % per) % WGY;
    // workgroups whose first window starts past L leave before any barrier
    if (m > L || m + 32 * wgy * WPG > L) return;
    const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int win = wgy * WPG + wave / H;
    const int cg0 = (wave % H) * CPW;             // this wave's first column group
    const int ncl = min(CPW, (nmap - (int)blockIdx.z * MPW - cg0 * CPG + CPG - 1) / CPG);   // groups with maps
    const int lw = m + 32 * win;
    const bool live = lw <= L;
    const int c0 = blockIdx.z * MPW;
    const int nb = (L - m + MF_TILE) / MF_TILE;
    const int bw = 2 * win;                        // the window's first block
    const long long plane = phi_plane(L, npair);
    // the staged item of thread (k): N, S phases of (pair, map) -> registers
    struct Ph { double2 a, b, c, d; };
    auto fetch = [&](int t, Ph (&pf)[PER]) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int i = threadIdx.x + NT * k;
            const int jp = GS_MF_AMAP ? i / MPW : i % MF_TILE, mp = GS_MF_AMAP ? i % MPW : i / MF_TILE;
            const int pr = MF_TILE * t + jp, map = c0 + mp;
            const double2 z = make_double2(0.0, 0.0);
            pf[k] = Ph{z, z, z, z};
            if (i < NIT && pr < npair && map < nmap) {
                const long long off = phi_at(m, pr, npair);
                const double2* P = phi + ((long long)map * ncm + cbase) * 2 * plane;
                pf[k].a = P[off];
                pf[k].b = P[plane + off];
                if constexpr (SPIN == 2) {
                    pf[k].c = P[2 * plane + off];
                    pf[k].d = P[3 * plane + off];
                }
            }
        }
    };
    f64x4 C[CPW][2];
#pragma unroll
    for (int c = 0; c < CPW; ++c) { C[c][0] = f64x4{0, 0, 0, 0}; C[c][1] = f64x4{0, 0, 0, 0}; }
    const int o = j & 3;
    const double s2 = (o == 0 || o == 3) ? -1.0 : 1.0;
    constexpr int NF = SPIN == 2 ? 2 : 1;
    // the lane's bases in the staged phases (row jp = 4 s + g, map (cg0 + c) ..):
    // spin 2 component o (a1) and 3 - o (a2), spin 0 re / im
    const double* spo = SPIN == 2 ? sp_ + g * RW + (cg0 * 4 + (j >> 2)) * HV + o
                                  : sp_ + g * RW + (cg0 * 8 + (j >> 1)) * HV + (j & 1);
    const double* spr = sp_ + g * RW + (cg0 * 4 + (j >> 2)) * HV + 3 - o;
    // tile t's window: false if it lies wholly below the tile's onset; bj / okb
    // the lane's block and whether it is stored
    // (prv: the row above the lane's first row -- the previous block's last --
    // is stored; the lane's l for p = 0 is that block's row 2 (j & 7))
    struct Tw { const double* blk; bool any, okb, prv; };
    auto twin = [&](int t) __attribute__((always_inline)) -> Tw {
        const long long ti = (long long)m * T.ntile + t;
        const int b0 = T.b0[ti];
        const bool any = live && bw + 1 >= b0 && bw < nb;    // wave-uniform
        const int bj = bw + (j >> 3);
        const bool okb = any && bj >= b0 && bj < nb;
        return Tw{okb ? T.tab + (T.off[ti] + bj - b0) * MF_BLK : T.tab, any, okb, okb && bj - 1 >= b0};
    };
    // the per-slice values of a tile (pairs 4 s + g): lambda at the lane's rows
    // 2 (j & 7) + p, spin 2 also the row above p = 0's and the pair's geometry.
    // Unconditional loads (a lane whose block is not stored reads the first
    // block; its values are zeroed where they are used)
    constexpr int NG = SPIN == 2 ? 5 : 2;
    auto tload = [&](const Tw& w, int t, int s, double (&gv)[4][NG]) __attribute__((always_inline)) {
        const double* bp = w.blk;
        const int row = 2 * (j & 7);
        gv[s][0] = *mf_chk(T, bp + row * MF_TILE + 4 * s + g);
        gv[s][1] = *mf_chk(T, bp + (row + 1) * MF_TILE + 4 * s + g);
        if constexpr (SPIN == 2) {
            const double* up = (j & 7) ? bp + (row - 1) * MF_TILE : (w.prv ? bp - MF_BLK + 15 * MF_TILE : T.tab);
            gv[s][2] = *mf_chk(T, up + 4 * s + g);
            const PairGeom* ge = D.geom + min(MF_TILE * t + 4 * s + g, npair - 1);
            gv[s][3] = ge->x;
            gv[s][4] = ge->is2;
        }
    };
    // spin 2: the lane's per-l coefficients of F1 / F2 (l = lw + 2 j + p)
    double cP[2], cQ[2], cR[2], cT[2], cRm[2];
    if constexpr (SPIN == 2) {
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const LegCoef c = D.coef[cidx(L, m, m) + min(lw + 2 * j + p, L) - m];
            cP[p] = c.P; cQ[p] = c.Q; cR[p] = c.R; cT[p] = c.T; cRm[p] = c.Rm;
        }
    }
    auto stage = [&](const Ph (&pf)[PER], double* sbuf) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int i = threadIdx.x + NT * k;
            if (i >= NIT) continue;
            const int jp = GS_MF_AMAP ? i / MPW : i % MF_TILE, mp = GS_MF_AMAP ? i % MPW : i / MF_TILE;
            double* dp = sbuf + jp * RW + mp * HV;                           // N + S
            double* dm = dp + MPW * HV;                                      // N - S
            const Ph& q = pf[k];
            if constexpr (SPIN == 2) {          // a = Q north, b = Q south, c = U north, d = U south
                dp[0] = q.a.x + q.b.x; dp[1] = q.a.y + q.b.y; dp[2] = q.c.x + q.d.x; dp[3] = q.c.y + q.d.y;
                dm[0] = q.a.x - q.b.x; dm[1] = q.a.y - q.b.y; dm[2] = q.c.x - q.d.x; dm[3] = q.c.y - q.d.y;
            } else {
                dp[0] = q.a.x + q.b.x; dp[1] = q.a.y + q.b.y; dm[0] = q.a.x - q.b.x; dm[1] = q.a.y - q.b.y;
            }
        }
    };
    // the tiles summed: all, or (pflag) those with weight -- a tile without
    // adds exact zeros, so skipping it leaves every bit of the sums
    int ntl = T.ntile;
    if (pflag) {
        if (threadIdx.x < 64) {
            int cnt = 0;
            for (int b = 0; b < T.ntile; b += 64) {
                const bool f = b + lane < T.ntile && tile_support(pflag, b + lane, npair);
                const unsigned long long msk = __ballot(f);
                if (f) tl_[cnt + __popcll(msk & ((1ull << lane) - 1))] = b + lane;
                cnt += __popcll(msk);
            }
            if (lane == 0) ntl_ = cnt;
        }
        __syncthreads();
        ntl = ntl_;
    }
    auto tile = [&](int i) __attribute__((always_inline)) {
        return pflag ? __builtin_amdgcn_readfirstlane(tl_[i]) : i;
    };
    Ph pf[PER];
    double gv[4][NG];
    const int t0 = ntl > 0 ? tile(0) : 0;
    Tw cur = twin(t0);
#pragma unroll
    for (int s = 0; s < 4; ++s) tload(cur, t0, s, gv);
    fetch(t0, pf);
    if (GS_MF_ADB) {
        if (ntl > 0) stage(pf, sp_);
        if (ntl > 1) fetch(tile(1), pf);
        __syncthreads();
    }
    // tile t: stage its phases, issue the next tile's phases, then t's MFMAs;
    // each slice's table registers are refilled with the next tile's values as
    // soon as its MFMAs are issued (their latency hides behind the rest of the
    // tile).  GS_MF_ADB: tile i's phases were staged during tile i - 1 (buffer
    // i & 1); tile i + 1's are staged now into the other buffer and tile i + 2's
    // loaded, and one barrier ends the tile (the staging visible, the buffer
    // read by every wave before it is written again)
    for (int i = 0; i < ntl; ++i) {
        const int t = tile(i);
        const bool more = i + 1 < ntl;
        const int tn = more ? tile(i + 1) : t;
        int bo = 0;
        if (GS_MF_ADB) {
            bo = (i & 1) * (MF_TILE * RW);
            if (more) stage(pf, sp_ + (MF_TILE * RW - bo));
            if (i + 2 < ntl) fetch(tile(i + 2), pf);
        } else {
            __syncthreads();
            stage(pf, sp_);
            __syncthreads();
            if (more) fetch(tn, pf);
        }
        const double* so = spo + bo;
        const double* sr = spr + bo;
        const Tw nxt = twin(tn);
        // A operands of slice s (a1 / a2 per parity and column group), read one
        // slice ahead of their MFMAs; every load unconditional, only the MFMAs
        // under the wave-uniform window test (see the synthesis)
        double aq[2][2][CPW][NF];
        auto ldsA = [&](int s, double (&a)[2][CPW][NF]) __attribute__((always_inline)) {
#pragma unroll
            for (int p = 0; p < 2; ++p)
#pragma unroll
                for (int c = 0; c < CPW; ++c) {
                    if constexpr (SPIN == 2) {
                        a[p][c][0] = so[s * 4 * RW + p * MPW * HV + c * 4 * HV];           // (N +- S)[o]
                        a[p][c][1] = sr[s * 4 * RW + (1 - p) * MPW * HV + c * 4 * HV];     // (N -+ S)[3 - o]
                    } else {
                        a[p][c][0] = so[s * 4 * RW + p * MPW * HV + c * 8 * HV];
                    }
                }
        };
        ldsA(0, aq[0]);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            if (s + 1 < 4) ldsA(s + 1, aq[(s + 1) & 1]);
            __builtin_amdgcn_sched_barrier(0);
            if (cur.any) {
                mf_prio_hi();
#pragma unroll
                for (int p = 0; p < 2; ++p) {
                    double gz[NF];
                    if constexpr (SPIN == 2) {
                        // F1 / F2 at (l = lw + 2 j + p, pair 16 t + 4 s + g): the VALU
                        // kernels' expressions on the table's lambda_l, lambda_{l-1}
                        const double w0 = gv[s][p];
                        const double w1 = p ? gv[s][0] : (((j & 7) || cur.prv) ? gv[s][2] : 0.0);
                        const double is2 = gv[s][4], xis2 = gv[s][3] * is2;
                        const double f1 = fma(cR[p] * xis2, w1, -fma(cP[p], is2, cQ[p]) * w0);
                        const double f2 = fma(cRm[p] * is2, w1, -(cT[p] * xis2) * w0);
                        gz[0] = cur.okb ? f1 : 0.0;
                        gz[1] = cur.okb ? f2 : 0.0;
                    } else {
                        gz[0] = cur.okb ? gv[s][p] : 0.0;
                    }
#pragma unroll
                    for (int c = 0; c < CPW; ++c) {
                        if (c >= ncl) continue;     // (a column group without maps: no MFMAs)
                        // F1 takes the parity-p combination (p = 0: +, 1: -), F2 the other
                        if constexpr (SPIN == 2) {
                            C[c][p] = mfma64(aq[s & 1][p][c][0], gz[0], C[c][p]);
                            C[c][p] = mfma64(s2 * aq[s & 1][p][c][1], gz[1], C[c][p]);
                        } else {
                            C[c][p] = mfma64(aq[s & 1][p][c][0], gz[0], C[c][p]);
                        }
                    }
                }
                mf_prio_lo();
            }
            __builtin_amdgcn_sched_barrier(0);
            tload(nxt, tn, s, gv);                  // (the last tile reloads its own: harmless)
            __builtin_amdgcn_sched_barrier(0);
        }
        cur = nxt;
        if (GS_MF_ADB) __syncthreads();
    }
    if (!live) return;
    // D layout: lane (g, j) holds rows g + 4 r = col index, col j = l index:
    // spin 2: map 4 c + r, part g (E re, E im, B re, B im); spin 0: map 8 c +
    // (g + 4 r) / 2, part (g + 4 r) % 2
    const double f = SPIN == 2 ? -w : w;
    constexpr double SQ2 = 1.41421356237309504880;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const int l = lw + 2 * j + p;
        if (l > L) continue;
        const long long ic = cidx(L, l, m);
#pragma unroll
        for (int c = 0; c < CPW; ++c) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = g + 4 * r;
                const int map = SPIN == 2 ? c0 + (cg0 + c) * 4 + r : c0 + (cg0 + c) * 8 + row / 2;
                const int comp = SPIN == 2 ? cbase + (g >> 1) : cbase;
                const int part = SPIN == 2 ? (g & 1) : (row & 1);
                if (map >= nmap) continue;
                const double v = f * C[c][p][r];
                double* out = alm + ((long long)map * ncm + comp) * alm_comp_stride(layout, L);
                if (layout == GS_ALM_COMPLEX) {
                    double* d = out + 2 * ic + part;
                    *d = acc ? *d + v : v;
                } else if (m == 0) {
                    if (part == 0) { double* d = out + l; *d = acc ? *d + v : v; }
                } else {
                    double* d = out + 2 * ic - (L + 1) + part;
                    *d = acc ? *d + SQ2 * v : SQ2 * v;
                }
            }
        }
    }
}

inline unsigned nblocks(long long n, int bs) { return (unsigned)std::max<long long>(1, (n + bs - 1) / bs); }
inline hipStream_t S(void* s) { return (hipStream_t)s; }

}  // namespace

// ============================================================================
// plan
// ============================================================================
struct gs_sht {
    int nside = 0, L = 0, npair = 0, ngroup = 0, nlm = 0, ntile = 0, Mmax = 0;
    // Legendre launch shapes chosen for occupancy (~4 waves per SIMD): ring
    // pairs per lane (sr) and m pairing, synthesis and analysis
    int syn_sr = 2, syn_paired = 1, ana_sr = 4, ana_paired = 1;
    // l-segments (0: none): the state table's granularity seg, and per launch
    // kind the segment length (a multiple of seg) -- synthesis, and analysis
    // per ncomp with its own ring groups per lane (index ncomp)
    int seg = 0;
    int syn_seg = 0;
    int ana_sr_nc[4] = {4, 4, 4, 4}, ana_seg_nc[4] = {0, 0, 0, 0};
    int* segoff = nullptr;
    double2* sst = nullptr;
    int* sstk = nullptr;
    long long npix = 0;
    PairGeom* geom = nullptr;
    LegCoef* coef = nullptr;
    AnaCoef* acoef = nullptr;    // [nlm + 4] the analysis' form (AnaCoef)
    double* acq = nullptr;       // [L + 1] Q_l
    int* lstart = nullptr;
    double2* st = nullptr;
    int* stk = nullptr;
    double2* tw = nullptr;
    double2* bsk = nullptr;
    double2* phi = nullptr;      // [3][2] planes of phi_plane(L, npair) (phi_at)
    double2* part = nullptr;     // [ntile][3][nlm]
    double2* gscr = nullptr;     // global FFT scratch for M > LDS_FFT_MAX
    double2* sscr = nullptr;     // split rings: [comp][slot][split_n] half-transform scratch
    int nsplit = 0, split_n = 0;
    int lds_fft_max = LDS_FFT_MAX;   // FFT lengths held in LDS (GS_SHT_LDS_FFT_MAX lowers it: tests)
    int ring_tw2 = 0;                // GS_SHT_RING_TW2=1: the two-level twiddle tables for every LDS ring class (tests)
    double* mapw = nullptr;      // [cap][3][npix] Jacobi residual maps
    double2* ain = nullptr;      // [cap][3][nlm] a_lm in healpy complex order
    int cap = 1;                 // maps of a batch the per-map workspace (phi, part, ain, mapw) holds
    // batched small maps: the Legendre stage on the fp64 matrix cores from a
    // plan-time table (gs_sht_set_mfma); mf = 1 routes every transform of the
    // plan (any batch size: results do not depend on it) through it
    int mf = 0;
    double* mf_tab = nullptr;
    long long* mf_off = nullptr;
    int* mf_b0 = nullptr;
    int mf_ntile = 0;
    long long mf_bytes = 0;
    long long mf_nblk = 0;
    MfTab mftab() const { return MfTab{mf_tab, mf_off, mf_b0, mf_ntile, mf_nblk}; }
    // ring classes by FFT length
    std::vector<int> cls_M;      // M of each class
    std::vector<int> cls_n;      // pairs in the class
    std::vector<int*> cls_pairs; // device lists
    // small maps: every ring pair in ONE ring-stage launch (FFT lengths up to
    // merged_M, all in LDS; largest rings first) instead of one latency-bound
    // launch per length class; 0 pairs = per-class launches
    int* merged_pairs = nullptr;
    int merged_n = 0, merged_M = 0;
    // ring-pair support of the current weighted analysis (k_pair_support)
    int* support = nullptr;
    // registered weights (gs_sht_register_weights): their pair classes (k_ring_classes)
    // and per-(pair, row) ring constants, computed once and reused by every
    // weighted transform given the same pointer
    const double* wreg = nullptr;
    int wreg_nc = 0;
    int* wsup = nullptr;
    double2* wconst = nullptr;
    // the short-ring classes run on a side stream beside the largest class
    // (fork / join by events, graph-capturable); 0 = all on the caller's stream
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    long long bytes = 0;
    ShtDev dev() const {
        ShtDev D;
        D.L = L; D.npair = npair; D.ngroup = ngroup; D.nlm = nlm;
        D.geom = geom; D.coef = coef; D.lstart = lstart; D.st = st; D.stk = stk;
        D.seg = seg; D.segmul = 1; D.segoff = segoff; D.sst = sst; D.sstk = sstk;
        return D;
    }
    // a launch whose segments are sl l long (a multiple of the table's seg)
    ShtDev devseg(int sl) const {
        ShtDev D = dev();
        D.seg = sl;
        D.segmul = (seg > 0 && sl > 0) ? sl / seg : 1;
        return D;
    }
};

namespace {

template <typename T>
int sht_alloc(gs_sht* p, T** dst, size_t n) {
    GS_CHECK(hipMalloc((void**)dst, std::max<size_t>(n, 1) * sizeof(T)));
    p->bytes += (long long)(std::max<size_t>(n, 1) * sizeof(T));
    return 0;
}

void sht_free(gs_sht* p) {
    void* bufs[] = {p->geom, p->coef, p->acoef, p->acq, p->lstart, p->st, p->stk, p->tw, p->bsk, p->phi, p->part, p->gscr, p->sscr,
                    p->mapw, p->ain, p->segoff, p->sst, p->sstk, p->merged_pairs, p->mf_tab, p->mf_off, p->mf_b0, p->support,
                    p->wsup, p->wconst};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    for (int* b : p->cls_pairs)
        if (b) (void)hipFree(b);
    if (p->ev_fork) (void)hipEventDestroy(p->ev_fork);
    if (p->ev_join) (void)hipEventDestroy(p->ev_join);
    if (p->side) (void)hipStreamDestroy(p->side);
    delete p;
}

int check_sht(const gs_sht* p) { return p ? 0 : set_error("null SHT plan"); }

int ilog2(int v) { int r = 0; while ((1 << r) < v) ++r; return r; }

}  // namespace

extern "C" {

int gs_sht_create(int nside, int lmax, gs_sht** out) {
    if (!out) return set_error("gs_sht_create: null out");
    *out = nullptr;
    if (nside < 1 || nside > 8192 || (nside & (nside - 1))) return set_error("gs_sht_create: nside must be a power of two <= 8192");
    if (lmax < 0 || lmax > 4 * nside) return set_error("gs_sht_create: lmax out of range (0..4 nside)");
    gs_sht* p = new gs_sht();
    if (const char* e = gs_detail::option("GS_SHT_RING_TW2")) p->ring_tw2 = std::atoi(e) != 0;
    if (const char* e = gs_detail::option("GS_SHT_LDS_FFT_MAX")) {
        const int v = std::atoi(e);
        if (v >= 16 && v <= LDS_FFT_MAX && (v & (v - 1)) == 0) p->lds_fft_max = v;
    }
    const int N = nside, L = lmax;
    p->nside = N; p->L = L; p->npair = 2 * N; p->ngroup = (p->npair + 63) / 64;
    p->nlm = (L + 1) * (L + 2) / 2;
    p->npix = 12LL * N * N;
    {
        // the largest ring count per lane (and m pairing) that still gives ~4 waves
        // per SIMD (1024 SIMDs); small maps fall back to one ring group per lane and
        // unpaired m.  GS_SHT_SYN / GS_SHT_ANA = "sr,paired" override (tests)
        auto waves = [&](int sr, int paired) {
            return (long long)(paired ? L / 2 + 1 : L + 1) * ((p->ngroup + sr - 1) / sr);
        };
        auto pick = [&](std::initializer_list<std::pair<int, int>> opts, const char* env, int& sr, int& paired) {
            sr = 1; paired = 0;
            for (auto o : opts)
                if (waves(o.first, o.second) >= 4096) { sr = o.first; paired = o.second; break; }
            if (const char* e = gs_detail::option(env)) {
                int a = 0, b = 0;
                if (std::sscanf(e, "%d,%d", &a, &b) == 2) { sr = a; paired = b ? 1 : 0; }
            }
        };
        pick({{2, 1}, {1, 1}, {1, 0}}, "GS_SHT_SYN", p->syn_sr, p->syn_paired);
        pick({{4, 1}, {2, 1}, {1, 1}, {1, 0}}, "GS_SHT_ANA", p->ana_sr, p->ana_paired);
        if ((p->syn_sr != 1 && p->syn_sr != 2 && p->syn_sr != 4) || (p->ana_sr != 1 && p->ana_sr != 2 && p->ana_sr != 4)) {
            delete p;
            return set_error("gs_sht_create: bad GS_SHT_SYN / GS_SHT_ANA override");
        }
    }
    // small maps (one ring group per lane, unpaired m: still few waves per SIMD,
    // each walking up to L + 1 recurrence steps in a latency-bound chain): split
    // every m's l range into segments entered with a plan-time recurrence state
    // -- independent waves with short chains.  Default: synthesis and TEB
    // analysis in 64-l segments with one ring group per lane; T and spin-2
    // analysis in 32-l segments with two ring groups per lane (half the
    // per-chunk wave reductions per ring pair; N_side 256 spin-2 map2alm 0.176 ->
    // 0.162 ms, TEB slower so it keeps the first shape), all from one table at
    // 32-l granularity.  GS_SHT_SEG (0 = off) / GS_SHT_ANA set one segment length
    // and one analysis shape for every launch (tests)
    {
        const char* e = gs_detail::option("GS_SHT_SEG");
        const bool small = p->ana_sr == 1 && !p->ana_paired;
        int sg = small ? 64 : 0;
        if (e) sg = std::atoi(e);
        if (sg < 0 || (sg & 1) || (sg > 0 && sg % ANA_C != 0)) {
            delete p;
            return set_error("gs_sht_create: GS_SHT_SEG must be 0 or a positive multiple of 4");
        }
        p->seg = sg >= L + 1 ? 0 : sg;
        p->syn_seg = p->seg;
        for (int nc = 1; nc <= 3; ++nc) { p->ana_sr_nc[nc] = p->ana_sr; p->ana_seg_nc[nc] = p->seg; }
        if (small && !e && !gs_detail::option("GS_SHT_ANA") && p->seg == 64) {
            p->seg = 32;
            for (int nc = 1; nc <= 2; ++nc) { p->ana_sr_nc[nc] = 2; p->ana_seg_nc[nc] = 32; }
        }
    }
    p->ntile = 0;
    for (int nc = 1; nc <= 3; ++nc)
        p->ntile = std::max(p->ntile, (p->ngroup + 4 * p->ana_sr_nc[nc] - 1) / (4 * p->ana_sr_nc[nc]));
    // ---- geometry (ring pair r: north ring r+1, south ring 4N-1-r) ----
    std::vector<PairGeom> geom(p->npair);
    int Mmax = 2;
    for (int r = 0; r < p->npair; ++r) {
        const int i = r + 1;
        PairGeom g{};
        if (i < N) {
            const double omx = (double)i * i / (3.0 * N * N);   // 1 - x, exact-ish
            g.x = 1.0 - omx;
            const double s2 = omx * (2.0 - omx);
            g.s = std::sqrt(s2);
            g.is2 = 1.0 / s2;
            g.nphi = 4 * i;
            g.phi_half = 1;
            g.startN = 2LL * i * (i - 1);
            g.startS = p->npix - 2LL * i * (i + 1);
        } else {
            g.x = 4.0 / 3.0 - 2.0 * i / (3.0 * N);
            const double s2 = (1.0 - g.x) * (1.0 + g.x);
            g.s = std::sqrt(s2);
            g.is2 = 1.0 / s2;
            g.nphi = 4 * N;
            g.phi_half = ((i - N) % 2 == 0) ? 1 : 0;
            g.startN = 2LL * N * (N - 1) + (long long)(i - N) * 4 * N;
            const int is = 4 * N - i;   // mirrored ring (same as i at the equator)
            g.startS = (is == i) ? -1 : 2LL * N * (N - 1) + (long long)(is - N) * 4 * N;
        }
        const bool pow2 = (g.nphi & (g.nphi - 1)) == 0;
        g.M = pow2 ? g.nphi : (1 << ilog2(2 * g.nphi - 1));
        g.split = 0;
        g.sslot = -1;
        if (!pow2 && g.M > p->lds_fft_max && g.nphi % 2 == 0) {
            const int Mh = 1 << ilog2(g.nphi - 1);          // Bluestein length for nphi / 2
            if (Mh <= p->lds_fft_max && Mh >= g.nphi) { g.M = Mh; g.split = 1; }
        }
        g.logM = ilog2(g.M);
        g.bs_off = -1;
        Mmax = std::max(Mmax, g.M);
        geom[r] = g;
    }
    long long bs_total = 0;
    std::vector<int> bs_pairs;
    for (int r = 0; r < p->npair; ++r) {
        if (geom[r].M != geom[r].nphi) {          // kernel V (M) then the chirp (the transform's length)
            geom[r].bs_off = bs_total;
            bs_total += geom[r].M + (geom[r].split ? geom[r].nphi / 2 : geom[r].nphi);
            bs_pairs.push_back(r);
        }
        if (geom[r].split) geom[r].sslot = p->nsplit++;
    }
    p->Mmax = Mmax;
    // ---- recurrence coefficients ----
    std::vector<LegCoef> coef(p->nlm);
    for (int m = 0; m <= L; ++m) {
        const long long base = (long long)m * (2 * L + 1 - m) / 2;
        for (int l = m; l <= L; ++l) {
            LegCoef c{};
            const double dl = l, dm = m;
            if (l > m) {
                c.a = std::sqrt((4.0 * dl * dl - 1.0) / (dl * dl - dm * dm));
                c.b = std::sqrt(((dl - 1.0) * (dl - 1.0) - dm * dm) / (4.0 * (dl - 1.0) * (dl - 1.0) - 1.0));
            }
            if (l >= 2) {
                const double cl = 2.0 / std::sqrt((dl - 1.0) * dl * (dl + 1.0) * (dl + 2.0));
                const double f = std::sqrt((2.0 * dl + 1.0) / (2.0 * dl - 1.0) * (dl * dl - dm * dm));
                c.P = cl * (dl - dm * dm);
                c.Q = cl * 0.5 * dl * (dl - 1.0);
                c.R = cl * f;
                c.T = cl * dm * (dl - 1.0);
                c.Rm = cl * dm * f;
            }
            coef[base + l] = c;
        }
    }
    std::vector<AnaCoef> acoef(p->nlm + 4, AnaCoef{});
    std::vector<double> acq(L + 1, 0.0);
    for (int l = 2; l <= L; ++l) acq[l] = coef[l].Q;          // m = 0 row: Q depends on l only
    for (int m = 0; m <= L; ++m) {
        const long long base = (long long)m * (2 * L + 1 - m) / 2;
        for (int l = m; l <= L; ++l) {
            const LegCoef& c = coef[base + l];
            AnaCoef& e = acoef[base + l];
            if (l < L) { e.a1 = coef[base + l + 1].a; e.b1 = coef[base + l + 1].b; }
            if (l >= 2) { e.P = c.P / c.Q; e.R = c.R / c.Q; e.T = c.T / c.Q; e.Rm = c.Rm / c.Q; }
        }
    }
    int rc = 0;
    rc |= sht_alloc(p, &p->geom, geom.size());
    rc |= sht_alloc(p, &p->coef, coef.size() + 1);   // + one zero entry past (L, L)
    rc |= sht_alloc(p, &p->acoef, acoef.size());
    rc |= sht_alloc(p, &p->acq, acq.size());
    rc |= sht_alloc(p, &p->lstart, (size_t)(L + 1) * p->ngroup);
    rc |= sht_alloc(p, &p->st, (size_t)(L + 1) * p->npair);
    rc |= sht_alloc(p, &p->stk, (size_t)(L + 1) * p->npair);
    rc |= sht_alloc(p, &p->tw, (size_t)Mmax / 2);
    rc |= sht_alloc(p, &p->bsk, (size_t)std::max<long long>(bs_total, 1));
    rc |= sht_alloc(p, &p->phi, (size_t)3 * 2 * phi_plane(L, p->npair));
    rc |= sht_alloc(p, &p->part, (size_t)p->ntile * 4 * 3 * p->nlm);   // one partial per analysis wave
    rc |= sht_alloc(p, &p->mapw, (size_t)3 * p->npix);
    rc |= sht_alloc(p, &p->ain, (size_t)3 * p->nlm);
    std::vector<int> segoff(L + 1, 0);
    long long segrows = 0;
    if (p->seg) {
        for (int m = 0; m <= L; ++m) {
            segoff[m] = (int)segrows;
            segrows += (L - m) / p->seg;                // segments s >= 1 of m: m + s seg <= L
        }
        rc |= sht_alloc(p, &p->segoff, (size_t)L + 1);
        rc |= sht_alloc(p, &p->sst, (size_t)std::max<long long>(segrows, 1) * p->npair);
        rc |= sht_alloc(p, &p->sstk, (size_t)std::max<long long>(segrows, 1) * p->npair);
    }
    if (rc) { sht_free(p); return -1; }
    if (p->seg && hipMemcpy(p->segoff, segoff.data(), segoff.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess) {
        sht_free(p);
        return set_error("gs_sht_create: segment table upload failed");
    }
    // ring classes by M
    std::vector<int> Ms;
    for (auto& g : geom) Ms.push_back(g.M);
    std::sort(Ms.begin(), Ms.end());
    Ms.erase(std::unique(Ms.begin(), Ms.end()), Ms.end());
    long long gscr_need = 0;
    for (int M : Ms) {
        std::vector<int> lst;
        for (int r = 0; r < p->npair; ++r)
            if (geom[r].M == M) lst.push_back(r);
        int* d = nullptr;
        if (hipMalloc((void**)&d, lst.size() * sizeof(int)) != hipSuccess ||
            hipMemcpy(d, lst.data(), lst.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess) {
            sht_free(p);
            return set_error("gs_sht_create: ring class upload failed");
        }
        p->cls_M.push_back(M);
        p->cls_n.push_back((int)lst.size());
        p->cls_pairs.push_back(d);
        if (M > p->lds_fft_max) gscr_need = std::max<long long>(gscr_need, 3LL * (long long)lst.size() * Mmax);
    }
    if (gscr_need && sht_alloc(p, &p->gscr, (size_t)gscr_need)) { sht_free(p); return -1; }
    {
        // one merged ring launch when every length fits a small LDS buffer
        // (GS_SHT_MERGE_RINGS=0/1 forces it off/on where legal).  Up to M = 4096
        // (N_side 512: two components of the longest Bluestein FFT fill the
        // 160-KB LDS): measured at N_side 512, 32 spin-2 maps, alm2map 9.95 ->
        // 9.11 ms, map2alm 10.66 -> 9.64 ms, and the f2 block maps take the
        // constant-ring (Parseval) route only here: masked ASIS 2702 -> 1613 ms
        // per 32-chain step (profiles/r06o_*)
        const int mmax = Ms.empty() ? 0 : Ms.back();
        bool merge = mmax <= 4096 && mmax <= p->lds_fft_max && p->nsplit == 0;
        if (const char* e = gs_detail::option("GS_SHT_MERGE_RINGS")) merge = std::atoi(e) != 0 && mmax <= p->lds_fft_max && p->nsplit == 0;
        if (merge && Ms.size() > 1) {
            std::vector<int> all(p->npair);
            for (int r = 0; r < p->npair; ++r) all[r] = r;
            std::stable_sort(all.begin(), all.end(), [&](int a, int b) { return geom[a].M > geom[b].M; });
            if (sht_alloc(p, &p->merged_pairs, all.size()) ||
                hipMemcpy(p->merged_pairs, all.data(), all.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess) {
                sht_free(p);
                return set_error("gs_sht_create: merged ring list upload failed");
            }
            p->merged_n = p->npair;
            p->merged_M = mmax;
        }
    }
    if (sht_alloc(p, &p->support, (size_t)p->npair)) { sht_free(p); return -1; }
    if (p->nsplit) {
        int nmax = 0;
        for (auto& g : geom) if (g.split) nmax = std::max(nmax, g.nphi);
        if (sht_alloc(p, &p->sscr, (size_t)3 * p->nsplit * nmax)) { sht_free(p); return -1; }
        p->split_n = nmax;
    }
    if (hipMemcpy(p->geom, geom.data(), geom.size() * sizeof(PairGeom), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(p->coef, coef.data(), coef.size() * sizeof(LegCoef), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(p->coef + coef.size(), 0, sizeof(LegCoef)) != hipSuccess ||
        hipMemcpy(p->acoef, acoef.data(), acoef.size() * sizeof(AnaCoef), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(p->acq, acq.data(), acq.size() * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) {
        sht_free(p);
        return set_error("gs_sht_create: table upload failed");
    }
    // ---- device-side tables ----
    double* lmm = nullptr;
    int* lmk = nullptr;
    if (hipMalloc((void**)&lmm, (size_t)(L + 1) * p->npair * sizeof(double)) != hipSuccess ||
        hipMalloc((void**)&lmk, (size_t)(L + 1) * p->npair * sizeof(int)) != hipSuccess) {
        if (lmm) (void)hipFree(lmm);
        sht_free(p);
        return set_error("gs_sht_create: out of device memory");
    }
    {
        const void* fns[] = {(const void*)k_sht_synth_ring<4>, (const void*)k_sht_synth_ring<8>,
                             (const void*)k_sht_synth_ring<4, PixAux>, (const void*)k_sht_synth_ring<8, PixAux>,
                             (const void*)k_sht_anal_ring<4>, (const void*)k_sht_anal_ring<8>};
        for (const void* f : fns)
            (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (std::max(LDS_FFT_MAX + 64 * 4, LDS_FFT_MAX + Mmax / 64 + 64) +
                                       ring_ph_entries(LDS_FFT_MAX)) * (int)sizeof(double2));
        const void* mc[] = {(const void*)k_sht_synth_ring_mc<8>, (const void*)k_sht_anal_ring_mc<8>,
                            (const void*)k_sht_apply_ring_mc<8, PixWeights>, (const void*)k_sht_apply_ring_mc<8, PixAux>,
                            (const void*)k_sht_parseval_ring_mc<8>};
        for (const void* f : mc)
            (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, RING_MC_LDS_MAX);
        (void)hipGetLastError();
    }
    hipLaunchKernelGGL(k_sht_twiddles, dim3(nblocks(Mmax / 2, 256)), dim3(256), 0, 0, Mmax, p->tw);
    hipLaunchKernelGGL(k_sht_lmm, dim3(nblocks(p->npair, 64)), dim3(64), 0, 0, L, p->npair, p->geom, lmm, lmk);
    hipLaunchKernelGGL(k_sht_onset, dim3(nblocks(p->npair, 256), L + 1), dim3(256), 0, 0, p->dev(), lmm, lmk,
                       p->lstart, p->st, p->stk);
    if (p->seg)
        hipLaunchKernelGGL(k_sht_segstate, dim3(nblocks(p->npair, 256), L + 1), dim3(256), 0, 0, p->dev());
    if (!bs_pairs.empty()) {
        int* dp = nullptr;
        if (hipMalloc((void**)&dp, bs_pairs.size() * sizeof(int)) == hipSuccess &&
            hipMemcpy(dp, bs_pairs.data(), bs_pairs.size() * sizeof(int), hipMemcpyHostToDevice) == hipSuccess) {
            hipLaunchKernelGGL(k_sht_bluestein_setup, dim3((unsigned)bs_pairs.size()), dim3(1024), 0, 0, dp,
                               p->geom, p->tw, Mmax, p->bsk);
        }
        (void)hipDeviceSynchronize();
        if (dp) (void)hipFree(dp);
    }
    const hipError_t e = hipDeviceSynchronize();
    (void)hipFree(lmm);
    (void)hipFree(lmk);
    if (e != hipSuccess || hipGetLastError() != hipSuccess) {
        sht_free(p);
        return set_error(std::string("gs_sht_create: setup kernels failed: ") + hipGetErrorString(e));
    }
    if (hipStreamCreateWithFlags(&p->side, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&p->ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&p->ev_join, hipEventDisableTiming) != hipSuccess) {
        sht_free(p);
        return set_error("gs_sht_create: side stream / events");
    }
    *out = p;
    return 0;
}

int gs_sht_destroy(gs_sht* p) {
    if (p) sht_free(p);
    return 0;
}

int gs_sht_info(const gs_sht* p, int* nside, int* lmax, long long* npix, long long* device_bytes) {
    if (check_sht(p)) return -1;
    if (nside) *nside = p->nside;
    if (lmax) *lmax = p->L;
    if (npix) *npix = p->npix;
    if (device_bytes) *device_bytes = p->bytes;
    return 0;
}

// LDS of a ring launch (double2 entries): the FFT buffer (M; global scratch
// instead when glob), the fold reduction of short rings (4 per thread) aliasing
// it, then the twiddle table (M / 2) when the total stays within RING_LDS_TW_MAX
// (twoff >= 0); else, for an LDS buffer, the two-level tables of twid (Mmax / 64
// + 64 entries at -2 - twoff: M = 8192 rings no longer wait on a global
// twiddle load in every FFT pass); glob: the plan's global table (twoff = -1)
constexpr size_t RING_LDS_TW_MAX = 96 * 1024;
static void ring_lds(int M, int bd, bool glob, bool short_red, int Mmax, size_t& lds, int& twoff, int& phoff,
                     bool tw2 = false) {
    const long long red = short_red ? 4LL * bd : 0;
    const long long r0 = glob ? red : std::max<long long>(M, red);
    const long long with_tw = r0 + M / 2;
    if (!glob && !tw2 && (size_t)with_tw * sizeof(double2) <= RING_LDS_TW_MAX) {
        twoff = (int)r0;
        lds = (size_t)with_tw * sizeof(double2);
    } else if (!glob) {
        twoff = -2 - (int)r0;
        lds = (size_t)(r0 + Mmax / 64 + 64) * sizeof(double2);
    } else {
        twoff = -1;
        lds = (size_t)r0 * sizeof(double2);
    }
    // then the ring's phase tables (ring_phases)
    phoff = (int)(lds / sizeof(double2));
    lds += (size_t)ring_ph_entries(M) * sizeof(double2);
}

static int sht_ring_class(gs_sht* p, size_t c, bool synth, int ncomp, const double* maps_in, double* maps_out,
                          hipStream_t st, const double2* phi = nullptr, const int* comp_lmax = nullptr,
                          int comp_div = 1, const double* wts = nullptr, int wnc = 3,
                          const gs::GsAuxPix* aux = nullptr) {
    if (!phi) phi = p->phi;
    const int M = p->cls_M[c];
    const bool glob = M > p->lds_fft_max;
    const int bd = ring_block(M);
    const bool nb8 = M / 2 > 4 * bd;
    size_t lds = 0;
    int twoff = -1;
    int phoff = 0;
    ring_lds(M, bd, glob, M < 8 * bd, p->Mmax, lds, twoff, phoff, p->ring_tw2);
    const dim3 grid(p->cls_n[c], ncomp);
    double2* scr = glob ? p->gscr : nullptr;
    if (synth && aux) {
        // the aux-variable step on the pixels as they leave (PixAux)
        const PixAux op{*aux};
        if (nb8)
            hipLaunchKernelGGL((k_sht_synth_ring<8, PixAux>), grid, dim3(bd), lds, st, p->L, p->npair, p->npix,
                               p->cls_pairs[c], p->geom, phi, p->tw, p->Mmax, p->bsk, scr, maps_out, p->sscr, p->nsplit,
                               p->split_n, comp_lmax, comp_div, twoff, phoff, op);
        else
            hipLaunchKernelGGL((k_sht_synth_ring<4, PixAux>), grid, dim3(bd), lds, st, p->L, p->npair, p->npix,
                               p->cls_pairs[c], p->geom, phi, p->tw, p->Mmax, p->bsk, scr, maps_out, p->sscr, p->nsplit,
                               p->split_n, comp_lmax, comp_div, twoff, phoff, op);
    } else if (synth) {
        if (nb8)
            hipLaunchKernelGGL(k_sht_synth_ring<8>, grid, dim3(bd), lds, st, p->L, p->npair, p->npix, p->cls_pairs[c],
                               p->geom, phi, p->tw, p->Mmax, p->bsk, scr, maps_out, p->sscr, p->nsplit, p->split_n,
                               comp_lmax, comp_div, twoff, phoff, PixNone{});
        else
            hipLaunchKernelGGL(k_sht_synth_ring<4>, grid, dim3(bd), lds, st, p->L, p->npair, p->npix, p->cls_pairs[c],
                               p->geom, phi, p->tw, p->Mmax, p->bsk, scr, maps_out, p->sscr, p->nsplit, p->split_n,
                               comp_lmax, comp_div, twoff, phoff, PixNone{});
    } else {
        if (nb8)
            hipLaunchKernelGGL(k_sht_anal_ring<8>, grid, dim3(bd), lds, st, p->L, p->npair, p->npix, p->cls_pairs[c],
                               p->geom, maps_in, p->tw, p->Mmax, p->bsk, scr, p->phi, p->sscr, p->nsplit, p->split_n, twoff, phoff, wts, wnc);
        else
            hipLaunchKernelGGL(k_sht_anal_ring<4>, grid, dim3(bd), lds, st, p->L, p->npair, p->npix, p->cls_pairs[c],
                               p->geom, maps_in, p->tw, p->Mmax, p->bsk, scr, p->phi, p->sscr, p->nsplit, p->split_n, twoff, phoff, wts, wnc);
    }
    GS_LAUNCH_CHECK(synth ? "k_sht_synth_ring" : "k_sht_anal_ring");
    return 0;
}

// Ring stage: one launch per FFT-length class.  The classes touch disjoint
// rings (and disjoint scratch: split rings own their sscr slot, the one
// global-scratch class stays on the caller's stream), so the short-ring
// classes -- a dozen small, latency-bound launches -- run on the plan's side
// stream while the largest class runs on the caller's.
// ncomp = every comp of the batch (maps b * wnc + c, contiguous); wts: wnc weight
// maps shared by the batch's maps
// components per ring workgroup in the merged launch (GS_SHT_RING_NC, default
// 2 -- measured at N_side 256, 16 spin-2 maps: 1 / 2 / 4 = 401 / 326 / 358 us
// synthesis ring stage; 1 = one component per workgroup, the k_sht_*_ring kernels): bounded by
// the LDS (NCB buffers of the longest FFT + its twiddles) and by 1024 threads
// at ring_block(M) threads (<= 8 values each) per component
static int ring_mc_ncb(int M, int ncomp) {
    // (2, 3, 4 measured: 2 is the fastest for the operator, synthesis and analysis)
    int ncb = std::min(2, ncomp);
    ncb = std::min(ncb, 1024 / ring_block(M));
    const int SB = std::max(M, 4 * ring_block(M));
    while (ncb > 1 && (size_t)(ncb * SB + M / 2) * sizeof(double2) > (size_t)RING_MC_LDS_MAX) --ncb;
    return ncb;
}

static int sht_rings(gs_sht* p, bool synth, int ncomp, const double* maps_in, double* maps_out, void* stream,
                     const double2* phi = nullptr, const int* comp_lmax = nullptr, int comp_div = 1, const double* wts = nullptr,
                     int wnc = 3, const int* pflag = nullptr, const int* pconst = nullptr,
                     const gs::GsAuxPix* aux = nullptr) {
    if (aux && p->merged_n > 0) return set_error("sht_rings: the aux store runs on the per-class ring stage");
    if (p->merged_n > 0) {
        // all ring pairs in one launch: the block size and LDS of the longest FFT
        // (shorter rings leave threads idle; their fold reduction uses the
        // J = block / K aliases per bin pair, as a short-ring class does)
        const int M = p->merged_M, bd = ring_block(M);
        const double2* ph = phi ? phi : p->phi;
        const int ncb = ring_mc_ncb(M, ncomp);
        if (ncb > 1) {
            // ring_block(M) threads per component, as the one-component kernels (the
            // fold's alias split J, hence its summation order, is the same)
            // (a component's buffer also holds its fold reduction: 4 per thread)
            const int bdm = ncb * bd, SB = std::max(M, 4 * bd), toff = ncb * SB;
            const size_t ldsm = (size_t)(ncb * SB + M / 2) * sizeof(double2);
            const int ncg = (ncomp + ncb - 1) / ncb;
            const dim3 gm((unsigned)(8 * ((p->merged_n + 15) / 16) * 2 * ncg));
            if (synth)
                hipLaunchKernelGGL(k_sht_synth_ring_mc<8>, gm, dim3(bdm), ldsm, S(stream), p->L, p->npair, p->npix,
                                   p->merged_pairs, p->geom, ph, p->tw, p->Mmax, p->bsk, maps_out, ncomp, ncb, SB,
                                   toff, comp_lmax, comp_div, p->merged_n, pconst);
            else
                hipLaunchKernelGGL(k_sht_anal_ring_mc<8>, gm, dim3(bdm), ldsm, S(stream), p->L, p->npair, p->npix,
                                   p->merged_pairs, p->geom, maps_in, p->tw, p->Mmax, p->bsk, p->phi, ncomp, ncb, SB,
                                   toff, wts, wnc, p->merged_n, pflag);
            GS_LAUNCH_CHECK(synth ? "k_sht_synth_ring_mc" : "k_sht_anal_ring_mc");
            return 0;
        }
        if (pconst) return set_error("sht_rings: Parseval block maps need the multi-component ring stage");
        const bool nb8 = M / 2 > 4 * bd;
        size_t lds = 0;
        int twoff = -1;
        int phoff = 0;
        ring_lds(M, bd, false, true, p->Mmax, lds, twoff, phoff, p->ring_tw2);
        phoff = -1;                                 // as the multi-component kernels: direct sincospi
        const dim3 grid(p->merged_n, ncomp);
        if (synth) {
            if (nb8)
                hipLaunchKernelGGL(k_sht_synth_ring<8>, grid, dim3(bd), lds, S(stream), p->L, p->npair, p->npix,
                                   p->merged_pairs, p->geom, ph, p->tw, p->Mmax, p->bsk, nullptr, maps_out, p->sscr,
                                   p->nsplit, p->split_n, comp_lmax, comp_div, twoff, phoff, PixNone{});
            else
                hipLaunchKernelGGL(k_sht_synth_ring<4>, grid, dim3(bd), lds, S(stream), p->L, p->npair, p->npix,
                                   p->merged_pairs, p->geom, ph, p->tw, p->Mmax, p->bsk, nullptr, maps_out, p->sscr,
                                   p->nsplit, p->split_n, comp_lmax, comp_div, twoff, phoff, PixNone{});
        } else {
            if (nb8)
                hipLaunchKernelGGL(k_sht_anal_ring<8>, grid, dim3(bd), lds, S(stream), p->L, p->npair, p->npix,
                                   p->merged_pairs, p->geom, maps_in, p->tw, p->Mmax, p->bsk, nullptr, p->phi, p->sscr,
                                   p->nsplit, p->split_n, twoff, phoff, wts, wnc);
            else
                hipLaunchKernelGGL(k_sht_anal_ring<4>, grid, dim3(bd), lds, S(stream), p->L, p->npair, p->npix,
                                   p->merged_pairs, p->geom, maps_in, p->tw, p->Mmax, p->bsk, nullptr, p->phi, p->sscr,
                                   p->nsplit, p->split_n, twoff, phoff, wts, wnc);
        }
        GS_LAUNCH_CHECK(synth ? "k_sht_synth_ring (merged)" : "k_sht_anal_ring (merged)");
        return 0;
    }
    if (pconst) return set_error("sht_rings: Parseval block maps need the merged ring stage");
    const size_t ncls = p->cls_M.size();
    size_t big = 0;
    for (size_t c = 1; c < ncls; ++c)
        if ((long long)p->cls_n[c] * p->cls_M[c] > (long long)p->cls_n[big] * p->cls_M[big]) big = c;
    const bool fork = p->side && ncls > 1;
    if (fork) {
        GS_CHECK(hipEventRecord(p->ev_fork, S(stream)));
        GS_CHECK(hipStreamWaitEvent(p->side, p->ev_fork, 0));
    }
    for (size_t c = 0; c < ncls; ++c) {
        const bool on_side = fork && c != big && p->cls_M[c] <= p->lds_fft_max;
        if (sht_ring_class(p, c, synth, ncomp, maps_in, maps_out, on_side ? p->side : S(stream), phi, comp_lmax,
                           comp_div, wts, wnc, aux))
            return -1;
    }
    if (fork) {
        GS_CHECK(hipEventRecord(p->ev_join, p->side));
        GS_CHECK(hipStreamWaitEvent(S(stream), p->ev_join, 0));
    }
    return 0;
}

// ---- batches of maps (chains) ------------------------------------------------
// A batch of B maps shares the plan's tables; every Legendre / ring / finish
// launch carries the batch in its grid (Legendre: blockIdx.z; ring and finish:
// the comp index b * ncomp + c), so one launch serves all B maps and a small map
// (N_side <= 256: a fraction of the GPU per map) fills the chip.  A map's
// arithmetic does not depend on B: map b of a batch is bit-identical to the same
// map transformed alone.  Plans whose ring stage needs the global FFT scratch or
// split rings (large maps: N_side >= 1024) run a batch as B single-map passes --
// one map already fills the GPU there.
static bool sht_batch_native(const gs_sht* p) { return p->gscr == nullptr && p->nsplit == 0; }

// per-map workspace for B maps (grown outside a capture only)
static int sht_reserve(gs_sht* p, int nmap, hipStream_t st) {
    if (nmap <= p->cap) return 0;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
        return set_error("gs_sht: a batch larger than the plan's reserved maps inside a graph capture "
                         "(call gs_sht_reserve first)");
    GS_CHECK(hipDeviceSynchronize());
    double2 *phi = nullptr, *part = nullptr, *ain = nullptr;
    double* mapw = nullptr;
    const size_t n = (size_t)nmap;
    if (hipMalloc((void**)&phi, n * 3 * 2 * phi_plane(p->L, p->npair) * sizeof(double2)) != hipSuccess ||
        hipMalloc((void**)&part, n * p->ntile * 4 * 3 * p->nlm * sizeof(double2)) != hipSuccess ||
        hipMalloc((void**)&ain, n * 3 * p->nlm * sizeof(double2)) != hipSuccess ||
        hipMalloc((void**)&mapw, n * 3 * p->npix * sizeof(double)) != hipSuccess) {
        for (void* q : {(void*)phi, (void*)part, (void*)ain, (void*)mapw})
            if (q) (void)hipFree(q);
        return set_error("gs_sht_reserve: out of device memory");
    }
    (void)hipFree(p->phi); (void)hipFree(p->part); (void)hipFree(p->ain); (void)hipFree(p->mapw);
    const long long old = (long long)p->cap;
    p->bytes += (long long)(n - old) * (long long)(3 * 2 * phi_plane(p->L, p->npair) * 16 +
                                                    (long long)p->ntile * 4 * 3 * p->nlm * 16 + 3LL * p->nlm * 16 +
                                                    3LL * p->npix * 8);
    p->phi = phi; p->part = part; p->ain = ain; p->mapw = mapw;
    p->cap = nmap;
    return 0;
}

// ---- the matrix-core Legendre stage (plans with mf set) --------------------------
constexpr int MF_CGW = 4;         // 16-column groups per workgroup (16 maps spin 2, 32 spin 0)

// launch shapes: 4 column groups per wave in both table kernels and 256-thread
// analysis workgroups.  Measured (N_side 256, 16 spin-2 maps, rocprofv3
// averages, XCD-aware orders): synthesis CPW 4 / 2 = 550 / 598 us; analysis
// (CPW, NT) (4, 256) / (4, 512) / (2, 512) = 737 / 825 / 1040 us
constexpr int MFS_CPW = 4, MFA_CPW = 4, MFA_NT = 256;

extern "C++" {
template <int CPW, bool RIN>
static void sht_synth_mfma_r(gs_sht* p, int nmap, int ncomp, hipStream_t st, const int* pflag, const double* areal,
                             const double* bl) {
    const ShtDev D = p->dev();
    const MfTab T = p->mftab();
    const unsigned ty = (unsigned)((p->mf_ntile + 3) / 4);
    const dim3 blk(256 * (MF_CGW / CPW));
    // (GS_MF_SYN_XCD 1: 1-D over whole phase blocks)
    const int nmb = (p->L + 1 + PHI_MB - 1) / PHI_MB;
    const unsigned gx = GS_MF_SYN_XCD ? (unsigned)(((nmb + 7) / 8) * 8 * PHI_MB * ty) : ty;
    const unsigned gy = GS_MF_SYN_XCD ? 1u : (unsigned)(p->L + 1);
    if (ncomp != 2) {               // T (spin 0): comp 0
        const dim3 g(gx, gy, (unsigned)((nmap + 8 * MF_CGW - 1) / (8 * MF_CGW)));
        hipLaunchKernelGGL((k_sht_synth_mfma<0, MF_CGW, CPW, RIN>), g, blk, 0, st, D, T, p->ain, p->phi, nmap, ncomp,
                           0, pflag, areal, bl);
    }
    if (ncomp != 1) {               // E, B -> Q, U: comps ncomp - 2, ncomp - 1
        const dim3 g(gx, gy, (unsigned)((nmap + 4 * MF_CGW - 1) / (4 * MF_CGW)));
        hipLaunchKernelGGL((k_sht_synth_mfma<2, MF_CGW, CPW, RIN>), g, blk, 0, st, D, T, p->ain, p->phi, nmap, ncomp,
                           ncomp - 2, pflag, areal, bl);
    }
}

template <int CPW, int NT>
static void sht_anal_mfma_v(gs_sht* p, int nmap, int ncomp, int layout, int acc, double* alm, hipStream_t st,
                            const int* pflag) {
    const ShtDev D = p->dev();
    const MfTab T = p->mftab();
    const double w = 4.0 * PI / (double)p->npix;
    constexpr int WPG = NT / 64 / (MF_CGW / CPW);    // windows per workgroup
    const int nwin = (p->L + 1 + 31) / 32;           // 32-l windows of m = 0
    const int wgy = (nwin + WPG - 1) / WPG;
    const int nmb = (p->L + 1 + PHI_MB - 1) / PHI_MB;   // phase blocks of 4 m, dealt to 8 XCDs
    const unsigned nx = (unsigned)(((nmb + 7) / 8) * 8 * PHI_MB * wgy);
    if (ncomp != 2) {
        const dim3 g(nx, 1, (unsigned)((nmap + 8 * MF_CGW - 1) / (8 * MF_CGW)));
        hipLaunchKernelGGL((k_sht_anal_mfma<0, MF_CGW, CPW, NT>), g, dim3(NT), 0, st, D, T, p->phi, nmap, ncomp, 0, w,
                           layout, acc, alm, pflag);
    }
    if (ncomp != 1) {
        const dim3 g(nx, 1, (unsigned)((nmap + 4 * MF_CGW - 1) / (4 * MF_CGW)));
        hipLaunchKernelGGL((k_sht_anal_mfma<2, MF_CGW, CPW, NT>), g, dim3(NT), 0, st, D, T, p->phi, nmap, ncomp,
                           ncomp - 2, w, layout, acc, alm, pflag);
    }
}
}  // extern "C++"

// areal: the caller's real-layout a_lm (and beam bl) read by the kernel itself
// instead of the plan's ain (filled by k_sht_alm_in)
static int sht_synth_mfma(gs_sht* p, int nmap, int ncomp, hipStream_t st, const int* pflag = nullptr,
                          const double* areal = nullptr, const double* bl = nullptr) {
    if (areal) sht_synth_mfma_r<MFS_CPW, true>(p, nmap, ncomp, st, pflag, areal, bl);
    else sht_synth_mfma_r<MFS_CPW, false>(p, nmap, ncomp, st, pflag, nullptr, nullptr);
    GS_LAUNCH_CHECK("k_sht_synth_mfma");
    return 0;
}

static int sht_anal_mfma(gs_sht* p, int nmap, int ncomp, int layout, int acc, double* alm, hipStream_t st,
                         const int* pflag = nullptr) {
    sht_anal_mfma_v<MFA_CPW, MFA_NT>(p, nmap, ncomp, layout, acc, alm, st, pflag);
    GS_LAUNCH_CHECK("k_sht_anal_mfma");
    return 0;
}

// the ring-pair support flags of a weighted analysis on the table path, or
// nullptr: no skipping (more tiles than the analysis' list holds)
// (the registered weights' classes when wts is the registered array: computed
// once; otherwise k_pair_support for this call)
// *out = nullptr: no skipping.  A failed launch is an error (the sticky error
// is reported, not cleared).
static int sht_support(gs_sht* p, const double* wts, int wnc, hipStream_t st, const int** out) {
    *out = nullptr;
    const int nt = (p->npair + 15) / 16;
    if (!p->mf || !wts || nt > MF_TL_MAX || nt != p->mf_ntile) return 0;
    if (wts == p->wreg && wnc == p->wreg_nc && p->wsup) { *out = p->wsup; return 0; }
    hipLaunchKernelGGL(k_pair_support, dim3(p->npair), dim3(256), 0, st, p->npix, p->geom, wts, wnc, p->support);
    GS_LAUNCH_CHECK("k_pair_support");
    *out = p->support;
    return 0;
}

// the registered ring constants for these weights (nullptr: not registered, or
// the constant-ring forms turned off by GS_SHT_CONST_RINGS=0)
static bool const_rings_on() {                     // read per call: tests A/B it in one process
    const char* e = gs_detail::option("GS_SHT_CONST_RINGS");
    return !e || atoi(e) != 0;
}
static const double2* sht_wconst(const gs_sht* p, const double* wts, int wnc) {
    return const_rings_on() && wts && wts == p->wreg && wnc == p->wreg_nc ? p->wconst : nullptr;
}

// build (on = 1) or drop (0) the plan's Legendre tables
static int sht_set_mfma(gs_sht* p, int on) {
    if (!on) {
        p->mf = 0;
        return 0;
    }
    if (p->mf_tab) { p->mf = 1; return 0; }
    const int L = p->L, npair = p->npair;
    const int ntile = (npair + MF_TILE - 1) / MF_TILE;
    double* lmm = nullptr;
    int* lmk = nullptr;
    int* b0d = nullptr;
    auto fail = [&](const char* what) {
        if (lmm) (void)hipFree(lmm);
        if (lmk) (void)hipFree(lmk);
        if (b0d) (void)hipFree(b0d);
        return set_error(std::string("gs_sht_set_mfma: ") + what);
    };
    if (hipMalloc((void**)&lmm, (size_t)(L + 1) * npair * sizeof(double)) != hipSuccess ||
        hipMalloc((void**)&lmk, (size_t)(L + 1) * npair * sizeof(int)) != hipSuccess ||
        hipMalloc((void**)&b0d, (size_t)(L + 1) * ntile * sizeof(int)) != hipSuccess)
        return fail("out of device memory");
    hipLaunchKernelGGL(k_sht_lmm, dim3(nblocks(npair, 64)), dim3(64), 0, 0, L, npair, p->geom, lmm, lmk);
    hipLaunchKernelGGL(k_mf_onset, dim3(nblocks(npair, 256), L + 1), dim3(256), 0, 0, p->dev(), lmm, lmk, b0d);
    std::vector<int> b0((size_t)(L + 1) * ntile);
    if (hipMemcpy(b0.data(), b0d, b0.size() * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
        return fail("onset pass failed");
    std::vector<long long> off(b0.size());
    long long nblk = 0;
    for (int m = 0; m <= L; ++m) {
        const int nb = (L - m + MF_TILE) / MF_TILE;
        for (int t = 0; t < ntile; ++t) {
            const size_t i = (size_t)m * ntile + t;
            off[i] = nblk;
            nblk += std::max(0, nb - b0[i]);
        }
    }
    double* tab = nullptr;
    long long* offd = nullptr;
    if (hipMalloc((void**)&tab, (size_t)std::max(1LL, nblk) * MF_BLK * sizeof(double)) != hipSuccess)
        return fail("out of device memory (table)");
    if (hipMalloc((void**)&offd, off.size() * sizeof(long long)) != hipSuccess ||
        hipMemcpy(offd, off.data(), off.size() * sizeof(long long), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(tab);
        if (offd) (void)hipFree(offd);
        return fail("offset upload failed");
    }
    p->mf_tab = tab; p->mf_off = offd; p->mf_b0 = b0d; p->mf_ntile = ntile; p->mf_nblk = std::max(1LL, nblk);
    b0d = nullptr;
    hipLaunchKernelGGL(k_mf_fill, dim3(nblocks(npair, 256), L + 1), dim3(256), 0, 0, p->dev(), lmm, lmk, p->mftab());
    const hipError_t e = hipDeviceSynchronize();
    (void)hipFree(lmm);
    (void)hipFree(lmk);
    lmm = nullptr; lmk = nullptr;
    if (e != hipSuccess || hipGetLastError() != hipSuccess) return set_error("gs_sht_set_mfma: table fill failed");
    p->mf_bytes = nblk * MF_BLK * (long long)sizeof(double) + (long long)off.size() * 12;
    p->bytes += p->mf_bytes;
    p->mf = 1;
    return 0;
}

// synthesis of B maps (alm [B][ncomp][n], maps [B][ncomp][Npix]); bl (real layout
// only): the per-l beam applied on the input load
static int sht_alm2map(gs_sht* p, int nmap, int ncomp, int layout, const double* alm, const double* bl, double* maps,
                       void* stream, const gs::GsAuxPix* aux = nullptr) {
    if (check_sht(p)) return -1;
    if (ncomp < 1 || ncomp > 3) return set_error("gs_sht_alm2map: ncomp must be 1 (T), 2 (E,B) or 3 (T,E,B)");
    if (layout != GS_ALM_REAL && layout != GS_ALM_COMPLEX) return set_error("gs_sht_alm2map: bad layout");
    if (bl && layout != GS_ALM_REAL) return set_error("gs_sht_alm2map: the beamed input needs the real layout");
    if (!alm || !maps) return set_error("gs_sht_alm2map: null argument");
    if (nmap < 1) return set_error("gs_sht_alm2map: nmap < 1");
    if (nmap > 1 && !sht_batch_native(p)) {
        const long long as = ncomp * alm_comp_stride(layout, p->L), ms = (long long)ncomp * p->npix;
        for (int b = 0; b < nmap; ++b)
            if (sht_alm2map(p, 1, ncomp, layout, alm + b * as, bl, maps + b * ms, stream)) return -1;
        return 0;
    }
    if (sht_reserve(p, nmap, S(stream))) return -1;
    if (aux && (p->mf || p->merged_n > 0 || nmap > 1))
        return set_error("gs_sht_alm2map: the aux store is for one map on the per-class ring stage");
    if (p->mf && layout == GS_ALM_REAL) {
        // the table kernel reads the real layout (and the beam) itself
        if (sht_synth_mfma(p, nmap, ncomp, S(stream), nullptr, alm, bl)) return -1;
        return sht_rings(p, true, nmap * ncomp, nullptr, maps, stream, nullptr, nullptr, 1, nullptr, ncomp);
    }
    const long long nin = (long long)nmap * ncomp * p->nlm;
    // the batch's comps are contiguous: the input pass sees B * ncomp comps
    // (the on-the-fly synthesis takes the spin-2 a_lm scaled by Q_l: AnaCoef)
    hipLaunchKernelGGL(k_sht_alm_in, dim3(nblocks(nin, 256)), dim3(256), 0, S(stream), p->L, p->nlm, nmap * ncomp, alm,
                       layout, p->ain, bl, ncomp, p->mf ? nullptr : p->acq);
    GS_LAUNCH_CHECK("k_sht_alm_in");
    if (p->mf) {
        if (sht_synth_mfma(p, nmap, ncomp, S(stream))) return -1;
        return sht_rings(p, true, nmap * ncomp, nullptr, maps, stream, nullptr, nullptr, 1, nullptr, ncomp);
    }
    const int syn_nseg = p->syn_seg ? (p->L + p->syn_seg) / p->syn_seg : 1;
    if (p->syn_seg > 0 && p->syn_seg <= 64 && p->syn_sr == 1 && !p->syn_paired && syn_nseg <= 16) {
        // small maps: l-segmented synthesis, one wave per segment (<= 64 l: the
        // wave's LDS slice stages 64 l of coefficients and a_lm)
        const dim3 g2(p->L + 1, p->ngroup, nmap), b2(64 * syn_nseg);
        const size_t lds = (size_t)syn_nseg * (66 * 8 + 3 * 64 * 2) * sizeof(double);
#define GS_SS(NC) hipLaunchKernelGGL((k_sht_synth_leg_seg<NC>), g2, b2, lds, S(stream), p->devseg(p->syn_seg), p->acoef, \
                                     p->ain, p->phi)
        if (ncomp == 1) GS_SS(1); else if (ncomp == 2) GS_SS(2); else GS_SS(3);
#undef GS_SS
        GS_LAUNCH_CHECK("k_sht_synth_leg_seg");
        return sht_rings(p, true, nmap * ncomp, nullptr, maps, stream, nullptr, nullptr, 1, nullptr, ncomp, nullptr,
                         nullptr, aux);
    }
    const dim3 grid(p->syn_paired ? p->L / 2 + 1 : p->L + 1, (p->ngroup + 4 * p->syn_sr - 1) / (4 * p->syn_sr), nmap);
#define GS_SL(NC, SR) hipLaunchKernelGGL((k_sht_synth_leg<NC, SR>), grid, dim3(LEG_BLOCK), 0, S(stream), p->dev(), \
                                         p->acoef, p->ain, p->phi, p->syn_paired)
#define GS_SL2(NC) do { if (p->syn_sr == 4) GS_SL(NC, 4); else if (p->syn_sr == 2) GS_SL(NC, 2); else GS_SL(NC, 1); } while (0)
    if (ncomp == 1) GS_SL2(1); else if (ncomp == 2) GS_SL2(2); else GS_SL2(3);
#undef GS_SL2
#undef GS_SL
    GS_LAUNCH_CHECK("k_sht_synth_leg");
    return sht_rings(p, true, nmap * ncomp, nullptr, maps, stream, nullptr, nullptr, 1, nullptr, ncomp, nullptr,
                     nullptr, aux);
}

int gs_sht_alm2map(gs_sht* p, int ncomp, int layout, const double* alm, double* maps, void* stream) {
    return sht_alm2map(p, 1, ncomp, layout, alm, nullptr, maps, stream);
}

// analysis of B maps (maps [B][ncomp][Npix] -> alm [B][ncomp][n]); wts: ncomp
// weight maps shared by the batch (the product wts * maps is transformed)
static int sht_analysis(gs_sht* p, int nmap, int ncomp, int layout, const double* maps, double* alm, int acc,
                        void* stream, const double* wts = nullptr) {
    if (nmap > 1 && !sht_batch_native(p)) {
        const long long as = ncomp * alm_comp_stride(layout, p->L), ms = (long long)ncomp * p->npix;
        for (int b = 0; b < nmap; ++b)
            if (sht_analysis(p, 1, ncomp, layout, maps + b * ms, alm + b * as, acc, stream, wts)) return -1;
        return 0;
    }
    if (sht_reserve(p, nmap, S(stream))) return -1;
    const int* sup = nullptr;
    if (sht_support(p, wts, ncomp, S(stream), &sup)) return -1;
    if (sht_rings(p, false, nmap * ncomp, maps, nullptr, stream, nullptr, nullptr, 1, wts, ncomp, sup))
        return -1;
    if (p->mf) return sht_anal_mfma(p, nmap, ncomp, layout, acc, alm, S(stream), sup);
    const int sr = p->ana_sr_nc[ncomp], sl = p->ana_seg_nc[ncomp];
    const int ntile = (p->ngroup + 4 * sr - 1) / (4 * sr);
    const int nsegz = sl ? (p->L + sl) / sl : 1;
    const dim3 grid(p->ana_paired ? p->L / 2 + 1 : p->L + 1, ntile, nsegz * nmap);
    const ShtDev D = p->devseg(sl);
#define GS_AL(NC, SR) do { if (sl > 0 && sl <= 64) \
        hipLaunchKernelGGL((k_sht_anal_leg<NC, SR, true>), grid, dim3(LEG_BLOCK), 0, S(stream), D, p->acoef, \
                           p->phi, p->part, p->ana_paired); \
    else hipLaunchKernelGGL((k_sht_anal_leg<NC, SR, false>), grid, dim3(LEG_BLOCK), 0, S(stream), D, p->acoef, \
                            p->phi, p->part, p->ana_paired); } while (0)
#define GS_AL2(NC) do { if (sr == 4) GS_AL(NC, 4); else if (sr == 2) GS_AL(NC, 2); \
                        else GS_AL(NC, 1); } while (0)
    if (ncomp == 1) GS_AL2(1); else if (ncomp == 2) GS_AL2(2); else GS_AL2(3);
#undef GS_AL2
#undef GS_AL
    GS_LAUNCH_CHECK("k_sht_anal_leg");
    const double w = 4.0 * PI / (double)p->npix;
    const long long n = (long long)nmap * ncomp * p->nlm;
#define GS_AF(NC) hipLaunchKernelGGL((k_sht_anal_finish<NC>), dim3(nblocks(n, 256)), dim3(256), 0, S(stream), p->L, p->nlm, \
                                     ntile * 4, p->part, w, layout, acc, alm, nmap, p->acq)
    if (ncomp == 1) GS_AF(1); else if (ncomp == 2) GS_AF(2); else GS_AF(3);
#undef GS_AF
    GS_LAUNCH_CHECK("k_sht_anal_finish");
    return 0;
}

long long gs_sht_phi_plane(const gs_sht* p) { return p ? phi_plane(p->L, p->npair) : 0; }

// nmap chains (batch-native plans; others one chain per pass): alm_real
// [nmap][nfield][(L+1)^2], phib [nmap][K NCO][2][plane], maps [nmap][K NCO][Npix],
// blk_lmax [nmap][K] (each chain's copy of the blocks' largest l)
int gs_sht_synth_blocks(gs_sht* p, int nmap, int nfield, const double* alm_real, const int* blk, int K,
                        const int* blk_lmax, double* phib, double* maps, void* stream, int parseval) {
    if (check_sht(p)) return -1;
    if (nfield != 1 && nfield != 2) return set_error("gs_sht_synth_blocks: nfield must be 1 (T) or 2 (E,B)");
    if (K < 1 || nmap < 1 || !alm_real || !blk || !blk_lmax || !phib || !maps)
        return set_error("gs_sht_synth_blocks: null argument");
    const int nco = nfield == 1 ? 1 : 2;
    const long long plane = phi_plane(p->L, p->npair);
    if (nmap > 1 && !sht_batch_native(p)) {
        for (int b = 0; b < nmap; ++b)
            if (gs_sht_synth_blocks(p, 1, nfield, alm_real + (long long)b * nfield * (p->L + 1) * (p->L + 1), blk, K,
                                    blk_lmax + (long long)b * K, phib + (long long)b * K * nco * 2 * plane * 2,
                                    maps + (long long)b * K * nco * p->npix, stream, parseval))
                return -1;
        return 0;
    }
    if (nmap > 1 && sht_reserve(p, nmap, S(stream))) return -1;
    double2* ph = reinterpret_cast<double2*>(phib);
    const char* bme = gs_detail::option("GS_SHT_BLOCKS_MFMA");
    if (p->mf && nfield == 2 && !(bme && atoi(bme) == 0)) {
        // the tables: every chain of the batch in one matrix-core launch (both
        // fields' passes; grid tile x phase block x (chain group, field))
        const dim3 g((unsigned)p->mf_ntile, (unsigned)((p->L + 4) / 4), (unsigned)(2 * ((nmap + 7) / 8)));
        hipLaunchKernelGGL(k_sht_blocks_mfma<2>, g, dim3(256), (size_t)(p->L + 1) * sizeof(int), S(stream), p->dev(),
                           p->mftab(), alm_real, nmap, blk, K, ph);
        GS_LAUNCH_CHECK("k_sht_blocks_mfma");
    } else {
    const long long nin = (long long)nmap * nfield * p->nlm;
    hipLaunchKernelGGL(k_sht_alm_in, dim3(nblocks(nin, 256)), dim3(256), 0, S(stream), p->L, p->nlm, nmap * nfield,
                       alm_real, GS_ALM_REAL, p->ain, nullptr);
    GS_LAUNCH_CHECK("k_sht_alm_in");
    const long long cst = (long long)K * nco * 2 * plane;
    // one launch per chain: the planes are written 16 B per lane at a 64-B stride,
    // each 64-B run completed by the workgroups of its four m, which one chain's
    // launch keeps co-resident (all chains in one grid measured 24.4 against 19.1
    // ms for 16 chains at N_side 256: the runs' pieces then reach L2 too far apart)
    const int bsr = p->syn_sr >= 2 ? 2 : 1;           // ring groups per lane (the block kernels: 1 or 2)
    const dim3 grid(p->syn_paired ? p->L / 2 + 1 : p->L + 1, (p->ngroup + 4 * bsr - 1) / (4 * bsr), 1);
    // staged variant when m = 0's coefficients, a_lm and block indices fit 64 KB
    // of LDS (GS_SHT_BLK_STAGE=0 turns it off: tests)
    const size_t stg = (size_t)(p->L + 1) * (4 * sizeof(double2) + nfield * (sizeof(double2) + sizeof(int)));
    const char* stg_env = gs_detail::option("GS_SHT_BLK_STAGE");
    const bool stage_off = stg_env && atoi(stg_env) == 0;
    const bool use_stg = stg <= 64 * 1024 && !stage_off;
#define GS_SB(NF, SR) do { if (use_stg) hipLaunchKernelGGL((k_sht_synth_blocks<NF, SR, true>), grid, dim3(LEG_BLOCK), \
                                         stg, S(stream), p->dev(), p->coef, p->ain + b * nfield * p->nlm, blk, \
                                         ph + b * cst, p->syn_paired, cst); \
    else hipLaunchKernelGGL((k_sht_synth_blocks<NF, SR, false>), grid, dim3(LEG_BLOCK), 0, S(stream), p->dev(), \
                            p->coef, p->ain + b * nfield * p->nlm, blk, ph + b * cst, p->syn_paired, cst); } while (0)
    for (long long b = 0; b < nmap; ++b) {
        if (nfield == 1) { if (bsr == 2) GS_SB(1, 2); else GS_SB(1, 1); }
        else { if (bsr == 2) GS_SB(2, 2); else GS_SB(2, 1); }
    }
#undef GS_SB
    GS_LAUNCH_CHECK("k_sht_synth_blocks");
    }
    // ring stage: the plan's FFT scratch (global / split rings) holds three comps,
    // so rings that need it run three comps per launch
    const int ncomp = nmap * K * nco;
    const bool scratch = p->gscr != nullptr || p->nsplit > 0;
    const int chunk = scratch ? nco * (3 / nco) : ncomp;    // whole blocks per launch
    for (int c0 = 0; c0 < ncomp; c0 += chunk) {
        const int nc = std::min(chunk, ncomp - c0);
        if (sht_rings(p, true, nc, nullptr, maps + (long long)c0 * p->npix, stream, ph + (long long)c0 * 2 * plane,
                      blk_lmax + c0 / nco, nco, nullptr, 3, nullptr, parseval ? p->wsup : nullptr))
            return -1;
    }
    return 0;
}

static int sht_map2alm(gs_sht* p, int nmap, int ncomp, int layout, const double* maps, double* alm, int niter,
                       void* stream) {
    if (check_sht(p)) return -1;
    if (ncomp < 1 || ncomp > 3) return set_error("gs_sht_map2alm: ncomp must be 1 (T), 2 (Q,U) or 3 (T,Q,U)");
    if (layout != GS_ALM_REAL && layout != GS_ALM_COMPLEX) return set_error("gs_sht_map2alm: bad layout");
    if (!alm || !maps) return set_error("gs_sht_map2alm: null argument");
    if (niter < 0) return set_error("gs_sht_map2alm: niter < 0");
    if (nmap < 1) return set_error("gs_sht_map2alm: nmap < 1");
    if (nmap > 1 && !sht_batch_native(p)) {
        const long long as = ncomp * alm_comp_stride(layout, p->L), ms = (long long)ncomp * p->npix;
        for (int b = 0; b < nmap; ++b)
            if (sht_map2alm(p, 1, ncomp, layout, maps + b * ms, alm + b * as, niter, stream)) return -1;
        return 0;
    }
    if (sht_analysis(p, nmap, ncomp, layout, maps, alm, 0, stream)) return -1;
    for (int it = 0; it < niter; ++it) {
        // a += map2alm(m - alm2map(a))   (healpy iter = niter)
        if (sht_alm2map(p, nmap, ncomp, layout, alm, nullptr, p->mapw, stream)) return -1;
        const long long n = (long long)nmap * ncomp * p->npix;
        hipLaunchKernelGGL(k_sub_maps, dim3(nblocks(n, 256)), dim3(256), 0, S(stream), n, maps, p->mapw);
        GS_LAUNCH_CHECK("k_sub_maps");
        if (sht_analysis(p, nmap, ncomp, layout, p->mapw, alm, 1, stream)) return -1;
    }
    return 0;
}

int gs_sht_map2alm(gs_sht* p, int ncomp, int layout, const double* maps, double* alm, int niter, void* stream) {
    return sht_map2alm(p, 1, ncomp, layout, maps, alm, niter, stream);
}

int gs_sht_alm2map_beamed(gs_sht* p, int ncomp, const double* alm_real, const double* bl, double* maps, void* stream) {
    if (!bl) return set_error("gs_sht_alm2map_beamed: null beam");
    return sht_alm2map(p, 1, ncomp, GS_ALM_REAL, alm_real, bl, maps, stream);
}

int gs_sht_map2alm_weighted(gs_sht* p, int ncomp, const double* maps, const double* weights, double* alm_real,
                            void* stream) {
    if (check_sht(p)) return -1;
    if (ncomp < 1 || ncomp > 3) return set_error("gs_sht_map2alm_weighted: ncomp must be 1 (T), 2 (Q,U) or 3 (T,Q,U)");
    if (!alm_real || !maps || !weights) return set_error("gs_sht_map2alm_weighted: null argument");
    return sht_analysis(p, 1, ncomp, GS_ALM_REAL, maps, alm_real, 0, stream, weights);
}

// register a weights array [wnc][Npix] (the masked context's N^-1, fixed for its
// lifetime): its pair support and constant-ring classes are computed once
// (k_ring_classes) and used by every weighted transform given the same pointer
// -- the support skip without a per-call pass, and the constant-ring forms of
// the fused operator (k_sht_apply_ring_mc).  The caller must not change the
// array while it is registered; weights = nullptr unregisters.
int gs_sht_register_weights(gs_sht* p, const double* weights, int wnc, void* stream) {
    if (check_sht(p)) return -1;
    p->wreg = nullptr;
    p->wreg_nc = 0;
    if (!weights) return 0;
    if (wnc < 1 || wnc > 3) return set_error("gs_sht_register_weights: wnc must be 1..3");
    if (!p->wsup && sht_alloc(p, &p->wsup, (size_t)p->npair)) return -1;
    if (!p->wconst && sht_alloc(p, &p->wconst, (size_t)p->npair * 3)) return -1;
    hipLaunchKernelGGL(k_ring_classes, dim3(p->npair), dim3(256), 0, S(stream), p->npix, p->geom, weights, wnc,
                       p->wsup, p->wconst);
    GS_LAUNCH_CHECK("k_ring_classes");
    p->wreg = weights;
    p->wreg_nc = wnc;
    return 0;
}

// the registered weights' pair classes: counts of class 0 (no weight), 1
// (weighted, varying on a ring) and 3 (constant on both rings)
int gs_sht_ring_class_counts(const gs_sht* p, int counts[3]) {
    if (check_sht(p)) return -1;
    counts[0] = counts[1] = counts[2] = 0;
    if (!p->wreg) return 0;
    std::vector<int> h((size_t)p->npair);
    GS_CHECK(hipMemcpy(h.data(), p->wsup, h.size() * sizeof(int), hipMemcpyDeviceToHost));
    for (int v : h) ++counts[v == 0 ? 0 : (v & 2 ? 2 : 1)];
    return 0;
}

// f2 block maps in Parseval coordinates on the registered weights' constant
// pairs: available when the block ring stage runs the merged multi-component
// kernels (small maps) with registered weights of nfield rows
int gs_sht_blocks_parseval(const gs_sht* p, int nfield, int ncomp_total) {
    if (!p || !const_rings_on() || !p->wreg || p->wreg_nc != nfield || p->merged_n <= 0) return 0;
    return ring_mc_ncb(p->merged_M, ncomp_total) > 1 ? 1 : 0;
}

// maps [ncomp][Npix] -> Parseval coordinates on the registered constant pairs, in
// place (the f2 residual, to match block maps made with parseval = 1)
int gs_sht_parseval_maps(gs_sht* p, int ncomp, double* maps, void* stream) {
    if (check_sht(p)) return -1;
    if (!p->wreg || p->merged_n <= 0 || !maps || ncomp < 1) return set_error("gs_sht_parseval_maps: not available");
    const int M = p->merged_M, bd = ring_block(M);
    const int ncb = std::max(1, ring_mc_ncb(M, ncomp));
    const int bdm = ncb * bd, SB = std::max(M, 4 * bd), toff = ncb * SB;
    const size_t ldsm = (size_t)(ncb * SB + M / 2) * sizeof(double2);
    const int ncg = (ncomp + ncb - 1) / ncb;
    const dim3 gm((unsigned)(8 * ((p->merged_n + 15) / 16) * 2 * ncg));
    hipLaunchKernelGGL(k_sht_parseval_ring_mc<8>, gm, dim3(bdm), ldsm, S(stream), p->npix, p->merged_pairs, p->geom,
                       p->tw, p->Mmax, p->bsk, maps, ncomp, ncb, SB, toff, p->merged_n, p->wsup);
    GS_LAUNCH_CHECK("k_sht_parseval_ring_mc");
    return 0;
}

int gs_sht_set_mfma(gs_sht* p, int on) {
    if (check_sht(p)) return -1;
    if (on && !sht_batch_native(p))
        return set_error("gs_sht_set_mfma: the Legendre tables are for small maps (no split-ring FFT plan)");
    if (on && !p->mf_tab) {
        // one lambda plane, 8 B per (l, m, ring pair) before the onset skip
        // (0.54 GB at N_side 256 / l_max 512, 4.3 GB at N_side 512 / l_max
        // 1024); budget GS_SHT_MFMA_MAX_GB (default 16 GB)
        double gb = 16.0;
        if (const char* e = gs_detail::option("GS_SHT_MFMA_MAX_GB")) gb = std::atof(e);
        const double need = 8.0 * (double)p->npair * (double)p->nlm / 1e9;
        if (need > gb) return set_error("gs_sht_set_mfma: the Legendre table exceeds GS_SHT_MFMA_MAX_GB");
    }
    return sht_set_mfma(p, on);
}

int gs_sht_mfma_info(const gs_sht* p, int* on, long long* table_bytes) {
    if (check_sht(p)) return -1;
    if (on) *on = p->mf;
    if (table_bytes) *table_bytes = p->mf_bytes;
    return 0;
}

int gs_sht_reserve(gs_sht* p, int nmap, void* stream) {
    if (check_sht(p)) return -1;
    if (nmap < 1) return set_error("gs_sht_reserve: nmap < 1");
    return sht_batch_native(p) ? sht_reserve(p, nmap, S(stream)) : 0;
}

int gs_sht_alm2map_batch(gs_sht* p, int nmap, int ncomp, int layout, const double* alm, const double* bl,
                         double* maps, void* stream) {
    return sht_alm2map(p, nmap, ncomp, layout, alm, bl, maps, stream);
}

// alm_out = map2alm(weights x alm2map(bl x alm_in)) (real layout): on the
// table path with the multi-component ring stage the maps never leave LDS
// (k_sht_apply_ring_mc); otherwise the two transforms through maps_scratch
int gs_sht_apply_weighted_batch(gs_sht* p, int nmap, int ncomp, const double* alm_in, const double* bl,
                                const double* weights, double* maps_scratch, double* alm_out, void* stream) {
    if (check_sht(p)) return -1;
    if (ncomp < 1 || ncomp > 3 || nmap < 1 || !alm_in || !weights || !alm_out)
        return set_error("gs_sht_apply_weighted_batch: bad argument");
    const int M = p->merged_M;
    const int ncb = (p->mf && p->merged_n > 0) ? ring_mc_ncb(M, nmap * ncomp) : 1;
    if (ncb < 2) {
        if (!maps_scratch) return set_error("gs_sht_apply_weighted_batch: this plan needs maps_scratch");
        if (sht_alm2map(p, nmap, ncomp, GS_ALM_REAL, alm_in, bl, maps_scratch, stream)) return -1;
        return gs_sht_map2alm_batch(p, nmap, ncomp, GS_ALM_REAL, maps_scratch, weights, alm_out, 0, stream);
    }
    if (sht_reserve(p, nmap, S(stream))) return -1;
    // pairs / tiles without weight: no synthesis, zero phases, skipped in the analysis
    const int* sup = nullptr;
    if (sht_support(p, weights, ncomp, S(stream), &sup)) return -1;
    if (sht_synth_mfma(p, nmap, ncomp, S(stream), sup, alm_in, bl)) return -1;
    {
        const int bd = ring_block(M), bdm = ncb * bd, SB = std::max(M, 4 * bd), toff = ncb * SB;
        const size_t ldsm = (size_t)(ncb * SB + M / 2) * sizeof(double2);
        const int nc = nmap * ncomp, ncg = (nc + ncb - 1) / ncb;
        const dim3 gm((unsigned)(8 * ((p->merged_n + 15) / 16) * 2 * ncg));
        const PixWeights op{weights, ncomp, p->npix, sup && sup == p->wsup ? sht_wconst(p, weights, ncomp) : nullptr};
        hipLaunchKernelGGL((k_sht_apply_ring_mc<8, PixWeights>), gm, dim3(bdm), ldsm, S(stream), p->L, p->npair,
                           p->npix, p->merged_pairs, p->geom, p->phi, p->tw, p->Mmax, p->bsk, nc, ncb, SB, toff, op,
                           p->merged_n, sup);
        GS_LAUNCH_CHECK("k_sht_apply_ring_mc");
    }
    return sht_anal_mfma(p, nmap, ncomp, GS_ALM_REAL, 0, alm_out, S(stream), sup);
}

// the aux-variable step's v | s and s | v analysis in one pass (gs_masked's
// masked CR, CenteredGibbs.py:693-717): alm_out = map2alm(y) (real layout, iter
// 0) with y = the v | s update (GsAuxPix, which also writes v) of alm2map(bl x
// alm_in), nmap chains of ncomp fields, the maps never leaving LDS.  Returns 1
// when the plan has no fused path (the caller then runs the two transforms and
// its pixel kernel); bit-identical to those.
int gs_sht_aux_pass_batch(gs_sht* p, int nmap, int ncomp, const double* alm_in, const double* bl, const void* aux,
                          double* alm_out, void* stream) {
    if (check_sht(p)) return -1;
    if (ncomp < 1 || ncomp > 3 || nmap < 1 || !alm_in || !aux || !alm_out)
        return set_error("gs_sht_aux_pass_batch: bad argument");
    const char* fe = gs_detail::option("GS_SHT_FUSED_AUX");
    if (fe && std::atoi(fe) == 0) return 1;
    if (!p->mf && p->merged_n == 0 && nmap == 1) {
        // large maps (per-class ring stage, the on-the-fly Legendre kernels): the
        // v | s step runs on the synthesised pixels as the ring stage stores them,
        // so A b s is never written and read back; y = v + N^-1 d goes to the
        // plan's map workspace and the analysis reads it from there (the same
        // bits as the synthesis, k_mc_v and the analysis in turn)
        if (sht_reserve(p, nmap, S(stream))) return -1;
        const gs::GsAuxPix* a = reinterpret_cast<const gs::GsAuxPix*>(aux);
        if (sht_alm2map(p, nmap, ncomp, GS_ALM_REAL, alm_in, bl, p->mapw, stream, a)) return -1;
        return sht_analysis(p, nmap, ncomp, GS_ALM_REAL, p->mapw, alm_out, 0, stream);
    }
    const int M = p->merged_M;
    const int ncb = (p->mf && p->merged_n > 0) ? ring_mc_ncb(M, nmap * ncomp) : 1;
    if (ncb < 2) return 1;
    if (sht_reserve(p, nmap, S(stream))) return -1;
    if (sht_synth_mfma(p, nmap, ncomp, S(stream), nullptr, alm_in, bl)) return -1;
    {
        const int bd = ring_block(M), bdm = ncb * bd, SB = std::max(M, 4 * bd), toff = ncb * SB;
        const size_t ldsm = (size_t)(ncb * SB + M / 2) * sizeof(double2);
        const int nc = nmap * ncomp, ncg = (nc + ncb - 1) / ncb;
        const dim3 gm((unsigned)(8 * ((p->merged_n + 15) / 16) * 2 * ncg));
        const PixAux op{*reinterpret_cast<const gs::GsAuxPix*>(aux)};
        hipLaunchKernelGGL((k_sht_apply_ring_mc<8, PixAux>), gm, dim3(bdm), ldsm, S(stream), p->L, p->npair, p->npix,
                           p->merged_pairs, p->geom, p->phi, p->tw, p->Mmax, p->bsk, nc, ncb, SB, toff, op, p->merged_n,
                           nullptr);
        GS_LAUNCH_CHECK("k_sht_apply_ring_mc (aux)");
    }
    if (sht_anal_mfma(p, nmap, ncomp, GS_ALM_REAL, 0, alm_out, S(stream), nullptr)) return -1;
    return 0;
}

int gs_sht_map2alm_batch(gs_sht* p, int nmap, int ncomp, int layout, const double* maps, const double* weights,
                         double* alm, int niter, void* stream) {
    if (weights) {
        if (layout != GS_ALM_REAL) return set_error("gs_sht_map2alm_batch: weights need the real layout");
        if (niter != 0) return set_error("gs_sht_map2alm_batch: weights need niter 0");
        if (check_sht(p)) return -1;
        if (ncomp < 1 || ncomp > 3 || nmap < 1 || !maps || !alm) return set_error("gs_sht_map2alm_batch: bad argument");
        if (nmap > 1 && !sht_batch_native(p)) {
            const long long as = ncomp * alm_comp_stride(layout, p->L), ms = (long long)ncomp * p->npix;
            for (int b = 0; b < nmap; ++b)
                if (sht_analysis(p, 1, ncomp, layout, maps + b * ms, alm + b * as, 0, stream, weights)) return -1;
            return 0;
        }
        return sht_analysis(p, nmap, ncomp, layout, maps, alm, 0, stream, weights);
    }
    return sht_map2alm(p, nmap, ncomp, layout, maps, alm, niter, stream);
}

}  // extern "C"
