// sht_cpu.cpp -- C++/OpenMP HEALPix RING spherical-harmonic transforms
// (TEST / MEASUREMENT INFRASTRUCTURE: only tests/, __graft_entry__ and
// bench.py's cpu_baseline load it; the product path never does).
//
// The CPU leg of the SHT-bound benchmarks (SURVEY.md 8d "C++/OpenMP
// SHT for transforms"): the reference calls healpy (libsharp / ducc0) for
// hp.alm2map / hp.map2alm (CenteredGibbs.py:204,298,505,513,698,717,751,773,791,812;
// NonCenteredGibbs.py:155,350; utils.py:89,104), which is absent offline.  This is
// a restatement of the same transforms with the conventions of oracle/sht.py
// (HEALPix geometry, Condon-Shortley lambda_lm, Zaldarriaga-Seljak spin-2 F1/F2,
// Q + iU = -sum (a_E + i a_B) 2Y_lm, map2alm = w * exact adjoint, healpy Jacobi
// iterations), checked against that dense oracle in tests/test_oracle_sht.py.
//
// Algorithm (libsharp's structure, plain C++):
//   * per m (OpenMP dynamic over m) and ring pair (north/south share |z|): the
//     normalised three-term recurrence of lambda_lm in l with a scale exponent
//     (value = v * 2^(SCALE k)), so sin^m theta never underflows; the north and
//     south ring sums split by the parity of l + m;
//   * per ring (OpenMP over rings): the phase sums by an FFT of the ring length
//     (radix-2 for powers of two, Bluestein otherwise), aliasing m -> m mod nphi.
// Layout: healpy complex m-major a_lm (idx = m (2L + 1 - m) / 2 + l), interleaved
// (re, im) doubles; comps 1 = T (spin 0), 2 = E,B <-> Q,U (spin 2), 3 = T,E,B <-> T,Q,U.
#include <cmath>
#include <complex>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <vector>
#include <omp.h>

namespace {

using cplx = std::complex<double>;
constexpr double PI = 3.14159265358979323846;
constexpr int SCALE = 256;                         // scale step of the recurrence: 2^256
const double BIG = std::ldexp(1.0, SCALE);
const double IBIG = std::ldexp(1.0, -SCALE);

struct Ring { double z, phi0; long long start; int nphi; };

std::vector<Ring> rings_of(int N) {
    std::vector<Ring> r(4 * N - 1);
    const long long npix = 12LL * N * N;
    for (int k = 0; k < 4 * N - 1; ++k) {
        const int i = k + 1;
        Ring& g = r[k];
        if (i < N) {
            g.z = 1.0 - (double)i * i / (3.0 * N * N); g.nphi = 4 * i; g.phi0 = PI / (4.0 * i);
            g.start = 2LL * i * (i - 1);
        } else if (i <= 3 * N) {
            g.z = 4.0 / 3.0 - 2.0 * i / (3.0 * N); g.nphi = 4 * N;
            g.phi0 = ((i - N) % 2 == 0 ? 0.5 : 0.0) * PI / (2.0 * N);
            g.start = 2LL * N * (N - 1) + (long long)(i - N) * 4 * N;
        } else {
            const int ii = 4 * N - i;
            g.z = -(1.0 - (double)ii * ii / (3.0 * N * N)); g.nphi = 4 * ii; g.phi0 = PI / (4.0 * ii);
            g.start = npix - 2LL * ii * (ii + 1);
        }
    }
    return r;
}

// ---- FFT: iterative radix-2 for powers of two, Bluestein otherwise ----------
struct Fft {
    int n = 0, m = 0;                      // length, Bluestein power-of-two length (0: radix-2 direct)
    std::vector<cplx> tw;                  // twiddles of the power-of-two transform
    std::vector<cplx> chirp, kern;         // Bluestein chirp w_k = e^{-i pi k^2 / n}, FFT of its conjugate
    static bool pow2(int x) { return x > 0 && (x & (x - 1)) == 0; }
    static void radix2(std::vector<cplx>& a, int len, const std::vector<cplx>& tw, bool inverse) {
        for (int i = 1, j = 0; i < len; ++i) {
            int bit = len >> 1;
            for (; j & bit; bit >>= 1) j ^= bit;
            j ^= bit;
            if (i < j) std::swap(a[i], a[j]);
        }
        for (int s = 2; s <= len; s <<= 1) {
            const int h = s >> 1, step = len / s;
            for (int b = 0; b < len; b += s)
                for (int k = 0; k < h; ++k) {
                    const cplx w = inverse ? std::conj(tw[k * step]) : tw[k * step];
                    const cplx u = a[b + k], v = a[b + k + h] * w;
                    a[b + k] = u + v;
                    a[b + k + h] = u - v;
                }
        }
    }
    explicit Fft(int len) : n(len) {
        const int base = pow2(n) ? n : [&] { int p = 1; while (p < 2 * n - 1) p <<= 1; return p; }();
        tw.resize(base / 2 + 1);
        for (int k = 0; k <= base / 2; ++k) tw[k] = std::polar(1.0, -2.0 * PI * k / base);
        if (pow2(n)) return;
        m = base;
        chirp.resize(n);
        for (int k = 0; k < n; ++k) {
            const double ph = PI * (double)((long long)k * k % (2LL * n)) / n;
            chirp[k] = std::polar(1.0, -ph);
        }
        kern.assign(m, cplx(0, 0));
        kern[0] = std::conj(chirp[0]);
        for (int k = 1; k < n; ++k) kern[k] = kern[m - k] = std::conj(chirp[k]);
        radix2(kern, m, tw, false);
    }
    // out[k] = sum_j in[j] e^{-+2 pi i jk / n} (forward: -, inverse: +; no 1/n)
    void run(std::vector<cplx>& a, bool inverse, std::vector<cplx>& work) const {
        if (m == 0) { radix2(a, n, tw, inverse); return; }
        work.assign(m, cplx(0, 0));
        for (int k = 0; k < n; ++k) work[k] = (inverse ? std::conj(a[k]) : a[k]) * chirp[k];
        radix2(work, m, tw, false);
        for (int k = 0; k < m; ++k) work[k] *= kern[k];
        radix2(work, m, tw, true);
        const double s = 1.0 / m;
        for (int k = 0; k < n; ++k) {
            const cplx v = work[k] * chirp[k] * s;
            a[k] = inverse ? std::conj(v) : v;
        }
    }
};

struct Plan {
    int N, L, nring, npair;
    std::vector<Ring> rings;
    std::map<int, std::unique_ptr<Fft>> ffts;
    Plan(int nside, int lmax) : N(nside), L(lmax) {
        rings = rings_of(N);
        nring = (int)rings.size();
        npair = 2 * N;                      // ring pairs k and nring-1-k; k = 2N-1 is the equator (alone)
        for (const Ring& r : rings)
            if (!ffts.count(r.nphi)) ffts[r.nphi] = std::make_unique<Fft>(r.nphi);
    }
    long long nlm() const { return (long long)(L + 1) * (L + 2) / 2; }
    long long idx(int l, int m) const { return (long long)m * (2 * L + 1 - m) / 2 + l; }
};

// per-m recurrence constants: lambda_l = a_l (x lambda_{l-1} - b_l lambda_{l-2});
// spin-2: c_l, f_l = sqrt((2l+1)/(2l-1) (l^2 - m^2))
struct MCoef { std::vector<double> a, b, c, f; double lmm_log2, lmm_sign; };

MCoef coef_m(int L, int m) {
    MCoef k;
    k.a.assign(L + 2, 0.0); k.b.assign(L + 2, 0.0); k.c.assign(L + 2, 0.0); k.f.assign(L + 2, 0.0);
    for (int l = m + 2; l <= L; ++l) {
        k.a[l] = std::sqrt((4.0 * l * l - 1.0) / ((double)l * l - (double)m * m));
        k.b[l] = std::sqrt((((double)l - 1.0) * (l - 1.0) - (double)m * m) / (4.0 * (l - 1.0) * (l - 1.0) - 1.0));
    }
    for (int l = std::max(m, 2); l <= L; ++l) {
        k.c[l] = 2.0 / std::sqrt(((double)l - 1.0) * l * (l + 1.0) * (l + 2.0));
        k.f[l] = std::sqrt((2.0 * l + 1.0) / (2.0 * l - 1.0) * ((double)l * l - (double)m * m));
    }
    // lambda_mm = (-1)^m sqrt((2m+1)/(4 pi) prod_{k<=m} (2k-1)/(2k)) sin^m: log2 of the sin-free part
    double lg = std::log2(1.0 / (4.0 * PI) * (2.0 * m + 1.0));
    for (int q = 1; q <= m; ++q) lg += std::log2((2.0 * q - 1.0) / (2.0 * q));
    k.lmm_log2 = 0.5 * lg;
    k.lmm_sign = (m & 1) ? -1.0 : 1.0;
    return k;
}

// Ring-pair blocks of RB lanes: the recurrence of lambda_lm(x) in l for RB
// ring pairs at once (the lane loops vectorise), each lane with its own scale
// exponent (value = v 2^(SCALE e)); a lane contributes only when e >= -1
// (below that the value is < 2^-SCALE).  Per l the lanes' true lambda_lm and
// lambda_{l-1,m} are in lam[], lam1[].
constexpr int RB = 8;

struct Block {
    int n;                                   // live lanes (ring pairs) in this block
    int pr[RB];                              // ring pair (north ring) index
    double x[RB], is2[RB];
};

struct Walker {
    double v0[RB], v1[RB], fac[RB], lam[RB], lam1[RB];
    int e[RB];
    void start(const MCoef& k, int m, const Block& B) {
        for (int r = 0; r < RB; ++r) {
            const double x = r < B.n ? B.x[r] : 0.5;
            const double s = std::sqrt((1.0 - x) * (1.0 + x));
            const double l2 = k.lmm_log2 + m * std::log2(s);
            e[r] = (int)std::floor(l2 / SCALE);
            v1[r] = k.lmm_sign * std::exp2(l2 - (double)e[r] * SCALE);
            v0[r] = 0.0;
        }
    }
    // true values of (v1, v0) into (lam, lam1); returns whether any lane contributes
    bool values() {
        bool any = false;
        for (int r = 0; r < RB; ++r) {
            fac[r] = e[r] == 0 ? 1.0 : (e[r] == -1 ? IBIG : 0.0);
            lam[r] = v1[r] * fac[r];
            lam1[r] = v0[r] * fac[r];
            any |= fac[r] != 0.0;
        }
        return any;
    }
    void step_first(int m, const Block& B) {           // lambda_{m+1,m} = x sqrt(2m+3) lambda_mm
        const double c = std::sqrt(2.0 * m + 3.0);
        for (int r = 0; r < RB; ++r) {
            const double vn = B.x[r] * c * v1[r];
            v0[r] = v1[r];
            v1[r] = vn;
        }
    }
    void step(const MCoef& k, int l, const Block& B) {
        const double al = k.a[l], bl = k.b[l];
        for (int r = 0; r < RB; ++r) {
            const double vn = al * (B.x[r] * v1[r] - bl * v0[r]);
            v0[r] = v1[r];
            v1[r] = vn;
            const bool up = std::fabs(vn) > BIG && e[r] < 0;
            v1[r] = up ? vn * IBIG : vn;
            v0[r] = up ? v0[r] * IBIG : v0[r];
            e[r] += up ? 1 : 0;
        }
    }
};

std::vector<Block> blocks_of(const Plan& P) {
    std::vector<Block> out;
    for (int p0 = 0; p0 < P.npair; p0 += RB) {
        Block B{};
        B.n = std::min(RB, P.npair - p0);
        for (int r = 0; r < RB; ++r) {
            const int pr = p0 + std::min(r, B.n - 1);
            B.pr[r] = pr;
            B.x[r] = P.rings[pr].z;
            B.is2[r] = 1.0 / ((1.0 - B.x[r]) * (1.0 + B.x[r]));
        }
        out.push_back(B);
    }
    return out;
}

// phase[ring][m] (ring-major, m <= L), re / im
struct Phases {
    std::vector<double> re, im;
    explicit Phases(size_t n = 0) : re(n, 0.0), im(n, 0.0) {}
};

void synth_legendre(const Plan& P, int comps, const double* alm, Phases* ph) {
    const int L = P.L;
    const long long nlm = P.nlm();
    const bool t0 = comps & 1, s2 = comps & 2;
    const double* aT = alm;
    const double* aE = alm + (t0 ? 2 * nlm : 0);
    const double* aB = aE + 2 * nlm;
    const std::vector<Block> blocks = blocks_of(P);
#pragma omp parallel for schedule(dynamic, 1)
    for (int mm = 0; mm <= L; ++mm) {
        const int m = (mm & 1) ? L - mm / 2 : mm / 2;        // large and small m interleaved
        const MCoef k = coef_m(L, m);
        for (const Block& B : blocks) {
            // [parity][lane]: 0 = even l + m (same sign north / south), 1 = odd
            double T[2][2][RB] = {}, Q[2][2][RB] = {}, U[2][2][RB] = {};     // [parity][re/im][lane]
            Walker w;
            w.start(k, m, B);
            for (int l = m; l <= L; ++l) {
                if (l == m + 1) w.step_first(m, B);
                else if (l > m + 1) w.step(k, l, B);
                if (!w.values()) continue;
                const long long i = 2 * P.idx(l, m);
                const int pa = (l + m) & 1, pb = pa ^ 1;
                if (t0) {
                    const double ar = aT[i], ai = aT[i + 1];
                    for (int r = 0; r < RB; ++r) { T[pa][0][r] += ar * w.lam[r]; T[pa][1][r] += ai * w.lam[r]; }
                }
                if (s2 && l >= 2) {
                    const double er = aE[i], ei = aE[i + 1], br = aB[i], bi = aB[i + 1];
                    const double cl = k.c[l], fl = k.f[l], lm2 = (double)l - (double)m * m, h = 0.5 * l * (l - 1.0);
                    for (int r = 0; r < RB; ++r) {
                        const double x = B.x[r], is2 = B.is2[r], lam = w.lam[r], lam1 = w.lam1[r];
                        const double F1 = cl * (-(lm2 * is2 + h) * lam + fl * x * is2 * lam1);
                        const double F2 = cl * m * is2 * (-(l - 1.0) * x * lam + fl * lam1);
                        // Q = -(e F1 + i b F2), U = -(b F1 - i e F2); F2 has the opposite parity
                        Q[pa][0][r] -= er * F1; Q[pa][1][r] -= ei * F1;
                        Q[pb][0][r] += bi * F2; Q[pb][1][r] -= br * F2;
                        U[pa][0][r] -= br * F1; U[pa][1][r] -= bi * F1;
                        U[pb][0][r] -= ei * F2; U[pb][1][r] += er * F2;
                    }
                }
            }
            for (int r = 0; r < B.n; ++r) {
                const int pr = B.pr[r], south = P.nring - 1 - pr;
                auto put = [&](Phases& o, double (&A)[2][2][RB]) {
                    o.re[(long long)pr * (L + 1) + m] = A[0][0][r] + A[1][0][r];
                    o.im[(long long)pr * (L + 1) + m] = A[0][1][r] + A[1][1][r];
                    if (south != pr) {
                        o.re[(long long)south * (L + 1) + m] = A[0][0][r] - A[1][0][r];
                        o.im[(long long)south * (L + 1) + m] = A[0][1][r] - A[1][1][r];
                    }
                };
                int c = 0;
                if (t0) put(ph[c++], T);
                if (s2) { put(ph[c], Q); put(ph[c + 1], U); }
            }
        }
    }
}

void synth_rings(const Plan& P, int ncomp, const Phases* ph, double* maps) {
    const int L = P.L;
    const long long npix = 12LL * P.N * P.N;
#pragma omp parallel
    {
        std::vector<cplx> a, work;
#pragma omp for schedule(dynamic, 4)
        for (int r = 0; r < P.nring; ++r) {
            const Ring& g = P.rings[r];
            const Fft& f = *P.ffts.at(g.nphi);
            for (int c = 0; c < ncomp; ++c) {
                a.assign(g.nphi, cplx(0, 0));
                for (int m = 0; m <= L; ++m) {
                    const long long q = (long long)r * (L + 1) + m;
                    const cplx G = cplx(ph[c].re[q], ph[c].im[q]) * std::polar(1.0, m * g.phi0) * (m ? 2.0 : 1.0);
                    a[m % g.nphi] += G;
                }
                f.run(a, true, work);
                for (int j = 0; j < g.nphi; ++j) maps[c * npix + g.start + j] = a[j].real();
            }
        }
    }
}

void anal_rings(const Plan& P, int ncomp, const double* maps, Phases* ph) {
    const int L = P.L;
    const long long npix = 12LL * P.N * P.N;
#pragma omp parallel
    {
        std::vector<cplx> a, work;
#pragma omp for schedule(dynamic, 4)
        for (int r = 0; r < P.nring; ++r) {
            const Ring& g = P.rings[r];
            const Fft& f = *P.ffts.at(g.nphi);
            for (int c = 0; c < ncomp; ++c) {
                a.resize(g.nphi);
                for (int j = 0; j < g.nphi; ++j) a[j] = cplx(maps[c * npix + g.start + j], 0.0);
                f.run(a, false, work);
                for (int m = 0; m <= L; ++m) {
                    const cplx v = a[m % g.nphi] * std::polar(1.0, -m * g.phi0);
                    ph[c].re[(long long)r * (L + 1) + m] = v.real();
                    ph[c].im[(long long)r * (L + 1) + m] = v.imag();
                }
            }
        }
    }
}

void anal_legendre(const Plan& P, int comps, const Phases* ph, double* alm) {
    const int L = P.L;
    const long long nlm = P.nlm();
    const bool t0 = comps & 1, s2 = comps & 2;
    double* aT = alm;
    double* aE = alm + (t0 ? 2 * nlm : 0);
    double* aB = aE + 2 * nlm;
    const double w = 4.0 * PI / (12.0 * P.N * P.N);
    const std::vector<Block> blocks = blocks_of(P);
#pragma omp parallel
    {
        std::vector<double> acc;                       // per l: T re/im, E re/im, B re/im
#pragma omp for schedule(dynamic, 1)
        for (int mm = 0; mm <= L; ++mm) {
            const int m = (mm & 1) ? L - mm / 2 : mm / 2;
            const MCoef k = coef_m(L, m);
            acc.assign(6 * (size_t)(L + 1), 0.0);
            for (const Block& B : blocks) {
                // per lane: [parity][re/im] sums (0: north + south, 1: north - south), zero on dead lanes
                double T[2][2][RB] = {}, Q[2][2][RB] = {}, U[2][2][RB] = {};
                for (int r = 0; r < B.n; ++r) {
                    const int pr = B.pr[r], south = P.nring - 1 - pr;
                    const bool pair = south != pr;
                    auto get = [&](const Phases& o, double (&A)[2][2][RB]) {
                        const long long qn = (long long)pr * (L + 1) + m, qs = (long long)south * (L + 1) + m;
                        const double nr = o.re[qn], ni = o.im[qn];
                        const double sr = pair ? o.re[qs] : 0.0, si = pair ? o.im[qs] : 0.0;
                        A[0][0][r] = nr + sr; A[0][1][r] = ni + si;
                        A[1][0][r] = nr - sr; A[1][1][r] = ni - si;
                    };
                    int c = 0;
                    if (t0) get(ph[c++], T);
                    if (s2) { get(ph[c], Q); get(ph[c + 1], U); }
                }
                Walker wk;
                wk.start(k, m, B);
                for (int l = m; l <= L; ++l) {
                    if (l == m + 1) wk.step_first(m, B);
                    else if (l > m + 1) wk.step(k, l, B);
                    if (!wk.values()) continue;
                    const int pa = (l + m) & 1, pb = pa ^ 1;
                    double* o = acc.data() + 6 * (size_t)l;
                    if (t0) {
                        double sr = 0, si = 0;
                        for (int r = 0; r < RB; ++r) { sr += wk.lam[r] * T[pa][0][r]; si += wk.lam[r] * T[pa][1][r]; }
                        o[0] += sr; o[1] += si;
                    }
                    if (s2 && l >= 2) {
                        const double cl = k.c[l], fl = k.f[l], lm2 = (double)l - (double)m * m, h = 0.5 * l * (l - 1.0);
                        double er = 0, ei = 0, br = 0, bi = 0;
                        for (int r = 0; r < RB; ++r) {
                            const double x = B.x[r], is2 = B.is2[r], lam = wk.lam[r], lam1 = wk.lam1[r];
                            const double F1 = cl * (-(lm2 * is2 + h) * lam + fl * x * is2 * lam1);
                            const double F2 = cl * m * is2 * (-(l - 1.0) * x * lam + fl * lam1);
                            // a_E = -(F1 Q + i F2 U), a_B = -(F1 U - i F2 Q)
                            er += -F1 * Q[pa][0][r] + F2 * U[pb][1][r];
                            ei += -F1 * Q[pa][1][r] - F2 * U[pb][0][r];
                            br += -F1 * U[pa][0][r] - F2 * Q[pb][1][r];
                            bi += -F1 * U[pa][1][r] + F2 * Q[pb][0][r];
                        }
                        o[2] += er; o[3] += ei; o[4] += br; o[5] += bi;
                    }
                }
            }
            for (int l = m; l <= L; ++l) {
                const long long i = 2 * P.idx(l, m);
                const double* o = acc.data() + 6 * (size_t)l;
                if (t0) { aT[i] = w * o[0]; aT[i + 1] = w * o[1]; }
                if (s2) { aE[i] = w * o[2]; aE[i + 1] = w * o[3]; aB[i] = w * o[4]; aB[i + 1] = w * o[5]; }
            }
        }
    }
}

int ncomp_of(int comps) { return (comps & 1 ? 1 : 0) + (comps & 2 ? 2 : 0); }

void alm2map_impl(const Plan& P, int comps, const double* alm, double* maps) {
    const int nc = ncomp_of(comps);
    std::vector<Phases> ph(nc, Phases((size_t)P.nring * (P.L + 1)));
    synth_legendre(P, comps, alm, ph.data());
    synth_rings(P, nc, ph.data(), maps);
}

void map2alm_adj(const Plan& P, int comps, const double* maps, double* alm) {
    const int nc = ncomp_of(comps);
    std::vector<Phases> ph(nc, Phases((size_t)P.nring * (P.L + 1)));
    anal_rings(P, nc, maps, ph.data());
    anal_legendre(P, comps, ph.data(), alm);
}

}  // namespace

extern "C" {

// maps [ncomp][12 N^2]; alm [ncomp][nlm] complex interleaved; comps 1 T, 2 EB, 3 TEB
int shtc_alm2map(int nside, int lmax, int comps, const double* alm, double* maps, int nthreads) {
    if (nside < 1 || lmax < 0 || comps < 1 || comps > 3 || !alm || !maps) return -1;
    if (nthreads > 0) omp_set_num_threads(nthreads);
    Plan P(nside, lmax);
    alm2map_impl(P, comps, alm, maps);
    return 0;
}

// healpy map2alm(iter): a = A^+ m, then iter Jacobi steps a += A^+ (m - A a)
int shtc_map2alm(int nside, int lmax, int comps, const double* maps, double* alm, int iter, int nthreads) {
    if (nside < 1 || lmax < 0 || comps < 1 || comps > 3 || !alm || !maps || iter < 0) return -1;
    if (nthreads > 0) omp_set_num_threads(nthreads);
    Plan P(nside, lmax);
    const int nc = ncomp_of(comps);
    const long long npix = 12LL * nside * nside, n2 = 2 * P.nlm() * nc;
    map2alm_adj(P, comps, maps, alm);
    if (iter > 0) {
        std::vector<double> resid((size_t)nc * npix), da((size_t)n2);
        for (int it = 0; it < iter; ++it) {
            alm2map_impl(P, comps, alm, resid.data());
            for (long long q = 0; q < (long long)nc * npix; ++q) resid[q] = maps[q] - resid[q];
            map2alm_adj(P, comps, resid.data(), da.data());
            for (long long q = 0; q < n2; ++q) alm[q] += da[q];
        }
    }
    return 0;
}

}  // extern "C"
