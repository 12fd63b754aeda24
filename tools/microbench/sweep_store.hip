// Store-only replica of the CR sweep's output stream (gfx950): the same task
// tiling (4 waves = 256 consecutive l, `tm` rows of m), the same XCD remap and
// the same addresses (F fields NR apart per chain, chains F*NR apart), with no
// compute.  `fstride` / `cstride` override the field / chain strides (doubles)
// to test whether the address pattern or the kernel shape limits the stream.
#include <hip/hip_runtime.h>
#include <stdint.h>
#if defined(PLAIN)
#define NTS(v, p) (*(p) = (v))
#else
#define NTS(v, p) __builtin_nontemporal_store(v, p)
#endif
typedef double dbl2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_store(int L, int nchains, int tm, const int2* __restrict__ tasks, double* s,
                                               long long fstride, long long cstride, int mode, int nitems) {
  // mode 0: one workgroup per item, XCD remap; 1: no remap; 2: persistent grid-stride (grid = gridDim.x)
  for (int item = blockIdx.x; item < nitems; item += (mode == 2 ? gridDim.x : nitems)) {
    int wg = item;
    if (mode == 0) {
        const int nwg = nitems, xcd = item & 7, q8 = nwg >> 3, r8 = nwg & 7;
        wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (item >> 3);
    }
    int pair = wg / nchains, chain = wg % nchains;
    const int lane = threadIdx.x & 63;
    int2 gc = tasks[pair];
    if (mode == 8) {           // per-workgroup table: (g, c, chain) triples
        const int3 e = reinterpret_cast<const int3*>(tasks)[wg];
        gc = make_int2(e.x, e.y); chain = e.z;
    }
    if (gc.x < 0) continue;
    const int ntile = (L + 64) / 64;
    const int t = 4 * gc.x + (threadIdx.x >> 6);
    if (t >= ntile) continue;
    const int lhi = L - 64 * t;
    const int m0 = gc.y * tm, m1 = min(m0 + tm, lhi + 1);
    const int ell_lo = lhi - 63, ell = ell_lo + lane;
    if (m0 >= m1 || ell_lo < 0 || m1 - 1 > ell_lo) continue;     // off-diagonal blocks only
    double* sc = s + (long long)chain * cstride;
    int m = m0 == 0 ? 1 : m0;
    long long i = (long long)m * (2 * L + 1 - m) / 2 + ell;
    for (; m < m1; ++m) {
        const long long r = 2 * i - (L + 1);
        if (mode == 7) {
            // segment of the workgroup: tiles 4g..4g+3 = l from lw = ell_lo(wave 3) to ell_hi(wave 0);
            // the lowest l of the segment is at tile 4g+3 -> wave 3, lane 0
            const int t3 = min(4 * gc.x + 3, ntile - 1);
            const int lseg = max(L - 64 * t3 - 63, 0);
            const long long iseg = (long long)m * (2 * L + 1 - m) / 2 + lseg;
            const int w = threadIdx.x >> 6;
            const int nseg = (L - 64 * 4 * gc.x) - lseg + 1;          // entries in the segment
#pragma unroll
            for (int f = 0; f < 3; ++f) {
                double* A = sc + f * fstride + 2 * iseg - (L + 1);
                const uintptr_t a = reinterpret_cast<uintptr_t>(A);
                double* A0 = reinterpret_cast<double*>(a & ~(uintptr_t)127);
                const uintptr_t aend = a + (uintptr_t)nseg * 16;
                // wave (3 - w) writes aligned KB number w of the segment (order irrelevant for timing)
                for (int kb = w; kb * 1024 < (int)(aend - (uintptr_t)A0); kb += 4) {
                    double* q = A0 + kb * 128 + 2 * lane;
                    const uintptr_t qa = reinterpret_cast<uintptr_t>(q);
                    if (qa >= a && qa + 16 <= aend) {
                        dbl2 v; v.x = (double)m; v.y = (double)f;
                        NTS(v, reinterpret_cast<dbl2*>(q));
                    } else if (qa + 8 == a || (qa < aend && qa + 16 > aend)) {
                        NTS((double)f, qa + 8 == a ? q + 1 : q);
                    }
                }
            }
            i += L - m;
            continue;
        }
#pragma unroll
        for (int f = 0; f < 3; ++f) {
            dbl2 v; v.x = (double)m; v.y = (double)f;
            double* q0 = mode == 3 ? s + ((((long long)item * 4 + (threadIdx.x >> 6)) * tm + (m - m0)) * 3 + f) * 128 + 2 * lane
                                  : mode == 4 ? s + (((long long)f * nitems * 4 + (long long)item * 4 + (threadIdx.x >> 6)) * tm + (m - m0)) * 128 + 2 * lane
                                  : sc + f * fstride + r;
            // mode 6: every wave store realigned to a 128-B line (timing experiment: wrong data)
            double* q = mode == 6 ? reinterpret_cast<double*>((reinterpret_cast<uintptr_t>(sc + f * fstride + r - 2 * lane) & ~(uintptr_t)127)) + 2 * lane
                      : mode == 5 ? reinterpret_cast<double*>(reinterpret_cast<uintptr_t>(sc + f * fstride + r) & ~(uintptr_t)15) : q0;
            NTS(v.x, q);
            NTS(v.y, q + 1);
        }
        i += L - m;
    }
  }
}

// full-row workgroups: 16 waves = tiles 0..15 (l = 1..L at L = 1024), one chunk of
// tm rows; lanes with l < m masked (diagonal), waves wholly below the chunk exit
__global__ __launch_bounds__(1024) void k_store_rows(int L, int nchains, int tm, double* s, int align) {
    const int nchunk = L / tm + 1;
    const int b = blockIdx.x;
    const int c = b / nchains, chain = b % nchains;     // consecutive blocks: chains of one chunk
    const int t = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int lhi = L - 64 * t, ell = lhi - 63 + lane;
    const int m0 = max(c * tm, 1), m1 = min(c * tm + tm, L + 1);
    const long long NR = (long long)(L + 1) * (L + 1);
    double* sc = s + (long long)chain * 3 * NR;
    if (align == 2) {
        // flat write-out: the chunk's rows are one contiguous range per field; write it
        // as 128-B-aligned 1-KB blocks (partial lines only at the two chunk ends)
        const long long i0 = (long long)m0 * (2 * L + 1 - m0) / 2 + m0;             // (l = m0, m0)
        const long long i1 = (long long)m1 * (2 * L + 1 - m1) / 2 + m1;             // (l = m1, m1)
        for (int f = 0; f < 3; ++f) {
            const uintptr_t a = reinterpret_cast<uintptr_t>(sc + f * NR + 2 * i0 - (L + 1));
            const uintptr_t e = reinterpret_cast<uintptr_t>(sc + f * NR + 2 * i1 - (L + 1));
            const uintptr_t a0 = a & ~(uintptr_t)127;
            for (uintptr_t kb = a0 + (uintptr_t)t * 1024; kb < e; kb += 16 * 1024) {
                const uintptr_t qa = kb + (uintptr_t)lane * 16;
                if (qa >= a && qa + 16 <= e) {
                    typedef double d2 __attribute__((ext_vector_type(2)));
                    d2 v; v.x = (double)m0; v.y = (double)f;
                    NTS(v, reinterpret_cast<d2*>(qa));
                } else if (qa + 8 == a) {
                    NTS((double)f, reinterpret_cast<double*>(qa + 8));
                } else if (qa < e && qa + 16 > e) {
                    NTS((double)f, reinterpret_cast<double*>(qa));
                }
            }
        }
        return;
    }
    if (lhi < m0) return;
    long long i = (long long)m0 * (2 * L + 1 - m0) / 2 + ell;
    for (int m = m0; m < m1; ++m) {
        if (ell >= m) {
            const long long r = 2 * i - (L + 1);
#pragma unroll
            for (int f = 0; f < 3; ++f) {
                double* q = sc + f * NR + r;
                if (align) q = reinterpret_cast<double*>(reinterpret_cast<uintptr_t>(q) & ~(uintptr_t)15);
                NTS((double)m, q);
                NTS((double)f, q + 1);
            }
        }
        i += L - m;
    }
    (void)nchunk;
}

extern "C" int run_rows(int L, int nchains, int tm, double* s, int align, void* stream) {
    const int nchunk = L / tm + 1;
    hipLaunchKernelGGL(k_store_rows, dim3((unsigned)(nchunk * nchains)), dim3(1024), 0, (hipStream_t)stream, L, nchains,
                       tm, s, align);
    return (int)hipGetLastError();
}

extern "C" int run(int L, int nchains, int tm, const int2* tasks, int ntask, double* s, long long fstride,
                   long long cstride, int mode, int grid, void* stream) {
    const int nitems = mode == 8 ? ntask : ntask * nchains;
    hipLaunchKernelGGL(k_store, dim3((unsigned)(mode == 2 ? grid : nitems)), dim3(256), 0, (hipStream_t)stream, L,
                       nchains, tm, tasks, s, fstride, cstride, mode, nitems);
    return (int)hipGetLastError();
}
