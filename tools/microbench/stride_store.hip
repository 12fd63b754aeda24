// Write-stream locality micro-benchmark (gfx950): nw waves each issue R stores
// of 1 KB (16 B per lane, non-temporal); groups of G waves interleave their 1-KB
// chunks, so a wave's consecutive stores are G KB apart and the G waves of a
// group cover one dense region.  G = 1: each wave writes one contiguous run.
#include <hip/hip_runtime.h>
typedef double dbl2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void k_stride(double* out, int R, int G, int nt) {
    const long long w = blockIdx.x * 4LL + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const long long grp = w / G, wi = w % G;
    for (int k = 0; k < R; ++k) {
        const long long kb = grp * (long long)R * G + (long long)k * G + wi;   // 1-KB chunk index
        dbl2 v; v.x = (double)k; v.y = (double)w;
        dbl2* q = reinterpret_cast<dbl2*>(out + kb * 128) + lane;
        if (nt) __builtin_nontemporal_store(v, q); else *q = v;
    }
}
extern "C" int run(double* out, long long nkb, int R, int G, int nt, void* stream) {
    const long long nw = nkb / R;
    hipLaunchKernelGGL(k_stride, dim3((unsigned)(nw / 4)), dim3(256), 0, (hipStream_t)stream, out, R, G, nt);
    return (int)hipGetLastError();
}
