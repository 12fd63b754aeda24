// Store-pattern micro-benchmark for the CR sweep's output stream (gfx950).
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef double dbl2u __attribute__((ext_vector_type(2), aligned(8)));
typedef double dbl2a __attribute__((ext_vector_type(2), aligned(16)));

// A: each lane one 16-B aligned store per iteration, wave = 1 KiB contiguous
template <bool NT>
__global__ void k_vec16(double* out, long long n2) {
    for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < n2; k += (long long)gridDim.x * blockDim.x) {
        dbl2a v; v.x = (double)k; v.y = (double)(k + 1);
        if (NT) __builtin_nontemporal_store(v, reinterpret_cast<dbl2a*>(out) + k);
        else reinterpret_cast<dbl2a*>(out)[k] = v;
    }
}
// B: two 8-B stores per lane at 16-B stride (the sweep's (re, im) pattern)
template <bool NT>
__global__ void k_pair8(double* out, long long n2) {
    for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < n2; k += (long long)gridDim.x * blockDim.x) {
        if (NT) { __builtin_nontemporal_store((double)k, out + 2 * k); __builtin_nontemporal_store((double)k + 1, out + 2 * k + 1); }
        else { out[2 * k] = (double)k; out[2 * k + 1] = (double)k + 1; }
    }
}
// C: misaligned 16-B stores (pair starts at an odd slot)
template <bool NT>
__global__ void k_vec16u(double* out, long long n2) {
    for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < n2 - 1; k += (long long)gridDim.x * blockDim.x) {
        dbl2u v; v.x = (double)k; v.y = (double)(k + 1);
        if (NT) __builtin_nontemporal_store(v, reinterpret_cast<dbl2u*>(out + 1 + 2 * k));
        else *reinterpret_cast<dbl2u*>(out + 1 + 2 * k) = v;
    }
}
// D: the sweep's access shape: rows of 128 doubles per wave, row stride S doubles,
// 3 fields NR apart, 8-B pair stores; grid of waves each doing `rows` rows
template <bool NT>
__global__ void k_rows(double* out, long long NR, int rows, long long stride) {
    const long long w = blockIdx.x * 4LL + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const long long base = (w / 8) * rows * stride + (w % 8) * 128;
    for (int m = 0; m < rows; ++m) {
        const long long r = base + m * stride + 2 * lane;
        for (int f = 0; f < 3; ++f) {
            if (NT) { __builtin_nontemporal_store(1.0 * m, out + f * NR + r); __builtin_nontemporal_store(2.0, out + f * NR + r + 1); }
            else { out[f * NR + r] = 1.0 * m; out[f * NR + r + 1] = 2.0; }
        }
    }
}

extern "C" int run(int which, int nt, double* out, long long n_doubles, int grid, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    const long long n2 = n_doubles / 2;
    switch (which) {
    case 0: if (nt) hipLaunchKernelGGL(k_vec16<true>, grid, 256, 0, s, out, n2); else hipLaunchKernelGGL(k_vec16<false>, grid, 256, 0, s, out, n2); break;
    case 1: if (nt) hipLaunchKernelGGL(k_pair8<true>, grid, 256, 0, s, out, n2); else hipLaunchKernelGGL(k_pair8<false>, grid, 256, 0, s, out, n2); break;
    case 2: if (nt) hipLaunchKernelGGL(k_vec16u<true>, grid, 256, 0, s, out, n2); else hipLaunchKernelGGL(k_vec16u<false>, grid, 256, 0, s, out, n2); break;
    case 3: {
        // 3 fields of NR = n/3 doubles; rows of 1024 doubles (8 waves x 128) stride 1024
        const long long NR = n_doubles / 3; const int rows = 64; const long long stride = 1024;
        const long long nw = NR / (rows * stride) * 8;
        if (nt) hipLaunchKernelGGL(k_rows<true>, (unsigned)(nw / 4), 256, 0, s, out, NR, rows, stride);
        else hipLaunchKernelGGL(k_rows<false>, (unsigned)(nw / 4), 256, 0, s, out, NR, rows, stride);
        break; }
    }
    return (int)hipGetLastError();
}
