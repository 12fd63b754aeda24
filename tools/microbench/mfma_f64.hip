// Throughput of v_mfma_f64_16x16x4_f64 on gfx950 (tools/microbench/mfma_f64.py):
// each wave issues n x 4 independent MFMAs (4 accumulators); mode 1 adds 8
// independent v_fma_f64 per MFMA (VALU beside the matrix pipe, same wave).
#include <hip/hip_runtime.h>
typedef double f64x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_mfma(double* out, int n, int mode) {
    const double a = threadIdx.x * 1e-3, b = blockIdx.x * 1e-4;
    f64x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    double v[8];
    for (int i = 0; i < 8; ++i) v[i] = a + i;
    for (int i = 0; i < n; ++i) {
        c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, b, c3, 0, 0, 0);
        if (mode == 1) {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = fma(v[j], a, b);
        }
    }
    double s = c0[0] + c1[1] + c2[2] + c3[3];
    for (int i = 0; i < 8; ++i) s += v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
extern "C" void run(int mode, double* out, int nblk, int n, void* stream) {
    hipLaunchKernelGGL(k_mfma, dim3(nblk), dim3(256), 0, (hipStream_t)stream, out, n, mode);
}
