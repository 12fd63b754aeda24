#include <hip/hip_runtime.h>
#define GS_RSQ_SQRT
#include "../../gibbssampler_amd/csrc/gs_rng.h"
__global__ void k(const double* t, double* out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x; if (i >= n) return;
    out[2 * i] = gs::bm_sqrt(t[i]); out[2 * i + 1] = sqrt(t[i]);
}
extern "C" int run(const double* t, double* out, int n) { hipLaunchKernelGGL(k, (n + 255) / 256, 256, 0, 0, t, out, n); return hipDeviceSynchronize(); }
