// Accuracy check of the custom Box-Muller math (bm_log, bm_sincos2pi) vs ocml.
#include "../../gibbssampler_amd/csrc/gs_rng.h"
__global__ void k(const double* u, double* out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x; if (i >= n) return;
    double s, c, s2, c2;
    gs::bm_sincos2pi(u[i], s, c);
    sincospi(2.0 * u[i], &s2, &c2);
    out[6 * i + 0] = gs::bm_log(u[i]); out[6 * i + 1] = log(u[i]);
    out[6 * i + 2] = s; out[6 * i + 3] = s2; out[6 * i + 4] = c; out[6 * i + 5] = c2;
}
extern "C" int run(const double* u, double* out, int n) { hipLaunchKernelGGL(k, (n + 255) / 256, 256, 0, 0, u, out, n); return hipDeviceSynchronize(); }
