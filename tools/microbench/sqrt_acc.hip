#include <hip/hip_runtime.h>
// sqrt(t), t >= 0: hardware reciprocal square root (~2^-29 relative) and one
// Newton step (error ~2^-58), then r = t y; exact 0 at t = 0 (measured as a
// Box-Muller radius candidate in r01; the product sweep keeps sqrt())
__device__ __forceinline__ double rsq_sqrt(double t) {
    double y = __builtin_amdgcn_rsq(t);
    const double h = 0.5 * t;
    y = y * fma(-h * y, y, 1.5);
    return t > 0.0 ? t * y : 0.0;
}
__global__ void k(const double* t, double* out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x; if (i >= n) return;
    out[2 * i] = rsq_sqrt(t[i]); out[2 * i + 1] = sqrt(t[i]);
}
extern "C" int run(const double* t, double* out, int n) { hipLaunchKernelGGL(k, (n + 255) / 256, 256, 0, 0, t, out, n); return hipDeviceSynchronize(); }
