// Calibration kernels for rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 with the
// CR sweep's access widths (8-byte loads/stores, lane pairs at 16-byte stride).
#include <hip/hip_runtime.h>
__global__ void k_read_pair8(const double* in, double* out, long long n2) {
    double acc = 0.0;
    for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < n2; k += (long long)gridDim.x * blockDim.x)
        acc += in[2 * k] * in[2 * k + 1];
    if (acc == 1.2345) out[0] = acc;   // keep the loads live, write nothing
}
__global__ void k_write_pair8(double* out, long long n2) {
    for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < n2; k += (long long)gridDim.x * blockDim.x) {
        __builtin_nontemporal_store((double)k, out + 2 * k);
        __builtin_nontemporal_store((double)k + 0.5, out + 2 * k + 1);
    }
}
extern "C" int run(int which, double* a, double* b, long long n, void* s) {
    if (which == 0) hipLaunchKernelGGL(k_read_pair8, 8192, 256, 0, (hipStream_t)s, a, b, n / 2);
    else hipLaunchKernelGGL(k_write_pair8, 8192, 256, 0, (hipStream_t)s, a, n / 2);
    return (int)hipStreamSynchronize((hipStream_t)s);
}
