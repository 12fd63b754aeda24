// Issue-rate micro-benchmark (gfx950): cycles per wave-instruction of
// v_mad_u64_u32, v_fma_f64, v_mul_lo_u32 and v_bitop3_b32, 8 independent chains per lane.
#include <hip/hip_runtime.h>
#include <stdint.h>
template <int OP>
__global__ __launch_bounds__(256) void k_rate(uint64_t* out, int n) {
    uint32_t a[8]; uint64_t p[8]; double d[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { a[k] = threadIdx.x * 7 + k; p[k] = a[k]; d[k] = 1.0 + k * 1e-3; }
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if constexpr (OP == 0) { p[k] = (uint64_t)0xD2511F53u * (uint32_t)p[k] + (p[k] >> 32); }
            else if constexpr (OP == 1) { d[k] = fma(d[k], 1.0000001, 1e-9); }
            else if constexpr (OP == 2) { a[k] = a[k] * 0xCD9E8D57u + 1u; }
            else { uint32_t r; asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a[k]), "v"(a[(k + 1) & 7]), "v"(a[(k + 2) & 7])); a[k] = r; }
        }
    }
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += p[k] + a[k] + (uint64_t)d[k];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
extern "C" int run(int op, uint64_t* out, int nblk, int n, void* st) {
    hipStream_t s = (hipStream_t)st;
    if (op == 0) hipLaunchKernelGGL(k_rate<0>, dim3(nblk), dim3(256), 0, s, out, n);
    else if (op == 1) hipLaunchKernelGGL(k_rate<1>, dim3(nblk), dim3(256), 0, s, out, n);
    else if (op == 2) hipLaunchKernelGGL(k_rate<2>, dim3(nblk), dim3(256), 0, s, out, n);
    else hipLaunchKernelGGL(k_rate<3>, dim3(nblk), dim3(256), 0, s, out, n);
    return (int)hipGetLastError();
}
