// Issue-rate micro-benchmark (gfx950): cycles per wave-instruction of the VALU
// instruction classes in the CR sweep's loop (k_cr_sweep<3,0,false,0>), at 1, 2,
// 4 and 8 waves per SIMD, measured on the shader clock.
//
// Each kernel runs NCH = 8 independent chains per lane of one instruction (or an
// interleaved pair of two), no dependence between the chains inside an
// iteration.  An empty `asm volatile("" : "+v"(x))` after each operation keeps
// the compiler from folding or hoisting it (it emits no instruction); the
// instruction under test is the compiler's own (builtins, never asm text), so
// the hazard recognizer sees it as in the product kernels -- the r05 version
// issued v_bitop3 through inline asm, which the recognizer pads with s_nop.
// tools/microbench/valu_rate.py checks every kernel's loop in the ISA (the
// instruction count of the class under test) before trusting its number.
//
// Timing: every wave reads s_memtime (shader clock) and s_memrealtime (100 MHz)
// around its loop and its hardware slot (HW_ID: SIMD, CU, SH, SE; XCC_ID); the
// host groups waves by SIMD, so cycles per instruction = (last end - first
// start on that SIMD) / (waves on it x instructions per wave), independent of
// how the dispatcher spread the workgroups, and the clock = memtime ticks per
// realtime tick x 100 MHz.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define BAR(x) asm volatile("" : "+v"(x))

enum Op {
    OP_FMA_F64, OP_MUL_F64, OP_ADD_F64, OP_MIN_F64, OP_MAD_U64_U32, OP_BITOP3, OP_ADD_U32, OP_XOR_B32,
    OP_LSHR_B32, OP_CNDMASK, OP_ALIGNBIT, OP_BFE_U32, OP_MED3_I32, OP_LSHL_B64, OP_CVT_F64_U32, OP_CVT_I32_F64,
    OP_LDEXP_F64, OP_FREXP_MANT_F64, OP_RSQ_F64, OP_MUL_LO_U32,
    // interleaved pairs (one of each per chain and iteration)
    MIX_FMA_BITOP3, MIX_FMA_ADDU32, MIX_FMA_MAD64, MIX_BITOP3_MAD64, MIX_FMA_CVT,
    NOPS
};

template <int OP>
__device__ __forceinline__ void step(uint32_t (&a)[8], uint64_t (&p)[8], double (&d)[8], uint32_t b, uint32_t s,
                                     uint64_t q, double c1, const double c2, int e) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        if constexpr (OP == OP_FMA_F64) { d[k] = fma(d[k], c1, c2); BAR(d[k]); }
        else if constexpr (OP == OP_MUL_F64) { d[k] = d[k] * c1; BAR(d[k]); }
        else if constexpr (OP == OP_ADD_F64) { d[k] = d[k] + c1; BAR(d[k]); }
        else if constexpr (OP == OP_MIN_F64) { d[k] = fmin(d[k], c1); BAR(d[k]); }
        else if constexpr (OP == OP_MAD_U64_U32) { p[k] = (uint64_t)0xD2511F53u * (uint32_t)p[k] + q; BAR(p[k]); }
        else if constexpr (OP == OP_BITOP3) { a[k] = __builtin_amdgcn_bitop3_b32(a[k], b, a[(k + 1) & 7], 0x96); BAR(a[k]); }
        else if constexpr (OP == OP_ADD_U32) { a[k] = a[k] + b; BAR(a[k]); }
        else if constexpr (OP == OP_XOR_B32) { a[k] = a[k] ^ b; BAR(a[k]); }
        else if constexpr (OP == OP_LSHR_B32) { a[k] = a[k] >> s; BAR(a[k]); }
        else if constexpr (OP == OP_CNDMASK) { a[k] = (b & 1u) ? a[k] : s; BAR(a[k]); }
        else if constexpr (OP == OP_ALIGNBIT) { a[k] = __builtin_amdgcn_alignbit(a[k], b, 6); BAR(a[k]); }
        else if constexpr (OP == OP_BFE_U32) { a[k] = (a[k] >> 5) & 0x7FFFFu; BAR(a[k]); }
        else if constexpr (OP == OP_MED3_I32) { a[k] = (uint32_t)min(max((int)a[k], 0), 127); BAR(a[k]); }
        else if constexpr (OP == OP_LSHL_B64) { p[k] = p[k] << s; BAR(p[k]); }
        else if constexpr (OP == OP_CVT_F64_U32) { d[k] = (double)a[k]; BAR(d[k]); BAR(a[k]); }
        else if constexpr (OP == OP_CVT_I32_F64) { a[k] = (uint32_t)(int)d[k]; BAR(a[k]); BAR(d[k]); }
        else if constexpr (OP == OP_LDEXP_F64) { d[k] = ldexp(d[k], e); BAR(d[k]); }
        else if constexpr (OP == OP_FREXP_MANT_F64) { d[k] = __builtin_amdgcn_frexp_mant(d[k]); BAR(d[k]); }
        else if constexpr (OP == OP_RSQ_F64) { d[k] = __builtin_amdgcn_rsq(d[k]); BAR(d[k]); }
        else if constexpr (OP == OP_MUL_LO_U32) { a[k] = a[k] * 0xCD9E8D57u; BAR(a[k]); }
        else if constexpr (OP == MIX_FMA_BITOP3) {
            d[k] = fma(d[k], c1, c2); BAR(d[k]);
            a[k] = __builtin_amdgcn_bitop3_b32(a[k], b, a[(k + 1) & 7], 0x96); BAR(a[k]);
        } else if constexpr (OP == MIX_FMA_ADDU32) {
            d[k] = fma(d[k], c1, c2); BAR(d[k]);
            a[k] = a[k] + b; BAR(a[k]);
        } else if constexpr (OP == MIX_FMA_MAD64) {
            d[k] = fma(d[k], c1, c2); BAR(d[k]);
            p[k] = (uint64_t)0xD2511F53u * (uint32_t)p[k] + q; BAR(p[k]);
        } else if constexpr (OP == MIX_BITOP3_MAD64) {
            a[k] = __builtin_amdgcn_bitop3_b32(a[k], b, a[(k + 1) & 7], 0x96); BAR(a[k]);
            p[k] = (uint64_t)0xD2511F53u * (uint32_t)p[k] + q; BAR(p[k]);
        } else if constexpr (OP == MIX_FMA_CVT) {
            d[k] = fma(d[k], c1, c2); BAR(d[k]);
            double t = (double)a[k]; BAR(t); BAR(a[k]);
        }
    }
}

// rec[wave] = {memtime start, end, realtime start, end, hw_id, xcc_id}
template <int OP>
__global__ __launch_bounds__(256) void k_rate(uint64_t* __restrict__ rec, uint64_t* __restrict__ sink, int n,
                                              uint32_t s, int e, double c1) {
    uint32_t a[8]; uint64_t p[8]; double d[8];
    const uint32_t b = threadIdx.x * 0x9E3779B9u + 1u;
    const uint64_t q = (uint64_t)b << 7;
    const double c2 = 1e-9 * (double)(threadIdx.x & 7);
#pragma unroll
    for (int k = 0; k < 8; ++k) { a[k] = threadIdx.x * 7 + k; p[k] = a[k] * 3ull; d[k] = 1.0 + k * 1e-3; }
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < n; ++i) {
        step<OP>(a, p, d, b, s, q, c1, c2, e);
        step<OP>(a, p, d, b, s, q, c1, c2, e);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += p[k] + a[k] + (uint64_t)__double_as_longlong(d[k]);
    sink[blockIdx.x * 256 + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) {
        const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);    // HW_REG_HW_ID
        const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID
        uint64_t* o = rec + 6 * (size_t)w;
        o[0] = t0; o[1] = t1; o[2] = r0; o[3] = r1; o[4] = hw; o[5] = xcc;
    }
}

template <int OP>
static void launch(int nblk, uint64_t* rec, uint64_t* sink, int n, hipStream_t st) {
    hipLaunchKernelGGL(k_rate<OP>, dim3(nblk), dim3(256), 0, st, rec, sink, n, 5u, 3, 1.0000001);
}

template <int... OPS>
static void dispatch(int op, int nblk, uint64_t* rec, uint64_t* sink, int n, hipStream_t st,
                     std::integer_sequence<int, OPS...>) {
    ((op == OPS ? launch<OPS>(nblk, rec, sink, n, st) : void()), ...);
}

extern "C" int valu_rate_nops() { return NOPS; }

extern "C" int valu_rate_run(int op, uint64_t* rec, uint64_t* sink, int nblk, int n, void* stream) {
    if (op < 0 || op >= NOPS || nblk <= 0 || n <= 0) return -1;
    dispatch(op, nblk, rec, sink, n, (hipStream_t)stream, std::make_integer_sequence<int, NOPS>{});
    return (int)hipGetLastError();
}
