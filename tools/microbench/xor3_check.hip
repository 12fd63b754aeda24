#include <hip/hip_runtime.h>
#define GS_XOR3
#include "../../gibbssampler_amd/csrc/gs_rng.h"
__global__ void k(uint32_t* out) { uint4 w = gs::philox(threadIdx.x, 0, 0, 0, gs::Key{0, 0}); out[4*threadIdx.x] = w.x; out[4*threadIdx.x+1] = w.y; out[4*threadIdx.x+2] = w.z; out[4*threadIdx.x+3] = w.w; }
extern "C" int run(uint32_t* out) { hipLaunchKernelGGL(k, 1, 64, 0, 0, out); return hipDeviceSynchronize(); }
