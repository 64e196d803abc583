// hfa_common.h — shared helpers for the libhfa C-ABI (gfx950 / CDNA4 only).
//
// Error convention (SURVEY.md §8b "C-ABI the build must export"): every entry point returns int
// status, 0 = OK, negative = argument error (HFA_EINVAL) or -(hipError_t).  The message of the last
// failure on the calling thread is returned by hfa_last_error().  Calls are stream-ordered on the
// hipStream_t passed in, never synchronise, never allocate persistent memory and never free caller
// memory, so they are capturable into a hipGraph.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#define HFA_OK 0
#define HFA_EINVAL (-1000)

namespace hfa {

void set_error(const char* fmt, ...);

inline int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: launch failed: %s", what, hipGetErrorString(e));
        return -(int)e;
    }
    return HFA_OK;
}

constexpr int kWave = 64;

__device__ __forceinline__ float neg_inf() { return -__builtin_inff(); }

// Wave-wide reductions over 64 lanes (ds_swizzle/DPP via __shfl_xor).
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// erf-GELU exactly as torch's default F.gelu / HF ACT2FN["gelu"]: 0.5 x (1 + erf(x / sqrt 2)).
__device__ __forceinline__ float gelu_erf(float x) {
    return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f));
}

// torch Hardswish: x * relu6(x + 3) / 6.
__device__ __forceinline__ float hardswish(float x) {
    float r = fminf(fmaxf(x + 3.0f, 0.0f), 6.0f);
    return x * r / 6.0f;
}

}  // namespace hfa
