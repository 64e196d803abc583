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
// Compute units of the calling thread's current device (hipDeviceProp_t::multiProcessorCount, cached per device);
// 256 on a whole MI355X, fewer on a partitioned one.  Grid-shape rules use it instead of a constant.
int device_cus();
// Workgroup cap for the row-streaming kernels (split_f16, LayerNorm, lattice prologue) on this host thread
// (hfa_set_grid_cap; 0 = none): a capped launch runs its rows in a grid-stride loop over at most this many
// workgroups.  task.submit caps the side pass's launches, whose tens of thousands of one-row workgroups otherwise
// cost the encoder beside them more than their work (profiles/r06/side_cost_decomposition.txt).
int grid_cap();
inline int capped(long long want) {
    const int cap = grid_cap();
    return (int)(cap > 0 && want > cap ? cap : want);
}

inline int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: launch failed: %s", what, hipGetErrorString(e));
        return -(int)e;
    }
    return HFA_OK;
}

constexpr int kWave = 64;

// ---- LDS-DMA (buffer_load_dwordx4 ... lds): one wave-instruction copies 64 x 16 B from per-lane byte offsets
// into 1 KiB of LDS at a wave-uniform address (lane-linear).  An offset past the descriptor's num_records reads
// zeros (scripts/probes/dma_oob.hip).  Completion is tracked only by vmcnt: wait_vm_barrier<N> then read.
__device__ __forceinline__ unsigned lds_addr(const void* ptr) {
    return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)ptr;
}

__device__ __forceinline__ void dma16(unsigned voff, __amdgpu_buffer_rsrc_t rsrc, unsigned soff, unsigned lds) {
    // M0 is compiler-reserved: set and restore it inside the statement that uses it.  soff / lds are wave-uniform;
    // readfirstlane states it where the divergence analysis cannot prove it
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(rsrc), "s"(__builtin_amdgcn_readfirstlane(soff)),
                   "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm_barrier() {
    // this wave's DMAs except the newest N landed, its LDS reads retired, then every wave of the block
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" :: "i"(N) : "memory");
}

constexpr unsigned DMA_OOB = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

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

// Branch-free erf: the two ranges of ROCm's device erff (|x| < 1: odd polynomial in x^2; |x| >= 1:
// 1 - exp(-q(|x|))) are both evaluated with the same constants and fma order and then selected, so the
// result is bit-identical to erff (tests/test_kernels_gpu.py) while lanes of a wave never diverge.
__device__ __forceinline__ float erf_nb(float x) {
    const float ax = fabsf(x);
    const float t = x * x;
    float s = fmaf(t, __uint_as_float(0xba1345e1u), __uint_as_float(0x3ba10414u));
    s = fmaf(t, s, __uint_as_float(0xbcdac9b8u));
    s = fmaf(t, s, __uint_as_float(0x3de703beu));
    s = fmaf(t, s, __uint_as_float(0xbec09330u));
    s = fmaf(t, s, __uint_as_float(0x3e0375d0u));
    s = fmaf(ax, s, ax);
    float q = fmaf(ax, __uint_as_float(0x378e98abu), __uint_as_float(0xb9c68948u));
    q = fmaf(ax, q, __uint_as_float(0x3b7cd369u));
    q = fmaf(ax, q, __uint_as_float(0xbcc618b2u));
    q = fmaf(ax, q, __uint_as_float(0x3dda74e4u));
    q = fmaf(ax, q, __uint_as_float(0x3f228afdu));
    q = fmaf(ax, q, __uint_as_float(0x3e03c728u));
    q = fmaf(ax, q, ax);
    const float l = 1.0f - expf(-q);
    return copysignf(ax < 1.0f ? s : l, x);
}

// erf-GELU as torch's default F.gelu / HF ACT2FN["gelu"]: 0.5 x (1 + erf(x / sqrt 2)), with the device erff
// (two-range, ~32 VALU ops).  Kept as the bit-exact reference of gelu_fast's self-test.
__device__ __forceinline__ float gelu_erf(float x) {
    return 0.5f * x * (1.0f + erf_nb(x * 0.70710678118654752440f));
}

// Low planes of two values whose high planes h (f16 pair, from one v_cvt_pk_f16_f32) are known: f16(2^11 v - 2^11 h)
// for each half, as two v_fma_mix ops that read h's halves in place (the compiler re-converts each value to a
// scalar f16 first).  x2048 = 2^11 v (exact); the fma is exact (|v - h| <= half an f16 ulp of v), so its one
// rounding to f16 equals the round-1 form f16((v - f32(h)) * 2^11) bit for bit.  c2048 = 2048.0f in a register
// (gfx9 VOP3P takes no literal).
__device__ __forceinline__ unsigned split_lo_pair(unsigned h, float x2048_0, float x2048_1, float c2048) {
    unsigned r;
    asm("v_fma_mixlo_f16 %0, -%1, %4, %2 op_sel_hi:[1,0,0]\n\t"
                 "v_fma_mixhi_f16 %0, -%1, %4, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
                 : "=&v"(r)
                 : "v"(h), "v"(x2048_0), "v"(x2048_1), "v"(c2048));
    return r;
}

typedef _Float16 h2v __attribute__((ext_vector_type(2)));
typedef float f2v __attribute__((ext_vector_type(2)));

// Split-f16 planes of two f32 values (hi = f16(v), lo = f16((v - hi) 2^11), bit for bit the scalar form): one
// v_cvt_pk_f16_f32 and two v_fma_mix (split_lo_pair) instead of 2 x (cvt, cvt back, sub, mul, cvt).  nanacc: the
// planes' range check as one v_pk_fma_f16 per pair -- hi * 0 + acc turns an inf (|v| >= 65520) or NaN hi into a
// NaN that persists; test it once at the end (range_bad).
__device__ __forceinline__ void split_pair(float a, float b, unsigned& hi, unsigned& lo, h2v& nanacc, float c2048) {
    const h2v hp = __builtin_convertvector((f2v){a, b}, h2v);
    nanacc = hp * (h2v){(_Float16)0.0f, (_Float16)0.0f} + nanacc;
    hi = __builtin_bit_cast(unsigned, hp);
    lo = split_lo_pair(hi, a * 2048.0f, b * 2048.0f, c2048);
}
__device__ __forceinline__ bool range_bad(h2v nanacc) { return nanacc[0] != nanacc[0] || nanacc[1] != nanacc[1]; }

// The GELU of every fused epilogue.  With E = erfc(|x| / sqrt 2) = 1 - erf(|x| / sqrt 2):
//   GELU(x) = x - (x / 2) E for x >= 0 and (x / 2) E for x < 0, i.e. max(x, 0) - |x / 2| E  (one fma),
// and E = exp2(q(a)), a = min(|x|, 3.95 sqrt 2), q(a) = a R7(a) fitted to log2 erfc(a / sqrt 2) on [0, 3.95 sqrt 2]
// (erfc-weighted least squares toward minimax, scripts/fit_gelu_erf.py): 13 VALU ops (|x| and -|x/2| are source
// modifiers; one v_exp_f32), against 19 for the round-1 form 0.5 x (1 + sign(z)(1 - exp(-q))).  In f32 it is within
// 1.21 |x| 2^-24 of the f64 GELU everywhere (the f32 formula 0.5 x (1 + erf) with a correctly rounded erf: 1.7 |x|
// 2^-24, its cancellation floor) and within 4.9 ulp where x > -1.5 (scripts/fit_gelu_erf.py emulates it; degree 8
// buys only 1.19 / 4.0).  Past the clamp E stays erfc(3.95) = 1.9e-8, i.e. an error <= 1e-8 |x|, inside the same
// bound.  x = +inf gives NaN (the range flags catch both).
__device__ __forceinline__ float gelu_fast(float x) {
    const float a = fminf(fabsf(x), 5.58614357f);
    float q = __uint_as_float(0xb64b3c2au);
    q = fmaf(q, a, __uint_as_float(0x382ef466u));
    q = fmaf(q, a, __uint_as_float(0xb94eba72u));
    q = fmaf(q, a, __uint_as_float(0xb8e94e0eu));
    q = fmaf(q, a, __uint_as_float(0x3be669ecu));
    q = fmaf(q, a, __uint_as_float(0xbd56f121u));
    q = fmaf(q, a, __uint_as_float(0xbeeb1e17u));
    q = fmaf(q, a, __uint_as_float(0xbf935766u));
    const float e = __builtin_amdgcn_exp2f(a * q);
    return fmaf(-fabsf(0.5f * x), e, fmaxf(x, 0.0f));
}


// torch Hardswish: x * relu6(x + 3) / 6.
__device__ __forceinline__ float hardswish(float x) {
    float r = fminf(fmaxf(x + 3.0f, 0.0f), 6.0f);
    return x * r / 6.0f;
}

}  // namespace hfa
