// conv.hip — the first layer of the Hubert CNN feature extractor (C_in = 1, k = 10, stride 5, 512 channels).
//
// Replaces FeatureExtractor conv0 + GroupNorm(512, 512) + GELU (networks/hubert/model.py:98-99,108; HF
// HubertGroupNormConvLayer) and, for the LN-conv (large) variant, the raw conv0 (+bias) that feeds a
// LayerNorm+GELU (HF HubertLayerNormConvLayer).  conv1..6 are dense contractions and go through the MFMA
// implicit GEMM (gemm.hip).
//
// conv0 does 10 MACs per output and writes 512 f32 channels per output frame (~65 MB per 10 s utterance):
// it is HBM-store bound.  GroupNorm(512, 512) normalises each channel over ALL T, so the statistics need a
// full pass before any output can be written.  Recomputing conv0 (10 FMAs) is far cheaper than writing and
// re-reading 65 MB, so:
//   pass 1 (stats):  conv0 on the fly, per-chunk per-channel f64 sum / sum-of-squares partials (no output);
//   pass 2 (reduce): mean / rstd per (batch, channel);
//   pass 3 (apply):  conv0 again, normalise, GELU, channels-last split-plane store [B, T0, 512] that conv1's
//                    implicit GEMM reads directly.  Split-plane output (the encoder's default path): the conv on
//                    the f16 MFMA with the three split products packed in one K step (conv0_packed_kernel); f32
//                    output: the explicit fmaf chain on the VALU (conv0_apply_kernel).
// (Since round 3 passes 1-2 are the lag-product statistics below; the conv re-run is hfa_conv0_tuning mode 1.)
#include "hfa_common.h"

namespace {

constexpr int C0 = 512;        // channels
constexpr int KW = 10;         // kernel width
constexpr int ST = 5;          // stride
constexpr int CH = 256;        // output frames per chunk
constexpr int NT = 256;        // threads: 2 channels per thread

__device__ __forceinline__ float conv10(const float* w, const float* xs) {
    float v = 0.0f;
#pragma unroll
    for (int j = 0; j < KW; ++j) v = fmaf(w[j], xs[j], v);
    return v;
}

__device__ __forceinline__ void stage_chunk(float* xs, const float* xb, int t0, int nt, int N) {
    const int n = nt * ST + (KW - ST);
    for (int i = threadIdx.x; i < n; i += NT) {
        const int idx = t0 * ST + i;
        xs[i] = idx < N ? xb[idx] : 0.0f;
    }
}

__global__ __launch_bounds__(NT) void conv0_stats_kernel(int N, int T0, const float* __restrict__ x, long long x_bs,
                                                         const float* __restrict__ w0, double* __restrict__ part,
                                                         const int32_t* __restrict__ t0_len) {
    __shared__ float xs[CH * ST + KW];
    const int b = blockIdx.y, chunk = blockIdx.x;
    const int t0 = chunk * CH;
    const int T0b = t0_len ? t0_len[b] : T0;       // a variable-length batch: statistics over this row's frames
    const int nt = max(0, min(CH, T0b - t0));
    stage_chunk(xs, x + b * x_bs, t0, nt, N);
    const int c0 = threadIdx.x * 2;
    float wa[KW], wb[KW];
#pragma unroll
    for (int j = 0; j < KW; ++j) {
        wa[j] = w0[c0 * KW + j];
        wb[j] = w0[(c0 + 1) * KW + j];
    }
    __syncthreads();
    double sa = 0.0, qa = 0.0, sb = 0.0, qb = 0.0;
    for (int t = 0; t < nt; ++t) {
        const float va = conv10(wa, xs + t * ST);
        const float vb = conv10(wb, xs + t * ST);
        sa += va; qa += (double)va * va;
        sb += vb; qb += (double)vb * vb;
    }
    double* pp = part + ((size_t)(b * gridDim.x + chunk) * C0 + c0) * 2;
    pp[0] = sa; pp[1] = qa; pp[2] = sb; pp[3] = qb;
}

// One block per (64 channels, batch row): 4 partitions of the chunks per channel summed in parallel, then combined
// in a fixed order (deterministic, independent of the batch it runs in).
__global__ __launch_bounds__(NT) void conv0_reduce_kernel(int T0, int nchunk, const double* __restrict__ part,
                                                          float eps, float* __restrict__ stats,
                                                          const int32_t* __restrict__ t0_len) {
    const int b = blockIdx.y;
    const int c = blockIdx.x * 64 + (threadIdx.x & 63), q4 = threadIdx.x >> 6;
    if (t0_len) T0 = t0_len[b];
    double s = 0.0, q = 0.0;
    for (int k = q4; k < nchunk; k += 4) {
        const double* pp = part + ((size_t)(b * nchunk + k) * C0 + c) * 2;
        s += pp[0];
        q += pp[1];
    }
    __shared__ double red[2][4][64];
    red[0][q4][threadIdx.x & 63] = s;
    red[1][q4][threadIdx.x & 63] = q;
    __syncthreads();
    if (q4 == 0) {
        const int l = threadIdx.x;
        s = (red[0][0][l] + red[0][1][l]) + (red[0][2][l] + red[0][3][l]);
        q = (red[1][0][l] + red[1][1][l]) + (red[1][2][l] + red[1][3][l]);
        const double mean = s / T0;
        double var = q / T0 - mean * mean;
        if (var < 0) var = 0;
        stats[(b * C0 + c) * 2] = (float)mean;
        stats[(b * C0 + c) * 2 + 1] = (float)(1.0 / sqrt(var + (double)eps));
    }
}

// ---- GroupNorm(512, 512) statistics from the wave's lag products (the default; conv0_stats_kernel with mode 1) ----
// conv0 has one input channel and no bias here, so a channel's statistics over the frames are forms in its 10 taps:
// sum_t v_c(t) = w_c . S and sum_t v_c(t)^2 = w_c^T G w_c with S_j = sum_t x[5t + j], G_jk = sum_t x[5t + j] x[5t + k]
// -- 10 + 55 numbers per utterance instead of re-running the 512-channel conv.  f64 throughout (the products of two
// f32 are exact in f64): the statistics of the exact conv outputs, where the conv pass summed them after their f32
// rounding (relative differences ~1e-16 in the sums; the f32 mean / rstd agree to the last bit or one ulp).
constexpr int GCH = 4096;      // frames per block of the lag-product pass (8 blocks per 10 s row)
constexpr int NGR = 65;        // 10 sums + 55 products
__global__ __launch_bounds__(256) void conv0_gram_kernel(int T0, const float* __restrict__ x, long long x_bs,
                                                         double* __restrict__ part, const int32_t* __restrict__ t0_len) {
    const int b = blockIdx.y, chunk = blockIdx.x;
    const int T0b = t0_len ? t0_len[b] : T0;
    const float* xb = x + b * x_bs;
    double acc[NGR];
#pragma unroll
    for (int i = 0; i < NGR; ++i) acc[i] = 0.0;
    for (int k = 0; k < GCH / 256; ++k) {
        const int t = chunk * GCH + k * 256 + threadIdx.x;
        if (t < T0b) {                                  // frame t reads x[5t .. 5t + 9], inside the row
            double xv[KW];
#pragma unroll
            for (int j = 0; j < KW; ++j) xv[j] = (double)xb[(long long)t * ST + j];
            int q = 0;
#pragma unroll
            for (int j = 0; j < KW; ++j) acc[q++] += xv[j];
#pragma unroll
            for (int j = 0; j < KW; ++j)
#pragma unroll
                for (int i = j; i < KW; ++i, ++q) acc[q] = fma(xv[j], xv[i], acc[q]);
        }
    }
    __shared__ double red[4][NGR];                      // fixed order: lane butterfly, then the 4 waves in order
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < NGR; ++i) {
        const double v = hfa::wave_sum_d(acc[i]);
        if (lane == 0) red[wave][i] = v;
    }
    __syncthreads();
    if (threadIdx.x < NGR) {
        const int i = threadIdx.x;
        part[((size_t)b * gridDim.x + chunk) * NGR + i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
    }
}

// One block of 512 threads (one per channel) per batch row: the chunk partials summed in order, then each channel's
// mean and rstd from its taps.
__global__ __launch_bounds__(C0) void conv0_gram_stats_kernel(int T0, int nchunk, const double* __restrict__ part,
                                                              const float* __restrict__ w0, float eps,
                                                              float* __restrict__ stats,
                                                              const int32_t* __restrict__ t0_len) {
    const int b = blockIdx.x, c = threadIdx.x;
    __shared__ double sg[NGR];
    if (c < NGR) {
        double s = 0.0;
        for (int k = 0; k < nchunk; ++k) s += part[((size_t)b * nchunk + k) * NGR + c];
        sg[c] = s;
    }
    __syncthreads();
    const int T = t0_len ? t0_len[b] : T0;
    double w[KW];
#pragma unroll
    for (int j = 0; j < KW; ++j) w[j] = (double)w0[c * KW + j];
    double s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int j = 0; j < KW; ++j) s1 = fma(w[j], sg[j], s1);
    int q = KW;
#pragma unroll
    for (int j = 0; j < KW; ++j)
#pragma unroll
        for (int i = j; i < KW; ++i, ++q) s2 += (i == j ? 1.0 : 2.0) * (w[j] * w[i]) * sg[q];
    const double mean = s1 / T;
    double var = s2 / T - mean * mean;
    if (var < 0) var = 0;
    stats[(b * C0 + c) * 2] = (float)mean;
    stats[(b * C0 + c) * 2 + 1] = (float)(1.0 / sqrt(var + (double)eps));
}

// mode 0: GroupNorm(stats) + affine + GELU; mode 1: + bias, no norm, no act (LN variant feeds a LayerNorm).
// OUTS: write the output as split-f16 planes (gemm.hip gemm_split_kernel operand: hi = f16(v), lo = f16((v - hi)
// * 2^11), plane 1 at +y_sp halves) instead of f32 — the same bytes, and conv1 then runs on the f16 MFMA.
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int MODE, bool OUTS>
__global__ __launch_bounds__(NT) void conv0_apply_kernel(int N, int T0, const float* __restrict__ x, long long x_bs,
                                                         const float* __restrict__ w0, const float* __restrict__ stats,
                                                         const float* __restrict__ gamma, const float* __restrict__ beta,
                                                         const float* __restrict__ bias, void* __restrict__ yv,
                                                         long long y_bs, long long y_sp, int* __restrict__ oflow) {
    __shared__ float xs[CH * ST + KW];
    const int b = blockIdx.y, chunk = blockIdx.x;
    const int t0 = chunk * CH;
    const int nt = min(CH, T0 - t0);
    stage_chunk(xs, x + b * x_bs, t0, nt, N);
    const int c0 = threadIdx.x * 2;
    float wa[KW], wb[KW];
#pragma unroll
    for (int j = 0; j < KW; ++j) {
        wa[j] = w0[c0 * KW + j];
        wb[j] = w0[(c0 + 1) * KW + j];
    }
    float sa = 1.f, ha = 0.f, sb = 1.f, hb = 0.f;
    float ma = 0.f, ra = 1.f, mb = 0.f, rb = 1.f;
    if (MODE == 0) {
        ma = stats[(b * C0 + c0) * 2]; ra = stats[(b * C0 + c0) * 2 + 1];
        mb = stats[(b * C0 + c0 + 1) * 2]; rb = stats[(b * C0 + c0 + 1) * 2 + 1];
        sa = ra * gamma[c0]; ha = beta[c0]; sb = rb * gamma[c0 + 1]; hb = beta[c0 + 1];   // rstd * gamma folded
    } else {
        ha = bias ? bias[c0] : 0.f;
        hb = bias ? bias[c0 + 1] : 0.f;
    }
    __syncthreads();
    float* yb = reinterpret_cast<float*>(yv) + b * y_bs + (long long)t0 * C0 + c0;
    _Float16* yh = reinterpret_cast<_Float16*>(yv) + b * y_bs + (long long)t0 * C0 + c0;
    bool bad = false;
    for (int t = 0; t < nt; ++t) {
        float va = conv10(wa, xs + t * ST);
        float vb = conv10(wb, xs + t * ST);
        if (MODE == 0) {
            va = hfa::gelu_fast((va - ma) * sa + ha);
            vb = hfa::gelu_fast((vb - mb) * sb + hb);
        } else {
            va += ha;
            vb += hb;
        }
        if constexpr (OUTS) {
            asm volatile("" : "+v"(va), "+v"(vb));   // split the rounded f32 values (no multiply-into-cvt fusion)
            bad |= !(__builtin_fabsf(va) < 65504.0f) || !(__builtin_fabsf(vb) < 65504.0f);
            f16x2 v1, v2;
            v1[0] = (_Float16)va;
            v1[1] = (_Float16)vb;
            v2[0] = (_Float16)((va - (float)v1[0]) * 2048.0f);
            v2[1] = (_Float16)((vb - (float)v1[1]) * 2048.0f);
            *reinterpret_cast<f16x2*>(yh + (long long)t * C0) = v1;
            *reinterpret_cast<f16x2*>(yh + (long long)t * C0 + y_sp) = v2;
        } else {
            *reinterpret_cast<float2*>(yb + (long long)t * C0) = make_float2(va, vb);
        }
    }
    if (OUTS && bad && oflow) *oflow = 1;
}

// Split-plane output with 8 channels per lane: a wave stores one frame's 512 channels as 16-B pieces per plane
// (1 KiB per wave-instruction instead of 256 B); 4 frames in flight per block.  Per element the same scalar
// operations in the same order as conv0_apply_kernel<MODE, true> (bit-identical outputs).  No packed-f32 math
// (Makefile NO_PK_F32).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

template <int MODE>
__global__ __launch_bounds__(NT) void conv0_apply8_kernel(int N, int T0, const float* __restrict__ x, long long x_bs,
                                                          const float* __restrict__ w0, const float* __restrict__ stats,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta,
                                                          const float* __restrict__ bias, _Float16* __restrict__ yh,
                                                          long long y_bs, long long y_sp, int* __restrict__ oflow) {
    __shared__ float xs[CH * ST + KW];
    const int b = blockIdx.y, chunk = blockIdx.x;
    const int t0 = chunk * CH;
    const int nt = min(CH, T0 - t0);
    stage_chunk(xs, x + b * x_bs, t0, nt, N);
    const int c0 = (threadIdx.x & 63) * 8, fr = threadIdx.x >> 6;
    float w[8][KW], m[8], r[8], sc[8], sh[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
#pragma unroll
        for (int j = 0; j < KW; ++j) w[c][j] = w0[(c0 + c) * KW + j];
        if (MODE == 0) {
            m[c] = stats[(b * C0 + c0 + c) * 2];
            r[c] = stats[(b * C0 + c0 + c) * 2 + 1];
            sc[c] = r[c] * gamma[c0 + c];   // rstd * gamma folded
            sh[c] = beta[c0 + c];
        } else {
            m[c] = 0.f;
            r[c] = sc[c] = 1.f;
            sh[c] = bias ? bias[c0 + c] : 0.f;
        }
    }
    __syncthreads();
    _Float16* yb = yh + b * y_bs + (long long)t0 * C0 + c0;
    bool bad = false;
    for (int t = fr; t < nt; t += NT / 64) {
        f16x8 h1, h2;
        const float* xt = xs + t * ST;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            float v = conv10(w[c], xt);
            if (MODE == 0) v = hfa::gelu_fast((v - m[c]) * sc[c] + sh[c]);
            else v += sh[c];
            asm volatile("" : "+v"(v));   // split the rounded f32 value: no fusing its last multiply into the f16 cvt
            bad |= !(__builtin_fabsf(v) < 65504.0f);
            h1[c] = (_Float16)v;
            h2[c] = (_Float16)((v - (float)h1[c]) * 2048.0f);
        }
        *reinterpret_cast<f16x8*>(yb + (long long)t * C0) = h1;
        *reinterpret_cast<f16x8*>(yb + (long long)t * C0 + y_sp) = h2;
    }
    if (bad && oflow) *oflow = 1;
}


// ---- conv0 on the f32-input MFMA --------------------------------------------------------------------------------
// v_mfma_f32_16x16x4_f32 is bit for bit a k-ordered fmaf chain, D = fma(a3, b3, fma(a2, b2, fma(a1, b1, fma(a0, b0, C))))
// (cdna_hip_programming.md §3, "FP32-input MFMA"), so the 10-tap conv as three MFMAs (taps 0-3, 4-7, 8-11 with
// w10 = w11 = 0, C = 0 first) gives exactly conv10's values: the apply pass below is bit-identical to
// conv0_apply8_kernel.  Measured (scripts/conv0_bench.py, B = 32 x 10 s): no faster (559-576 vs 531-565 us), so it
// is hfa_conv0_tuning mode 2, not the default -- the apply pass is bound by VALU issue (~38 VALU ops per output in apply8, ~30 here: GELU ~21 of them; 2.1 GB written would take ~0.35 ms
// at the 6 TB/s store rate), and the f32 MFMA (32 cycles per 16x16x4 per SIMD) takes most of what it frees.  The
// same conv in the statistics pass with f64 accumulation was slower (254 vs 176 us: 131 VGPRs), so that pass stays
// on the VALU.
// Block: 8 waves over a CH-frame chunk; wave w owns channels 64 w + [0, 64) as four 16-channel MFMA blocks and walks
// the chunk in groups of 16 frames.  MFMA rows are channels, columns frames.  Block 2p + q, row r -> channel
// 64 w + 32 p + 8 (r >> 2) + 4 q + (r & 3): lane l (g = l >> 4, frame j = l & 15) then holds, in the D tiles of
// blocks 2p and 2p + 1, channels 64 w + 32 p + 8 g + [0, 8) of frame j -- one 16-B split-plane piece per pair.
constexpr int MNT = 512;
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void stage_chunk_m(float* xs, const float* xb, int t0, int nt, int N) {
    const int n = nt * ST + (KW - ST);                  // samples of frames < nt; zeros beyond (taps 10, 11 and
    for (int i = threadIdx.x; i < CH * ST + 12; i += MNT) {   // frames >= nt read them)
        const int idx = t0 * ST + i;
        xs[i] = (i < n && idx < N) ? xb[idx] : 0.0f;
    }
}

__device__ __forceinline__ void conv0_wfrag(const float* __restrict__ w0, int wave, int lane, float (&wf)[4][3]) {
    const int i = lane & 15, k = lane >> 4;
#pragma unroll
    for (int blk = 0; blk < 4; ++blk) {
        const int ch = 64 * wave + 32 * (blk >> 1) + 8 * (i >> 2) + 4 * (blk & 1) + (i & 3);
#pragma unroll
        for (int s = 0; s < 3; ++s) wf[blk][s] = 4 * s + k < KW ? w0[ch * KW + 4 * s + k] : 0.0f;
    }
}

// conv0 of frames f0 + [0, 16) for the wave's four channel blocks
__device__ __forceinline__ void conv0_group(const float* xs, int f0, int lane, const float (&wf)[4][3],
                                            f32x4 (&d)[4]) {
    const float* xl = xs + ST * (f0 + (lane & 15)) + (lane >> 4);
    float xb[3];
#pragma unroll
    for (int s = 0; s < 3; ++s) xb[s] = xl[4 * s];
#pragma unroll
    for (int blk = 0; blk < 4; ++blk) {
        d[blk] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int s = 0; s < 3; ++s) d[blk] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[blk][s], xb[s], d[blk], 0, 0, 0);
    }
}

template <int MODE>
__global__ __launch_bounds__(MNT) void conv0_apply_mfma_kernel(int N, int T0, const float* __restrict__ x,
                                                               long long x_bs, const float* __restrict__ w0,
                                                               const float* __restrict__ stats,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ beta,
                                                               const float* __restrict__ bias,
                                                               _Float16* __restrict__ yh, long long y_bs,
                                                               long long y_sp, int* __restrict__ oflow) {
    __shared__ float xs[CH * ST + 12];
    const int b = blockIdx.y, chunk = blockIdx.x;
    const int t0 = chunk * CH;
    const int nt = min(CH, T0 - t0);
    stage_chunk_m(xs, x + b * x_bs, t0, nt, N);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, j = lane & 15;
    float wf[4][3];
    conv0_wfrag(w0, wave, lane, wf);
    float m[16], r[16], sc[16], sh[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) {
        const int ch = 64 * wave + 32 * (c >> 3) + 8 * g + (c & 7);
        if (MODE == 0) {
            m[c] = stats[(b * C0 + ch) * 2];
            r[c] = stats[(b * C0 + ch) * 2 + 1];
            sc[c] = r[c] * gamma[ch];
            sh[c] = beta[ch];
        } else {
            m[c] = 0.f;
            r[c] = sc[c] = 1.f;
            sh[c] = bias ? bias[ch] : 0.f;
        }
    }
    __syncthreads();
    _Float16* yb = yh + b * y_bs + (long long)t0 * C0 + 64 * wave + 8 * g;
    bool bad = false;
    for (int f0 = 0; f0 < nt; f0 += 16) {
        f32x4 d[4];
        conv0_group(xs, f0, lane, wf, d);
        const bool live = f0 + j < nt;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            f16x8 h1, h2;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int c = 8 * p + e;
                float v = d[2 * p + (e >> 2)][e & 3];
                if (MODE == 0) v = hfa::gelu_fast((v - m[c]) * sc[c] + sh[c]);
                else v += sh[c];
                asm volatile("" : "+v"(v));   // split the rounded f32 value: no fusing its last multiply into the cvt
                bad |= live && !(__builtin_fabsf(v) < 65504.0f);
                h1[e] = (_Float16)v;
                h2[e] = (_Float16)fmaf((float)h1[e], -2048.0f, v * 2048.0f);   // exact: 2^11 (v - h1)
            }
            if (live) {
                _Float16* dst = yb + (long long)(f0 + j) * C0 + 32 * p;
                *reinterpret_cast<f16x8*>(dst) = h1;
                *reinterpret_cast<f16x8*>(dst + y_sp) = h2;
            }
        }
    }
    if (bad && oflow) *oflow = 1;
}

// ---- conv0 on the f16 MFMA, the three split products packed in one K = 32 step (the split-plane apply pass) -------
// The 10-tap conv of 16 channels x 16 frames is ONE v_mfma_f32_16x16x32_f16: A (rows = channels) holds
// [2^11 w1 (taps 0-9) | w2 (taps 0-9) | w1 (taps 0-9) | mean pair], B (columns = frames) [x1 | x1 | x2 | -1 -1], with
// w = w1 + 2^-11 w2 and x = x1 + 2^-11 x2 the split-f16 pairs of gemm.hip, so D = 2^11 w1 x1 + w2 x1 + w1 x2 =
// 2^11 (w . x) to the scheme's 2^-22 (every f16 x f16 product exact in the f32 accumulator).  Slots 30 and 31 carry
// 2^11 mean as an f16 pair (A) against -1 (B), so D = 2^11 (v - mean) and GroupNorm is one fma: D (rstd gamma
// 2^-11) + beta (|mean| >= 32 overflows the pair and is flagged like |w| >= 32).  What is left on the VALU is
// GroupNorm, GELU (hfa::gelu_fast, 13 ops), the plane split (one v_cvt_pk_f16_f32 and two v_fma_mix per pair) and a
// packed-f16 range check: ~18 VALU ops per output against ~36 in conv0_apply8_kernel, whose explicit fmaf chain (and
// its 72 LDS reads per frame: the compiler re-read the 10 samples for every channel) made that pass VALU-issue bound.
// Block: 8 waves over a CH-frame chunk.  The chunk's B columns are packed once into LDS (64 B per frame: one
// ds_read_b128 per lane per 16 frames, conflict-free); wave w owns channels 64 w + [0, 64) as four 16-channel MFMA
// blocks with the row map of conv0_apply_mfma_kernel (lane l then holds channels 64 w + 32 p + 8 (l >> 4) + [0, 8)
// of frame l & 15 for p = 0, 1: one 16-B piece per plane) and walks the chunk's 16 frame groups.  |w| >= 32
// overflows 2^11 w1 to inf, which the output check flags (the range guard then re-runs the batch on the f32 path,
// whose conv0 is the exact VALU kernel).  The f32-output conv0 (hfa_conv0_f32) stays on conv0_apply_kernel.
// Stores (STORE): the MFMA layout gives a store instruction 16 frames x 64 B; STORE 1 (default) passes each wave's
// 16 x 64 channels through its own XOR-swizzled LDS tile so one instruction writes 8 frames x 128 B (whole lines),
// STORE 2 through a block-wide double-buffered tile (one 1-KiB row per instruction, one barrier per group), STORE 0
// stores straight from the accumulator layout.  Measured (scripts/conv0_bench.py, B = 32 x 10 s, conv0 in all):
// STORE 0 0.51-0.56 ms, 1 0.457-0.466 (0.440-0.443 with non-temporal stores, the default), 2 0.468; the VALU apply
// pass 0.53-0.57; a persistent-block form (next chunk's samples prefetched into registers) 0.60-0.65.  Ablations:
// STORE 0 without plane stores 0.33-0.35 ms, without GELU 0.47; STORE 1 without GELU 0.43.
constexpr int PNT = 512;

// NT: STORE 1's plane stores non-temporal (streaming; the 2.1 GB per batch are far past the 256 MB Infinity Cache
// anyway): 0.466 -> 0.440 ms per batch (mode 8 = without).  (The timing ablations quoted above -- no plane stores,
// no GELU -- were builds of this kernel for measurement only; they are not in the library.)
template <int MODE, int STORE, bool NT = true>
__global__ __launch_bounds__(PNT) void conv0_packed_kernel(int N, int T0, const float* __restrict__ x,
                                                           long long x_bs, const float* __restrict__ w0,
                                                           const float* __restrict__ stats,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta,
                                                           const float* __restrict__ bias,
                                                           _Float16* __restrict__ yh, long long y_bs, long long y_sp,
                                                           int* __restrict__ oflow) {
    __shared__ __attribute__((aligned(16))) _Float16 bcol[CH * 32];   // [frame][32 k-slots]
    // STORE 1: [wave][plane][row][8 chunks of 16 B]; STORE 2: [buf][plane][row][64 chunks of 16 B]
    __shared__ __attribute__((aligned(16))) uint4 otile[STORE == 1 ? PNT / 64 : STORE == 2 ? 2 : 1][2]
                                                       [STORE == 1 ? 16 * 8 : STORE == 2 ? 16 * 64 : 1];
    const int b = blockIdx.y, chunk = blockIdx.x;
    const int t0 = chunk * CH;
    const int nt = min(CH, T0 - t0);
    {   // pack: thread (frame f, half h) splits samples 5 (t0 + f) + 5 h + [0, 5) into slots k, 10 + k and 20 + k
        const int f = threadIdx.x >> 1, h = threadIdx.x & 1;
        const float* xb = x + b * x_bs + (long long)(t0 + f) * ST + 5 * h;
        const long long rem = (long long)N - ((long long)(t0 + f) * ST + 5 * h);   // samples left in the row
        _Float16* col = bcol + f * 32;
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const float v = (f < nt && i < rem) ? xb[i] : 0.0f;
            const _Float16 v1 = (_Float16)v;
            const _Float16 v2 = (_Float16)((v - (float)v1) * 2048.0f);
            col[5 * h + i] = v1;
            col[10 + 5 * h + i] = v1;
            col[20 + 5 * h + i] = v2;
        }
        if (h) col[30] = col[31] = (_Float16)-1.0f;   // against the mean's slots of A (zero in mode 1)
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, j = lane & 15;
    // A fragments: block 2p + q, row i = lane & 15 -> channel 64 wave + 32 p + 8 (i >> 2) + 4 q + (i & 3);
    // k-slots 8 g + [0, 8)
    f16x8 af[4];
    bool bad = false;
#pragma unroll
    for (int blk = 0; blk < 4; ++blk) {
        const int i = j;
        const int ch = 64 * wave + 32 * (blk >> 1) + 8 * (i >> 2) + 4 * (blk & 1) + (i & 3);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int k = 8 * g + e;
            const int tap = k < 10 ? k : k < 20 ? k - 10 : k < 30 ? k - 20 : 0;
            const float w = k < 30 ? w0[ch * KW + tap] : 0.0f;
            const _Float16 w1 = (_Float16)w;
            const float w1f = (float)w1;
            bad |= !(__builtin_fabsf(w) < 32.0f);
            af[blk][e] = k < 10 ? (_Float16)(w1f * 2048.0f) : k < 20 ? (_Float16)((w - w1f) * 2048.0f) : w1;
        }
        if (MODE == 0 && g == 3) {   // slots 30, 31: 2^11 mean as an f16 pair (hi + lo, 22 bits) against B = -1
            const float m2 = 2048.0f * stats[(b * C0 + ch) * 2];
            const _Float16 mh = (_Float16)m2;
            af[blk][6] = mh;
            af[blk][7] = (_Float16)(m2 - (float)mh);
            bad |= !(__builtin_fabsf(m2) < 65504.0f);
        } else if (g == 3) {
            af[blk][6] = af[blk][7] = (_Float16)0.0f;
        }
    }
    // per-channel constants of the lane's 16 channels: c = 8 p + e <-> channel 64 wave + 32 p + 8 g + e
    float sc[16], sh[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) {
        const int ch = 64 * wave + 32 * (c >> 3) + 8 * g + (c & 7);
        if (MODE == 0) {
            sc[c] = stats[(b * C0 + ch) * 2 + 1] * gamma[ch] * (1.0f / 2048.0f);   // rstd gamma 2^-11
            sh[c] = beta[ch];
        } else {
            sc[c] = 1.0f / 2048.0f;
            sh[c] = bias ? bias[ch] : 0.0f;
        }
    }
    __syncthreads();
    // Range check on the packed high planes: |v| >= 65520 rounds to inf, a NaN stays NaN, and h * 0 + acc turns
    // either into a NaN that persists (the planes represent every |v| < 65520 exactly to the scheme's precision:
    // the low plane then holds |v - h1| * 2^11 <= 2^15).  Frames past the chunk's nt come from zero samples: finite.
    const f16x2 zero2 = {(_Float16)0.0f, (_Float16)0.0f};
    f16x2 nanacc = zero2;
    const float c2048 = 2048.0f;
    int tb = 0;
    _Float16* yb = yh + b * y_bs + (long long)t0 * C0;
    for (int f0 = 0; f0 < nt; f0 += 16) {
        const f16x8 bx = *reinterpret_cast<const f16x8*>(bcol + (f0 + j) * 32 + 8 * g);
        f32x4 d[4];
#pragma unroll
        for (int blk = 0; blk < 4; ++blk)
            d[blk] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[blk], bx, f32x4{0.0f, 0.0f, 0.0f, 0.0f}, 0, 0, 0);
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            unsigned h1[4], h2[4];   // f16 pairs
#pragma unroll
            for (int e = 0; e < 8; e += 2) {
                float v[2];
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int c = 8 * p + e + u;
                    v[u] = fmaf(d[2 * p + ((e + u) >> 2)][(e + u) & 3], sc[c], sh[c]);
                    if (MODE == 0) v[u] = hfa::gelu_fast(v[u]);
                    asm volatile("" : "+v"(v[u]));   // split the rounded f32 value: no fusing its last fma into the cvt
                }
                const f16x2 hp = __builtin_convertvector((f32x2){v[0], v[1]}, f16x2);   // one v_cvt_pk_f16_f32
                nanacc = hp * zero2 + nanacc;   // stays 0 unless a high plane is inf / NaN (v_pk_fma_f16)
                h1[e >> 1] = __builtin_bit_cast(unsigned, hp);
                h2[e >> 1] = hfa::split_lo_pair(h1[e >> 1], v[0] * 2048.0f, v[1] * 2048.0f, c2048);
            }
            const uint4 o1 = make_uint4(h1[0], h1[1], h1[2], h1[3]), o2 = make_uint4(h2[0], h2[1], h2[2], h2[3]);
            if (STORE == 1) {   // row j, 16-B chunk 4 p + g of the wave's 128-B row segment, XOR-swizzled
                const int slot = j * 8 + ((4 * p + g) ^ (j & 7));
                otile[wave][0][slot] = o1;
                otile[wave][1][slot] = o2;
            } else if (STORE == 2) {   // row j, chunk 8 wave + 4 p + g of the 1-KiB row, XOR-swizzled by the row
                const int slot = j * 64 + ((8 * wave + 4 * p + g) ^ j);
                otile[tb][0][slot] = o1;
                otile[tb][1][slot] = o2;
            } else if (f0 + j < nt) {
                _Float16* dst = yb + (long long)(f0 + j) * C0 + 64 * wave + 32 * p + 8 * g;
                *reinterpret_cast<uint4*>(dst) = o1;
                *reinterpret_cast<uint4*>(dst + y_sp) = o2;
            }
        }
        if (STORE == 1) {   // lane (row r = lane >> 3 + 8 hf, chunk c = lane & 7): 8 rows x 128 B
            const int c = lane & 7;     // (wave-local tile: LDS ops of one wave complete in order, no barrier)
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
                const int r = (lane >> 3) + 8 * hf;
                const int slot = r * 8 + (c ^ (r & 7));
                const uint4 v1 = otile[wave][0][slot], v2 = otile[wave][1][slot];
                if (f0 + r < nt) {
                    _Float16* dst = yb + (long long)(f0 + r) * C0 + 64 * wave + 8 * c;
                    if (NT) {   // non-temporal (streaming) stores
                        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
                        __builtin_nontemporal_store(u32x4{v1.x, v1.y, v1.z, v1.w}, reinterpret_cast<u32x4*>(dst));
                        __builtin_nontemporal_store(u32x4{v2.x, v2.y, v2.z, v2.w}, reinterpret_cast<u32x4*>(dst + y_sp));
                    } else {
                        *reinterpret_cast<uint4*>(dst) = v1;
                        *reinterpret_cast<uint4*>(dst + y_sp) = v2;
                    }
                }
            }
        } else if (STORE == 2) {   // wave w stores rows 2 w, 2 w + 1: one 1-KiB row per instruction
            __syncthreads();
#pragma unroll
            for (int rr = 0; rr < 2; ++rr) {
                const int r = 2 * wave + rr;
                const int slot = r * 64 + (lane ^ r);
                const uint4 v1 = otile[tb][0][slot], v2 = otile[tb][1][slot];
                if (f0 + r < nt) {
                    _Float16* dst = yb + (long long)(f0 + r) * C0 + 8 * lane;
                    *reinterpret_cast<uint4*>(dst) = v1;
                    *reinterpret_cast<uint4*>(dst + y_sp) = v2;
                }
            }
            tb ^= 1;   // the other buffer's readers passed this group's barrier before anyone writes it again
        }
    }
    bad |= nanacc[0] != nanacc[0] || nanacc[1] != nanacc[1];
    if (bad && oflow) *oflow = 1;
}

thread_local int g_conv0_mode = 0;   // hfa_conv0_tuning: 0 packed f16 MFMA apply (default), 1 round 1, 2 f32-MFMA
                                     // apply, 3 VALU apply (conv0_apply8_kernel)

}  // namespace

extern "C" {

long long hfa_conv0_workspace_bytes(int B, int N) {
    const int T0 = N >= KW ? (N - KW) / ST + 1 : 0;
    const int nchunk = (T0 + CH - 1) / CH;
    return (long long)B * nchunk * C0 * 2 * sizeof(double) + (long long)B * C0 * 2 * sizeof(float) + 64;
}

namespace {
int conv0_launch(int B, int N, const float* x, long long x_bs, const float* w0, const float* bias, int norm,
                 const float* gamma, const float* beta, float eps, void* workspace, void* y, long long y_bs,
                 long long y_sp, bool outs, int* oflow, const int32_t* t0_len, hipStream_t stream) {
    const char* fn = outs ? "hfa_conv0_split" : "hfa_conv0_f32";
    if (B < 0 || N < KW) {
        hfa::set_error("%s: need N >= %d samples (got %d)", fn, KW, N);
        return HFA_EINVAL;
    }
    if (B == 0) return HFA_OK;
    if (!x || !w0 || !y || (norm && (!gamma || !beta || !workspace)) || ((uintptr_t)y & 7) || y_bs % 2 ||
        (outs && y_sp % 2)) {
        hfa::set_error("%s: bad pointer arguments", fn);
        return HFA_EINVAL;
    }
    const int T0 = (N - KW) / ST + 1;
    const int nchunk = (T0 + CH - 1) / CH;
    dim3 grid(nchunk, B);
    const bool vec8 = ((uintptr_t)y & 15) == 0 && y_bs % 8 == 0 && y_sp % 8 == 0;   // 16-B plane pieces
    if (norm) {
        double* part = reinterpret_cast<double*>(workspace);
        float* stats = reinterpret_cast<float*>(part + (size_t)B * nchunk * C0 * 2);
        if (g_conv0_mode != 1) {
            const int ng = (T0 + GCH - 1) / GCH;                      // <= nchunk: fits the partials region
            hipLaunchKernelGGL(conv0_gram_kernel, dim3(ng, B), dim3(256), 0, stream, T0, x, x_bs, part, t0_len);
            hipLaunchKernelGGL(conv0_gram_stats_kernel, dim3(B), dim3(C0), 0, stream, T0, ng, part, w0, eps, stats,
                               t0_len);
        } else {
            hipLaunchKernelGGL(conv0_stats_kernel, grid, dim3(NT), 0, stream, N, T0, x, x_bs, w0, part, t0_len);
            hipLaunchKernelGGL(conv0_reduce_kernel, dim3(C0 / 64, B), dim3(NT), 0, stream, T0, nchunk, part, eps,
                               stats, t0_len);
        }
#define HFA_PACKED(MODE_, STORE_, STATS_)                                                                             \
    hipLaunchKernelGGL((conv0_packed_kernel<MODE_, STORE_>), grid, dim3(PNT), 0, stream, N, T0, x, x_bs, w0,           \
                       STATS_, gamma, beta, bias, reinterpret_cast<_Float16*>(y), y_bs, y_sp, oflow)
        if (outs && vec8 && g_conv0_mode == 0) HFA_PACKED(0, 1, stats);
        else if (outs && vec8 && g_conv0_mode == 4) HFA_PACKED(0, 0, stats);
        else if (outs && vec8 && g_conv0_mode == 7) HFA_PACKED(0, 2, stats);
        else if (outs && vec8 && g_conv0_mode == 8)
            hipLaunchKernelGGL((conv0_packed_kernel<0, 1, false>), grid, dim3(PNT), 0, stream, N, T0, x, x_bs, w0,
                               stats, gamma, beta, bias, reinterpret_cast<_Float16*>(y), y_bs, y_sp, oflow);
        else if (outs && vec8 && g_conv0_mode == 10)   // mode 0 held to 2 workgroups per CU (16 KiB of unused LDS)
            hipLaunchKernelGGL((conv0_packed_kernel<0, 1, true>), grid, dim3(PNT), 16 * 1024, stream, N, T0, x, x_bs,
                               w0, stats, gamma, beta, bias, reinterpret_cast<_Float16*>(y), y_bs, y_sp, oflow);
        else if (outs && vec8 && g_conv0_mode == 2)
            hipLaunchKernelGGL((conv0_apply_mfma_kernel<0>), grid, dim3(MNT), 0, stream, N, T0, x, x_bs, w0, stats,
                               gamma, beta, bias, reinterpret_cast<_Float16*>(y), y_bs, y_sp, oflow);
        else if (outs && vec8)
            hipLaunchKernelGGL((conv0_apply8_kernel<0>), grid, dim3(NT), 0, stream, N, T0, x, x_bs, w0, stats, gamma,
                               beta, bias, reinterpret_cast<_Float16*>(y), y_bs, y_sp, oflow);
        else if (outs)
            hipLaunchKernelGGL((conv0_apply_kernel<0, true>), grid, dim3(NT), 0, stream, N, T0, x, x_bs, w0, stats,
                               gamma, beta, bias, y, y_bs, y_sp, oflow);
        else
            hipLaunchKernelGGL((conv0_apply_kernel<0, false>), grid, dim3(NT), 0, stream, N, T0, x, x_bs, w0, stats,
                               gamma, beta, bias, y, y_bs, y_sp, oflow);
    } else if (outs && vec8 && (g_conv0_mode == 0 || g_conv0_mode >= 4)) {   // the packed modes
        HFA_PACKED(1, 1, nullptr);
    } else if (outs && vec8 && g_conv0_mode == 2) {
        hipLaunchKernelGGL((conv0_apply_mfma_kernel<1>), grid, dim3(MNT), 0, stream, N, T0, x, x_bs, w0, nullptr,
                           nullptr, nullptr, bias, reinterpret_cast<_Float16*>(y), y_bs, y_sp, oflow);
    } else if (outs && vec8) {
        hipLaunchKernelGGL((conv0_apply8_kernel<1>), grid, dim3(NT), 0, stream, N, T0, x, x_bs, w0, nullptr, nullptr,
                           nullptr, bias, reinterpret_cast<_Float16*>(y), y_bs, y_sp, oflow);
    } else if (outs) {
        hipLaunchKernelGGL((conv0_apply_kernel<1, true>), grid, dim3(NT), 0, stream, N, T0, x, x_bs, w0, nullptr,
                           nullptr, nullptr, bias, y, y_bs, y_sp, oflow);
    } else {
        hipLaunchKernelGGL((conv0_apply_kernel<1, false>), grid, dim3(NT), 0, stream, N, T0, x, x_bs, w0, nullptr,
                           nullptr, nullptr, bias, y, y_bs, y_sp, oflow);
    }
#undef HFA_PACKED
    return hfa::check_launch(fn);
}
}  // namespace

// x [B, N] (row stride x_bs) -> y [B, T0, 512] channels-last (row stride 512, batch stride y_bs).
// norm = 1: GroupNorm(512,512)+GELU (gamma/beta required, workspace of hfa_conv0_workspace_bytes);
// norm = 0: raw conv + bias (bias may be NULL).  t0_len (optional, device [B]): per-row frame counts of a
// variable-length batch — the GroupNorm statistics cover frames < t0_len[b] only (rows beyond are don't-care).
int hfa_conv0_f32(int B, int N, const float* x, long long x_bs, const float* w0, const float* bias, int norm,
                  const float* gamma, const float* beta, float eps, void* workspace, float* y, long long y_bs,
                  const int32_t* t0_len, hipStream_t stream) {
    return conv0_launch(B, N, x, x_bs, w0, bias, norm, gamma, beta, eps, workspace, y, y_bs, 0, false, nullptr,
                        t0_len, stream);
}

// As hfa_conv0_f32, output as split-f16 planes ys (plane 1 at +y_sp halves; strides in halves); *oflow is raised
// when an output leaves f16 range.
int hfa_conv0_split(int B, int N, const float* x, long long x_bs, const float* w0, const float* bias, int norm,
                    const float* gamma, const float* beta, float eps, void* workspace, uint16_t* ys, long long y_bs,
                    long long y_sp, int* oflow, const int32_t* t0_len, hipStream_t stream) {
    return conv0_launch(B, N, x, x_bs, w0, bias, norm, gamma, beta, eps, workspace, ys, y_bs, y_sp, true, oflow,
                        t0_len, stream);
}

// Kernel choice for A/B timing and the parity tests (split-plane output; the f32 output is always the VALU kernel):
// 0 (default) the lag-product statistics and the packed f16-MFMA apply pass (conv0_packed_kernel), 1 the round-1
// passes (the conv re-run on the VALU for the statistics, conv0_apply8_kernel), 2 the lag-product statistics with the
// f32-MFMA apply pass (bit-identical to 3; measured 0.575-0.620 vs 0.566-0.571 ms per batch, scripts/conv0_bench.py),
// 3 the lag-product statistics with conv0_apply8_kernel (the round-2 default), 4 mode 0 with its stores straight
// from the MFMA layout, 7 with its stores through a block-wide LDS tile, 8 with plain (not non-temporal) stores, 10
// held to 2 workgroups per CU (room for a side-stream GEMM workgroup beside it); 5, 6 and 9 were timing ablations
// (wrong outputs by construction) and are rejected.  Per calling thread.
int hfa_conv0_tuning(int mode) {
    if (mode < 0 || mode > 10 || mode == 5 || mode == 6 || mode == 9) {
        hfa::set_error("hfa_conv0_tuning: mode %d is not 0-4, 7, 8 or 10", mode);
        return HFA_EINVAL;
    }
    g_conv0_mode = mode;
    return HFA_OK;
}

}  // extern "C"
