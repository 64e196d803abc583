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
// (Since round 3 passes 1-2 are the lag-product statistics below: no conv re-run; round 4 retired the alternatives.)
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

// ---- GroupNorm(512, 512) statistics from the wave's lag products ----------------------------------------------
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
// blocks (block 2p + q, row i -> channel 64 w + 32 p + 8 (i >> 2) + 4 q + (i & 3), so lane l holds channels
// 64 w + 32 p + 8 (l >> 4) + [0, 8) of frame l & 15 for p = 0, 1: one 16-B piece per plane) and walks the chunk's 16
// frame groups.  |w| >= 32 overflows 2^11 w1 to inf, which the output check flags (the range guard then re-runs the
// batch on the f32 path, whose conv0 is the exact VALU kernel).  The f32-output conv0 (hfa_conv0_f32) stays on
// conv0_apply_kernel.
// Stores: the MFMA layout gives a store instruction 16 frames x 64 B; each wave passes its 16 x 64 channels through
// its own XOR-swizzled LDS tile so one instruction writes 8 frames x 128 B (whole lines), non-temporal (the 2.1 GB
// per batch are far past the 256 MB Infinity Cache).  Measured (scripts/conv0_bench.py, B = 32 x 10 s, conv0 in all;
// the alternatives are in git history, round 3): stores straight from the accumulator layout 0.51-0.56 ms, this tile
// 0.457-0.466 (0.440-0.443 non-temporal), a block-wide 1-KiB-row tile 0.468, the VALU apply pass 0.53-0.57, a
// persistent-block form 0.60-0.65.  Ablations (measurement builds only): without plane stores 0.33-0.35 ms, without
// GELU 0.43.
constexpr int PNT = 512;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(PNT) void conv0_packed_kernel(int N, int T0, const float* __restrict__ x,
                                                           long long x_bs, const float* __restrict__ w0,
                                                           const float* __restrict__ stats,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta,
                                                           const float* __restrict__ bias,
                                                           _Float16* __restrict__ yh, long long y_bs, long long y_sp,
                                                           int* __restrict__ oflow) {
    __shared__ __attribute__((aligned(16))) _Float16 bcol[CH * 32];   // [frame][32 k-slots]
    __shared__ __attribute__((aligned(16))) uint4 otile[PNT / 64][2][16 * 8];   // [wave][plane][row][8 x 16 B]
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
            const int slot = j * 8 + ((4 * p + g) ^ (j & 7));   // row j, 16-B chunk 4 p + g, XOR-swizzled
            otile[wave][0][slot] = o1;
            otile[wave][1][slot] = o2;
        }
        // the wave's tile is written by one lane map and read by another: order the LDS accesses inside the wave
        // (gemm.hip store_split_lds does the same; no block barrier, the tile is the wave's own)
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        const int c = lane & 7;         // lane (row r = lane >> 3 + 8 hf, chunk c = lane & 7): 8 rows x 128 B
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            const int r = (lane >> 3) + 8 * hf;
            const int slot = r * 8 + (c ^ (r & 7));
            const uint4 v1 = otile[wave][0][slot], v2 = otile[wave][1][slot];
            if (f0 + r < nt) {
                _Float16* dst = yb + (long long)(f0 + r) * C0 + 64 * wave + 8 * c;
                __builtin_nontemporal_store(u32x4{v1.x, v1.y, v1.z, v1.w}, reinterpret_cast<u32x4*>(dst));
                __builtin_nontemporal_store(u32x4{v2.x, v2.y, v2.z, v2.w}, reinterpret_cast<u32x4*>(dst + y_sp));
            }
        }
        // the next group's tile writes follow this group's reads
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }
    bad |= nanacc[0] != nanacc[0] || nanacc[1] != nanacc[1];
    if (bad && oflow) *oflow = 1;
}

}  // namespace

extern "C" {

long long hfa_conv0_workspace_bytes(int B, int N) {
    const int T0 = N >= KW ? (N - KW) / ST + 1 : 0;
    const int ng = (T0 + GCH - 1) / GCH;
    return (long long)B * ng * NGR * sizeof(double) + (long long)B * C0 * 2 * sizeof(float) + 64;
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
        const int ng = (T0 + GCH - 1) / GCH;
        float* stats = reinterpret_cast<float*>(part + (size_t)B * ng * NGR);
        hipLaunchKernelGGL(conv0_gram_kernel, dim3(ng, B), dim3(256), 0, stream, T0, x, x_bs, part, t0_len);
        hipLaunchKernelGGL(conv0_gram_stats_kernel, dim3(B), dim3(C0), 0, stream, T0, ng, part, w0, eps, stats, t0_len);
        if (outs && vec8)
            hipLaunchKernelGGL((conv0_packed_kernel<0>), grid, dim3(PNT), 0, stream, N, T0, x, x_bs, w0, stats, gamma,
                               beta, bias, reinterpret_cast<_Float16*>(y), y_bs, y_sp, oflow);
        else if (outs)
            hipLaunchKernelGGL((conv0_apply_kernel<0, true>), grid, dim3(NT), 0, stream, N, T0, x, x_bs, w0, stats,
                               gamma, beta, bias, y, y_bs, y_sp, oflow);
        else
            hipLaunchKernelGGL((conv0_apply_kernel<0, false>), grid, dim3(NT), 0, stream, N, T0, x, x_bs, w0, stats,
                               gamma, beta, bias, y, y_bs, y_sp, oflow);
    } else if (outs && vec8) {
        hipLaunchKernelGGL((conv0_packed_kernel<1>), grid, dim3(PNT), 0, stream, N, T0, x, x_bs, w0, nullptr, nullptr,
                           nullptr, bias, reinterpret_cast<_Float16*>(y), y_bs, y_sp, oflow);
    } else if (outs) {
        hipLaunchKernelGGL((conv0_apply_kernel<1, true>), grid, dim3(NT), 0, stream, N, T0, x, x_bs, w0, nullptr,
                           nullptr, nullptr, bias, y, y_bs, y_sp, oflow);
    } else {
        hipLaunchKernelGGL((conv0_apply_kernel<1, false>), grid, dim3(NT), 0, stream, N, T0, x, x_bs, w0, nullptr,
                           nullptr, nullptr, bias, y, y_bs, y_sp, oflow);
    }
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

}  // extern "C"
