// norm.hip — LayerNorm / GroupNorm (+ fused activation) for channels-last [rows, C] activations.
//
// Replaces ATen layer_norm / group_norm (+ gelu / hardswish) on the path:
//   * Hubert: feature_projection LN (model.py:121; HF HubertFeatureProjection), encoder LN after pos-conv
//     (model.py:25,52; HF HubertEncoder.layer_norm), per-layer norm1/norm2 (post-LN) or pre-LN + final LN
//     (HF HubertEncoderLayerStableLayerNorm), LN-conv feature extractor of the large variant
//     (HF HubertLayerNormConvLayer: conv -> LN over channels -> GELU).
//   * UNet ResidualBasicBlock: GroupNorm(16) + Hardswish and LN + Hardswish (resnet_block.py:25-26, :42-45).
// HBM-bound: one wavefront per row, the row held in registers (C <= 4096), float4 loads, two-pass
// mean/variance in f32 like ATen's reference path, then y = (x - mean) * rstd * gamma + beta.
#include "hfa_common.h"
#include "hfa.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

enum { ACT_NONE = 0, ACT_GELU = 1, ACT_HARDSWISH = 2 };

__device__ __forceinline__ float act_apply(float v, int act) {
    if (act == ACT_GELU) return hfa::gelu_fast(v);
    if (act == ACT_HARDSWISH) return hfa::hardswish(v);
    return v;
}

// Row-per-wave LayerNorm; C % 4 == 0, C <= 64*4*VPL.  One row (wave index `wave`) per call.
template <int VPL>
__device__ __forceinline__ void layernorm_row(int wave, int lane, int C, const float* __restrict__ x, long long ldx,
                                                        const float* __restrict__ res, long long ldr,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, float eps, int act,
                                                        float* __restrict__ y, long long ldy, int T,
                                                        const int32_t* __restrict__ t_len,
                                                        _Float16* __restrict__ ys, long long ldys, long long sps,
                                                        int* __restrict__ oflow) {
    // ys (optional): the output also as split-f16 planes (gemm.hip's split operand: hi, (x - hi) * 2^11), so the
    // next split GEMM reads it without a separate conversion pass; *oflow raised for |y| >= 65504 / non-finite
    if (t_len && wave % T >= t_len[wave / T]) {     // padding row of a variable-length batch: zeros
        float* yr = y ? y + wave * ldy : nullptr;
        for (int c = lane * 4; c < C; c += 256) {
            if (yr) *reinterpret_cast<f32x4*>(yr + c) = f32x4{0.f, 0.f, 0.f, 0.f};
            if (ys) {
                const f16x4 z{(_Float16)0.f, (_Float16)0.f, (_Float16)0.f, (_Float16)0.f};
                *reinterpret_cast<f16x4*>(ys + wave * ldys + c) = z;
                *reinterpret_cast<f16x4*>(ys + sps + wave * ldys + c) = z;
            }
        }
        return;
    }
    const float* xr = x + wave * ldx;
    const float* rr = res ? res + wave * ldr : nullptr;
    f32x4 v[VPL];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
        const int c = (lane + i * 64) * 4;
        if (c < C) {
            v[i] = *reinterpret_cast<const f32x4*>(xr + c);
            if (rr) v[i] += *reinterpret_cast<const f32x4*>(rr + c);
        } else {
            v[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        s += (v[i][0] + v[i][1]) + (v[i][2] + v[i][3]);
    }
    const float mean = hfa::wave_sum(s) / (float)C;
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
        const int c = (lane + i * 64) * 4;
        if (c < C) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float d = v[i][e] - mean;
                ss += d * d;
            }
        }
    }
    const float var = hfa::wave_sum(ss) / (float)C;
    const float rstd = 1.0f / sqrtf(var + eps);
    float* yr = y ? y + wave * ldy : nullptr;      // y NULL: split planes only (the residual is read from them)
    hfa::h2v nanacc = {(_Float16)0.0f, (_Float16)0.0f};   // the planes' range check (hfa::split_pair)
    const float c2048 = 2048.0f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
        const int c = (lane + i * 64) * 4;
        if (c < C) {
            const f32x4 g = *reinterpret_cast<const f32x4*>(gamma + c);
            const f32x4 bb = *reinterpret_cast<const f32x4*>(beta + c);
            f32x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = act_apply((v[i][e] - mean) * rstd * g[e] + bb[e], act);
            if (yr) *reinterpret_cast<f32x4*>(yr + c) = o;
            if (ys) {
                uint2 h1, h2;
                hfa::split_pair(o[0], o[1], h1.x, h2.x, nanacc, c2048);
                hfa::split_pair(o[2], o[3], h1.y, h2.y, nanacc, c2048);
                *reinterpret_cast<uint2*>(ys + wave * ldys + c) = h1;
                *reinterpret_cast<uint2*>(ys + sps + wave * ldys + c) = h2;
            }
        }
    }
    if (hfa::range_bad(nanacc) && oflow) *oflow = 1;
}

// Rows wave, wave + 4 gridDim.x, ... (a capped grid, hfa::grid_cap)
template <int VPL>
__global__ __launch_bounds__(256) void layernorm_kernel(int rows, int C, const float* __restrict__ x, long long ldx,
                                                        const float* __restrict__ res, long long ldr,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, float eps, int act,
                                                        float* __restrict__ y, long long ldy, int T,
                                                        const int32_t* __restrict__ t_len,
                                                        _Float16* __restrict__ ys, long long ldys, long long sps,
                                                        int* __restrict__ oflow) {
    const int lane = threadIdx.x & 63;
    for (int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; wave < rows; wave += gridDim.x * (blockDim.x >> 6))
        layernorm_row<VPL>(wave, lane, C, x, ldx, res, ldr, gamma, beta, eps, act, y, ldy, T, t_len, ys, ldys, sps,
                           oflow);
}

// GroupNorm over a channels-last [T, C] slab per batch item: group g = channels [g*Cg, (g+1)*Cg) over all T.
// One workgroup per (batch, group); f64 accumulation of the statistics, then a second sweep applies the
// affine + activation.  (torch.nn.GroupNorm on [B, C, T]: biased variance, eps inside the sqrt.)
__global__ __launch_bounds__(256) void groupnorm_kernel(int T, int C, int G, const float* __restrict__ x,
                                                        long long x_bs, int ldx, const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, float eps, int act,
                                                        float* __restrict__ y, long long y_bs, int ldy,
                                                        const int32_t* __restrict__ t_len) {
    const int b = blockIdx.y, g = blockIdx.x;
    const int Cg = C / G;
    const float* xb = x + b * x_bs + g * Cg;
    float* yb = y + b * y_bs + g * Cg;
    const int Tb = t_len ? t_len[b] : T;            // variable-length batch: this row's frames only
    const int n = Tb * Cg;
    double s = 0.0, ss = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int t = i / Cg, c = i - t * Cg;
        const double v = xb[(long long)t * ldx + c];
        s += v;
        ss += v * v;
    }
    __shared__ double red[2][4];
    s = hfa::wave_sum_d(s);
    ss = hfa::wave_sum_d(ss);
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = s;
        red[1][threadIdx.x >> 6] = ss;
    }
    __syncthreads();
    double S = 0.0, SS = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
        S += red[0][w];
        SS += red[1][w];
    }
    const double mean_d = n > 0 ? S / n : 0.0;
    double var_d = n > 0 ? SS / n - mean_d * mean_d : 0.0;
    if (var_d < 0) var_d = 0;
    const float mean = (float)mean_d;
    const float rstd = (float)(1.0 / sqrt(var_d + (double)eps));
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int t = i / Cg, c = i - t * Cg;
        const float v = xb[(long long)t * ldx + c];
        yb[(long long)t * ldy + c] = act_apply((v - mean) * rstd * gamma[g * Cg + c] + beta[g * Cg + c], act);
    }
    for (int i = n + threadIdx.x; i < T * Cg; i += blockDim.x) {   // padding rows -> zeros
        const int t = i / Cg, c = i - t * Cg;
        yb[(long long)t * ldy + c] = 0.0f;
    }
}

// Long sequences with few (batch, group) pairs (a 5-minute utterance: B = 1, 16 groups) would leave the chip
// idle with one workgroup per pair: split T into P parts.  Pass 1 writes per-part f64 partial sums, pass 2
// reduces the P partials of its pair (P <= 64, same order in every block) and applies its part.
__global__ __launch_bounds__(256) void groupnorm_partial_kernel(int T, int C, int G, int P,
                                                                const float* __restrict__ x, long long x_bs,
                                                                int ldx, const int32_t* __restrict__ t_len,
                                                                double* __restrict__ part) {
    const int g = blockIdx.x, b = blockIdx.y, pi = blockIdx.z;
    const int Cg = C / G;
    const int Tb = t_len ? t_len[b] : T;
    const int rows = (Tb + P - 1) / P;
    const int t0 = pi * rows, t1 = min(Tb, t0 + rows);
    const float* xb = x + b * x_bs + g * Cg;
    double s = 0.0, ss = 0.0;
    const int n = max(0, t1 - t0) * Cg;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int t = t0 + i / Cg, c = i % Cg;
        const double v = xb[(long long)t * ldx + c];
        s += v;
        ss += v * v;
    }
    __shared__ double red[2][4];
    s = hfa::wave_sum_d(s);
    ss = hfa::wave_sum_d(ss);
    if ((threadIdx.x & 63) == 0) { red[0][threadIdx.x >> 6] = s; red[1][threadIdx.x >> 6] = ss; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double* pp = part + (((size_t)b * G + g) * P + pi) * 2;
        pp[0] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
        pp[1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    }
}

__global__ __launch_bounds__(256) void groupnorm_apply_kernel(int T, int C, int G, int P, const float* __restrict__ x,
                                                              long long x_bs, int ldx, const float* __restrict__ gamma,
                                                              const float* __restrict__ beta, float eps, int act,
                                                              float* __restrict__ y, long long y_bs, int ldy,
                                                              const int32_t* __restrict__ t_len,
                                                              const double* __restrict__ part) {
    const int g = blockIdx.x, b = blockIdx.y, pi = blockIdx.z;
    const int Cg = C / G;
    const int Tb = t_len ? t_len[b] : T;
    const double* pp = part + ((size_t)b * G + g) * P * 2;
    double S = 0.0, SS = 0.0;
    for (int k = 0; k < P; ++k) { S += pp[2 * k]; SS += pp[2 * k + 1]; }
    const long long n = (long long)Tb * Cg;
    const double mean_d = n > 0 ? S / n : 0.0;
    double var_d = n > 0 ? SS / n - mean_d * mean_d : 0.0;
    if (var_d < 0) var_d = 0;
    const float mean = (float)mean_d;
    const float rstd = (float)(1.0 / sqrt(var_d + (double)eps));
    const int rows = (T + P - 1) / P;                // this block's share of ALL T rows (padding rows -> 0)
    const int t0 = pi * rows, t1 = min(T, t0 + rows);
    const float* xb = x + b * x_bs + g * Cg;
    float* yb = y + b * y_bs + g * Cg;
    const int m = max(0, t1 - t0) * Cg;
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
        const int t = t0 + i / Cg, c = i % Cg;
        float o = 0.0f;
        if (t < Tb) o = act_apply((xb[(long long)t * ldx + c] - mean) * rstd * gamma[g * Cg + c] + beta[g * Cg + c], act);
        yb[(long long)t * ldy + c] = o;
    }
}

// Row-parallel GroupNorm for channels-last [T, C] with C % 4 == 0, Cg % 4 == 0, C <= 1024 (the UNet's GN(16) on
// 192 / 384 channels: a group is 12 / 24 channels, 48 / 96 B of a row, so one workgroup per (batch, group) reads
// short strided pieces).  Rows are cut into fixed parts of kGnRows rows; pass 1 (grid parts x B) reads whole rows with
// float4 loads, each thread on one fixed float4 column (one group) and every (256 / (C/4))-th row of the part, and
// writes f64 partial sums per (batch, part, group), reduced per group in a fixed order; pass 2 re-reduces a row's
// partials in part order (the parts of a row depend only on its own length: a row gives the same bits in any batch)
// and applies affine + activation to its part, writing f32 and / or split-f16 planes (the next split GEMM's operand).
constexpr int kGnRows = 32;

__global__ __launch_bounds__(256) void gn_rows_partial_kernel(int T, int C, int G, const float* __restrict__ x,
                                                              long long x_bs, int ldx,
                                                              const int32_t* __restrict__ t_len,
                                                              double* __restrict__ part) {
    const int pi = blockIdx.x, b = blockIdx.y, P = gridDim.x;
    const int C4 = C >> 2, Cg = C / G, rstep = 256 / C4;
    const int col = threadIdx.x % C4, r0 = threadIdx.x / C4;
    const int Tb = t_len ? t_len[b] : T;
    const int t0 = pi * kGnRows, t1 = min(Tb, t0 + kGnRows);
    double s = 0.0, ss = 0.0;
    if (r0 < rstep) {
        const float* xb = x + b * x_bs + col * 4;
        for (int t = t0 + r0; t < t1; t += rstep) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(xb + (long long)t * ldx);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                s += (double)v[e];
                ss += (double)v[e] * (double)v[e];
            }
        }
    }
    __shared__ double red[256][2];
    red[threadIdx.x][0] = s;
    red[threadIdx.x][1] = ss;
    __syncthreads();
    if (threadIdx.x < G) {                              // group g: columns [g Cg/4, (g+1) Cg/4) of every row lane
        const int g = threadIdx.x, c0 = g * (Cg >> 2), c1 = c0 + (Cg >> 2);
        double S = 0.0, SS = 0.0;
        for (int r = 0; r < rstep; ++r)
            for (int c = c0; c < c1; ++c) {
                S += red[r * C4 + c][0];
                SS += red[r * C4 + c][1];
            }
        double* pp = part + (((size_t)b * P + pi) * G + g) * 2;
        pp[0] = S;
        pp[1] = SS;
    }
}

// (b, g) statistics from S = sum x, SS = sum x^2 over the row's Tb * Cg values
__device__ __forceinline__ void gn_stat(double S, double SS, int Tb, int Cg, float eps, float* out) {
    const double n = (double)Tb * Cg;
    const double mean_d = Tb > 0 ? S / n : 0.0;
    double var_d = Tb > 0 ? SS / n - mean_d * mean_d : 0.0;
    if (var_d < 0) var_d = 0;
    out[0] = (float)mean_d;
    out[1] = (float)(1.0 / sqrt(var_d + (double)eps));
}

// Long rows (more than kGnStatParts parts, e.g. config 5's UNet level 0 at T = 25 840: 808 parts): the statistics once
// per batch row, before pass 2.  The parts are summed in part order exactly as pass 2 does in-block (the same bits),
// but staged through LDS in coalesced chunks: pass 2's per-block loop reads one dependent f64 pair per part and took
// ~125 us per call there, in every one of its 808 blocks at once.
constexpr int kGnStatParts = 64;

__global__ __launch_bounds__(256) void gn_rows_stats_kernel(int T, int Cg, int G, const int32_t* __restrict__ t_len,
                                                            const double* __restrict__ part, int P, float eps,
                                                            float* __restrict__ stats) {
    const int b = blockIdx.x;
    const int Tb = t_len ? t_len[b] : T;
    const int pb = (Tb + kGnRows - 1) / kGnRows;
    __shared__ double buf[kGnStatParts * 64 * 2];      // kGnStatParts parts x G <= 64 groups x (S, SS): 64 KiB
    double S = 0.0, SS = 0.0;
    for (int k0 = 0; k0 < pb; k0 += kGnStatParts) {
        const int n = (pb - k0 < kGnStatParts ? pb - k0 : kGnStatParts) * G * 2;
        const double* src = part + ((size_t)b * P + k0) * G * 2;
        for (int i = threadIdx.x; i < n; i += 256) buf[i] = src[i];
        __syncthreads();
        if (threadIdx.x < G) {
            const int g = threadIdx.x;
            for (int i = 2 * g; i < n; i += 2 * G) {
                S += buf[i];
                SS += buf[i + 1];
            }
        }
        __syncthreads();
    }
    if (threadIdx.x < G) gn_stat(S, SS, Tb, Cg, eps, stats + ((size_t)b * G + threadIdx.x) * 2);
}

__global__ __launch_bounds__(256) void gn_rows_apply_kernel(int T, int C, int G, const float* __restrict__ x,
                                                            long long x_bs, int ldx, const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, float eps, int act,
                                                            float* __restrict__ y, long long y_bs, int ldy,
                                                            const int32_t* __restrict__ t_len,
                                                            const double* __restrict__ part,
                                                            const float* __restrict__ stats,
                                                            _Float16* __restrict__ ys, long long ys_bs, int ldys,
                                                            long long sps, int* __restrict__ oflow) {
    const int pi = blockIdx.x, b = blockIdx.y, P = gridDim.x;
    const int C4 = C >> 2, Cg = C / G, rstep = 256 / C4;
    const int Tb = t_len ? t_len[b] : T;
    __shared__ float stat[64][2];                       // G <= 64: mean, rstd per group
    if (threadIdx.x < G) {
        const int g = threadIdx.x;
        if (stats) {                                    // long rows: gn_rows_stats_kernel summed the parts
            stat[g][0] = stats[((size_t)b * G + g) * 2];
            stat[g][1] = stats[((size_t)b * G + g) * 2 + 1];
        } else {
            const int pb = (Tb + kGnRows - 1) / kGnRows;   // this row's own parts, in order
            double S = 0.0, SS = 0.0;
            for (int k = 0; k < pb; ++k) {
                const double* pp = part + (((size_t)b * P + k) * G + g) * 2;
                S += pp[0];
                SS += pp[1];
            }
            gn_stat(S, SS, Tb, Cg, eps, &stat[g][0]);
        }
    }
    __syncthreads();
    const int col = threadIdx.x % C4, r0 = threadIdx.x / C4;
    if (r0 >= rstep) return;
    const int c = col * 4, g = c / Cg;
    const float mean = stat[g][0], rstd = stat[g][1];
    const f32x4 gm = *reinterpret_cast<const f32x4*>(gamma + c), bt = *reinterpret_cast<const f32x4*>(beta + c);
    const int t0 = pi * kGnRows, t1 = min(T, t0 + kGnRows);
    hfa::h2v nanacc = {(_Float16)0.0f, (_Float16)0.0f};   // the planes' range check (hfa::split_pair)
    const float c2048 = 2048.0f;
    for (int t = t0 + r0; t < t1; t += rstep) {
        f32x4 o = f32x4{0.f, 0.f, 0.f, 0.f};
        if (t < Tb) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(x + b * x_bs + (long long)t * ldx + c);
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = act_apply((v[e] - mean) * rstd * gm[e] + bt[e], act);
        }
        if (y) *reinterpret_cast<f32x4*>(y + b * y_bs + (long long)t * ldy + c) = o;
        if (ys) {
            uint2 h1, h2;
            hfa::split_pair(o[0], o[1], h1.x, h2.x, nanacc, c2048);
            hfa::split_pair(o[2], o[3], h1.y, h2.y, nanacc, c2048);
            _Float16* d = ys + b * ys_bs + (long long)t * ldys + c;
            *reinterpret_cast<uint2*>(d) = h1;
            *reinterpret_cast<uint2*>(d + sps) = h2;
        }
    }
    if (hfa::range_bad(nanacc) && oflow) *oflow = 1;
}

}  // namespace

extern "C" {

int hfa_layernorm_f32(int rows, int C, const float* x, long long ldx, const float* res, long long ldr,
                      const float* gamma, const float* beta, float eps, int act, float* y, long long ldy, int T,
                      const int32_t* t_len, hipStream_t stream) {
    return hfa_layernorm_split(rows, C, x, ldx, res, ldr, gamma, beta, eps, act, y, ldy, T, t_len, nullptr, 0, 0,
                               nullptr, stream);
}

int hfa_layernorm_split(int rows, int C, const float* x, long long ldx, const float* res, long long ldr,
                        const float* gamma, const float* beta, float eps, int act, float* y, long long ldy, int T,
                        const int32_t* t_len, uint16_t* ys_, long long ldys, long long sps, int* oflow,
                        hipStream_t stream) {
    _Float16* ys = reinterpret_cast<_Float16*>(ys_);
    if (ys && ((((uintptr_t)ys) & 7) || ldys % 4 || sps % 4)) {
        hfa::set_error("hfa_layernorm_split: split planes need 8-byte alignment and strides multiple of 4 halves");
        return HFA_EINVAL;
    }
    if (t_len && (T <= 0 || rows % T)) {
        hfa::set_error("hfa_layernorm_f32: t_len needs rows = B * T (T=%d, rows=%d)", T, rows);
        return HFA_EINVAL;
    }
    if (rows < 0 || C <= 0 || C % 4 || C > 4096 || act < 0 || act > 2) {
        hfa::set_error("hfa_layernorm_f32: bad sizes rows=%d C=%d (C%%4==0, C<=4096)", rows, C);
        return HFA_EINVAL;
    }
    if (rows == 0) return HFA_OK;
    if (!x || !gamma || !beta || (!y && !ys) ||
        (((uintptr_t)x | (uintptr_t)y | (uintptr_t)gamma | (uintptr_t)beta) & 15) || ldx % 4 || ldy % 4 ||
        (res && (((uintptr_t)res & 15) || ldr % 4))) {
        hfa::set_error("hfa_layernorm_split: operands must be non-null (y may be NULL with planes), 16-byte aligned, "
                       "strides multiple of 4");
        return HFA_EINVAL;
    }
    const int blocks = hfa::capped((rows + 3) / 4);
    const int vpl = (C + 255) / 256;
#define HFA_LN(V)                                                                                               \
    hipLaunchKernelGGL(layernorm_kernel<V>, dim3(blocks), dim3(256), 0, stream, rows, C, x, ldx, res, ldr, gamma, \
                       beta, eps, act, y, ldy, T, t_len, ys, ldys, sps, oflow)
    if (vpl <= 1) HFA_LN(1);
    else if (vpl <= 2) HFA_LN(2);
    else if (vpl <= 3) HFA_LN(3);
    else if (vpl <= 4) HFA_LN(4);
    else if (vpl <= 8) HFA_LN(8);
    else HFA_LN(16);
#undef HFA_LN
    return hfa::check_launch("hfa_layernorm_f32");
}

long long hfa_groupnorm_workspace_bytes(int B, int T, int C, int G) {
    (void)C;
    const long long a = (long long)B * G * 64 * 2 * sizeof(double) + 64;                      // split-T path
    const long long r = (long long)B * ((T + kGnRows - 1) / kGnRows) * G * 2 * sizeof(double)   // row-parallel path
                        + (long long)B * G * 2 * sizeof(float);                                 // its long-row stats
    return a > r ? a : r;
}

static bool gn_rows_ok(int C, int G) { return C % 4 == 0 && (C / G) % 4 == 0 && C <= 1024 && G <= 64 && C % G == 0; }

int hfa_groupnorm_split(int B, int T, int C, int G, const float* x, long long x_bs, int ldx, const float* gamma,
                        const float* beta, float eps, int act, float* y, long long y_bs, int ldy, const int32_t* t_len,
                        uint16_t* ys_, long long ys_bs, int ldys, long long sps, int* oflow, void* workspace,
                        hipStream_t stream) {
    _Float16* ys = reinterpret_cast<_Float16*>(ys_);
    if (B < 0 || T < 0 || C <= 0 || G <= 0 || act < 0 || act > 2 || !gn_rows_ok(C, G) || B > 65535) {
        hfa::set_error("hfa_groupnorm_split: bad sizes (C %% 4, (C/G) %% 4, C <= 1024, G <= 64)");
        return HFA_EINVAL;
    }
    if (B == 0 || T == 0) return HFA_OK;
    if (!x || !gamma || !beta || (!y && !ys) || !workspace ||
        (((uintptr_t)x | (uintptr_t)gamma | (uintptr_t)beta | (uintptr_t)y) & 15) || ldx % 4 || x_bs % 4 ||
        (y && (ldy % 4 || y_bs % 4)) || (ys && ((((uintptr_t)ys) & 7) || ldys % 4 || ys_bs % 4 || sps % 4))) {
        hfa::set_error("hfa_groupnorm_split: null or misaligned operand (16-B rows; 8-B plane rows; workspace)");
        return HFA_EINVAL;
    }
    const int P = (T + kGnRows - 1) / kGnRows;
    double* part = reinterpret_cast<double*>(workspace);
    float* stats = P > kGnStatParts ? reinterpret_cast<float*>(part + (size_t)B * P * G * 2) : nullptr;
    hipLaunchKernelGGL(gn_rows_partial_kernel, dim3(P, B), dim3(256), 0, stream, T, C, G, x, x_bs, ldx, t_len, part);
    if (stats)
        hipLaunchKernelGGL(gn_rows_stats_kernel, dim3(B), dim3(256), 0, stream, T, C / G, G, t_len, part, P, eps, stats);
    // (the apply pass may write y in place of x: every partial of the batch row is complete at this launch boundary)
    hipLaunchKernelGGL(gn_rows_apply_kernel, dim3(P, B), dim3(256), 0, stream, T, C, G, x, x_bs, ldx, gamma, beta,
                       eps, act, y, y_bs, ldy, t_len, part, stats, ys, ys_bs, ldys, sps, oflow);
    return hfa::check_launch("hfa_groupnorm_split");
}

int hfa_groupnorm_f32(int B, int T, int C, int G, const float* x, long long x_bs, int ldx, const float* gamma,
                      const float* beta, float eps, int act, float* y, long long y_bs, int ldy, const int32_t* t_len,
                      void* workspace, hipStream_t stream) {
    if (B < 0 || T < 0 || C <= 0 || G <= 0 || C % G || act < 0 || act > 2) {
        hfa::set_error("hfa_groupnorm_f32: bad sizes");
        return HFA_EINVAL;
    }
    if (B == 0 || T == 0) return HFA_OK;
    if (!x || !gamma || !beta || !y) {
        hfa::set_error("hfa_groupnorm_f32: null pointer");
        return HFA_EINVAL;
    }
    if (workspace && gn_rows_ok(C, G) && B <= 65535 &&
        !(((uintptr_t)x | (uintptr_t)gamma | (uintptr_t)beta | (uintptr_t)y) & 15) && ldx % 4 == 0 &&
        x_bs % 4 == 0 && ldy % 4 == 0 && y_bs % 4 == 0)
        return hfa_groupnorm_split(B, T, C, G, x, x_bs, ldx, gamma, beta, eps, act, y, y_bs, ldy, t_len, nullptr, 0,
                                   0, 0, nullptr, workspace, stream);
    // general shapes: one workgroup per (batch, group), or T split when that grid cannot fill the chip
    const long long per_pair = (long long)T * (C / G);
    int P = 1;
    if (workspace && (long long)B * G < 512 && per_pair > 65536) {
        P = (int)min(64LL, max(1LL, 1024LL / ((long long)B * G)));
        P = (int)min((long long)P, max(1LL, per_pair / 16384));
    }
    if (P > 1) {
        double* part = reinterpret_cast<double*>(workspace);
        // (the apply pass writes y in place of x only after every partial of its pair is complete: separate launch)
        hipLaunchKernelGGL(groupnorm_partial_kernel, dim3(G, B, P), dim3(256), 0, stream, T, C, G, P, x, x_bs, ldx,
                           t_len, part);
        hipLaunchKernelGGL(groupnorm_apply_kernel, dim3(G, B, P), dim3(256), 0, stream, T, C, G, P, x, x_bs, ldx,
                           gamma, beta, eps, act, y, y_bs, ldy, t_len, part);
    } else {
        hipLaunchKernelGGL(groupnorm_kernel, dim3(G, B), dim3(256), 0, stream, T, C, G, x, x_bs, ldx, gamma, beta,
                           eps, act, y, y_bs, ldy, t_len);
    }
    return hfa::check_launch("hfa_groupnorm_f32");
}

}  // extern "C"
