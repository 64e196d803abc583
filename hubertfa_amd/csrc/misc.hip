// misc.hip — bandwidth kernels around the encoder: frame-grid gather, wave normalisation, padding,
// element-wise add, and the sinc resampler entry point (a pad + the MFMA implicit GEMM of gemm.hip).
#include "hfa_common.h"
#include "hfa.h"

extern "C" int hfa_conv_gemm_f32(int M, int N, int K, int Zb, int G, const float* A, long long sAb, long long sAg,
                                 int ldx, int stride, int pad, int Cg, int Tin, const float* W, long long sWg, int ldw,
                                 const float* bias, long long sBg, const float* R, long long sRb, long long sRg,
                                 int ldr, float* C, long long sCb, long long sCg, int ldc, int epilogue,
                                 hipStream_t stream);

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// UnitsEncoder.encode nearest-frame gather (tools/encoder.py:56-59):
//   index[k] = clamp(round(f32(ratio) * f32(k)), max=U-1) (torch f32 promotion, round half to even);
//   out[b, k, :] = units[b, index[k], :] for k < n_frames; rows n_frames..T_pad-1 are zero (UNet pad,
//   networks/layer/backbone/unet.py:103-106).  One wavefront per output row, float4 copies.
// Snapshot-and-clear of device flags (the split range guard's per-batch flags): snap[i] = flags[i], flags[i] = 0.
__global__ __launch_bounds__(64) void flag_take_kernel(int n, int* __restrict__ flags, int* __restrict__ snap) {
    for (int i = threadIdx.x; i < n; i += 64) {
        snap[i] = flags[i];
        flags[i] = 0;
    }
}

__global__ __launch_bounds__(256) void units_gather_kernel(int U, int C, const float* __restrict__ units,
                                                           long long u_bs, int u_ld, int n_frames, int T_pad,
                                                           float ratio, float* __restrict__ out, long long o_bs,
                                                           int o_ld, const int32_t* __restrict__ nf_b,
                                                           const int32_t* __restrict__ U_b) {
    const int b = blockIdx.y;
    const int k = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (k >= T_pad) return;
    const int nf = nf_b ? nf_b[b] : n_frames;      // per-utterance lengths of a variable-length batch
    const int Ub = U_b ? U_b[b] : U;
    float* orow = out + b * o_bs + (long long)k * o_ld;
    if (k >= nf) {
        for (int c = lane * 4; c < C; c += 256) *reinterpret_cast<f32x4*>(orow + c) = f32x4{0.f, 0.f, 0.f, 0.f};
        return;
    }
    int idx = (int)rintf(__fmul_rn(ratio, (float)k));
    idx = idx < Ub - 1 ? idx : Ub - 1;
    const float* irow = units + b * u_bs + (long long)idx * u_ld;
    for (int c = lane * 4; c < C; c += 256) *reinterpret_cast<f32x4*>(orow + c) = *reinterpret_cast<const f32x4*>(irow + c);
}

// Zero rows t >= lens[b] of a [B, T, C] tensor (the padding rows of a variable-length batch, which convs with
// padding and GroupNorm must see as zeros / not at all).
__global__ __launch_bounds__(256) void mask_rows_kernel(int T, int C, float* __restrict__ x, long long x_bs, int ldx,
                                                        const int32_t* __restrict__ lens) {
    const int b = blockIdx.y;
    const int t0 = lens[b];
    const long long n = (long long)(T - t0) * C;
    float* xb = x + b * x_bs;
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        const int t = t0 + (int)(i / C), c = (int)(i % C);
        xb[(long long)t * ldx + c] = 0.0f;
    }
}

// Wav2Vec2FeatureExtractor zero_mean_unit_var_norm (transformers feature_extraction_wav2vec2.py): per row
// (x - mean) / sqrt(var + 1e-7), biased variance, f64 statistics.  Two launches so a row is spread over the chip:
// wav_stats_kernel sums fixed chunks of a row into f64 partials (kWavChunks per row, fixed order: deterministic),
// wav_apply_kernel re-reduces a row's partials in order and normalises its tile (float4 where aligned).
constexpr int kWavChunks = 64;

__global__ __launch_bounds__(256) void wav_stats_kernel(int N, const float* __restrict__ x, long long x_bs,
                                                        const int32_t* __restrict__ lens, double* __restrict__ part) {
    const int b = blockIdx.y, c = blockIdx.x;
    const int Nb = lens ? lens[b] : N;                // statistics over this utterance's samples only
    const int per = (Nb + kWavChunks - 1) / kWavChunks;
    const int i0 = c * per, i1 = min(Nb, i0 + per);
    const float* xr = x + b * x_bs;
    double s = 0.0, ss = 0.0;
    for (int i = i0 + threadIdx.x; i < i1; i += 256) {
        const double v = xr[i];
        s += v;
        ss += v * v;
    }
    __shared__ double red[2][4];
    s = hfa::wave_sum_d(s);
    ss = hfa::wave_sum_d(ss);
    if ((threadIdx.x & 63) == 0) { red[0][threadIdx.x >> 6] = s; red[1][threadIdx.x >> 6] = ss; }
    __syncthreads();
    if (threadIdx.x == 0) {
        part[(b * kWavChunks + c) * 2] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
        part[(b * kWavChunks + c) * 2 + 1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    }
}

__global__ __launch_bounds__(256) void wav_apply_kernel(int N, const float* __restrict__ x, long long x_bs, float eps,
                                                        float* __restrict__ y, long long y_bs,
                                                        const int32_t* __restrict__ lens,
                                                        const double* __restrict__ part, bool vec) {
    const int b = blockIdx.y;
    const int Nb = lens ? lens[b] : N;
    __shared__ float sh[2];
    if (threadIdx.x == 0) {
        double S = 0.0, SS = 0.0;
        for (int c = 0; c < kWavChunks; ++c) {
            S += part[(b * kWavChunks + c) * 2];
            SS += part[(b * kWavChunks + c) * 2 + 1];
        }
        const double mean = Nb > 0 ? S / Nb : 0.0;
        double var = Nb > 0 ? SS / Nb - mean * mean : 0.0;
        if (var < 0) var = 0;
        sh[0] = (float)mean;
        sh[1] = (float)sqrt((double)(float)var + (double)eps);
    }
    __syncthreads();
    const float meanf = sh[0], den = sh[1];
    const float* xr = x + b * x_bs;
    float* yr = y + b * y_bs;
    const int i0 = blockIdx.x * 4096;
    if (vec) {
        for (int i = i0 + threadIdx.x * 4; i < min(N, i0 + 4096); i += 1024) {
            if (i + 3 < N) {
                const f32x4 v = *reinterpret_cast<const f32x4*>(xr + i);
                f32x4 o;
#pragma unroll
                for (int t = 0; t < 4; ++t) o[t] = i + t < Nb ? (v[t] - meanf) / den : 0.0f;
                *reinterpret_cast<f32x4*>(yr + i) = o;
            } else {
                for (int t = 0; t < 4 && i + t < N; ++t) yr[i + t] = i + t < Nb ? (xr[i + t] - meanf) / den : 0.0f;
            }
        }
    } else {
        for (int i = i0 + threadIdx.x; i < min(N, i0 + 4096); i += 256) yr[i] = i < Nb ? (xr[i] - meanf) / den : 0.0f;
    }
}

// y[b, i] = x[b, i - left] inside [0, N), else 0, for i < N_out.
__global__ __launch_bounds__(256) void pad_rows_kernel(int N, const float* __restrict__ x, long long x_bs, int left,
                                                       int N_out, float* __restrict__ y, long long y_bs) {
    const int b = blockIdx.y;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < N_out; i += gridDim.x * 256) {
        const int s = i - left;
        y[b * y_bs + i] = (s >= 0 && s < N) ? x[b * x_bs + s] : 0.0f;
    }
}

// Split planes of a zero-padded row: y[p][b][i] (i < Lp) of v = x[b, i - front] inside [0, N), else 0 (the resampler's
// sinc padding): hi = f16(v), lo = f16((v - hi) * 2^11); 8 samples per thread, 16-B plane stores; raises *oflow for
// |v| >= 65504 or a non-finite v.
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
__global__ __launch_bounds__(256) void pad_split_kernel(int N, int Lp, int front, const float* __restrict__ x,
                                                        long long x_bs, _Float16* __restrict__ y, long long y_bs,
                                                        long long y_sp, int* __restrict__ oflow) {
    const int b = blockIdx.y;
    bool bad = false;
    for (int i0 = (blockIdx.x * 256 + threadIdx.x) * 8; i0 < Lp; i0 += gridDim.x * 256 * 8) {
        f16x8_t h1, h2;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int s = i0 + k - front;
            const float v = (s >= 0 && s < N) ? x[b * x_bs + s] : 0.0f;
            bad |= !(__builtin_fabsf(v) < 65504.0f);
            h1[k] = (_Float16)v;
            h2[k] = (_Float16)((v - (float)h1[k]) * 2048.0f);
        }
        *reinterpret_cast<f16x8_t*>(y + b * y_bs + i0) = h1;
        *reinterpret_cast<f16x8_t*>(y + b * y_bs + i0 + y_sp) = h2;
    }
    if (bad && oflow) *oflow = 1;
}

__global__ __launch_bounds__(256) void add_kernel(long long n4, const f32x4* __restrict__ a,
                                                  const f32x4* __restrict__ b, f32x4* __restrict__ o) {
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) o[i] = a[i] + b[i];
}

__global__ __launch_bounds__(256) void erf_check_kernel(long long n, const float* __restrict__ x,
                                                        float* __restrict__ y_nb, float* __restrict__ y_ref) {
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        y_nb[i] = hfa::erf_nb(x[i]);
        y_ref[i] = erff(x[i]);
    }
}

__global__ __launch_bounds__(256) void gelu_check_kernel(long long n, const float* __restrict__ x,
                                                         float* __restrict__ y) {
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) y[i] = hfa::gelu_fast(x[i]);
}

inline int grid1d(long long n, int per = 256, int cap = 8192) {
    long long g = (n + per - 1) / per;
    return (int)(g < 1 ? 1 : (g > cap ? cap : g));
}

}  // namespace

extern "C" {

int hfa_units_gather_f32(int B, int U, int C, const float* units, long long u_bs, int u_ld, int n_frames, int T_pad,
                         float ratio, float* out, long long o_bs, int o_ld, const int32_t* n_frames_b,
                         const int32_t* U_b, hipStream_t stream) {
    if (B < 0 || U < 1 || C <= 0 || C % 4 || n_frames < 0 || T_pad < n_frames || u_ld % 4 || o_ld % 4 ||
        u_bs % 4 || o_bs % 4 || (((uintptr_t)units | (uintptr_t)out) & 15)) {
        hfa::set_error("hfa_units_gather_f32: bad arguments");
        return HFA_EINVAL;
    }
    if (B == 0 || T_pad == 0) return HFA_OK;
    hipLaunchKernelGGL(units_gather_kernel, dim3((T_pad + 3) / 4, B), dim3(256), 0, stream, U, C, units, u_bs, u_ld,
                       n_frames, T_pad, ratio, out, o_bs, o_ld, n_frames_b, U_b);
    return hfa::check_launch("hfa_units_gather_f32");
}

int hfa_mask_rows_f32(int B, int T, int C, float* x, long long x_bs, int ldx, const int32_t* lens,
                      hipStream_t stream) {
    if (B < 0 || T < 0 || C < 1 || !x || !lens || ldx < C) {
        hfa::set_error("hfa_mask_rows_f32: bad arguments");
        return HFA_EINVAL;
    }
    if (B == 0 || T == 0) return HFA_OK;
    hipLaunchKernelGGL(mask_rows_kernel, dim3(grid1d((long long)T * C, 256, 512), B), dim3(256), 0, stream, T, C, x,
                       x_bs, ldx, lens);
    return hfa::check_launch("hfa_mask_rows_f32");
}

long long hfa_wav_normalize_workspace_bytes(int B) { return B > 0 ? (long long)B * kWavChunks * 2 * 8 : 0; }

int hfa_wav_normalize_f32(int B, int N, const float* x, long long x_bs, float eps, float* y, long long y_bs,
                          const int32_t* lens, void* workspace, hipStream_t stream) {
    if (B < 0 || N <= 0 || !x || !y || (B > 0 && !workspace) || B > 65535) {
        hfa::set_error("hfa_wav_normalize_f32: bad arguments");
        return HFA_EINVAL;
    }
    if (B == 0) return HFA_OK;
    double* part = static_cast<double*>(workspace);
    hipLaunchKernelGGL(wav_stats_kernel, dim3(kWavChunks, B), dim3(256), 0, stream, N, x, x_bs, lens, part);
    const bool vec = ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0 && x_bs % 4 == 0 && y_bs % 4 == 0;
    hipLaunchKernelGGL(wav_apply_kernel, dim3((N + 4095) / 4096, B), dim3(256), 0, stream, N, x, x_bs, eps, y, y_bs,
                       lens, part, vec);
    return hfa::check_launch("hfa_wav_normalize_f32");
}

int hfa_pad_rows_f32(int B, int N, const float* x, long long x_bs, int left, int N_out, float* y, long long y_bs,
                     hipStream_t stream) {
    if (B < 0 || N < 0 || N_out < 0 || !x || !y) {
        hfa::set_error("hfa_pad_rows_f32: bad arguments");
        return HFA_EINVAL;
    }
    if (B == 0 || N_out == 0) return HFA_OK;
    hipLaunchKernelGGL(pad_rows_kernel, dim3(grid1d(N_out, 256, 1024), B), dim3(256), 0, stream, N, x, x_bs, left,
                       N_out, y, y_bs);
    return hfa::check_launch("hfa_pad_rows_f32");
}

// Self-test: the branch-free erf used by every GELU epilogue vs the device library's erff.
int hfa_selftest_erf(long long n, const float* x, float* y_nb, float* y_ref, hipStream_t stream) {
    if (n < 0 || !x || !y_nb || !y_ref) {
        hfa::set_error("hfa_selftest_erf: bad arguments");
        return HFA_EINVAL;
    }
    if (n == 0) return HFA_OK;
    hipLaunchKernelGGL(erf_check_kernel, dim3(grid1d(n)), dim3(256), 0, stream, n, x, y_nb, y_ref);
    return hfa::check_launch("hfa_selftest_erf");
}

// Self-test: the GELU every fused epilogue applies (hfa::gelu_fast), element-wise.
int hfa_selftest_gelu(long long n, const float* x, float* y, hipStream_t stream) {
    if (n < 0 || !x || !y) {
        hfa::set_error("hfa_selftest_gelu: bad arguments");
        return HFA_EINVAL;
    }
    if (n == 0) return HFA_OK;
    hipLaunchKernelGGL(gelu_check_kernel, dim3(grid1d(n)), dim3(256), 0, stream, n, x, y);
    return hfa::check_launch("hfa_selftest_gelu");
}

int hfa_flag_take(int n, int* flags, int* snap, hipStream_t stream) {
    if (n < 0 || (n > 0 && (!flags || !snap))) {
        hfa::set_error("hfa_flag_take: bad arguments");
        return HFA_EINVAL;
    }
    if (n == 0) return HFA_OK;
    hipLaunchKernelGGL(flag_take_kernel, dim3(1), dim3(64), 0, stream, n, flags, snap);
    return hfa::check_launch("hfa_flag_take");
}

int hfa_add_f32(long long n, const float* a, const float* b, float* out, hipStream_t stream) {
    if (n < 0 || n % 4 || (((uintptr_t)a | (uintptr_t)b | (uintptr_t)out) & 15)) {
        hfa::set_error("hfa_add_f32: n must be a multiple of 4 and operands 16-byte aligned");
        return HFA_EINVAL;
    }
    if (n == 0) return HFA_OK;
    hipLaunchKernelGGL(add_kernel, dim3(grid1d(n / 4)), dim3(256), 0, stream, n / 4,
                       reinterpret_cast<const f32x4*>(a), reinterpret_cast<const f32x4*>(b),
                       reinterpret_cast<f32x4*>(out));
    return hfa::check_launch("hfa_add_f32");
}

// torchaudio Resample (sinc_interp_hann) as pad + implicit GEMM (tools/load_wav.py:7, tools/encoder.py:46-48):
//   xpad = pad(x, (width, width + orig)); out[f*new + p] = sum_k xpad[f*orig + k] * kernel[p][k]
// orig/new are the gcd-reduced rates, kernel [new][Kpad] (taps 2*width+orig zero-padded to Kpad % 16 == 0).
// y must hold F*new floats per row (F = N/orig + 1, y_bs >= F*new); the valid length is ceil(new*N/orig).
long long hfa_resample_workspace_bytes(int B, int N, int orig, int Kpad) {
    const long long F = N / orig + 1;
    return (long long)B * (F * orig + Kpad + 4) * sizeof(float) + 64;
}

int hfa_resample_f32(int B, int N, const float* x, long long x_bs, int orig, int newr, const float* kernel, int Kpad,
                     int width, void* workspace, float* y, long long y_bs, hipStream_t stream) {
    if (B < 0 || N <= 0 || orig <= 0 || newr <= 0 || Kpad % 16 || Kpad < 2 * width + orig || !x || !kernel ||
        !workspace || !y) {
        hfa::set_error("hfa_resample_f32: bad arguments");
        return HFA_EINVAL;
    }
    if (B == 0) return HFA_OK;
    const long long F = N / orig + 1;
    if (y_bs < F * newr) {
        hfa::set_error("hfa_resample_f32: y_bs=%lld < F*new=%lld", y_bs, F * newr);
        return HFA_EINVAL;
    }
    const long long plen = F * orig + Kpad + 4;
    float* xpad = reinterpret_cast<float*>(workspace);
    int rc = hfa_pad_rows_f32(B, N, x, x_bs, width, (int)plen, xpad, plen, stream);
    if (rc) return rc;
    return hfa_conv_gemm_f32((int)F, newr, Kpad, B, 1, xpad, plen, 0, orig, 1, 0, Kpad, (int)F, kernel, 0, Kpad,
                             nullptr, 0, nullptr, 0, 0, 0, y, y_bs, 0, newr, 0, stream);
}

// The same resampler on the split-f16 GEMM (f32-class accuracy): the padded rows as split planes in the workspace,
// then one implicit GEMM whose A rows start 16-B aligned.  G = 1 (orig % 8 == 0): frame f at f * orig.  G = 8
// (orig % 8 == 1, e.g. 441): frames f = 8 m + g as 8 groups, group g's row m at g (orig - 1) + 8 orig m (8-aligned),
// i.e. 'g' samples before frame f's true start, so group g's taps are the kernel shifted right by g (Wg [2][G][new][Kg]
// split planes, built by the caller; Kg % 32 == 0, Kg >= 2 width + orig + G - 1); output frame f row = C + g new +
// m * 8 new.  y holds F8 * 8 * new floats per row for G = 8 (F8 = ceil(F / 8)), F * new for G = 1.
// ---- a two-stage sinc chain at its row edges (hfa_resample_chain_edges) -----------------------------------------
// torchaudio's ceil(as_tensor(a * n / b)): the quotient rounded to float32 before the ceil (resample.target_length)
__device__ __forceinline__ int ceil_f32_quot(long long a, long long n, long long b) {
    const float q = (float)((double)(a * n) / (double)b);
    return (int)__builtin_ceilf(q);
}

// The frame a slot stands for: slot s < FL is left frame s, slot FL + j the j-th frame of the right edge (from the
// first whose second-stage window reaches len_u); -1 when the row has no such frame.
__device__ __forceinline__ int chain_slot_frame(int slot, int FL, int len_u, int len_y, int P, int Q, int tail,
                                                int y_cols) {
    int i;
    if (slot < FL) {
        i = slot;
    } else {
        const int num = len_u - tail;
        i = (num <= 0 ? 0 : (num + Q - 1) / Q) + (slot - FL);
    }
    return (P * i >= len_y || P * i >= y_cols) ? -1 : i;
}

// Edge pass, part 1: one thread per sample of a slot's intermediate window u[Q i - wd_width, + kwd), computed as the
// first stage computes it (x zero outside [0, Nb); a sequential f32 FMA chain over its kwu taps, k-major taps wu_t
// [kwu][Q] so consecutive phases read consecutive addresses) and zero outside [0, len_u) as the second stage's
// padding has it; into the workspace [B][FS][kwd].  Many small workgroups: each CU streams few tap bytes.
constexpr int kChainUThreads = 128, kChainQW = 32, kChainParts = 16;
__global__ __launch_bounds__(kChainUThreads) void chain_window_kernel(int N, const int32_t* __restrict__ lens,
                                                                      const float* __restrict__ x, long long x_bs,
                                                                      int P, int Q, const float* __restrict__ wu_t,
                                                                      int kwu, int wu_width, int kwd, int wd_width,
                                                                      int FL, int FS, int y_cols,
                                                                      float* __restrict__ uw) {
    const int b = blockIdx.z, slot = blockIdx.y, t = blockIdx.x * kChainUThreads + threadIdx.x;
    const int Nb = lens ? min(lens[b], N) : N;      // (a row never reads past N)
    if (Nb <= 0 || t >= kwd) return;
    const int len_u = ceil_f32_quot(Q, Nb, P);
    const int len_y = ceil_f32_quot(P, len_u, Q);
    const int i = chain_slot_frame(slot, FL, len_u, len_y, P, Q, kwd - 1 - wd_width, y_cols);
    if (i < 0) return;
    const int r = Q * i - wd_width + t;
    float v = 0.0f;
    if (r >= 0 && r < len_u) {
        const int f = r / Q, ph = r - f * Q;
        const int s0 = P * f - wu_width;
        const int k0 = s0 < 0 ? -s0 : 0, k1 = Nb - s0 < kwu ? Nb - s0 : kwu;
        const float* w = wu_t + ph;
        const float* xr = x + b * x_bs + s0;
#pragma unroll 8
        for (int k = k0; k < k1; ++k) v = __builtin_fmaf(w[k * Q], xr[k], v);
    }
    uw[((long long)b * FS + slot) * kwd + t] = v;
}

// Edge pass, part 2: one workgroup per (slice of kChainQW output phases, slot, row): the window (LDS) against the
// slice's columns of the second stage's taps (k-major wd_t [kwd][P]), kChainParts partial FMA chains per output over
// consecutive l ranges, summed in a fixed order -- the same bits for a row in any batch.
__global__ __launch_bounds__(kChainQW * kChainParts) void chain_frame_kernel(int N, const int32_t* __restrict__ lens,
                                                                             int P, int Q, int kwd, int wd_width,
                                                                             const float* __restrict__ wd_t, int FL,
                                                                             int FS, const float* __restrict__ uw,
                                                                             float* __restrict__ y, long long y_bs,
                                                                             int y_cols) {
    extern __shared__ float su[];                          // [kwd] window, then [kChainParts][kChainQW] partial sums
    float* part = su + kwd;
    const int b = blockIdx.z, slot = blockIdx.y, q0 = blockIdx.x * kChainQW;
    const int Nb = lens ? min(lens[b], N) : N;      // (a row never reads past N)
    if (Nb <= 0) return;
    const int len_u = ceil_f32_quot(Q, Nb, P);
    const int len_y = ceil_f32_quot(P, len_u, Q);
    const int i = chain_slot_frame(slot, FL, len_u, len_y, P, Q, kwd - 1 - wd_width, y_cols);
    if (i < 0) return;
    const float* u = uw + ((long long)b * FS + slot) * kwd;
    for (int t = threadIdx.x; t < kwd; t += kChainQW * kChainParts) su[t] = u[t];
    __syncthreads();
    const int ql = threadIdx.x % kChainQW, pt = threadIdx.x / kChainQW, q = q0 + ql;
    const int span = (kwd + kChainParts - 1) / kChainParts;
    const int l0 = pt * span, l1 = l0 + span < kwd ? l0 + span : kwd;
    float acc = 0.0f;
    if (q < P) {
        const float* w = wd_t + q;
#pragma unroll 8
        for (int l = l0; l < l1; ++l) acc = __builtin_fmaf(w[l * P], su[l], acc);
    }
    part[pt * kChainQW + ql] = acc;
    __syncthreads();
    if (pt == 0 && q < P) {
        const int n = P * i + q;
        if (n < len_y && n < y_cols) {
            float sum = part[ql];
#pragma unroll
            for (int k = 1; k < kChainParts; ++k) sum += part[k * kChainQW + ql];
            y[b * y_bs + n] = sum;
        }
    }
}

static long long resample_split_lp(int N, int orig, int Kg, int G) {
    const long long F = N / orig + 1;
    const long long rows = G == 1 ? F : (F + 7) / 8;
    const long long need = G == 1 ? (F - 1) * orig + Kg : 7LL * (orig - 1) + (rows - 1) * 8 * orig + Kg;
    return (need + 7) / 8 * 8;
}

long long hfa_resample_split_workspace_bytes(int B, int N, int orig, int Kg, int G) {
    if (B < 0 || N <= 0 || orig <= 0 || (G != 1 && G != 8)) return -1;
    return 2LL * B * resample_split_lp(N, orig, Kg, G) * 2 + 64;
}

int hfa_resample_split(int B, int N, const float* x, long long x_bs, int orig, int newr, const uint16_t* Wg, int Kg,
                       int G, int width, void* workspace, float* y, long long y_bs, int* oflow, hipStream_t stream) {
    if (B < 0 || N <= 0 || orig <= 0 || newr <= 0 || width < 0 || !x || !Wg || !workspace || !y ||
        !(G == 1 ? orig % 8 == 0 : (G == 8 && orig % 8 == 1)) || Kg % 32 || Kg < 2 * width + orig + G - 1 ||
        ((uintptr_t)workspace & 15)) {
        hfa::set_error("hfa_resample_split: bad arguments (G = 1 needs orig %% 8 == 0, G = 8 orig %% 8 == 1; "
                       "Kg %% 32 == 0 and >= 2 width + orig + G - 1)");
        return HFA_EINVAL;
    }
    if (B == 0) return HFA_OK;
    const long long F = N / orig + 1;
    const long long rows = G == 1 ? F : (F + 7) / 8;
    if (y_bs < rows * (G == 1 ? 1 : 8) * newr) {
        hfa::set_error("hfa_resample_split: y_bs=%lld too small", y_bs);
        return HFA_EINVAL;
    }
    const long long Lp = resample_split_lp(N, orig, Kg, G);
    if (Lp >= (1LL << 30) / 2) {
        hfa::set_error("hfa_resample_split: row too long");
        return HFA_EINVAL;
    }
    _Float16* planes = reinterpret_cast<_Float16*>(workspace);
    hipLaunchKernelGGL(pad_split_kernel, dim3(grid1d(Lp / 8, 256, 1024), B), dim3(256), 0, stream, N, (int)Lp, width,
                       x, x_bs, planes, Lp, (long long)B * Lp, oflow);
    if (int rc = hfa::check_launch("hfa_resample_split")) return rc;
    const int ldx = G == 1 ? orig : 8 * orig;
    return hfa_conv_gemm_split((int)rows, newr, Kg, B, G, reinterpret_cast<const uint16_t*>(planes), (long long)B * Lp,
                               Lp, G == 1 ? 0 : orig - 1, ldx, 1, 0, Kg, (int)rows, Wg, (long long)G * newr * Kg,
                               (long long)newr * Kg, Kg, nullptr, 0, nullptr, 0, 0, 0, nullptr, 0, y, nullptr, 0, y_bs,
                               G == 1 ? 0 : newr, G == 1 ? newr : 8 * newr, 0, oflow, stream);
}

static inline int chain_slots(int Q, int kwd, int wd_width) {
    return (wd_width + Q - 1) / Q + (kwd - 1 - wd_width) / Q + 2;   // left frames + right frames (+ slack)
}

long long hfa_resample_chain_edges_workspace_bytes(int B, int Q, int kwd, int wd_width) {
    if (B < 0 || Q <= 0 || kwd <= 0 || wd_width < 0 || wd_width >= kwd) return -1;
    return (long long)B * chain_slots(Q, kwd, wd_width) * kwd * 4 + 64;
}

int hfa_resample_chain_edges(int B, int N, const int32_t* lens, const float* x, long long x_bs, int P, int Q,
                             const float* wu_t, int kwu, int wu_width, const float* wd_t, int kwd, int wd_width,
                             void* workspace, float* y, long long y_bs, int y_cols, hipStream_t stream) {
    if (B < 0 || B > 65535 || N <= 0 || !x || P <= 0 || Q <= 0 || !wu_t || kwu <= 0 || wu_width < 0 || !wd_t ||
        kwd <= 0 || wd_width < 0 || wd_width >= kwd || !workspace || ((uintptr_t)workspace & 15) || !y ||
        y_cols < 0 || y_bs < y_cols || (long long)(kwd + kChainParts * kChainQW) * 4 > 64 * 1024 ||
        (long long)Q * N / P > (1LL << 30)) {
        hfa::set_error("hfa_resample_chain_edges: bad arguments");
        return HFA_EINVAL;
    }
    if (B == 0 || y_cols == 0) return HFA_OK;
    const int FL = (wd_width + Q - 1) / Q, FS = chain_slots(Q, kwd, wd_width);
    float* uw = static_cast<float*>(workspace);
    hipLaunchKernelGGL(chain_window_kernel, dim3((kwd + kChainUThreads - 1) / kChainUThreads, FS, B),
                       dim3(kChainUThreads), 0, stream, N, lens, x, x_bs, P, Q, wu_t, kwu, wu_width, kwd, wd_width,
                       FL, FS, y_cols, uw);
    if (int rc = hfa::check_launch("hfa_resample_chain_edges")) return rc;
    hipLaunchKernelGGL(chain_frame_kernel, dim3((P + kChainQW - 1) / kChainQW, FS, B), dim3(kChainQW * kChainParts),
                       (kwd + kChainParts * kChainQW) * sizeof(float), stream, N, lens, P, Q, kwd, wd_width, wd_t, FL,
                       FS, uw, y, y_bs, y_cols);
    return hfa::check_launch("hfa_resample_chain_edges");
}

}  // extern "C"
