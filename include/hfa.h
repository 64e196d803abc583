/* hfa.h — C ABI of libhfa.so: hand-written gfx950 (MI355X, CDNA4) kernels for the HubertFA inference path.
 *
 * Conventions (all entry points):
 *   - return 0 on success, HFA_EINVAL (-1000) on a bad argument, -(hipError_t) on a HIP launch error;
 *     hfa_last_error() gives the calling thread's last message.
 *   - every pointer is a DEVICE pointer owned by the caller (except the host-side WAV reader's), the library
 *     never allocates persistent memory and never frees caller memory.
 *   - stream-ordered on `stream`, no implicit synchronisation, re-entrant across streams/threads, so every
 *     call can be captured into a hipGraph.  The *_tuning hooks (benchmark overrides) set state of the calling
 *     thread only (thread-local), so they never change another thread's launches.
 *   - plain pointers and sizes only (no torch types); layouts are row-major with the strides named.
 *
 *   - variable-length batches: the optional `const int32_t*` length arrays ([B], device) give each row's own
 *     length; statistics (GroupNorm, conv0's GroupNorm, wave normalisation) and attention keys cover that
 *     length only, and padding rows come out as zeros (or don't-care where stated), so every utterance gets
 *     the result it would get alone — the reference runs one utterance at a time.  NULL = all rows full.
 *
 * Each entry cites the reference interface it replaces (paths relative to the HubertFA repository).
 */
#ifndef HFA_H_
#define HFA_H_

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HFA_EINVAL (-1000)

/* ---- library ------------------------------------------------------------------------------------------- */
const char* hfa_last_error(void);
/* HFA_ABI_VERSION: bumped on every incompatible change of an entry point's arguments or of the set of entry points
 * (INTEGRATION.md §4 lists the changes); bindings check hfa_abi_version() == the version they were written for. */
#define HFA_ABI_VERSION 2
int hfa_abi_version(void);
const char* hfa_build_arch(void);

/* ---- WAV front end (hubertfa_amd/csrc/wav.cpp; HOST memory, no stream, never touches the GPU) ----------------
 * Replace torchaudio.load in tools/load_wav.py:5 (default normalize=True): RIFF/WAVE, PCM 8/16/24/32-bit or IEEE
 * float 32/64, plain or WAVE_FORMAT_EXTENSIBLE; samples scaled as torchaudio (uint8 (x-128)/128, int16 / 2^15,
 * 24-bit / 2^23, int32 / 2^31, f64 rounded to f32).  A data chunk longer than the file ends at end of file.
 * hfa_wav_info reads the headers only (frames per channel, channels, sample rate): the length-sorted batch plan
 * and the multi-GPU shard costs need every file's length before any is decoded.
 * hfa_wav_read decodes channel `channel` (0-based; the reference keeps waveform[0]) into dst[frames], or every
 * channel planar into dst[channels][frames] with channel = -1; `capacity` is dst's size in floats (HFA_EINVAL
 * if the samples do not fit).  `path` is a NUL-terminated file name; both are re-entrant. */
int hfa_wav_info(const char* path, int64_t* frames, int32_t* channels, int32_t* sample_rate);
int hfa_wav_read(const char* path, int32_t channel, float* dst, int64_t capacity, int64_t* frames,
                 int32_t* sample_rate);

/* ---- alignment decoder (hubertfa_amd/csrc/viterbi.hip) ------------------------------------------------------
 * hfa_viterbi_forward replaces AlignmentDecoder.forward_pass, tools/alignment_decoder.py:170-230 (numba JIT),
 * batched: utterance b has T[b] frames and S[b] states inside [Tmax, Smax] planes.
 *   prob_log [B,Tmax,Smax] f32, not_edge_log/edge_log [B,Tmax] f32, ph_seq_id [B,Smax] i32,
 *   curr [B,Smax] f64 (in/out, = curr_ph_max_prob_log), dp [B,Tmax,Smax] f32 (row 0 in, rows 1.. out),
 *   bt [B,Tmax,Smax] i8 (rows 1.. out; = backtrack_s), prob3_pad_len [B] i32 or NULL (=2 if S>=2 else 1).
 * Bit-exact with the reference (f32 sums, f64 curr*(T/S) term, strict '>' ties stay->advance->skip).
 * Smax <= 32768 (one wave up to 512 states, then 2-8 states per lane over up to 16 waves to 8192 states, then the
 * state range as segments of 8192 walked in order inside each time step). */
int hfa_viterbi_forward(int B, int Tmax, int Smax, const int32_t* T, const int32_t* S,
                        const int32_t* prob3_pad_len, const float* prob_log, const float* not_edge_log,
                        const float* edge_log, double* curr, float* dp, int8_t* bt, const int32_t* ph_seq_id,
                        hipStream_t stream);

/* The same DP over time steps [t_begin, t_end) only (t_begin >= 1; clipped to each utterance's T[b]): it continues
 * from dp row t_begin - 1 and from curr, and leaves curr for the next range, so consecutive ranges give the bits of
 * one whole call.  Lets the caller cut a long lattice (config 5: 25 839 steps, 13 ms on one CU) into pieces that
 * run beside the next batch's attention kernels.  Smax > 8192 (the segmented-state form): whole ranges only. */
int hfa_viterbi_forward_steps(int B, int Tmax, int Smax, const int32_t* T, const int32_t* S,
                              const int32_t* prob3_pad_len, const float* prob_log, const float* not_edge_log,
                              const float* edge_log, double* curr, float* dp, int8_t* bt, const int32_t* ph_seq_id,
                              int t_begin, int t_end, hipStream_t stream);
/* The largest Smax for which hfa_viterbi_forward_steps takes partial step ranges (8192: past it the segmented-state
 * form runs whole lattices only); callers that cut a DP into ranges ask the library instead of repeating it. */
int hfa_viterbi_range_max_states(void);

/* Tuning hook (tests, benchmarks): states per lane of the multi-wave forward DP, 2 / 4 / 8, 0 = automatic (4 up
 * to 4096 states, then 8); the same bits whatever the choice. */
int hfa_viterbi_tuning(int force_k);

/* hfa_viterbi_backtrack replaces the backward half of AlignmentDecoder._decode,
 * tools/alignment_decoder.py:263-288: end state, serial backtrack, frame_confidence = exp(diff([0]+dp_path)).
 * Outputs: ph_idx_seq/ph_time_int [B,Tmax] i32 (first n_out[b] valid, ascending t), frame_conf [B,Tmax] f32.
 * Smax <= 32768; any Tmax (past 64000 frames the chased path is kept in frame_conf's buffer instead of LDS). */
int hfa_viterbi_backtrack(int B, int Tmax, int Smax, const int32_t* T, const int32_t* S, const float* dp,
                          const int8_t* bt, const int32_t* ph_seq_id, int32_t* ph_idx_seq, int32_t* ph_time_int,
                          int32_t* n_out, float* frame_conf, hipStream_t stream);

/* hfa_lattice_prologue replaces the device half of AlignmentDecoder.decode, tools/alignment_decoder.py:35-84,
 * and _decode's lattice prep :239-242.  frame_logits row (b,t) at frame_logits + b*frame_bs + t*frame_ld
 * (V contiguous floats); edge logit at edge_logits + b*edge_bs + t*edge_ld.
 * Outputs: prob_log [B,Tmax,Smax] (= ph_prob_log[:, ph_seq_id]), edge_log/not_edge_log [B,Tmax] f32,
 * edge_diff [B,Tmax] f32, edge_prob [B,Tmax] f64 (may be NULL), ph_prob_log/ph_frame_pred [B,Tmax,V] (may be
 * NULL).  V <= 1024.  dp [B,Tmax,Smax] f32 / curr [B,Smax] f64 (both or neither): also _decode's DP
 * initialisation, tools/alignment_decoder.py:244-254 (dp row 0 and curr, as hfa_viterbi_init), from frame 0's
 * lattice row, so hfa_viterbi_forward can follow directly. */
int hfa_lattice_prologue(int B, int Tmax, int V, int Smax, const int32_t* T, const int32_t* S,
                         const float* frame_logits, long long frame_ld, long long frame_bs,
                         const float* edge_logits, long long edge_ld, long long edge_bs, const int32_t* ph_seq_id,
                         float* ph_prob_log, float* ph_frame_pred, float* prob_log, float* edge_log,
                         float* not_edge_log, float* edge_diff, double* edge_prob, float* dp, double* curr,
                         hipStream_t stream);
/* hfa_viterbi_init replaces _decode's initialisation, tools/alignment_decoder.py:244-254, for a lattice that did not
 * come through hfa_lattice_prologue: dp[b,0,0] = curr[b,0] = prob_log[b,0,0]; if ph_seq_id[b,0] == 0 and S[b] > 1
 * also dp[b,0,1] = curr[b,1] = prob_log[b,0,1]; every other dp[b,0,s] and curr[b,s] (s < Smax) = -inf; T[b] = 0:
 * the whole row -inf. */
int hfa_viterbi_init(int B, int Tmax, int Smax, const int32_t* T, const int32_t* S, const float* prob_log,
                     const int32_t* ph_seq_id, float* dp, double* curr, hipStream_t stream);

/* ---- dense contractions (hubertfa_amd/csrc/gemm.hip): f32 MFMA implicit GEMM ---------------------------------
 * C[z](m,n) = epi(sum_k A[z](m,k) W[z](n,k) + bias[zg*sBg + n]) + R[z](m,n),  z = zb*G + zg,
 * A[z](m,k): k = j*Cg + c, t = m*stride + j - pad, value X[zb*sAb + zg*sAg + t*ldx + c] if 0 <= t < Tin else 0.
 * W[z] row n at W + zg*sWg + n*ldw (K contiguous, conv weights in [Cout][k][Cin] im2col order).
 * epilogue: 0 none, 1 erf-GELU (applied before the residual add).  K % 16 == 0, Cg % 16 == 0, Cg | K.
 * Replaces ATen addmm (nn.Linear) and conv1d on the path:
 *   networks/hubert/model.py:100-114 (conv1-6), :122 (projection), :135-147 (grouped positional conv),
 *   :27-33 (nn.TransformerEncoderLayer in/out proj, linear1/2), transformers HubertAttention/HubertFeedForward,
 *   networks/layer/block/resnet_block.py:17-40 (k3 convs :18-24,27-33, shortcut :36-40), networks/layer/scaling/stride_conv.py:23-47
 *   (k2 s2 conv, ConvTranspose), networks/task/forced_alignment.py:53-55 (head). */
int hfa_conv_gemm_f32(int M, int N, int K, int Zb, int G, const float* A, long long sAb, long long sAg, int ldx,
                      int stride, int pad, int Cg, int Tin, const float* W, long long sWg, int ldw,
                      const float* bias, long long sBg, const float* R, long long sRb, long long sRg, int ldr,
                      float* C, long long sCb, long long sCg, int ldc, int epilogue, hipStream_t stream);
/* Tuning hook for benchmarks: force the staging pipeline of hfa_conv_gemm_f32 (16/32 = register-staged K-step,
 * 102/103 = LDS-DMA with 2/3 stages) and the tile configuration (1..7, see gemm.hip); 0 = automatic. */
int hfa_gemm_tuning(int force_pipe, int force_cfg);
/* Name (rocprof symbol stem) of the kernel instantiation hfa_conv_gemm_f32 launches for the same arguments, e.g.
 * "gemm_dma_kernel<1, 128, 128, 2, 2, 2, 4, true>"; thread-local storage, valid until the next call. */
const char* hfa_gemm_kernel_name(int M, int N, int K, int Zb, int G, const float* A, long long sAb, long long sAg,
                                 int ldx, int stride, int pad, int Cg, int Tin, const float* W, long long sWg, int ldw,
                                 const float* bias, long long sBg, const float* R, long long sRb, long long sRg,
                                 int ldr, float* C, long long sCb, long long sCg, int ldc, int epilogue);
/* Plain Linear: C[M,N] = epi(A[M,K] W[N,K]^T + bias) + R. */
int hfa_gemm_f32(int M, int N, int K, const float* A, int lda, const float* W, int ldw, const float* bias,
                 const float* R, int ldr, float* C, int ldc, int epilogue, hipStream_t stream);

/* ---- split-f16 GEMM (gemm.hip gemm_split_kernel) -------------------------------------------------------------
 * The same contractions as hfa_conv_gemm_f32 with f32-class accuracy on the f16 MFMA: every f32 operand x is
 * carried as two f16 planes, x1 = f16(x) and x2 = f16((x - x1) * 2^11) (plane 1 at +sAp / +sWp / +sCp halves;
 * every stride in halves), and A.W = A1.W1 + 2^-11 (A1.W2 + A2.W1), each partial product exact in f32.
 * Requirements: K a multiple of 32, Cg a multiple of 32 (or of 8 and >= 32: per-lane tap tracking, f32 C only); A/W 16-B aligned with 8-half strides; |x| < 65504 for every split value
 * (producers raise *oflow otherwise; the caller recomputes on the f32 path) and |w| < 32 for W (the large
 * single-accumulator tiles form 2^11 * w1 in f16; an overflow there yields a non-finite result, which also raises
 * *oflow).  Output: f32 C (+R, 16-B rows), or with Cs non-NULL and C NULL split planes of epi(acc + bias) (no R),
 * or with both non-NULL the f32 C and the split planes of that same final value (dual output).  Rs (instead of
 * R, f32 C alone): the residual as split planes (plane 1 at +sRp; strides sRb, sRg, ldr in halves), added as
 * hi + 2^-11 lo -- the residual stream carried by the planes a LayerNorm already wrote for the next GEMM.
 * epilogue | HFA_GEMM_F16: opt-in fast mode -- the high planes alone, one f16 product per MAC (A1.W1, f32
 * accumulation: f16-class accuracy, about 2.5x the split rate); ignored by the grouped positional conv kernels
 * (Cg not a multiple of 32 or N = 48/64 windows), which keep the three products. */
#define HFA_GEMM_F16 0x100
int hfa_conv_gemm_split(int M, int N, int K, int Zb, int G, const uint16_t* A, long long sAp, long long sAb,
                        long long sAg, int ldx, int stride, int pad, int Cg, int Tin, const uint16_t* W,
                        long long sWp, long long sWg, int ldw, const float* bias, long long sBg, const float* R,
                        long long sRb, long long sRg, int ldr, const uint16_t* Rs, long long sRp, float* C,
                        uint16_t* Cs, long long sCp, long long sCb, long long sCg, int ldc, int epilogue, int* oflow,
                        hipStream_t stream);
/* rocprof symbol stem of the split instantiation for an M x N x K contraction over Z = Zb*G (out_split: planes out;
 * stride 1 assumed, as the grouped positional conv's window kernel needs). */
const char* hfa_gemm_split_kernel_name(int M, int N, int K, int Z, int out_split, int epilogue, int Cg);
/* Tile override for the split GEMM (tests, benchmarks): 0 auto; 15 the N = 48 kernel (16x16x32 MFMA; chosen
 * automatically for N = 48 with f32 output, e.g. the grouped positional conv at Cg = 48); 16 the LDS-window
 * positional conv kernel; 17 / 18 / 19 / 20 the 256x256 / 128x128 / 128x64 / 256x64 tiles; 23 / 24 256x192 /
 * 192x256 (one round of 252 tiles for N = 768 at B*T = 15968 rows); 25 128x192 with two workgroups per CU.  Every
 * tile is a single-accumulator v_mfma_f32_16x16x32_f16 tile, so results do not depend on the tile.  Other values
 * (the retired tuning-only tiles 1-14, 21, 22, 26) return HFA_EINVAL and leave the override unchanged. */
int hfa_gemm_split_tuning(int cfg);
/* x [rows, cols] f32 (row stride ldx) -> split planes y (row stride ldy, plane 1 at +sp); raises *oflow (if
 * non-NULL) for |x| >= 65504 or a non-finite x. */
int hfa_split_f16(int rows, int cols, const float* x, long long ldx, uint16_t* y, long long ldy, long long sp,
                  int* oflow, hipStream_t stream);

/* ---- attention (hubertfa_amd/csrc/attention.hip) -----------------------------------------------------------
 * O = softmax(scale * Q K^T) V per (batch, head), head_dim 64, fp32 MFMA flash attention.
 * Q(b,h,i,d) at q + b*q_bs + i*q_ld + h*64 + d (same for k, v, o).
 * With key_len, O rows i >= key_len[b] (padding queries) are written as zeros.
 * Replaces nn.MultiheadAttention/SDPA in networks/hubert/model.py:27-32 and transformers
 * modeling_hubert.py HubertAttention (eager_attention_forward). */
int hfa_attention_f32(int B, int H, int L, int head_dim, float scale, const float* q, long long q_bs, int q_ld,
                      const float* k, long long k_bs, int k_ld, const float* v, long long v_bs, int v_ld, float* o,
                      long long o_bs, int o_ld, const int32_t* key_len, hipStream_t stream);
/* The same attention on split-f16 planes (see hfa_conv_gemm_split): Q, K, V read as plane pairs (plane 1 at
 * +q_sp / +k_sp / +v_sp halves), O written as plane pairs (+o_sp); every contraction is three exact f16 MFMA
 * products (f32-class accuracy).  Pointers 16-B aligned, strides multiples of 8 halves; |O| <= max |V|. */
int hfa_attention_split(int B, int H, int L, int head_dim, float scale, const uint16_t* q, long long q_sp,
                        long long q_bs, int q_ld, const uint16_t* k, long long k_sp, long long k_bs, int k_ld,
                        const uint16_t* v, long long v_sp, long long v_bs, int v_ld, uint16_t* o, long long o_sp,
                        long long o_bs, int o_ld, const int32_t* key_len, hipStream_t stream);
/* Waves (x 32 queries) per workgroup of hfa_attention_split: 4 or 8, 0 = automatic (the form whose grid gives the
 * busiest CU fewer query rows; on a tie 8 from 2048 keys).  Results do not depend on it (every query row sees the
 * same tiles in the same order). */
int hfa_attention_split_tuning(int waves);
/* MFMA form of hfa_attention_split (tuning / A-B; 0 = automatic = 16): 16 = v_mfma_f32_16x16x32_f16, 32 =
 * v_mfma_f32_32x32x16_f16 (the round-2..5 kernel).  The same products in the same key-tile order; outputs agree to
 * f32 rounding.  HFA_EINVAL for any other value. */
int hfa_attention_split_form(int form);
/* Name of the instantiation hfa_attention_split launches for (B, H, L) under the current tuning (profiler labels). */
const char* hfa_attention_split_kernel_name(int B, int H, int L);

/* ---- normalisation (hubertfa_amd/csrc/norm.hip); act: 0 none, 1 erf-GELU, 2 Hardswish -----------------------
 * y = act(LayerNorm(x (+ res)) * gamma + beta) over rows of C <= 4096 (C % 4 == 0).
 * Replaces LayerNorm in networks/hubert/model.py:25,121 and nn.TransformerEncoderLayer norm1/2,
 * transformers HubertFeatureProjection/HubertEncoder(*StableLayerNorm)/HubertLayerNormConvLayer,
 * networks/layer/block/resnet_block.py:42-45 (LN + Hardswish). */
int hfa_layernorm_f32(int rows, int C, const float* x, long long ldx, const float* res, long long ldr,
                      const float* gamma, const float* beta, float eps, int act, float* y, long long ldy, int T,
                      const int32_t* t_len, hipStream_t stream);
/* hfa_layernorm_f32 that also writes its output as split-f16 planes (see hfa_conv_gemm_split): ys row r at
 * ys + r*ldys, plane 1 at +sps halves (8-B aligned rows), so the consuming split GEMM needs no conversion pass;
 * *oflow raised for outputs outside f16 range.  y may be NULL: planes only (the consumers read the residual from
 * them, hfa_conv_gemm_split Rs). */
int hfa_layernorm_split(int rows, int C, const float* x, long long ldx, const float* res, long long ldr,
                        const float* gamma, const float* beta, float eps, int act, float* y, long long ldy, int T,
                        const int32_t* t_len, uint16_t* ys, long long ldys, long long sps, int* oflow,
                        hipStream_t stream);
/* GroupNorm(G, C) over a channels-last [B, T, C] tensor (+act).  Replaces resnet_block.py:25-26
 * (nn.GroupNorm(16, C) + nn.Hardswish). */
int hfa_groupnorm_f32(int B, int T, int C, int G, const float* x, long long x_bs, int ldx, const float* gamma,
                      const float* beta, float eps, int act, float* y, long long y_bs, int ldy, const int32_t* t_len,
                      void* workspace, hipStream_t stream);
/* Workspace for hfa_groupnorm_f32's split-T path (long rows, few (batch, group) pairs); NULL workspace = one
 * workgroup per pair. */
long long hfa_groupnorm_workspace_bytes(int B, int T, int C, int G);
/* GroupNorm (+act) of channels-last [B, T, C] (resnet_block.py:17-26, GroupNorm(16) + Hardswish) writing f32 y
 * and / or split-f16 planes ys (plane 1 at +sps halves; the next split GEMM's operand: the UNet block's second conv);
 * C % 4 == 0, (C/G) % 4 == 0, C <= 1024, G <= 64; workspace = hfa_groupnorm_workspace_bytes(B, T, C, G) bytes; rows
 * t >= t_len[b] are zeros and excluded from the statistics; *oflow raised for a plane value out of f16 range. */
int hfa_groupnorm_split(int B, int T, int C, int G, const float* x, long long x_bs, int ldx, const float* gamma,
                        const float* beta, float eps, int act, float* y, long long y_bs, int ldy, const int32_t* t_len,
                        uint16_t* ys, long long ys_bs, int ldys, long long sps, int* oflow, void* workspace,
                        hipStream_t stream);

/* ---- extractor conv0 (hubertfa_amd/csrc/conv.hip) ------------------------------------------------------------
 * x [B, N] -> y [B, T0, 512] channels-last, T0 = (N-10)/5+1.  norm=1: GroupNorm(512,512) + GELU
 * (networks/hubert/model.py:98-99,108; transformers HubertGroupNormConvLayer), needs a workspace of
 * hfa_conv0_workspace_bytes(B, N).  norm=0: conv + bias only (HubertLayerNormConvLayer's conv). */
long long hfa_conv0_workspace_bytes(int B, int N);
int hfa_conv0_f32(int B, int N, const float* x, long long x_bs, const float* w0, const float* bias, int norm,
                  const float* gamma, const float* beta, float eps, void* workspace, float* y, long long y_bs,
                  const int32_t* t0_len, hipStream_t stream);
/* hfa_conv0_f32 with the output written as split-f16 planes (see hfa_conv_gemm_split): ys [2][B][T0][512],
 * batch stride y_bs and plane stride y_sp in halves; *oflow raised for outputs outside f16 range. */
int hfa_conv0_split(int B, int N, const float* x, long long x_bs, const float* w0, const float* bias, int norm,
                    const float* gamma, const float* beta, float eps, void* workspace, uint16_t* ys, long long y_bs,
                    long long y_sp, int* oflow, const int32_t* t0_len, hipStream_t stream);

/* ---- glue (hubertfa_amd/csrc/misc.hip) -----------------------------------------------------------------------
 * Nearest-frame gather onto the DP grid, tools/encoder.py:56-59: idx[k] = min(rint(f32(ratio)*k), U-1),
 * out[b,k,:] = units[b,idx[k],:] for k < n_frames, zero rows up to T_pad (unet.py:103-106 padding). */
int hfa_units_gather_f32(int B, int U, int C, const float* units, long long u_bs, int u_ld, int n_frames, int T_pad,
                         float ratio, float* out, long long o_bs, int o_ld, const int32_t* n_frames_b,
                         const int32_t* U_b, hipStream_t stream);
/* Wav2Vec2FeatureExtractor zero-mean/unit-variance normalisation (tools/encoder.py:94-95), f64 statistics over each
 * row's own lens[b] samples; workspace: hfa_wav_normalize_workspace_bytes(B) bytes of device memory (row partials). */
long long hfa_wav_normalize_workspace_bytes(int B);
int hfa_wav_normalize_f32(int B, int N, const float* x, long long x_bs, float eps, float* y, long long y_bs,
                          const int32_t* lens, void* workspace, hipStream_t stream);
/* Zero rows t >= lens[b] of a [B, T, C] tensor (row t of batch b at x + b*x_bs + t*ldx): the padding rows of a
 * variable-length batch, which padded convs must read as zeros (reference: each utterance runs alone, B=1). */
int hfa_mask_rows_f32(int B, int T, int C, float* x, long long x_bs, int ldx, const int32_t* lens,
                      hipStream_t stream);
/* Zero padding of rows (networks/hubert/model.py:77 F.pad 40/40; resampler edge padding). */
int hfa_pad_rows_f32(int B, int N, const float* x, long long x_bs, int left, int N_out, float* y, long long y_bs,
                     hipStream_t stream);
/* Self-test: y_nb = the branch-free erf of every GELU epilogue, y_ref = device erff (must be bit-identical). */
int hfa_selftest_erf(long long n, const float* x, float* y_nb, float* y_ref, hipStream_t stream);
/* Self-test: y = the GELU applied by every fused epilogue (GEMM, LayerNorm/GroupNorm act, conv0). */
int hfa_selftest_gelu(long long n, const float* x, float* y, hipStream_t stream);
/* Range-guard bookkeeping (no reference counterpart: the split-f16 arithmetic's per-batch overflow flags): snap[i] =
 * flags[i], then flags[i] = 0, for i < n, stream-ordered (the batch's snapshot travels with its outputs). */
int hfa_flag_take(int n, int* flags, int* snap, hipStream_t stream);
/* Workgroup cap (no reference counterpart; 0 = none, the default) for this host thread's later launches of the
 * row-streaming kernels -- hfa_split_f16, hfa_layernorm_f32 / _split, hfa_lattice_prologue: a capped launch runs its
 * rows in a grid-stride loop over at most `wgs` workgroups (results identical).  The pipelined step enqueues its side
 * pass (UNet head + lattice, beside the next batch's encoder) under a cap: its tens of thousands of one-row
 * workgroups otherwise cost the encoder more than their work. */
int hfa_set_grid_cap(int wgs);
/* out = a + b (UNet skip connection, networks/layer/backbone/unet.py:114). */
int hfa_add_f32(long long n, const float* a, const float* b, float* out, hipStream_t stream);
/* torchaudio.transforms.Resample (sinc_interp_hann) as pad + MFMA GEMM (tools/load_wav.py:7,
 * tools/encoder.py:46-48).  orig/newr gcd-reduced; kernel [newr][Kpad]; y_bs >= (N/orig+1)*newr. */
/* The resampler on the split-f16 GEMM (f32-class): x padded and split into the workspace, then one split GEMM with
 * 16-B aligned rows.  G = 1 for orig % 8 == 0 (frame f at f * orig), G = 8 for orig % 8 == 1 (e.g. 44100 -> 16000:
 * frames 8m+g as 8 groups, group g's taps shifted right by g): Wg is [2][G][new][Kg] split planes of those taps
 * (Kg % 32 == 0, Kg >= 2 width + orig + G - 1).  y: F*new (G = 1) or ceil(F/8)*8*new (G = 8) floats per row;
 * the valid length is ceil(new*N/orig).  *oflow as hfa_split_f16. */
long long hfa_resample_split_workspace_bytes(int B, int N, int orig, int Kg, int G);
int hfa_resample_split(int B, int N, const float* x, long long x_bs, int orig, int newr, const uint16_t* Wg, int Kg,
                       int G, int width, void* workspace, float* y, long long y_bs, int* oflow, hipStream_t stream);
/* The composite of two sinc stages that return to the input rate (16 k -> 44.1 k -> 16 k: tools/load_wav.py:7 then
 * tools/encoder.py:46-48) runs as ONE hfa_resample_split pass (orig = newr = P, the composed taps); this entry
 * overwrites the output frames that pass cannot express -- those whose second-stage window reaches past the
 * intermediate row, where each stage alone zero-pads: the first ceil(wd_width / Q) frames and the frames from
 * ceil((len_u - (kwd - 1 - wd_width)) / Q) to the row's last output, computed as the two stages compute them
 * (f32): each frame's intermediate window into the workspace (hfa_resample_chain_edges_workspace_bytes), then the
 * frame's outputs.  P, Q: the first stage's gcd-reduced orig / new (the second's new / orig); wu_t [kwu][Q] and wd_t
 * [kwd][P] the stages' f32 taps, k-major; lens [B] per-row input lengths (NULL: N); len_u and the row's output
 * length follow torchaudio's float32-quotient ceil.  y: [B][y_bs] (y_cols columns exist); kwd + 512 floats fit
 * 64 KiB. */
long long hfa_resample_chain_edges_workspace_bytes(int B, int Q, int kwd, int wd_width);
int hfa_resample_chain_edges(int B, int N, const int32_t* lens, const float* x, long long x_bs, int P, int Q,
                             const float* wu_t, int kwu, int wu_width, const float* wd_t, int kwd, int wd_width,
                             void* workspace, float* y, long long y_bs, int y_cols, hipStream_t stream);
long long hfa_resample_workspace_bytes(int B, int N, int orig, int Kpad);
int hfa_resample_f32(int B, int N, const float* x, long long x_bs, int orig, int newr, const float* kernel, int Kpad,
                     int width, void* workspace, float* y, long long y_bs, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* HFA_H_ */
