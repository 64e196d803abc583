/* hfa.h — C ABI of libhfa.so: hand-written gfx950 (MI355X, CDNA4) kernels for the HubertFA inference path.
 *
 * Conventions (all entry points):
 *   - return 0 on success, HFA_EINVAL (-1000) on a bad argument, -(hipError_t) on a HIP launch error;
 *     hfa_last_error() gives the calling thread's last message.
 *   - every pointer is a DEVICE pointer owned by the caller; the library never allocates persistent memory
 *     and never frees caller memory.
 *   - stream-ordered on `stream`, no implicit synchronisation, re-entrant across streams/threads, so every
 *     call can be captured into a hipGraph.
 *   - plain pointers and sizes only (no torch types); layouts are row-major with the strides named.
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
int hfa_abi_version(void);
const char* hfa_build_arch(void);

/* ---- alignment decoder (hubertfa_amd/csrc/viterbi.hip) ------------------------------------------------------
 * hfa_viterbi_forward replaces AlignmentDecoder.forward_pass, tools/alignment_decoder.py:170-230 (numba JIT),
 * batched: utterance b has T[b] frames and S[b] states inside [Tmax, Smax] planes.
 *   prob_log [B,Tmax,Smax] f32, not_edge_log/edge_log [B,Tmax] f32, ph_seq_id [B,Smax] i32,
 *   curr [B,Smax] f64 (in/out, = curr_ph_max_prob_log), dp [B,Tmax,Smax] f32 (row 0 in, rows 1.. out),
 *   bt [B,Tmax,Smax] i8 (rows 1.. out; = backtrack_s), prob3_pad_len [B] i32 or NULL (=2 if S>=2 else 1).
 * Bit-exact with the reference (f32 sums, f64 curr*(T/S) term, strict '>' ties stay->advance->skip).
 * Smax <= 2048. */
int hfa_viterbi_forward(int B, int Tmax, int Smax, const int32_t* T, const int32_t* S,
                        const int32_t* prob3_pad_len, const float* prob_log, const float* not_edge_log,
                        const float* edge_log, double* curr, float* dp, int8_t* bt, const int32_t* ph_seq_id,
                        hipStream_t stream);

/* hfa_viterbi_backtrack replaces the backward half of AlignmentDecoder._decode,
 * tools/alignment_decoder.py:263-288: end state, serial backtrack, frame_confidence = exp(diff([0]+dp_path)).
 * Outputs: ph_idx_seq/ph_time_int [B,Tmax] i32 (first n_out[b] valid, ascending t), frame_conf [B,Tmax] f32.
 * Smax <= 32767, Tmax <= 65536. */
int hfa_viterbi_backtrack(int B, int Tmax, int Smax, const int32_t* T, const int32_t* S, const float* dp,
                          const int8_t* bt, const int32_t* ph_seq_id, int32_t* ph_idx_seq, int32_t* ph_time_int,
                          int32_t* n_out, float* frame_conf, hipStream_t stream);

/* hfa_lattice_prologue replaces the device half of AlignmentDecoder.decode, tools/alignment_decoder.py:35-84,
 * and _decode's lattice prep :239-242.  frame_logits row (b,t) at frame_logits + b*frame_bs + t*frame_ld
 * (V contiguous floats); edge logit at edge_logits + b*edge_bs + t*edge_ld.
 * Outputs: prob_log [B,Tmax,Smax] (= ph_prob_log[:, ph_seq_id]), edge_log/not_edge_log [B,Tmax] f32,
 * edge_diff [B,Tmax] f32, edge_prob [B,Tmax] f64 (may be NULL), ph_prob_log/ph_frame_pred [B,Tmax,V] (may be
 * NULL).  V <= 1024. */
int hfa_lattice_prologue(int B, int Tmax, int V, int Smax, const int32_t* T, const int32_t* S,
                         const float* frame_logits, long long frame_ld, long long frame_bs,
                         const float* edge_logits, long long edge_ld, long long edge_bs, const int32_t* ph_seq_id,
                         float* ph_prob_log, float* ph_frame_pred, float* prob_log, float* edge_log,
                         float* not_edge_log, float* edge_diff, double* edge_prob, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* HFA_H_ */
