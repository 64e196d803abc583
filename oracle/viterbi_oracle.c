/* viterbi_oracle.c — TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * A plain-C restatement of the HubertFA alignment DP, used by tests/ and by bench.py's cpu_baseline leg.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may load this library.
 *
 *   hfa_oracle_forward   <- AlignmentDecoder.forward_pass   /root/reference/tools/alignment_decoder.py:170-230
 *   hfa_oracle_backtrack <- AlignmentDecoder._decode (end state + backtrack + frame confidence) :263-288
 *
 * Pinned: tests/test_oracle.py checks it bit-exact (dp, bt, curr, path) against tests/golden/dp_cases.npz,
 * which tests/golden/gen_golden.py produced by running the reference itself (numba stubbed as identity).
 *
 * Numerics: f32 sums in f32, the curr*(T/S) term in f64, store rounds to f32.  Build with
 * -ffp-contract=off (oracle/Makefile) so no a*b+c is fused.
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>

/* dp [T*S] f32 (row 0 initialised by the caller), bt [T*S] int32 (row 0 = -1), curr [S] f64 in/out. */
void hfa_oracle_forward(int T, int S, const float* prob_log, const float* not_edge_log, const float* edge_log,
                        double* curr, float* dp, int32_t* bt, const int32_t* ph_seq_id, int prob3_pad_len) {
    const double ratio = (double)T / (double)S;
    const float ninf = -INFINITY;
    for (int t = 1; t < T; ++t) {
        const float* dprev = dp + (size_t)(t - 1) * S;
        const float* L = prob_log + (size_t)t * S;
        float* drow = dp + (size_t)t * S;
        int32_t* brow = bt + (size_t)t * S;
        const float E = edge_log[t], nE = not_edge_log[t];
        for (int i = 0; i < S; ++i) {
            float p1 = dprev[i] + L[i];
            p1 = p1 + nE;
            float p2 = ninf;
            if (i >= 1) {
                float a = dprev[i - 1] + L[i - 1];
                a = a + E;
                p2 = (float)((double)a + curr[i - 1] * ratio);
            }
            float p3 = ninf;
            if (i >= prob3_pad_len) {
                const int j = i - prob3_pad_len + 1;
                if (!(j < S - 1 && ph_seq_id[j] != 0)) {
                    const int k = i - prob3_pad_len;
                    float a = dprev[k] + L[k];
                    a = a + E;
                    p3 = (float)((double)a + curr[k] * ratio);
                }
            }
            float best = p1;
            int idx = 0;
            if (p2 > best) { best = p2; idx = 1; }
            if (p3 > best) { best = p3; idx = 2; }
            drow[i] = best;
            brow[i] = idx;
        }
        /* curr update only after the whole row (p2/p3 above read the previous step's curr) */
        for (int i = 0; i < S; ++i) {
            if (brow[i] == 0) {
                const double l = (double)L[i];
                if (l > curr[i]) curr[i] = l;
            } else if (brow[i] > 0) {
                curr[i] = (double)L[i];
            }
        }
        for (int i = 0; i < S; ++i)
            if (ph_seq_id[i] == 0) curr[i] = 0.0;
    }
}

/* Returns the number of emitted (ph_idx, t) pairs written (ascending t). frame_conf has T entries. */
int hfa_oracle_backtrack(int T, int S, const float* dp, const int32_t* bt, const int32_t* ph_seq_id,
                         int32_t* ph_idx_seq, int32_t* ph_time_int, float* frame_conf) {
    int s;
    if (S >= 2 && dp[(size_t)(T - 1) * S + S - 2] > dp[(size_t)(T - 1) * S + S - 1] && ph_seq_id[S - 1] == 0)
        s = S - 2;
    else
        s = S - 1;
    int n = 0;
    /* walk backwards, then reverse in place */
    for (int t = T - 1; t >= 0; --t) {
        frame_conf[t] = dp[(size_t)t * S + s];
        const int code = bt[(size_t)t * S + s];
        if (code != 0) {
            ph_idx_seq[n] = s;
            ph_time_int[n] = t;
            ++n;
            s -= code;
        }
    }
    for (int i = 0, j = n - 1; i < j; ++i, --j) {
        int32_t a = ph_idx_seq[i]; ph_idx_seq[i] = ph_idx_seq[j]; ph_idx_seq[j] = a;
        int32_t b = ph_time_int[i]; ph_time_int[i] = ph_time_int[j]; ph_time_int[j] = b;
    }
    /* np.exp(np.diff(np.pad(fc, (1, 0)))) in f32 */
    float prev = 0.0f;
    for (int t = 0; t < T; ++t) {
        const float v = frame_conf[t];
        frame_conf[t] = expf(v - prev);
        prev = v;
    }
    return n;
}
