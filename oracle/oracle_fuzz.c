/* oracle_fuzz.c — TEST INFRASTRUCTURE ONLY: drives the C restatement of the alignment DP (viterbi_oracle.c) over
 * random lattices under AddressSanitizer + UndefinedBehaviorSanitizer (oracle/Makefile target `sanitize`,
 * tests/test_sanitizers.py).  Shapes cover T = 1, S = 1, T < S (infeasible: all -inf), SP-framed and unframed state
 * sequences, consecutive SP states, -inf emissions and ties; the lattice is prepared as _decode does
 * (alignment_decoder.py:239-257: dp/curr row 0, bt = -1, prob3 pad 2 if S >= 2).  Checks: every emitted state is in
 * [0, S), times strictly ascend, n <= T, confidences are finite or NaN-free exp() of finite differences.
 * Exit 0 = all lattices passed and no sanitizer fired. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

void hfa_oracle_forward(int T, int S, const float* prob_log, const float* not_edge_log, const float* edge_log,
                        double* curr, float* dp, int32_t* bt, const int32_t* ph_seq_id, int prob3_pad_len);
int hfa_oracle_backtrack(int T, int S, const float* dp, const int32_t* bt, const int32_t* ph_seq_id,
                         int32_t* ph_idx_seq, int32_t* ph_time_int, float* frame_conf);

static uint64_t g_s = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(void) {                       /* xorshift64* */
    g_s ^= g_s >> 12; g_s ^= g_s << 25; g_s ^= g_s >> 27;
    return (uint32_t)((g_s * 0x2545F4914F6CDD1Dull) >> 32);
}
static float urand(void) { return (rnd() >> 8) * (1.0f / 16777216.0f); }

int main(int argc, char** argv) {
    const int cases = argc > 1 ? atoi(argv[1]) : 400;
    int bad = 0;
    for (int c = 0; c < cases; ++c) {
        const int T = c < 4 ? 1 + c : 1 + (int)(rnd() % 400);
        const int S = c % 7 == 0 ? 1 : 1 + (int)(rnd() % 150);
        const int mode = (int)(rnd() % 4);               /* 0 random ids, 1 SP-framed, 2 ties, 3 -inf holes */
        float* pl = malloc(sizeof(float) * (size_t)T * S);
        float* E = malloc(sizeof(float) * T);
        float* nE = malloc(sizeof(float) * T);
        double* curr = malloc(sizeof(double) * S);
        float* dp = malloc(sizeof(float) * (size_t)T * S);
        int32_t* bt = malloc(sizeof(int32_t) * (size_t)T * S);
        int32_t* ids = malloc(sizeof(int32_t) * S);
        int32_t* idx = malloc(sizeof(int32_t) * T);
        int32_t* tim = malloc(sizeof(int32_t) * T);
        float* fc = malloc(sizeof(float) * T);
        for (int i = 0; i < S; ++i)
            ids[i] = mode == 1 ? (i % 2 == 0 ? 0 : 1 + (int)(rnd() % 60)) : (int)(rnd() % 5 == 0 ? 0 : 1 + rnd() % 60);
        for (size_t i = 0; i < (size_t)T * S; ++i) {
            float v = mode == 2 ? -1.0f : logf(urand() + 1e-6f);
            if (mode == 3 && rnd() % 9 == 0) v = -INFINITY;
            pl[i] = v;
        }
        for (int t = 0; t < T; ++t) {
            const float e = urand();
            E[t] = logf(e + 1e-6f);
            nE[t] = logf(1.0f - e + 1e-6f);
        }
        for (int i = 0; i < S; ++i) curr[i] = -INFINITY;
        for (size_t i = 0; i < (size_t)T * S; ++i) { dp[i] = -INFINITY; bt[i] = -1; }
        dp[0] = pl[0];
        curr[0] = pl[0];
        if (ids[0] == 0 && S > 1) { dp[1] = pl[1]; curr[1] = pl[1]; }
        hfa_oracle_forward(T, S, pl, nE, E, curr, dp, bt, ids, S >= 2 ? 2 : 1);
        const int n = hfa_oracle_backtrack(T, S, dp, bt, ids, idx, tim, fc);
        int ok = n >= 0 && n <= T;
        for (int i = 0; ok && i < n; ++i) {
            ok = idx[i] >= 0 && idx[i] < S && tim[i] >= 0 && tim[i] < T && (i == 0 || tim[i] > tim[i - 1]);
        }
        if (!ok) {
            printf("lattice %d (T=%d S=%d mode=%d): bad path, n=%d\n", c, T, S, mode, n);
            ++bad;
        }
        free(pl); free(E); free(nE); free(curr); free(dp); free(bt); free(ids); free(idx); free(tim); free(fc);
    }
    printf("%d lattices, %d bad\n", cases, bad);
    return bad ? 1 : 0;
}
