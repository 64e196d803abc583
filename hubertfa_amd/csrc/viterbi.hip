// viterbi.hip — the alignment decoder's device path: lattice prologue, monotonic max-plus DP, backtrack.
//
// Replaces (reference, read-only at /root/reference):
//   * AlignmentDecoder.decode, device part    tools/alignment_decoder.py:35-84   -> hfa_lattice_prologue
//   * AlignmentDecoder._decode lattice prep   tools/alignment_decoder.py:239-242 -> hfa_lattice_prologue
//   * AlignmentDecoder.forward_pass (numba)   tools/alignment_decoder.py:170-230 -> hfa_viterbi_forward
//   * AlignmentDecoder._decode backtrack      tools/alignment_decoder.py:263-288 -> hfa_viterbi_backtrack
//
// Numerics: dp is f32, curr_ph_max_prob_log is f64.  prob1 = (dp+L)+nE in f32;
// prob2/prob3 = f32( f64( (dp+L)+E in f32 ) + curr*(T/S) in f64 ).  Ties resolve by strict '>' in the order
// stay(0) -> advance(1) -> skip(2).  This file is compiled with -ffp-contract=off and uses explicit
// __dmul_rn/__dadd_rn so no FMA contraction changes a rounding.  Result: dp/bt bit-exact with the reference.
//
// Parallel structure (one wavefront per utterance): dp[t,.] depends only on dp[t-1, s], dp[t-1, s-1],
// dp[t-1, s-2], so the front is the whole row t: each lane owns K contiguous states, T serial steps, the
// batch spreads over CUs.  The only cross-lane traffic per step is the two "q" values of the left neighbour
// lane (DPP/permute via __shfl_up).  Emission rows for t+1.. are prefetched a group ahead so the serial
// chain never waits on HBM.
#include <type_traits>

#include "hfa_common.h"

namespace {

using hfa::neg_inf;

// One workgroup per utterance: NW waves x 64 lanes, each lane owning K contiguous states; G time steps of
// emissions are prefetched one group ahead.  With NW > 1 the two boundary q values of each wave's last lane
// cross to the next wave through a double-buffered LDS slot (one barrier per time step).
// q of the lane one below (DPP wave_shr:1: a one-cycle VALU move, where __shfl_up is an LDS ds_bpermute on
// the step's critical path); lane 0 receives -inf.
__device__ __forceinline__ float from_lane_below(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(neg_inf()), __float_as_int(v), 0x138, 0xF, 0xF,
                                                      false));
}

// VEC: Smax % K == 0 and aligned planes, so a lane's K contiguous states are loaded and stored as vectors
// (dp K x f32, bt K bytes) instead of 2K scattered narrow accesses per time step.
//
// Emission pipeline: a ring of R groups of G time steps in registers.  Group r is computed, then its slot is
// refilled for the group R ahead, so (R - 1) * G steps of compute cover a refill's memory latency.  Every load is
// unconditional (rows past T, lanes past Smax read a clamped, valid address; their values are never used): loads
// in divergent branches defeat the compiler's vmcnt tracking, which then waits for every outstanding load (the
// refill just issued included) at the top of each group — the prefetch did nothing and each group paid a full
// memory round trip.  E and nE of a group are one vector load each (lane u holds step t0 + u) broadcast per step
// with v_readlane, instead of two scalar loads per step whose lgkmcnt(0) waits also catch the refills.
//
// CF: curr held as f32.  Every value the DP writes into curr is an f32 value (L, max(curr, L), 0) and so is the
// lattice prologue's initialisation, so when every incoming curr is one (checked by the kernel below) the f64
// max / select updates become f32 ones on one register -- the same bits, ~3 fewer VALU operations per state and
// step; the f64 form stays for a caller's arbitrary f64 curr.  Only the q term is computed in f64, as before.
template <int K, int NW, int G, int R, bool VEC, bool CF>
__device__ __forceinline__ void forward_body(
    int Tmax, int Smax, const int32_t* __restrict__ Tv, const int32_t* __restrict__ Sv,
    const int32_t* __restrict__ padv, const float* __restrict__ prob_log,
    const float* __restrict__ not_edge_log, const float* __restrict__ edge_log, double* __restrict__ curr_io,
    float* __restrict__ dp, int8_t* __restrict__ bt, const int32_t* __restrict__ ph_seq_id, int t_begin, int t_end) {
    using CT = typename std::conditional<CF, float, double>::type;
    static_assert(NW == 1 || K >= 2, "multi-wave DP needs >= 2 states per lane");
    static_assert(G <= 64 && R >= 2, "a group's E / nE fit one wave's lanes; at least two groups in flight");
    __shared__ float xq[2][NW][2];
    const int b = blockIdx.x;
    const int g = threadIdx.x;
    const int lane = g & 63, wave = g >> 6;
    const int T = Tv[b];
    const int S = Sv[b];
    // time steps [t0, te) of this utterance (a range call continues from dp row t0 - 1 and from curr)
    const int t0 = max(t_begin, 1), te = min(t_end, T);
    if (te <= t0 || S <= 0) return;
    const int pad = padv ? padv[b] : (S >= 2 ? 2 : 1);
    const size_t ts = (size_t)b * Tmax * Smax;
    const float* pl = prob_log + ts;
    float* d = dp + ts;
    int8_t* bb = bt + ts;
    const float* nEp = not_edge_log + (size_t)b * Tmax;
    const float* Ep = edge_log + (size_t)b * Tmax;
    const int32_t* ids = ph_seq_id + (size_t)b * Smax;
    double* cu = curr_io + (size_t)b * Smax;
    const double ratio = (double)T / (double)S;  // `T / S` (alignment_decoder.py:186), f64 true division

    const int s0 = g * K;
    const int sl = s0 < Smax ? s0 : 0;          // load column of this lane (clamped: lanes past Smax load row start)
    float dprev[K];
    CT curr[K];
    bool valid[K], zero[K], allow3[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int s = s0 + k;
        valid[k] = s < S;
        dprev[k] = valid[k] ? d[(size_t)(t0 - 1) * Smax + s] : neg_inf();
        curr[k] = valid[k] ? (CT)cu[s] : (CT)-__builtin_inf();
        zero[k] = valid[k] && ids[s] == 0;
        // prob3 (alignment_decoder.py:191-202): -inf for s < pad, and for s >= pad when
        // (s - pad + 1 < S - 1 and ph_seq_id[s - pad + 1] != 0).
        const int j = s - pad + 1;
        allow3[k] = valid[k] && s >= pad && !((j < S - 1) && ids[j] != 0);
    }

    float L[R][G][K], EV[R], nEV[R];
    auto load = [&](float (&Lr)[G][K], float& ev, float& nev, int t0) {
        const int te = min(t0 + lane, T - 1);
        ev = Ep[te];
        nev = nEp[te];
#pragma unroll
        for (int u = 0; u < G; ++u) {
            const float* src = pl + (size_t)min(t0 + u, T - 1) * Smax;
            if (VEC && K >= 2) {
#pragma unroll
                for (int k = 0; k < K; k += 2) {
                    const float2 v = *reinterpret_cast<const float2*>(src + sl + k);
                    Lr[u][k] = v.x;
                    Lr[u][k + 1] = v.y;
                }
            } else {
#pragma unroll
                for (int k = 0; k < K; ++k) Lr[u][k] = src[min(s0 + k, Smax - 1)];
            }
        }
    };
    // dp / bt rows go out through buffer stores: a lane past Smax gets an out-of-range offset, which the hardware
    // drops, so the stores need no branch either
    const int st_off = s0 < Smax ? s0 : 0x40000000;
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

    // one time step t from emission slot (r, u): the reference's arithmetic, state by state (see the header)
    auto step = [&](const float (&Lu)[K], float E, float nE, int t) __attribute__((always_inline)) {
        float a[K], q[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            a[k] = __fadd_rn(dprev[k], Lu[k]);                                       // dp + L     (f32)
            const float a2 = __fadd_rn(a[k], E);                                     //  + E       (f32)
            q[k] = (float)__dadd_rn((double)a2, __dmul_rn((double)curr[k], ratio));  //  + C*T/S   (f64)
        }
        // left neighbour lane's last two q values (states s0-1, s0-2)
        float qm1 = from_lane_below(q[K - 1]);
        float qm2 = (K >= 2) ? from_lane_below(q[K >= 2 ? K - 2 : 0]) : from_lane_below(qm1);
        if (NW > 1) {
            if (lane == 63) {
                xq[t & 1][wave][0] = q[K - 1];
                xq[t & 1][wave][1] = q[K >= 2 ? K - 2 : 0];
            }
            __syncthreads();
            if (lane == 0 && wave > 0) {
                qm1 = xq[t & 1][wave - 1][0];
                qm2 = xq[t & 1][wave - 1][1];
            }
        }
        const size_t row = (size_t)t * Smax;
        float bestv[K];
        unsigned long long bidx = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int s = s0 + k;
            const float p1 = __fadd_rn(a[k], nE);
            const float src1 = (k >= 1) ? q[k >= 1 ? k - 1 : 0] : qm1;
            const float src2 = (k >= 2) ? q[k >= 2 ? k - 2 : 0] : (k == 1 ? qm1 : qm2);
            // (state 0: src1 is the -inf lane 0 of wave 0 gets from below, so p2 = -inf as the reference's)
            const float p2 = src1;
            const float p3 = allow3[k] ? (pad == 1 ? src1 : src2) : neg_inf();
            float best = p1;
            int idx = 0;
            if (p2 > best) { best = p2; idx = 1; }
            if (p3 > best) { best = p3; idx = 2; }
            if (VEC) {
                bestv[k] = best;
                bidx |= (unsigned long long)idx << (8 * k);
            } else if (valid[k]) {
                d[row + s] = best;
                bb[row + s] = (int8_t)idx;
            }
            // max(curr, L) on a stay (:222), L on an advance or skip (:224), 0 on a zero-id state (:226-228)
            const CT Lc = (CT)Lu[k];
            curr[k] = (idx != 0 || Lc > curr[k]) ? Lc : curr[k];
            if (zero[k]) curr[k] = (CT)0;
            dprev[k] = best;
        }
        if (VEC) {     // states past S inside the Smax pitch get don't-care values
            const __amdgpu_buffer_rsrc_t rd = hfa::make_rsrc(d + row, (long long)Smax * 4);
            const __amdgpu_buffer_rsrc_t rb = hfa::make_rsrc(bb + row, Smax);
            const int od = st_off < 0x40000000 ? st_off * 4 : 0x40000000;
#pragma unroll
            for (int k = 0; k < K; k += 4) {
                if (K - k >= 4) {
                    u32x4 w;
                    w.x = __float_as_uint(bestv[k]);
                    w.y = __float_as_uint(bestv[k + 1 < K ? k + 1 : 0]);
                    w.z = __float_as_uint(bestv[k + 2 < K ? k + 2 : 0]);
                    w.w = __float_as_uint(bestv[k + 3 < K ? k + 3 : 0]);
                    __builtin_amdgcn_raw_buffer_store_b128(w, rd, od + 4 * k, 0, 0);
                } else if (K - k >= 2) {
                    u32x2 w;
                    w.x = __float_as_uint(bestv[k]);
                    w.y = __float_as_uint(bestv[k + 1 < K ? k + 1 : 0]);
                    __builtin_amdgcn_raw_buffer_store_b64(w, rd, od + 4 * k, 0, 0);
                } else {
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(bestv[k]), rd, od + 4 * k, 0, 0);
                }
            }
            if (K == 1) __builtin_amdgcn_raw_buffer_store_b8((unsigned char)bidx, rb, st_off, 0, 0);
            else if (K == 2) __builtin_amdgcn_raw_buffer_store_b16((unsigned short)bidx, rb, st_off, 0, 0);
            else if (K == 4) __builtin_amdgcn_raw_buffer_store_b32((unsigned int)bidx, rb, st_off, 0, 0);
            else {
                u32x2 w;
                w.x = (unsigned int)bidx;
                w.y = (unsigned int)(bidx >> 32);
                __builtin_amdgcn_raw_buffer_store_b64(w, rb, st_off, 0, 0);
            }
        }
    };

#pragma unroll
    for (int r = 0; r < R; ++r) load(L[r], EV[r], nEV[r], t0 + r * G);
    int tb = t0;
    // main loop: whole rounds of R groups, straight-line (no early exits: a branch around a refill would again
    // cost the vmcnt tracking); slot r holds steps tb + r G .. + G - 1 on entry
    for (; tb + R * G <= te; tb += R * G) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
#pragma unroll
            for (int u = 0; u < G; ++u)
                step(L[r][u], __int_as_float(__builtin_amdgcn_readlane(__float_as_int(EV[r]), u)),
                     __int_as_float(__builtin_amdgcn_readlane(__float_as_int(nEV[r]), u)), tb + r * G + u);
            load(L[r], EV[r], nEV[r], tb + (r + R) * G);   // refill this slot for the group R ahead
        }
    }
    // tail (< R G steps): the slots already hold them
#pragma unroll
    for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int u = 0; u < G; ++u) {
            const int t = tb + r * G + u;
            if (t < te)   // uniform over the workgroup
                step(L[r][u], __int_as_float(__builtin_amdgcn_readlane(__float_as_int(EV[r]), u)),
                     __int_as_float(__builtin_amdgcn_readlane(__float_as_int(nEV[r]), u)), t);
        }
    }
#pragma unroll
    for (int k = 0; k < K; ++k)
        if (valid[k]) cu[s0 + k] = (double)curr[k];
}

template <int K, int NW, int G, int R, bool VEC>
__global__ __launch_bounds__(64 * NW) void viterbi_forward_kernel(
    int Tmax, int Smax, const int32_t* __restrict__ Tv, const int32_t* __restrict__ Sv,
    const int32_t* __restrict__ padv, const float* __restrict__ prob_log,
    const float* __restrict__ not_edge_log, const float* __restrict__ edge_log, double* __restrict__ curr_io,
    float* __restrict__ dp, int8_t* __restrict__ bt, const int32_t* __restrict__ ph_seq_id, int t_begin, int t_end) {
    // f32 curr (CF) when every incoming curr of the utterance is an f32 value (NaN, or f64-only values: the f64 form)
    const int b = blockIdx.x, S = Sv[b];
    bool f32 = true;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int s = (int)threadIdx.x * K + k;
        if (s < S) {
            const double c = curr_io[(size_t)b * Smax + s];
            f32 = f32 && (double)(float)c == c;
        }
    }
    if (__syncthreads_and(f32))
        forward_body<K, NW, G, R, VEC, true>(Tmax, Smax, Tv, Sv, padv, prob_log, not_edge_log, edge_log, curr_io, dp,
                                             bt, ph_seq_id, t_begin, t_end);
    else
        forward_body<K, NW, G, R, VEC, false>(Tmax, Smax, Tv, Sv, padv, prob_log, not_edge_log, edge_log, curr_io, dp,
                                              bt, ph_seq_id, t_begin, t_end);
}

// S > 8192 (up to 32768 states, the backtrack's 15-bit path entries; the reference takes any S): the
// register-resident form above runs out of lanes (16 waves x 64 x 8), so the state range is walked as up to four
// segments of 8192 inside every time step, in order.  A lane's dp[t-1] and curr come back from global memory -- its own stores of the previous step, so
// no value crosses threads through memory -- and the two boundary q values cross waves through the LDS slots as
// above and segments through the last wave's slot of the previous iteration (read before this iteration's barrier,
// so the next write of that slot, which follows the barrier, cannot overtake it).  Per-state arithmetic identical to
// viterbi_forward_kernel (bit-exact with the oracle); slower per step (an HBM/L2 round trip per segment), which only
// the rare > 8192-phoneme utterance pays.
constexpr int kWideK = 8, kWideNW = 16, kWideSeg = kWideK * kWideNW * 64;

__global__ __launch_bounds__(64 * kWideNW) void viterbi_forward_wide_kernel(
    int Tmax, int Smax, const int32_t* __restrict__ Tv, const int32_t* __restrict__ Sv,
    const int32_t* __restrict__ padv, const float* __restrict__ prob_log,
    const float* __restrict__ not_edge_log, const float* __restrict__ edge_log, double* __restrict__ curr_io,
    float* __restrict__ dp, int8_t* __restrict__ bt, const int32_t* __restrict__ ph_seq_id) {
    constexpr int K = kWideK, NW = kWideNW;
    __shared__ float xq[2][NW][2];
    const int b = blockIdx.x;
    const int g = threadIdx.x;
    const int lane = g & 63, wave = g >> 6;
    const int T = Tv[b];
    const int S = Sv[b];
    if (T <= 1 || S <= 0) return;
    const int pad = padv ? padv[b] : (S >= 2 ? 2 : 1);
    const size_t ts = (size_t)b * Tmax * Smax;
    const float* pl = prob_log + ts;
    float* d = dp + ts;
    int8_t* bb = bt + ts;
    const float* nEp = not_edge_log + (size_t)b * Tmax;
    const float* Ep = edge_log + (size_t)b * Tmax;
    const int32_t* ids = ph_seq_id + (size_t)b * Smax;
    double* cu = curr_io + (size_t)b * Smax;
    const double ratio = (double)T / (double)S;
    const int nseg = (S + kWideSeg - 1) / kWideSeg;
    int it = 0;
    for (int t = 1; t < T; ++t) {
        const float E = Ep[t], nE = nEp[t];
        const size_t row = (size_t)t * Smax, prow = (size_t)(t - 1) * Smax;
        for (int seg = 0; seg < nseg; ++seg, ++it) {
            const int s0 = seg * kWideSeg + g * K;
            float carry1 = neg_inf(), carry2 = neg_inf();   // q of states s0 - 1, s0 - 2 from the previous segment
            if (seg > 0 && g == 0) {
                carry1 = xq[(it - 1) & 1][NW - 1][0];
                carry2 = xq[(it - 1) & 1][NW - 1][1];
            }
            float a[K], q[K], dprev[K], L[K];
            double curr[K];
            bool valid[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int s = s0 + k;
                valid[k] = s < S;
                dprev[k] = valid[k] ? d[prow + s] : neg_inf();
                curr[k] = valid[k] ? cu[s] : -__builtin_inf();
                L[k] = valid[k] ? pl[row + s] : 0.0f;
                a[k] = __fadd_rn(dprev[k], L[k]);
                const float a2 = __fadd_rn(a[k], E);
                q[k] = (float)__dadd_rn((double)a2, __dmul_rn(curr[k], ratio));
            }
            float qm1 = from_lane_below(q[K - 1]);
            float qm2 = from_lane_below(q[K - 2]);
            if (lane == 63) {
                xq[it & 1][wave][0] = q[K - 1];
                xq[it & 1][wave][1] = q[K - 2];
            }
            __syncthreads();
            if (lane == 0) {
                qm1 = wave > 0 ? xq[it & 1][wave - 1][0] : carry1;
                qm2 = wave > 0 ? xq[it & 1][wave - 1][1] : carry2;
            }
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int s = s0 + k;
                if (!valid[k]) continue;
                const int j = s - pad + 1;
                const bool allow3 = s >= pad && !((j < S - 1) && ids[j] != 0);
                const float p1 = __fadd_rn(a[k], nE);
                const float src1 = (k >= 1) ? q[k >= 1 ? k - 1 : 0] : qm1;
                const float src2 = (k >= 2) ? q[k >= 2 ? k - 2 : 0] : (k == 1 ? qm1 : qm2);
                const float p2 = (s == 0) ? neg_inf() : src1;
                const float p3 = allow3 ? (pad == 1 ? src1 : src2) : neg_inf();
                float best = p1;
                int idx = 0;
                if (p2 > best) { best = p2; idx = 1; }
                if (p3 > best) { best = p3; idx = 2; }
                d[row + s] = best;
                bb[row + s] = (int8_t)idx;
                const double Ld = (double)L[k];
                double c = curr[k];
                if (idx == 0) c = (Ld > c) ? Ld : c;
                else c = Ld;
                if (ids[s] == 0) c = 0.0;
                cu[s] = c;
            }
        }
    }
}

// Backtrack (alignment_decoder.py:263-288): one 256-thread workgroup per utterance.
//   1. end state: S-2 if S>=2 and dp[T-1,S-2] > dp[T-1,S-1] and ph_seq_id[S-1]==0 else S-1 (:269-272)
//   2. bt rows staged through LDS in chunks, one lane chases s(t) from T-1 down to 0 (serial by nature),
//      recording path[t] = s | emit<<15 in LDS (emit: bt[t,s] != 0, always at t == 0 where bt is -1).
//   3. all threads: frame_conf[t] = exp(dp[t,s_t] - dp[t-1,s_{t-1}]) (np.exp(np.diff(pad(fc,(1,0))))),
//      and an ordered compaction of the emitted (s, t) pairs.
constexpr int kBtThreads = 256;
constexpr int kBtChunkBytes = 32768;
constexpr int kBtLdsFrames = 64000;          // path in LDS up to this many frames (32 KB chunk + 125 KB path)

// GPATH: the chased path (state | emit << 31 per frame) goes to frame_conf's own memory in global memory instead of
// LDS (Tmax > kBtLdsFrames: a long-form lattice past 160 KB of LDS, reference: any T): the compaction reads it there
// (non-temporal loads: L2, never a stale L1 line), then the confidence pass overwrites it tile by tile, reading each
// tile's path entries before any of its stores and carrying the previous tile's last state through LDS.  Outputs are
// identical to the LDS form.
template <bool GPATH>
__global__ __launch_bounds__(kBtThreads) void viterbi_backtrack_kernel(
    int Tmax, int Smax, const int32_t* __restrict__ Tv, const int32_t* __restrict__ Sv,
    const float* __restrict__ dp, const int8_t* __restrict__ bt, const int32_t* __restrict__ ph_seq_id,
    int32_t* __restrict__ ph_idx_seq, int32_t* __restrict__ ph_time_int, int32_t* __restrict__ n_out,
    float* __restrict__ frame_conf) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    int8_t* chunk = reinterpret_cast<int8_t*>(smem);
    uint16_t* path = reinterpret_cast<uint16_t*>(smem + kBtChunkBytes);
    uint32_t* gpath = reinterpret_cast<uint32_t*>(frame_conf) + (size_t)blockIdx.x * Tmax;
    __shared__ int s_cur, s_carry;
    __shared__ int warp_cnt[kBtThreads / 64];

    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int T = Tv[b];
    const int S = Sv[b];
    const size_t ts = (size_t)b * Tmax * Smax;
    const float* d = dp + ts;
    const int8_t* bb = bt + ts;
    const int32_t* ids = ph_seq_id + (size_t)b * Smax;
    if (T <= 0 || S <= 0) {
        if (tid == 0) n_out[b] = 0;
        return;
    }
    if (tid == 0) {
        int s = S - 1;
        if (S >= 2 && d[(size_t)(T - 1) * Smax + S - 2] > d[(size_t)(T - 1) * Smax + S - 1] && ids[S - 1] == 0)
            s = S - 2;
        s_cur = s;
    }
    // Band staging + run-skipping chase.  The chased state only ever decreases (by 0..2 per frame), so a chunk of
    // rows [lo, hi] is staged for a band of BW columns ending at the current state (whole rows when Smax <= 128);
    // when the state leaves the band the next chunk restarts from that frame.  The chase itself is wave-parallel:
    // the 64 lanes read bt at the current state for the next 64 frames at once and the first non-zero code (a
    // ballot) ends the run of 'stay' frames — the path moves about once per T/S frames, so one LDS round trip
    // covers many frames instead of one per frame.
    const bool whole = Smax <= 128;
    const int lgb = whole ? (Smax <= 16 ? 4 : 32 - __builtin_clz(Smax - 1)) : 6;   // band: 2^lgb columns
    const int BW = 1 << lgb;                                       // (the LDS row pitch)
    const int R = kBtChunkBytes >> lgb;                            // rows per chunk
    const bool dw = (Smax & 3) == 0 && (reinterpret_cast<uintptr_t>(bb) & 3) == 0;
    const int lane = tid & 63, wv = tid >> 6;
    __syncthreads();
    int hi = T - 1;
    while (hi >= 0) {
        const int top = s_cur;
        const int lo = max(0, hi - R + 1);
        const int c0 = whole ? 0 : max(0, (top & ~3) + 4 - BW);    // 4-aligned, the band [c0, top | 3] holds top
        const int ncol = min(BW, Smax - c0);                       // staged columns (the rest of the band unused)
        const int total = (hi - lo + 1) << (lgb - 2);              // dwords of the chunk
        for (int i = tid; i < total; i += kBtThreads) {
            const int r = i >> (lgb - 2), c = (i & ((BW >> 2) - 1)) << 2;
            if (c >= ncol) continue;
            const int8_t* src = bb + (size_t)(lo + r) * Smax + c0 + c;
            if (dw) {
                *reinterpret_cast<int*>(chunk + r * BW + c) = *reinterpret_cast<const int*>(src);
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) chunk[r * BW + c + j] = c + j < ncol ? src[j] : 0;
            }
        }
        __syncthreads();
        if (wv == 0) {
            int s = top, t = hi;
            while (t >= lo && s >= c0) {
                const int tl = t - lane;                           // the frame this lane checks, at state s
                const bool inr = tl >= lo;
                const int code = !inr ? 0 : (tl == 0 ? -1 : (int)chunk[(tl - lo) * BW + (s - c0)]);
                const unsigned long long nz = __ballot(code != 0);
                const int last = min(63, t - lo);                  // the last lane inside the chunk
                const int first = nz ? __ffsll((long long)nz) - 1 : last;   // lanes 0..first are this run
                const bool emits = nz != 0;
                if (lane <= first && inr) {
                    const int emit = (lane == first && emits) ? 1 : 0;
                    if constexpr (GPATH) gpath[tl] = (uint32_t)s | ((uint32_t)emit << 31);
                    else path[tl] = (uint16_t)(s | (emit << 15));
                }
                if (emits) s -= __shfl(code, first);
                if (s < 0) s = 0;                                  // (only a corrupt bt gets here)
                t -= first + 1;
            }
            if (lane == 0) s_cur = s;
            hi = t;                                                // next frame to chase (state left the band:
        }                                                          // restart the band there)
        if (wv == 0 && lane == 0) s_carry = hi;
        __syncthreads();
        hi = s_carry;
        __syncthreads();
    }
    // confidence + ordered compaction of emitted (s, t)
    int base = 0;
    for (int t0 = 0; t0 < T; t0 += kBtThreads) {
        const int t = t0 + tid;
        int emit = 0, s = 0;
        if (t < T) {
            if constexpr (GPATH) {
                const uint32_t p = __builtin_nontemporal_load(gpath + t);
                s = (int)(p & 0x7fffffffu);
                emit = (int)(p >> 31);
            } else {
                const uint16_t p = path[t];
                s = p & 0x7fff;
                emit = p >> 15;
                const float v = d[(size_t)t * Smax + s];
                float vp = 0.0f;
                if (t > 0) vp = d[(size_t)(t - 1) * Smax + (path[t - 1] & 0x7fff)];
                frame_conf[(size_t)b * Tmax + t] = expf(v - vp);
            }
        }
        const unsigned long long m = __ballot(emit);
        const int lane = tid & 63, w = tid >> 6;
        const int before = __popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) warp_cnt[w] = __popcll(m);
        __syncthreads();
        int off = base;
        for (int i = 0; i < w; ++i) off += warp_cnt[i];
        int total = 0;
        for (int i = 0; i < kBtThreads / 64; ++i) total += warp_cnt[i];
        if (emit) {
            ph_idx_seq[(size_t)b * Tmax + off + before] = s;
            ph_time_int[(size_t)b * Tmax + off + before] = t;
        }
        base += total;
        __syncthreads();
    }
    if (tid == 0) n_out[b] = base;
    if constexpr (GPATH) {                      // confidences over the path, in place of it
        if (tid == 0) s_carry = 0;
        for (int t0 = 0; t0 < T; t0 += kBtThreads) {
            const int t = t0 + tid;
            int s = 0, sp = 0;
            __syncthreads();                    // s_carry of the previous tile is set
            if (t < T) {
                s = (int)(__builtin_nontemporal_load(gpath + t) & 0x7fffffffu);
                sp = tid > 0 ? (int)(__builtin_nontemporal_load(gpath + t - 1) & 0x7fffffffu) : s_carry;
            }
            __syncthreads();                    // every path entry of this tile has been read
            if (t < T) {
                if (tid == kBtThreads - 1) s_carry = s;
                const float v = d[(size_t)t * Smax + s];
                const float vp = t > 0 ? d[(size_t)(t - 1) * Smax + sp] : 0.0f;
                frame_conf[(size_t)b * Tmax + t] = expf(v - vp);
            }
        }
    }
}

// Lattice prologue: one wavefront per DP frame row (alignment_decoder.py:35-84, 239-242).
//   x = logits_f32 - 1e9*(v not in {0} U ph_seq_id)            (:37-40, :53)
//   ph_prob_log = log_softmax(x), ph_frame_pred = softmax(x)     (:56-65)
//   e = clamp((sigmoid(edge_logit) - 0.1) / 0.8, 0, 1)           (:68-71)
//   edge_diff[t] = e[t+1]-e[t] (0 at T-1)   edge_prob = clip(e[t] + e[t-1], 0, 1) in f64   (:83-84)
//   prob_log[t,s] = ph_prob_log[t, ph_seq_id[s]]; E = f32(log(edge_prob + 1e-6)); nE = f32(log(1-edge_prob+1e-6))
constexpr int kProThreads = 256;
constexpr int kMaxV = 1024;

// _decode's initialisation (tools/alignment_decoder.py:244-254): dp[0, 0] = L[0, 0] and curr[0] = L[0, 0]; if
// ph_seq_id[0] == 0 (and S > 1) also dp[0, 1] = curr[1] = L[0, 1]; every other dp[0, s] and curr[s] = -inf (curr in
// f64, as the reference's np.full).  row0 = {L[0, 0], L[0, 1]}, or null for an all -inf row (T = 0).  Threads
// i0, i0 + step, ... of the caller cover s < Smax (rows 1.. of dp and bt are written by the forward kernel).
__device__ __forceinline__ void dp_row0(int b, int Tmax, int Smax, int S, const int32_t* ids, const float* row0,
                                        int i0, int step, float* dp, double* curr) {
    const bool two = row0 && S > 1 && ids[0] == 0;
    for (int s = i0; s < Smax; s += step) {
        float v = neg_inf();
        if (row0 && s == 0) v = row0[0];
        else if (two && s == 1) v = row0[1];
        dp[(size_t)b * Tmax * Smax + s] = v;
        curr[(size_t)b * Smax + s] = (double)v;
    }
}

__global__ __launch_bounds__(256) void viterbi_init_kernel(int Tmax, int Smax, const int32_t* __restrict__ Tv,
                                                           const int32_t* __restrict__ Sv,
                                                           const float* __restrict__ prob_log,
                                                           const int32_t* __restrict__ ph_seq_id,
                                                           float* __restrict__ dp, double* __restrict__ curr) {
    const int b = blockIdx.x;
    const float* L0 = prob_log + (size_t)b * Tmax * Smax;
    const int S = Sv[b];
    const float row0[2] = {L0[0], Smax > 1 ? L0[1] : 0.0f};
    dp_row0(b, Tmax, Smax, S, ph_seq_id + (size_t)b * Smax, Tv[b] > 0 ? row0 : nullptr, threadIdx.x, 256, dp, curr);
}

// One frame t of batch b (one wave): masked log-softmax over V into lsm, the lattice row, edge terms, dp row 0.
__device__ __forceinline__ void lattice_frame(
    int t, int b, int T, int S, int V, int Tmax, int Smax, const int32_t* __restrict__ ids,
    const unsigned char* allowed, float* lsm_w, int lane, const float* __restrict__ frame_logits, long long f_ld,
    long long f_bs, const float* __restrict__ edge_logits, long long e_ld, long long e_bs,
    float* __restrict__ ph_prob_log, float* __restrict__ ph_frame_pred, float* __restrict__ prob_log,
    float* __restrict__ edge_log, float* __restrict__ not_edge_log, float* __restrict__ edge_diff,
    double* __restrict__ edge_prob_out, float* __restrict__ dp, double* __restrict__ curr) {
    const float* xr = frame_logits + b * f_bs + t * f_ld;
    float m = neg_inf();
    for (int v = lane; v < V; v += 64) {
        const float x = xr[v] - (allowed[v] ? 0.0f : 1e9f);
        lsm_w[v] = x;
        m = fmaxf(m, x);
    }
    m = hfa::wave_max(m);
    float sum = 0.0f;
    for (int v = lane; v < V; v += 64) sum += expf(lsm_w[v] - m);
    sum = hfa::wave_sum(sum);
    const float lse = logf(sum);
    const float inv = 1.0f / sum;
    for (int v = lane; v < V; v += 64) {
        const float xm = lsm_w[v] - m;
        const float lp = xm - lse;
        if (ph_prob_log) ph_prob_log[((size_t)b * Tmax + t) * V + v] = lp;
        if (ph_frame_pred) ph_frame_pred[((size_t)b * Tmax + t) * V + v] = expf(xm) * inv;
        lsm_w[v] = lp;
    }
    __builtin_amdgcn_wave_barrier();
    for (int s = lane; s < S; s += 64) {
        const int v = ids[s];
        prob_log[((size_t)b * Tmax + t) * Smax + s] = lsm_w[v];
    }
    if (t == 0 && dp) {          // _decode's dp / curr initialisation from this frame's lattice row (no extra launch)
        const float l0 = lsm_w[ids[0]], l1 = S > 1 ? lsm_w[ids[1]] : 0.0f;
        const float row0[2] = {l0, l1};
        dp_row0(b, Tmax, Smax, S, ids, row0, lane, 64, dp, curr);
    }
    if (lane == 0) {
        const float* er = edge_logits + b * e_bs;
        auto edge_pred = [&](int tt) {
            const float x = er[tt * e_ld];
            const float sg = 1.0f / (1.0f + expf(-x));
            return fminf(fmaxf((sg - 0.1f) / 0.8f, 0.0f), 1.0f);
        };
        const float e = edge_pred(t);
        const float en = (t + 1 < T) ? edge_pred(t + 1) : 0.0f;
        const float ep = (t > 0) ? edge_pred(t - 1) : 0.0f;
        edge_diff[(size_t)b * Tmax + t] = (t + 1 < T) ? (en - e) : 0.0f;
        double pr = (double)e + (double)ep;
        pr = pr < 0.0 ? 0.0 : (pr > 1.0 ? 1.0 : pr);
        if (edge_prob_out) edge_prob_out[(size_t)b * Tmax + t] = pr;
        edge_log[(size_t)b * Tmax + t] = (float)log(pr + 1e-6);
        not_edge_log[(size_t)b * Tmax + t] = (float)log(1.0 - pr + 1e-6);
    }
}

__global__ __launch_bounds__(kProThreads) void lattice_prologue_kernel(
    int Tmax, int V, int Smax, const int32_t* __restrict__ Tv, const int32_t* __restrict__ Sv,
    const float* __restrict__ frame_logits, long long f_ld, long long f_bs, const float* __restrict__ edge_logits,
    long long e_ld, long long e_bs, const int32_t* __restrict__ ph_seq_id, float* __restrict__ ph_prob_log,
    float* __restrict__ ph_frame_pred, float* __restrict__ prob_log, float* __restrict__ edge_log,
    float* __restrict__ not_edge_log, float* __restrict__ edge_diff, double* __restrict__ edge_prob_out,
    float* __restrict__ dp, double* __restrict__ curr) {
    __shared__ unsigned char allowed[kMaxV];
    __shared__ float lsm[kProThreads / 64][kMaxV];
    const int b = blockIdx.y;
    const int T = Tv[b];
    const int S = Sv[b];
    const int32_t* ids = ph_seq_id + (size_t)b * Smax;
    for (int v = threadIdx.x; v < V; v += kProThreads) allowed[v] = (v == 0);
    __syncthreads();
    for (int s = threadIdx.x; s < S; s += kProThreads) {
        const int v = ids[s];
        if (v >= 0 && v < V) allowed[v] = 1;
    }
    __syncthreads();
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // frames t = blockIdx.x * 4 + w, + 4 gridDim.x, ... (a capped grid, hfa::grid_cap); a wave's lsm row is reused
    const int tstride = gridDim.x * (kProThreads / 64);
    const int tfirst = blockIdx.x * (kProThreads / 64) + w;
    if (tfirst == 0 && T <= 0 && dp) dp_row0(b, Tmax, Smax, 0, ids, nullptr, lane, 64, dp, curr);   // T = 0: -inf row
    for (int t = tfirst; t < T; t += tstride) {
        lattice_frame(t, b, T, S, V, Tmax, Smax, ids, allowed, lsm[w], lane, frame_logits, f_ld, f_bs, edge_logits,
                      e_ld, e_bs, ph_prob_log, ph_frame_pred, prob_log, edge_log, not_edge_log, edge_diff,
                      edge_prob_out, dp, curr);
        __builtin_amdgcn_wave_barrier();
    }
}

thread_local int g_force_k = 0;   // hfa_viterbi_tuning: states per lane of the multi-wave DP (0 = automatic)

template <int K, int NW, int G, int R>
int launch_forward(int B, int Tmax, int Smax, const int32_t* T, const int32_t* S, const int32_t* pad,
                   const float* prob_log, const float* nE, const float* E, double* curr, float* dp, int8_t* bt,
                   const int32_t* ids, int t_begin, int t_end, hipStream_t st) {
    const bool vec = Smax % K == 0 && ((uintptr_t)prob_log % 16 == 0) && ((uintptr_t)dp % 16 == 0) &&
                     ((uintptr_t)bt % 8 == 0);
    if (vec)
        hipLaunchKernelGGL((viterbi_forward_kernel<K, NW, G, R, true>), dim3(B), dim3(64 * NW), 0, st, Tmax, Smax, T,
                           S, pad, prob_log, nE, E, curr, dp, bt, ids, t_begin, t_end);
    else
        hipLaunchKernelGGL((viterbi_forward_kernel<K, NW, G, R, false>), dim3(B), dim3(64 * NW), 0, st, Tmax, Smax, T,
                           S, pad, prob_log, nE, E, curr, dp, bt, ids, t_begin, t_end);
    return hfa::check_launch("hfa_viterbi_forward");
}

}  // namespace

extern "C" {

int hfa_viterbi_forward_steps(int B, int Tmax, int Smax, const int32_t* T, const int32_t* S,
                              const int32_t* prob3_pad_len, const float* prob_log, const float* not_edge_log,
                              const float* edge_log, double* curr, float* dp, int8_t* bt, const int32_t* ph_seq_id,
                              int t_begin, int t_end, hipStream_t stream) {
    if (B < 0 || Tmax < 0 || Smax < 0 || (B > 0 && (!T || !S || !prob_log || !not_edge_log || !edge_log ||
                                                     !curr || !dp || !bt || !ph_seq_id))) {
        hfa::set_error("hfa_viterbi_forward: bad arguments");
        return HFA_EINVAL;
    }
    if (t_begin < 1 || t_end < t_begin) {
        hfa::set_error("hfa_viterbi_forward_steps: bad step range [%d, %d)", t_begin, t_end);
        return HFA_EINVAL;
    }
    if (B == 0 || Tmax == 0 || Smax == 0 || t_begin >= Tmax || t_end == t_begin) return HFA_OK;
    // one wave while a lane holds <= 8 states; beyond that K states per lane over up to 16 waves (K = 8 by
    // default, or forced to 2/4 by hfa_viterbi_tuning: more waves, fewer states each, one barrier per step)
#define HFA_FWD(K, NW, G, R)                                                                                    \
    return launch_forward<K, NW, G, R>(B, Tmax, Smax, T, S, prob3_pad_len, prob_log, not_edge_log, edge_log, curr, \
                                       dp, bt, ph_seq_id, t_begin, t_end, stream)
    // R groups of G steps in flight (K * G * R emission registers per lane, within the VGPR budget of 64 * NW
    // threads: 512 up to 4 waves, 256 at 8, 128 at 16)
    const int per_lane = (Smax + 63) / 64;
    if (per_lane <= 1) HFA_FWD(1, 1, 8, 4);
    if (per_lane <= 2) HFA_FWD(2, 1, 8, 4);
    if (per_lane <= 4) HFA_FWD(4, 1, 8, 3);
    if (per_lane <= 8 && g_force_k == 0) HFA_FWD(8, 1, 4, 4);
    // measured (scripts/dp_bench.py, T = 25 839, S = 1 801, with the emission ring): 4 states per lane over 8
    // waves 0.51 us/step, 2 over 16 0.58, 8 over 4 0.65 (before the ring: 0.68 / 0.77 / 0.98) — the step is
    // VALU-issue bound over the CU's four SIMDs, and 4 states per lane balance that against the barrier's waves
    const int kk = g_force_k ? g_force_k : (Smax <= 4096 ? 4 : 8);
    if (kk == 2 && Smax <= 2048) {
        const int w = (Smax + 127) / 128;
        if (w <= 2) HFA_FWD(2, 2, 8, 4);
        if (w <= 4) HFA_FWD(2, 4, 8, 4);
        if (w <= 8) HFA_FWD(2, 8, 8, 4);
        HFA_FWD(2, 16, 8, 3);
    }
    if (kk == 4 && Smax <= 4096) {
        const int w = (Smax + 255) / 256;
        if (w <= 2) HFA_FWD(4, 2, 4, 4);
        if (w <= 4) HFA_FWD(4, 4, 4, 4);
        if (w <= 8) HFA_FWD(4, 8, 4, 4);
        HFA_FWD(4, 16, 4, 3);
    }
    const int waves = (Smax + 511) / 512;
    if (waves <= 2) HFA_FWD(8, 2, 4, 3);
    if (waves <= 4) HFA_FWD(8, 4, 4, 3);
    if (waves <= 8) HFA_FWD(8, 8, 4, 3);
    if (waves <= 16) HFA_FWD(8, 16, 2, 3);   // 1024 threads cap VGPRs at 128: shorter groups
#undef HFA_FWD
    if (Smax <= 4 * kWideSeg) {  // the segmented form, up to 32768 states (the backtrack's 15-bit path entries)
        if (t_begin != 1 || t_end < Tmax) {
            hfa::set_error("hfa_viterbi_forward_steps: Smax=%d > %d runs whole lattices only", Smax, kWideSeg);
            return HFA_EINVAL;
        }
        hipLaunchKernelGGL(viterbi_forward_wide_kernel, dim3(B), dim3(64 * kWideNW), 0, stream, Tmax, Smax, T, S,
                           prob3_pad_len, prob_log, not_edge_log, edge_log, curr, dp, bt, ph_seq_id);
        return hfa::check_launch("hfa_viterbi_forward");
    }
    hfa::set_error("hfa_viterbi_forward: Smax=%d exceeds 32768 states per utterance", Smax);
    return HFA_EINVAL;
}

int hfa_viterbi_forward(int B, int Tmax, int Smax, const int32_t* T, const int32_t* S,
                        const int32_t* prob3_pad_len, const float* prob_log, const float* not_edge_log,
                        const float* edge_log, double* curr, float* dp, int8_t* bt, const int32_t* ph_seq_id,
                        hipStream_t stream) {
    return hfa_viterbi_forward_steps(B, Tmax, Smax, T, S, prob3_pad_len, prob_log, not_edge_log, edge_log, curr, dp,
                                     bt, ph_seq_id, 1, Tmax > 1 ? Tmax : 1, stream);
}

int hfa_viterbi_range_max_states(void) { return kWideSeg; }

int hfa_viterbi_tuning(int force_k) {
    if (force_k != 0 && force_k != 2 && force_k != 4 && force_k != 8) {
        hfa::set_error("hfa_viterbi_tuning: states per lane must be 0 (automatic), 2, 4 or 8 (got %d)", force_k);
        return HFA_EINVAL;
    }
    g_force_k = force_k;
    return HFA_OK;
}

int hfa_viterbi_backtrack(int B, int Tmax, int Smax, const int32_t* T, const int32_t* S, const float* dp,
                          const int8_t* bt, const int32_t* ph_seq_id, int32_t* ph_idx_seq, int32_t* ph_time_int,
                          int32_t* n_out, float* frame_conf, hipStream_t stream) {
    if (B < 0 || Tmax < 0 || Smax < 0 || Smax > 32768) {
        hfa::set_error("hfa_viterbi_backtrack: bad sizes (Smax<=32768)");
        return HFA_EINVAL;
    }
    if (B == 0) return HFA_OK;
    if (!T || !S || !dp || !bt || !ph_seq_id || !ph_idx_seq || !ph_time_int || !n_out || !frame_conf) {
        hfa::set_error("hfa_viterbi_backtrack: null pointer");
        return HFA_EINVAL;
    }
    if (Tmax > kBtLdsFrames) {                  // long lattice: the path in global memory (frame_conf's buffer)
        hipLaunchKernelGGL(viterbi_backtrack_kernel<true>, dim3(B), dim3(kBtThreads), kBtChunkBytes, stream, Tmax,
                           Smax, T, S, dp, bt, ph_seq_id, ph_idx_seq, ph_time_int, n_out, frame_conf);
        return hfa::check_launch("hfa_viterbi_backtrack");
    }
    const size_t lds = kBtChunkBytes + sizeof(uint16_t) * (size_t)(Tmax > 0 ? Tmax : 1);
    if (lds > 65536) {
        hipError_t e = hipFuncSetAttribute((const void*)viterbi_backtrack_kernel<false>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) {
            hfa::set_error("hfa_viterbi_backtrack: cannot reserve %zu B of LDS: %s", lds, hipGetErrorString(e));
            return -(int)e;
        }
    }
    hipLaunchKernelGGL(viterbi_backtrack_kernel<false>, dim3(B), dim3(kBtThreads), lds, stream, Tmax, Smax, T, S, dp,
                       bt, ph_seq_id, ph_idx_seq, ph_time_int, n_out, frame_conf);
    return hfa::check_launch("hfa_viterbi_backtrack");
}

int hfa_lattice_prologue(int B, int Tmax, int V, int Smax, const int32_t* T, const int32_t* S,
                         const float* frame_logits, long long frame_ld, long long frame_bs,
                         const float* edge_logits, long long edge_ld, long long edge_bs, const int32_t* ph_seq_id,
                         float* ph_prob_log, float* ph_frame_pred, float* prob_log, float* edge_log,
                         float* not_edge_log, float* edge_diff, double* edge_prob, float* dp, double* curr,
                         hipStream_t stream) {
    if (B < 0 || Tmax < 0 || V <= 0 || V > kMaxV || Smax < 0) {
        hfa::set_error("hfa_lattice_prologue: bad sizes (0 < V <= %d)", kMaxV);
        return HFA_EINVAL;
    }
    if (B == 0 || Tmax == 0) return HFA_OK;
    if (!T || !S || !frame_logits || !edge_logits || !ph_seq_id || !prob_log || !edge_log || !not_edge_log ||
        !edge_diff || (!dp != !curr)) {
        hfa::set_error("hfa_lattice_prologue: null pointer (dp and curr go together)");
        return HFA_EINVAL;
    }
    const int tb = (Tmax + kProThreads / 64 - 1) / (kProThreads / 64);
    const int gx = hfa::capped((long long)tb * B) / B;
    dim3 grid(gx > 0 ? gx : 1, B);
    hipLaunchKernelGGL(lattice_prologue_kernel, grid, dim3(kProThreads), 0, stream, Tmax, V, Smax, T, S,
                       frame_logits, frame_ld, frame_bs, edge_logits, edge_ld, edge_bs, ph_seq_id, ph_prob_log,
                       ph_frame_pred, prob_log, edge_log, not_edge_log, edge_diff, edge_prob, dp, curr);
    return hfa::check_launch("hfa_lattice_prologue");
}

int hfa_viterbi_init(int B, int Tmax, int Smax, const int32_t* T, const int32_t* S, const float* prob_log,
                     const int32_t* ph_seq_id, float* dp, double* curr, hipStream_t stream) {
    if (B < 0 || Tmax < 0 || Smax < 0 || (B > 0 && Tmax > 0 && Smax > 0 &&
                                          (!T || !S || !prob_log || !ph_seq_id || !dp || !curr))) {
        hfa::set_error("hfa_viterbi_init: bad arguments");
        return HFA_EINVAL;
    }
    if (B == 0 || Tmax == 0 || Smax == 0) return HFA_OK;
    hipLaunchKernelGGL(viterbi_init_kernel, dim3(B), dim3(256), 0, stream, Tmax, Smax, T, S, prob_log, ph_seq_id, dp,
                       curr);
    return hfa::check_launch("hfa_viterbi_init");
}

}  // extern "C"
