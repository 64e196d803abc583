// attention.hip — fp32 flash attention on MFMA (v_mfma_f32_32x32x2_f32), head_dim 64, no mask (key length
// masking only), scale applied to Q (exact for power-of-two scales such as 64^-0.5 = 1/8).
//
// Replaces: torch scaled_dot_product_attention / nn.MultiheadAttention fast path in the bshall encoder
// (networks/hubert/model.py:27-32) and transformers HubertAttention eager path
// (modeling_hubert.py eager_attention_forward: softmax(q k^T * head_dim^-0.5) v).
//
// Structure: one workgroup = 4 waves = 128 queries of one (batch, head); each wave owns 32 queries.
// K/V tiles of 32 keys are staged through double-buffered LDS and shared by the 4 waves.
// The score tile is computed TRANSPOSED (S^T = K Q^T) so each lane holds one query column and 16 keys in its
// accumulator registers: the per-query max/sum is an in-register reduction plus one xor-32 lane swap, and the
// S^T accumulator registers are directly the B operand of O^T += V^T P^T (no LDS round trip for P).
// Online softmax (running max/sum per query) avoids materialising the L x L matrix.
#include "hfa_common.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int DH = 64;
constexpr int KB = 32;          // keys per tile
constexpr int QW = 32;          // queries per wave
constexpr int NW = 4;           // waves per workgroup
constexpr int LDK = DH + 4;     // padded LDS row (ds_read_b128 conflict-free)

struct AttnP {
    int B, H, L;
    float scale;
    const float* q; long long q_bs; int q_ld;
    const float* k; long long k_bs; int k_ld;
    const float* v; long long v_bs; int v_ld;
    float* o; long long o_bs; int o_ld;
};

__global__ __launch_bounds__(NW * 64) void attn_fwd_f32_kernel(const AttnP p) {
    __shared__ __attribute__((aligned(16))) float sK[2][KB * LDK];
    __shared__ __attribute__((aligned(16))) float sV[2][KB * LDK];

    const int bh = blockIdx.y;
    const int b = bh / p.H, hd = bh - b * p.H;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int r32 = lane & 31, half = lane >> 5;
    const int q0 = blockIdx.x * (QW * NW) + wave * QW;
    const int qi = q0 + r32;

    const float* Q = p.q + b * p.q_bs + hd * DH;
    const float* Kp = p.k + b * p.k_bs + hd * DH;
    const float* Vp = p.v + b * p.v_bs + hd * DH;

    // Q fragments: lane holds Q[qi][kk*8 + half*4 + e] * scale, kk = 0..7, e = 0..3
    f32x4 qf[DH / 8];
#pragma unroll
    for (int kk = 0; kk < DH / 8; ++kk) {
        if (qi < p.L) {
            f32x4 v = *reinterpret_cast<const f32x4*>(Q + (long long)qi * p.q_ld + kk * 8 + half * 4);
            qf[kk] = v * p.scale;
        } else {
            qf[kk] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }

    // K/V staging: 32 rows x 64 floats each = 512 float4 per matrix; 256 threads x 2 each
    f32x4 rk[2], rv[2];
    auto load_tile = [&](int key0) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int idx = tid + i * NW * 64;
            const int row = idx >> 4, c4 = (idx & 15) * 4;
            const int key = key0 + row;
            const bool ok = key < p.L;
            rk[i] = ok ? *reinterpret_cast<const f32x4*>(Kp + (long long)key * p.k_ld + c4) : f32x4{0.f, 0.f, 0.f, 0.f};
            rv[i] = ok ? *reinterpret_cast<const f32x4*>(Vp + (long long)key * p.v_ld + c4) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
    };
    auto store_tile = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int idx = tid + i * NW * 64;
            const int row = idx >> 4, c4 = (idx & 15) * 4;
            *reinterpret_cast<f32x4*>(&sK[buf][row * LDK + c4]) = rk[i];
            *reinterpret_cast<f32x4*>(&sV[buf][row * LDK + c4]) = rv[i];
        }
    };

    f32x16 oacc[2];
#pragma unroll
    for (int e = 0; e < 16; ++e) { oacc[0][e] = 0.f; oacc[1][e] = 0.f; }
    float m_run = -__builtin_inff(), l_run = 0.0f;

    const int nkb = (p.L + KB - 1) / KB;
    load_tile(0);
    store_tile(0);
    __syncthreads();
    for (int kb = 0; kb < nkb; ++kb) {
        const int cur = kb & 1;
        if (kb + 1 < nkb) load_tile((kb + 1) * KB);
        // S^T[j][i] = sum_d K[j][d] * Qs[i][d]
        f32x16 s;
#pragma unroll
        for (int e = 0; e < 16; ++e) s[e] = 0.f;
#pragma unroll
        for (int kk = 0; kk < DH / 8; ++kk) {
            const f32x4 kf = *reinterpret_cast<const f32x4*>(&sK[cur][r32 * LDK + kk * 8 + half * 4]);
#pragma unroll
            for (int e = 0; e < 4; ++e) s = __builtin_amdgcn_mfma_f32_32x32x2f32(kf[e], qf[kk][e], s, 0, 0, 0);
        }
        // mask keys beyond L; block max per query (this lane's 16 keys + partner lane's 16)
        const int key0 = kb * KB;
        float bm = -__builtin_inff();
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int j = key0 + (e & 3) + 8 * (e >> 2) + 4 * half;
            if (j >= p.L) s[e] = -__builtin_inff();
            bm = fmaxf(bm, s[e]);
        }
        bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
        const float m_new = fmaxf(m_run, bm);
        const float alpha = expf(m_run - m_new);
        float ls = 0.0f;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            s[e] = expf(s[e] - m_new);
            ls += s[e];
        }
        ls += __shfl_xor(ls, 32, 64);
        l_run = l_run * alpha + ls;
        m_run = m_new;
#pragma unroll
        for (int e = 0; e < 16; ++e) { oacc[0][e] *= alpha; oacc[1][e] *= alpha; }
        // O^T[d][i] += sum_j V[j][d] * P^T[j][i]; MFMA e uses key j(e, half) = (e&3) + 8(e>>2) + 4 half
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int j = (e & 3) + 8 * (e >> 2) + 4 * half;
            const float v0 = sV[cur][j * LDK + r32];
            const float v1 = sV[cur][j * LDK + 32 + r32];
            oacc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(v0, s[e], oacc[0], 0, 0, 0);
            oacc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(v1, s[e], oacc[1], 0, 0, 0);
        }
        if (kb + 1 < nkb) store_tile(cur ^ 1);
        __syncthreads();
    }

    // normalise and stage O[i][d] through LDS (reuse sK: 4 waves x 32 queries x 68 floats fits in 2*32*68)
    const float inv = 1.0f / l_run;
    float* stage = &sK[0][0] + wave * (QW * LDK / 2);  // 32 x 34? -> use two passes of 32 dims
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
        // each wave writes its 32 queries x 32 dims (dims dt*32..) into a private 32 x 33 slab
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int d = (e & 3) + 8 * (e >> 2) + 4 * half;
            stage[r32 * 33 + d] = oacc[dt][e] * inv;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        // 32 rows x 32 floats = 256 float4 -> 4 per lane, row-contiguous global stores
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int idx = lane + i * 64;
            const int row = idx >> 3, c4 = (idx & 7) * 4;
            const int qq = q0 + row;
            if (qq < p.L) {
                f32x4 v{stage[row * 33 + c4], stage[row * 33 + c4 + 1], stage[row * 33 + c4 + 2],
                        stage[row * 33 + c4 + 3]};
                *reinterpret_cast<f32x4*>(p.o + b * p.o_bs + (long long)qq * p.o_ld + hd * DH + dt * 32 + c4) = v;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

}  // namespace

extern "C" {

int hfa_attention_f32(int B, int H, int L, int head_dim, float scale, const float* q, long long q_bs, int q_ld,
                      const float* k, long long k_bs, int k_ld, const float* v, long long v_bs, int v_ld, float* o,
                      long long o_bs, int o_ld, hipStream_t stream) {
    if (head_dim != DH) {
        hfa::set_error("hfa_attention_f32: head_dim=%d unsupported (64 only)", head_dim);
        return HFA_EINVAL;
    }
    if (B < 0 || H < 1 || L < 0) {
        hfa::set_error("hfa_attention_f32: bad sizes");
        return HFA_EINVAL;
    }
    if (B == 0 || L == 0) return HFA_OK;
    if ((((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)o) & 15) || (q_ld | k_ld | v_ld | o_ld) % 4 ||
        (q_bs | k_bs | v_bs | o_bs) % 4) {
        hfa::set_error("hfa_attention_f32: operands must be 16-byte aligned with strides multiple of 4");
        return HFA_EINVAL;
    }
    AttnP p{B, H, L, scale, q, q_bs, q_ld, k, k_bs, k_ld, v, v_bs, v_ld, o, o_bs, o_ld};
    dim3 grid((L + QW * NW - 1) / (QW * NW), B * H);
    hipLaunchKernelGGL(attn_fwd_f32_kernel, grid, dim3(NW * 64), 0, stream, p);
    return hfa::check_launch("hfa_attention_f32");
}

}  // extern "C"
