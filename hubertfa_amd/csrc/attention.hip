// attention.hip — fp32 flash attention on MFMA (v_mfma_f32_32x32x2_f32), head_dim 64, no mask (key length
// masking only); scale * log2(e) is folded into Q (softmax evaluated as exp2, same value up to rounding).
//
// Replaces: torch scaled_dot_product_attention / nn.MultiheadAttention fast path in the bshall encoder
// (networks/hubert/model.py:27-32) and transformers HubertAttention eager path
// (modeling_hubert.py eager_attention_forward: softmax(q k^T * head_dim^-0.5) v).
//
// Structure: one workgroup = 4 waves = 128 queries of one (batch, head); each wave owns 32 queries.
// K/V tiles of 32 keys arrive by LDS-DMA (buffer_load ... lds, NS-stage ring, no VALU staging work: the f32 MFMA
// shares the vector ALU's issue, so VALU work in the loop costs MFMA time) and are shared by the 4 waves.
// The score tile is computed TRANSPOSED (S^T = K Q^T) so each lane holds one query column and 16 keys in its
// accumulator registers: the per-query max/sum is an in-register reduction plus one xor-32 lane swap, and the
// S^T accumulator registers are directly the B operand of O^T += V^T P^T (no LDS round trip for P).
// Online softmax in the log2 domain: scale*log2(e) is folded into Q, so p = exp2(s - m) is one v_exp_f32;
// the running reference max moves only when a query's max exceeds it by more than 8 (log2 units), so the
// output rescale runs about once per row.
#include "hfa_common.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int DH = 64;
constexpr int KB = 32;          // keys per tile
constexpr int QW = 32;          // queries per wave
constexpr int NW = 4;           // waves per workgroup
#ifndef HFA_ATTN_NS
#define HFA_ATTN_NS 2
#endif
constexpr int NS = HFA_ATTN_NS; // LDS stages (NS-1 key tiles in flight)
constexpr int TILE = KB * DH;   // floats per K (or V) tile image
constexpr float kSlack = 8.0f;  // stale-max slack of the online softmax (log2 units)

struct AttnP {
    int B, H, L;
    float scale;
    const float* q; long long q_bs; int q_ld;
    const float* k; long long k_bs; int k_ld;
    const float* v; long long v_bs; int v_ld;
    float* o; long long o_bs; int o_ld;
    const int32_t* key_len;     // optional [B]: per-row sequence lengths of a variable-length batch
};

__global__ __launch_bounds__(NW * 64) void attn_fwd_f32_kernel(const AttnP p) {
    // stage s: K image [32 rows][64] with 16-B chunks XOR-swizzled by (row & 15) (ds_read_b128 row reads by 32
    // rows stay conflict-free), then V image [32][64] unswizzled (read by ds_read2_b32 along rows)
    __shared__ __attribute__((aligned(16))) float smem[NS * 2 * TILE];

    // XCD-aware bijective remap (as in gemm.hip): the q-blocks of one (batch, head) get consecutive ids and so
    // share an XCD's L2 for their K/V tiles
    const int nwg = gridDim.x, orig = blockIdx.x;
    const int xcd = orig & 7, xq = nwg >> 3, xr = nwg & 7;
    const int wgid = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (orig >> 3);
    const int nqb = (p.L + QW * NW - 1) / (QW * NW);
    const int bh = wgid / nqb, qb = wgid - bh * nqb;
    const int b = bh / p.H, hd = bh - b * p.H;
    const int L = p.key_len ? p.key_len[b] : p.L;       // this row's length (queries and keys beyond: padding)
    if (qb * (QW * NW) >= L) return;                     // whole workgroup is padding (uniform exit)
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r32 = lane & 31, half = lane >> 5;
    const int q0 = qb * (QW * NW) + wave * QW;
    const int qi = q0 + r32;

    const float* Q = p.q + b * p.q_bs + hd * DH;
    const float* Kp = p.k + b * p.k_bs + hd * DH;
    const float* Vp = p.v + b * p.v_bs + hd * DH;
    const __amdgpu_buffer_rsrc_t rK = hfa::make_rsrc(Kp, ((long long)(L - 1) * p.k_ld + DH) * 4);
    const __amdgpu_buffer_rsrc_t rV = hfa::make_rsrc(Vp, ((long long)(L - 1) * p.v_ld + DH) * 4);

    // Q fragments: lane holds Q[qi][kk*8 + half*4 + e] * scale * log2(e), kk = 0..7, e = 0..3
    const float qscale = p.scale * 1.44269504088896340736f;
    f32x4 qf[DH / 8];
#pragma unroll
    for (int kk = 0; kk < DH / 8; ++kk) {
        if (qi < L) {
            f32x4 v = *reinterpret_cast<const f32x4*>(Q + (long long)qi * p.q_ld + kk * 8 + half * 4);
            qf[kk] = v * qscale;
        } else {
            qf[kk] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }

    // DMA geometry: 8 x 1 KiB wave-instructions per 32 x 64 image, 2 per wave; instruction d covers rows
    // (wave*2 + d)*4 + lane/16, LDS slot lane&15
    int rowd[2], kcol[2];
#pragma unroll
    for (int d = 0; d < 2; ++d) {
        rowd[d] = (wave * 2 + d) * 4 + (lane >> 4);
        kcol[d] = ((lane & 15) ^ (rowd[d] & 15)) * 4;
    }
    const unsigned lds0 = hfa::lds_addr(smem);
    auto issue = [&](int stage, int key0) {
        const unsigned kdst = lds0 + stage * 2 * TILE * 4 + wave * 2 * 1024;
        const unsigned vdst = kdst + TILE * 4;
#pragma unroll
        for (int d = 0; d < 2; ++d) {
            const int key = key0 + rowd[d];
            const bool ok = key < L;
            hfa::dma16(ok ? (unsigned)((key * p.k_ld + kcol[d]) * 4) : hfa::DMA_OOB, rK, 0u, kdst + d * 1024);
            hfa::dma16(ok ? (unsigned)((key * p.v_ld + (lane & 15) * 4) * 4) : hfa::DMA_OOB, rV, 0u, vdst + d * 1024);
        }
    };

    f32x16 oacc[2];
#pragma unroll
    for (int e = 0; e < 16; ++e) { oacc[0][e] = 0.f; oacc[1][e] = 0.f; }
    float m_run = -__builtin_inff(), l_run = 0.0f;

    // per-lane LDS read offsets (floats): K row r32 chunk (kk*2 + half) swizzled; V row j(e, half), column r32
    int krd[DH / 8];
#pragma unroll
    for (int kk = 0; kk < DH / 8; ++kk) krd[kk] = r32 * DH + (((kk * 2 + half) ^ (r32 & 15)) << 2);

    const int nkb = (L + KB - 1) / KB;
#pragma unroll
    for (int st = 0; st < NS - 1; ++st)
        if (st < nkb) issue(st, st * KB);
    if (nkb >= NS - 1) hfa::wait_vm_barrier<(NS - 2) * 4>();
    else hfa::wait_vm_barrier<0>();
    int stage = 0;
    for (int kb = 0; kb < nkb; ++kb) {
        const bool more = kb + NS - 1 < nkb;
        if (more) issue(stage == 0 ? NS - 1 : stage - 1, (kb + NS - 1) * KB);
        const float* sK = smem + stage * 2 * TILE;
        const float* sV = sK + TILE;
        // S^T[j][i] = sum_d K[j][d] * Qs[i][d]  (log2 units)
        f32x16 s;
#pragma unroll
        for (int e = 0; e < 16; ++e) s[e] = 0.f;
#pragma unroll
        for (int kk = 0; kk < DH / 8; ++kk) {
            const f32x4 kf = *reinterpret_cast<const f32x4*>(sK + krd[kk]);
#pragma unroll
            for (int e = 0; e < 4; ++e) s = __builtin_amdgcn_mfma_f32_32x32x2f32(kf[e], qf[kk][e], s, 0, 0, 0);
        }
        const int key0 = kb * KB;
        if (key0 + KB > L) {          // last, partial tile: keys >= L do not exist
#pragma unroll
            for (int e = 0; e < 16; ++e)
                if (key0 + (e & 3) + 8 * (e >> 2) + 4 * half >= L) s[e] = -__builtin_inff();
        }
        float bm = s[0];
#pragma unroll
        for (int e = 1; e < 16; ++e) bm = fmaxf(bm, s[e]);
        bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
        // Stale-max online softmax: the running reference m_run moves only when a query's max exceeds it by more
        // than kSlack (log2 units), so p = exp2(s - m_run) <= 2^kSlack stays far from overflow while the O/l
        // rescale (64 multiplies per lane) runs about once per row instead of on almost every 32-key tile (with
        // 32 queries per wave, SOME query's max moves on most tiles).  O and l share the reference, so the
        // normalised result is the same softmax; f32 keeps its relative precision at 2^8 as at 1.
        const float m_cand = fmaxf(m_run, bm);
        const bool move = m_cand > m_run + kSlack;          // first tile: m_run = -inf moves
        if (__builtin_amdgcn_ballot_w64(move)) {
            const float m_new = move ? m_cand : m_run;
            const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
            l_run *= alpha;
#pragma unroll
            for (int e = 0; e < 16; ++e) { oacc[0][e] *= alpha; oacc[1][e] *= alpha; }
            m_run = m_new;
        }
        float ls = 0.0f;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            s[e] = __builtin_amdgcn_exp2f(s[e] - m_run);
            ls += s[e];
        }
        ls += __shfl_xor(ls, 32, 64);
        l_run += ls;
        // O^T[d][i] += sum_j V[j][d] * P^T[j][i]; MFMA e uses key j(e, half) = (e&3) + 8(e>>2) + 4 half
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int j = (e & 3) + 8 * (e >> 2) + 4 * half;
            const float v0 = sV[j * DH + r32];
            const float v1 = sV[j * DH + 32 + r32];
            oacc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(v0, s[e], oacc[0], 0, 0, 0);
            oacc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(v1, s[e], oacc[1], 0, 0, 0);
        }
        if (kb + 1 < nkb) {                     // next tile landed; every wave done with this stage
            if (more) hfa::wait_vm_barrier<(NS - 2) * 4>();
            else hfa::wait_vm_barrier<0>();
        }
        stage = stage + 1 == NS ? 0 : stage + 1;
    }

    // normalise and stage O[i][d] through LDS (each wave a private 32 x 33 slab), row-contiguous stores
    __syncthreads();
    const float inv = 1.0f / l_run;
    float* slab = smem + wave * (QW * 33);
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int d = (e & 3) + 8 * (e >> 2) + 4 * half;
            slab[r32 * 33 + d] = oacc[dt][e] * inv;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int idx = lane + i * 64;
            const int row = idx >> 3, c4 = (idx & 7) * 4;
            const int qq = q0 + row;
            if (qq < L) {
                f32x4 v{slab[row * 33 + c4], slab[row * 33 + c4 + 1], slab[row * 33 + c4 + 2],
                        slab[row * 33 + c4 + 3]};
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
                      long long o_bs, int o_ld, const int32_t* key_len, hipStream_t stream) {
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
    if (((long long)(L - 1) * k_ld + DH) * 4 >= 0x7fffffffLL || ((long long)(L - 1) * v_ld + DH) * 4 >= 0x7fffffffLL) {
        hfa::set_error("hfa_attention_f32: K/V span exceeds 31-bit buffer offsets");
        return HFA_EINVAL;
    }
    AttnP p{B, H, L, scale, q, q_bs, q_ld, k, k_bs, k_ld, v, v_bs, v_ld, o, o_bs, o_ld, key_len};
    const long long nblk = (long long)((L + QW * NW - 1) / (QW * NW)) * B * H;
    if (nblk > 0x7fffffffLL) {
        hfa::set_error("hfa_attention_f32: grid too large");
        return HFA_EINVAL;
    }
    dim3 grid((unsigned)nblk);
    hipLaunchKernelGGL(attn_fwd_f32_kernel, grid, dim3(NW * 64), 0, stream, p);
    return hfa::check_launch("hfa_attention_f32");
}

}  // extern "C"
