// attention64.hip — split-f16 flash attention with 64 queries per wave (two 32-query halves), head_dim 64.
//
// Replaces the same reference operations as attention.hip's attn_fwd_split_kernel (networks/hubert/model.py:27-32,
// transformers modeling_hubert.py eager_attention_forward: softmax(q k^T * head_dim^-0.5) v), with the same
// arithmetic (three exact f16 MFMA products per f32-class product, stale-max online softmax in the exp2 domain, P
// split in registers, O at scale 2^11) and the same LDS images, so every query row gets the same bits as from the
// 32-query kernel.  What differs is the work per wave: a workgroup of 4 waves covers 256 queries of one
// (batch, head), one wave per SIMD (the whole register file: the score tiles of both halves, double-buffered, and
// the two output accumulators sit in AGPRs, so this file is built without the VGPR MFMA form), and every K / V
// fragment read from LDS feeds the MFMAs of both halves: half the LDS operand reads and half the LDS-DMA bytes per
// query of the 32-query kernel, and one half's softmax can issue between the other half's MFMAs.
#include "hfa_common.h"
#include "attn_params.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int DH = 64;               // head dim
constexpr int QH = 32;               // queries per half
constexpr int NH = 2;                // halves per wave
constexpr int NW = 4;                // waves per workgroup
constexpr int QWG = QH * NH * NW;    // queries per workgroup
constexpr int SKB = 64;              // keys per tile
constexpr int SPLANE = SKB * DH;     // halves per plane image (8 KiB)
constexpr int KST = 2 * SPLANE;      // halves per K (or V) stage, both planes
constexpr int PPW = 8 / NW;          // 1-KiB DMA pieces (8 keys) per plane per wave
constexpr float kLo = 1.0f / 2048.0f;
constexpr float kSlack = 8.0f;       // stale-max slack of the online softmax (log2 units)

__device__ __forceinline__ f16x4 lds_tr(const _Float16* base, int byte_off) {
    const auto* ptr = reinterpret_cast<const __attribute__((address_space(3))) s16x4*>(
        reinterpret_cast<const __attribute__((address_space(3))) char*>(
            (const __attribute__((address_space(3))) _Float16*)base) + byte_off);
    return __builtin_bit_cast(f16x4, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        const_cast<__attribute__((address_space(3))) s16x4*>(ptr)));
}

__global__ __launch_bounds__(NW * 64, 1) void attn_fwd_split64_kernel(const AttnSP p) {
    // K and V in 2-stage LDS-DMA rings, one tile ahead (64 KiB of LDS); no cross-tile score pipelining (its second
    // score buffer does not fit beside 64 queries' Q planes): the overlap is between the two halves.
    __shared__ __attribute__((aligned(16))) _Float16 smem[4 * KST];   // K0, K1, V0, V1

    const int nwg = gridDim.x, orig = blockIdx.x;
    const int xcd = orig & 7, xq = nwg >> 3, xr = nwg & 7;
    const int wgid = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (orig >> 3);
    const int nqb = (p.L + QWG - 1) / QWG;
    const int bh = wgid / nqb, qb = wgid - bh * nqb;
    const int b = bh / p.H, hd = bh - b * p.H;
    const int L = p.key_len ? p.key_len[b] : p.L;
    if (qb * QWG >= L) {                                 // whole workgroup is padding: zero its O rows, exit
        for (int i = threadIdx.x; i < QWG * (DH / 4); i += NW * 64) {
            const int qq = qb * QWG + i / (DH / 4), c4 = (i % (DH / 4)) * 4;
            if (qq < p.L) {
                _Float16* dst = p.o + b * p.o_bs + (long long)qq * p.o_ld + hd * DH + c4;
                const f16x4 z{(_Float16)0.f, (_Float16)0.f, (_Float16)0.f, (_Float16)0.f};
                *reinterpret_cast<f16x4*>(dst) = z;
                *reinterpret_cast<f16x4*>(dst + p.o_sp) = z;
            }
        }
        return;
    }
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r32 = lane & 31, half = lane >> 5;
    const int q0 = qb * QWG + wave * (QH * NH);         // half h: queries q0 + 32 h + r32

    const _Float16* Q = p.q + b * p.q_bs + hd * DH;
    const _Float16* Kp = p.k + b * p.k_bs + hd * DH;
    const _Float16* Vp = p.v + b * p.v_bs + hd * DH;
    const long long kbytes = ((long long)(L - 1) * p.k_ld + DH) * 2, vbytes = ((long long)(L - 1) * p.v_ld + DH) * 2;
    const __amdgpu_buffer_rsrc_t rK1 = hfa::make_rsrc(Kp, kbytes), rK2 = hfa::make_rsrc(Kp + p.k_sp, kbytes);
    const __amdgpu_buffer_rsrc_t rV1 = hfa::make_rsrc(Vp, vbytes), rV2 = hfa::make_rsrc(Vp + p.v_sp, vbytes);

    f16x8 q1[NH][DH / 16], q2[NH][DH / 16];
#pragma unroll
    for (int h = 0; h < NH; ++h) {
        const int qi = q0 + QH * h + r32;
#pragma unroll
        for (int kb = 0; kb < DH / 16; ++kb) {
            if (qi < L) {
                const _Float16* src = Q + (long long)qi * p.q_ld + kb * 16 + half * 8;
                q1[h][kb] = *reinterpret_cast<const f16x8*>(src);
                q2[h][kb] = *reinterpret_cast<const f16x8*>(src + p.q_sp);
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) q1[h][kb][j] = q2[h][kb][j] = (_Float16)0.0f;
            }
        }
    }

    int rowd[PPW], kch[PPW], vch[PPW];
#pragma unroll
    for (int d = 0; d < PPW; ++d) {
        rowd[d] = (wave * PPW + d) * 8 + (lane >> 3);
        kch[d] = (lane & 7) ^ ((rowd[d] >> 1) & 7);
        vch[d] = (lane & 7) ^ (((rowd[d] >> 1) & 1) << 2);
    }
    const unsigned lds0 = hfa::lds_addr(smem);
    auto issueK = [&](int stage, int key0) {
        const unsigned base = lds0 + stage * KST * 2 + wave * PPW * 1024;
#pragma unroll
        for (int d = 0; d < PPW; ++d) {
            const int key = key0 + rowd[d];
            const unsigned ko = key < L ? (unsigned)((key * p.k_ld + kch[d] * 8) * 2) : hfa::DMA_OOB;
            hfa::dma16(ko, rK1, 0u, base + d * 1024);
            hfa::dma16(ko, rK2, 0u, base + SPLANE * 2 + d * 1024);
        }
    };
    auto issueV = [&](int stage, int key0) {
        const unsigned base = lds0 + (2 + stage) * KST * 2 + wave * PPW * 1024;
#pragma unroll
        for (int d = 0; d < PPW; ++d) {
            const int key = key0 + rowd[d];
            const unsigned vo = key < L ? (unsigned)((key * p.v_ld + vch[d] * 8) * 2) : hfa::DMA_OOB;
            hfa::dma16(vo, rV1, 0u, base + d * 1024);
            hfa::dma16(vo, rV2, 0u, base + SPLANE * 2 + d * 1024);
        }
    };

    int kofs[DH / 16];
#pragma unroll
    for (int kb = 0; kb < DH / 16; ++kb) kofs[kb] = r32 * DH + (((kb * 2 + half) ^ ((r32 >> 1) & 7)) << 3);
    const int gi = lane & 15, gq = gi >> 2, gp = gi & 3;
    const int vrow = 4 * half + gq;
    const int vch0 = 2 * ((lane >> 4) & 1) + (gp >> 1);
    const int vfx = (((vrow >> 1) & 1) << 2);
    int vofs[2];
#pragma unroll
    for (int db = 0; db < 2; ++db) vofs[db] = vrow * (DH * 2) + (((4 * db + vch0) ^ vfx) << 4) + 8 * (gp & 1);

    const float qscale = p.scale * 1.44269504088896340736f;
    f16x8 q1s[NH][DH / 16], q2s[NH][DH / 16];
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
        for (int kb = 0; kb < DH / 16; ++kb) {
            q1s[h][kb] = q1[h][kb] * (_Float16)kLo;
            q2s[h][kb] = q2[h][kb] * (_Float16)kLo;
        }
    // one half's score tile (the K fragments are read once per half: the halves are interleaved with each other's
    // softmax, not with each other's MFMAs)
    auto scores = [&](const _Float16* sK, f32x16 (&sM)[2], int h) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
            for (int e = 0; e < 16; ++e) sM[kt][e] = 0.f;
#pragma unroll
            for (int kb = 0; kb < DH / 16; ++kb) {
                const f16x8 k1 = *reinterpret_cast<const f16x8*>(sK + kt * 32 * DH + kofs[kb]);
                const f16x8 k2 = *reinterpret_cast<const f16x8*>(sK + SPLANE + kt * 32 * DH + kofs[kb]);
                sM[kt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(k1, q1[h][kb], sM[kt], 0, 0, 0);
                sM[kt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(k1, q2s[h][kb], sM[kt], 0, 0, 0);
                sM[kt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(k2, q1s[h][kb], sM[kt], 0, 0, 0);
            }
        }
    };
    f32x16 o[NH][2];
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
        for (int e = 0; e < 16; ++e) o[h][0][e] = o[h][1][e] = 0.f;
    float m_run[NH], l_run[NH];
#pragma unroll
    for (int h = 0; h < NH; ++h) {
        m_run[h] = -__builtin_inff();
        l_run[h] = 0.0f;
    }

    const int nkb = (L + SKB - 1) / SKB;
    issueK(0, 0);
    issueV(0, 0);
    const float one = 1.0f;
    // softmax of one half's tile in place: s becomes q = 2^11 p (the running max and sum updated, O rescaled)
    auto softmax = [&](int t, f32x16 (&s)[2], float& mr, float& lr, f32x16 (&oh)[2]) {
        const int key0 = t * SKB;
        if (key0 + SKB > L) {
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int e = 0; e < 16; ++e)
                    if (key0 + kt * 32 + (e & 3) + 8 * (e >> 2) + 4 * half >= L) s[kt][e] = -__builtin_inff();
        }
        float bq[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) bq[c] = fmaxf(s[0][c], s[1][c]);
#pragma unroll
        for (int e = 4; e < 16; ++e) bq[e & 3] = fmaxf(bq[e & 3], fmaxf(s[0][e], s[1][e]));
        float bm = fmaxf(fmaxf(bq[0], bq[1]), fmaxf(bq[2], bq[3]));
        bm = fmaxf(bm, __shfl_xor(bm, 32, 64)) * qscale;
        const float m_cand = fmaxf(mr, bm);
        const bool move = m_cand > mr + kSlack;
        {   // branch-free (alpha = 1 exactly where the max does not move: the same bits), so the scheduler can
            // interleave this half's softmax with the other half's MFMAs
            const float m_new = move ? m_cand : mr;
            const float alpha = __builtin_amdgcn_exp2f(mr - m_new);
            lr *= alpha;
            asm volatile("" : "+v"(lr));   // keep l's rescale a separate rounding (no FMA with the sum below)
#pragma unroll
            for (int e = 0; e < 16; ++e) { oh[0][e] *= alpha; oh[1][e] *= alpha; }
            mr = m_new;
        }
        const float nref = 11.0f - (mr + kSlack);
        float ls = 0.0f;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                s[kt][e] = __builtin_amdgcn_exp2f(__builtin_fmaf(s[kt][e], qscale, nref));
                ls += s[kt][e];
            }
        ls += __shfl_xor(ls, 32, 64);
        lr += ls;
    };
    // tile t (K(t), V(t) landed at the previous barrier): K(t+1), V(t+1) go to the other stages under this tile's
    // work; the two halves' score tiles from one pass over the K fragments, then one half at a time: its softmax
    // (VALU) and its PV MFMAs, so the second half's softmax can issue between the first half's PV MFMAs
    f32x16 sc[NH][2];
    auto step = [&](int t) {
        const int st = t & 1;
        if (t + 1 < nkb) {
            issueK(st ^ 1, (t + 1) * SKB);
            issueV(st ^ 1, (t + 1) * SKB);
        }
        const _Float16* sK = smem + st * KST;
        const _Float16* sV = smem + (2 + st) * KST;
        auto pv = [&](int h) {
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) {
                    unsigned w1[4], w2[4];
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj) {
                        const float x0 = sc[h][kt][8 * ks + 2 * jj], x1 = sc[h][kt][8 * ks + 2 * jj + 1];
                        w1[jj] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){x0, x1}, f16x2));
                        w2[jj] = hfa::split_lo_pair(w1[jj], x0, x1, one);
                    }
                    const f16x8 p1s = __builtin_bit_cast(f16x8, make_uint4(w1[0], w1[1], w1[2], w1[3]));
                    const f16x8 p2 = __builtin_bit_cast(f16x8, make_uint4(w2[0], w2[1], w2[2], w2[3]));
                    const f16x8 p1 = p1s * (_Float16)kLo;
                    const int rb = (32 * kt + 16 * ks) * (DH * 2);
#pragma unroll
                    for (int db = 0; db < 2; ++db) {
                        const f16x4 a0 = lds_tr(sV, rb + vofs[db]);
                        const f16x4 a1 = lds_tr(sV, rb + 8 * DH * 2 + vofs[db]);
                        const f16x4 b0 = lds_tr(sV + SPLANE, rb + vofs[db]);
                        const f16x4 b1 = lds_tr(sV + SPLANE, rb + 8 * DH * 2 + vofs[db]);
                        const f16x8 v1 = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
                        const f16x8 v2 = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
                        o[h][db] = __builtin_amdgcn_mfma_f32_32x32x16_f16(v1, p1s, o[h][db], 0, 0, 0);
                        o[h][db] = __builtin_amdgcn_mfma_f32_32x32x16_f16(v1, p2, o[h][db], 0, 0, 0);
                        o[h][db] = __builtin_amdgcn_mfma_f32_32x32x16_f16(v2, p1, o[h][db], 0, 0, 0);
                    }
                }
        };
        // half A's softmax beside half B's score MFMAs, half B's softmax beside half A's PV MFMAs
        scores(sK, sc[0], 0);
        softmax(t, sc[0], m_run[0], l_run[0], o[0]);
        scores(sK, sc[1], 1);
        pv(0);
        softmax(t, sc[1], m_run[1], l_run[1], o[1]);
        pv(1);
        if (t + 1 < nkb) {
            hfa::wait_vm_barrier<0>();                     // K(t+1), V(t+1) landed; K(t), V(t) reads done
        }
    };
    hfa::wait_vm_barrier<0>();                             // Q, K(0), V(0) landed
    for (int t = 0; t < nkb; ++t) step(t);

    __syncthreads();
    float* slab = reinterpret_cast<float*>(smem) + wave * (QH * 33);
#pragma unroll
    for (int h = 0; h < NH; ++h) {
        const float inv = 1.0f / l_run[h];                 // o and l both carry the 2^11 scale
        const int qh0 = q0 + QH * h;
#pragma unroll
        for (int db = 0; db < 2; ++db) {
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int d = (e & 3) + 8 * (e >> 2) + 4 * half;
                slab[r32 * 33 + d] = o[h][db][e] * inv;
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int idx = lane + i * 64;
                const int row = idx >> 3, c4 = (idx & 7) * 4;
                const int qq = qh0 + row;
                if (qq < p.L) {                 // rows past this row's length: zeros (padding of a varlen batch)
                    f16x4 h1, h2;
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const float x = qq < L ? slab[row * 33 + c4 + t] : 0.0f;
                        h1[t] = (_Float16)x;
                        h2[t] = (_Float16)((x - (float)h1[t]) * 2048.0f);
                    }
                    _Float16* dst = p.o + b * p.o_bs + (long long)qq * p.o_ld + hd * DH + db * 32 + c4;
                    *reinterpret_cast<f16x4*>(dst) = h1;
                    *reinterpret_cast<f16x4*>(dst + p.o_sp) = h2;
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
}

}  // namespace

void launch_attn_split64(const AttnSP& p, hipStream_t stream) {
    const long long nblk = (long long)((p.L + QWG - 1) / QWG) * p.B * p.H;
    hipLaunchKernelGGL(attn_fwd_split64_kernel, dim3((unsigned)nblk), dim3(NW * 64), 0, stream, p);
}
