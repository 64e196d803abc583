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
constexpr int NS = 2;           // LDS stages (NS-1 key tiles in flight)
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
    if (qb * (QW * NW) >= L) {                           // whole workgroup is padding: zero its O rows, exit
        for (int i = threadIdx.x; i < QW * NW * (DH / 4); i += NW * 64) {
            const int qq = qb * (QW * NW) + i / (DH / 4), c4 = (i % (DH / 4)) * 4;
            if (qq < p.L)
                *reinterpret_cast<f32x4*>(p.o + b * p.o_bs + (long long)qq * p.o_ld + hd * DH + c4) =
                    f32x4{0.f, 0.f, 0.f, 0.f};
        }
        return;
    }
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
            if (qq < p.L) {                     // rows past this row's length: zeros (padding of a varlen batch)
                f32x4 v{slab[row * 33 + c4], slab[row * 33 + c4 + 1], slab[row * 33 + c4 + 2],
                        slab[row * 33 + c4 + 3]};
                if (qq >= L) v = f32x4{0.f, 0.f, 0.f, 0.f};
                *reinterpret_cast<f32x4*>(p.o + b * p.o_bs + (long long)qq * p.o_ld + hd * DH + dt * 32 + c4) = v;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// ---- split-f16 flash attention ---------------------------------------------------------------------------------
// Q, K, V and O as split-f16 plane pairs (x = x1 + 2^-11 x2, gemm.hip's split scheme): every product is three exact
// f16 x f16 MFMA products (scores: x1 y1 + x1 (2^-11 y2) + x2 (2^-11 y1) on one accumulator; output: one
// accumulator at scale 2^11), so the contractions keep f32-class accuracy while running on
// v_mfma_f32_32x32x16_f16.
// Same structure as attn_fwd_f32_kernel (S^T = K Q^T with one query per lane, stale-max online softmax in the
// exp2 domain, the P accumulator as the B operand of O^T += V^T P^T), with 64-key tiles and:
//   * K image [64 keys][8 chunks of 16 B] per plane, chunk c of row r at slot c ^ ((r >> 1) & 7): the
//     ds_read_b128 row reads of the 32x32x16 A operand are conflict-free;
//   * V image, same shape, chunk c of row r at slot c ^ (((r >> 1) & 1) << 2), read with ds_read_b64_tr_b16
//     (4 keys x 16 d per 16-lane group, delivered column-major): the V^T operand with no transposing pass;
//   * P split in registers (p <= 2^8 under the stale max, far inside f16 range); the scale * log2(e) factor
//     multiplies the f32 score (Q stays exactly the producer's planes);
//   * O normalised in f32 and written back as split planes for the out-projection's split GEMM.
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int SKB = 64;              // keys per tile
constexpr int SPLANE = SKB * DH;     // halves per plane image (8 KiB)
constexpr float kLo = 1.0f / 2048.0f;

struct AttnSP {
    int B, H, L;
    float scale;
    const _Float16* q; long long q_sp, q_bs; int q_ld;
    const _Float16* k; long long k_sp, k_bs; int k_ld;
    const _Float16* v; long long v_sp, v_bs; int v_ld;
    _Float16* o; long long o_sp, o_bs; int o_ld;
    const int32_t* key_len;
};

__device__ __forceinline__ f16x4 lds_tr(const _Float16* base, int byte_off) {
    const auto* ptr = reinterpret_cast<const __attribute__((address_space(3))) s16x4*>(
        reinterpret_cast<const __attribute__((address_space(3))) char*>(
            (const __attribute__((address_space(3))) _Float16*)base) + byte_off);
    return __builtin_bit_cast(f16x4, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        const_cast<__attribute__((address_space(3))) s16x4*>(ptr)));
}

// Since round 3: P's planes as one v_cvt_pk_f16_f32 per pair (2^11 p1 = RNE f16 of q) and the exact remainder by
// two v_fma_mix (hfa::split_lo_pair: f16(q - p1) read straight from the packed pair), 1.5 VALU ops per score instead
// of and + cvt + sub + cvt (4); and the tile loop unrolled by two with the current and next score tiles in swapped
// register sets (no 32-register copy per tile).  (The round-2 loop is in git history.)
template <int SNW>
__global__ __launch_bounds__(SNW * 64, 2) void attn_fwd_split_kernel(const AttnSP p) {
    // Software-pipelined: iteration t issues the score MFMAs of tile t+1, then runs tile t's softmax (VALU) while
    // those MFMAs execute, then tile t's PV MFMAs.  K runs one tile further ahead than V in separate 2-stage rings
    // (K(t+1) must have landed when iteration t starts, V(t) only by its PV), so the LDS stays 64 KiB (2 per CU).
    // The output uses one accumulator at scale 2^11: P is taken relative to m_run + kSlack (p <= 1, so 2^11 p1 is
    // exact in f16) and O += V1 (2^11 P1) + V1 P2 + V2 P1.
    // SNW waves of 32 queries share each K/V tile (8 waves halve the LDS-DMA stream per query at L ~ 500)
    constexpr int KST = 2 * SPLANE;                      // halves per K (or V) stage, both planes
    constexpr int NW = SNW, PPW = 8 / SNW;               // 1-KiB DMA pieces (8 keys) per plane per wave
    static_assert(SNW == 4 || SNW == 8, "4 or 8 waves");
    __shared__ __attribute__((aligned(16))) _Float16 smem[4 * KST];   // K0, K1, V0, V1

    const int nwg = gridDim.x, orig = blockIdx.x;
    const int xcd = orig & 7, xq = nwg >> 3, xr = nwg & 7;
    const int wgid = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (orig >> 3);
    const int nqb = (p.L + QW * NW - 1) / (QW * NW);
    const int bh = wgid / nqb, qb = wgid - bh * nqb;
    const int b = bh / p.H, hd = bh - b * p.H;
    const int L = p.key_len ? p.key_len[b] : p.L;
    if (qb * (QW * NW) >= L) {                           // whole workgroup is padding: zero its O rows, exit
        for (int i = threadIdx.x; i < QW * NW * (DH / 4); i += NW * 64) {
            const int qq = qb * (QW * NW) + i / (DH / 4), c4 = (i % (DH / 4)) * 4;
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
    const int q0 = qb * (QW * NW) + wave * QW;
    const int qi = q0 + r32;

    const _Float16* Q = p.q + b * p.q_bs + hd * DH;
    const _Float16* Kp = p.k + b * p.k_bs + hd * DH;
    const _Float16* Vp = p.v + b * p.v_bs + hd * DH;
    const long long kbytes = ((long long)(L - 1) * p.k_ld + DH) * 2, vbytes = ((long long)(L - 1) * p.v_ld + DH) * 2;
    const __amdgpu_buffer_rsrc_t rK1 = hfa::make_rsrc(Kp, kbytes), rK2 = hfa::make_rsrc(Kp + p.k_sp, kbytes);
    const __amdgpu_buffer_rsrc_t rV1 = hfa::make_rsrc(Vp, vbytes), rV2 = hfa::make_rsrc(Vp + p.v_sp, vbytes);

    f16x8 q1[DH / 16], q2[DH / 16];
#pragma unroll
    for (int kb = 0; kb < DH / 16; ++kb) {
        if (qi < L) {
            const _Float16* src = Q + (long long)qi * p.q_ld + kb * 16 + half * 8;
            q1[kb] = *reinterpret_cast<const f16x8*>(src);
            q2[kb] = *reinterpret_cast<const f16x8*>(src + p.q_sp);
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) q1[kb][j] = q2[kb][j] = (_Float16)0.0f;
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
    // One score accumulator: k1 q1 + k1 (2^-11 q2) + k2 (2^-11 q1), the two small products on Q planes pre-scaled
    // once per wave (2^-11 q2 is the exact residual q - q1; an f16 subnormal below 2^-14, i.e. an absolute error
    // <= 2^-25 |k| per product, under the f32 score's own rounding) -- no second accumulator, no combine pass.
    // Against the two-accumulator form (main + correction, combined by one FMA per score): 0.092 -> 0.087 ms per
    // layer (base), 0.118 -> 0.112 (large), 215 -> 204 VGPRs (profiles/r02/attn_single_acc_ab.txt).
    f16x8 q1s[DH / 16], q2s[DH / 16];
#pragma unroll
    for (int kb = 0; kb < DH / 16; ++kb) {
        q1s[kb] = q1[kb] * (_Float16)kLo;
        q2s[kb] = q2[kb] * (_Float16)kLo;
    }
    auto scores = [&](const _Float16* sK, f32x16 (&sM)[2]) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
            for (int e = 0; e < 16; ++e) sM[kt][e] = 0.f;
#pragma unroll
            for (int kb = 0; kb < DH / 16; ++kb) {
                const f16x8 k1 = *reinterpret_cast<const f16x8*>(sK + kt * 32 * DH + kofs[kb]);
                const f16x8 k2 = *reinterpret_cast<const f16x8*>(sK + SPLANE + kt * 32 * DH + kofs[kb]);
                sM[kt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(k1, q1[kb], sM[kt], 0, 0, 0);
                sM[kt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(k1, q2s[kb], sM[kt], 0, 0, 0);
                sM[kt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(k2, q1s[kb], sM[kt], 0, 0, 0);
            }
        }
    };
    f32x16 o[2];
#pragma unroll
    for (int e = 0; e < 16; ++e) o[0][e] = o[1][e] = 0.f;
    float m_run = -__builtin_inff(), l_run = 0.0f;

    const int nkb = (L + SKB - 1) / SKB;
    issueK(0, 0);
    issueV(0, 0);
    if (nkb > 1) issueK(1, SKB);
    hfa::wait_vm_barrier<0>();
    f32x16 sA[2], sB[2];
    scores(smem, sA);
    __syncthreads();                                       // every wave's K(0) reads done before K(2) lands there
    const float one = 1.0f;
    // tile t: s holds its scores, the next tile's go to nM (the caller swaps the two sets every tile)
    auto step = [&](int t, f32x16 (&s)[2], f32x16 (&nM)[2]) {
        const int st = t & 1;
        if (t + 2 < nkb) issueK(st, (t + 2) * SKB);        // K(t) was read by iteration t - 1's scores
        if (t + 1 < nkb) issueV(st ^ 1, (t + 1) * SKB);    // V(t - 1) was read by iteration t - 1's PV
        if (t + 1 < nkb) scores(smem + (st ^ 1) * KST, nM);   // tile t + 1, in flight during softmax(t)
        const int key0 = t * SKB;
        if (key0 + SKB > L) {
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int e = 0; e < 16; ++e)
                    if (key0 + kt * 32 + (e & 3) + 8 * (e >> 2) + 4 * half >= L) s[kt][e] = -__builtin_inff();
        }
        float bq[4];                                       // four independent max3 chains
#pragma unroll
        for (int c = 0; c < 4; ++c) bq[c] = fmaxf(s[0][c], s[1][c]);
#pragma unroll
        for (int e = 4; e < 16; ++e) bq[e & 3] = fmaxf(bq[e & 3], fmaxf(s[0][e], s[1][e]));
        float bm = fmaxf(fmaxf(bq[0], bq[1]), fmaxf(bq[2], bq[3]));
        bm = fmaxf(bm, __shfl_xor(bm, 32, 64)) * qscale;
        const float m_cand = fmaxf(m_run, bm);
        const bool move = m_cand > m_run + kSlack;
        if (__builtin_amdgcn_ballot_w64(move)) {
            const float m_new = move ? m_cand : m_run;
            const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
            l_run *= alpha;
#pragma unroll
            for (int e = 0; e < 16; ++e) { o[0][e] *= alpha; o[1][e] *= alpha; }
            m_run = m_new;
        }
        // q = 2^11 p, p = exp2(qscale s - m_run - kSlack) <= 1, so q <= 2048 is an f16 normal down to p = 2^-25
        const float nref = 11.0f - (m_run + kSlack);
        float ls = 0.0f;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                s[kt][e] = __builtin_amdgcn_exp2f(__builtin_fmaf(s[kt][e], qscale, nref));
                ls += s[kt][e];
            }
        ls += __shfl_xor(ls, 32, 64);
        l_run += ls;
        const _Float16* sV = smem + (2 + st) * KST;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                f16x8 p1, p2, p1s;
                // 2^11 p1 = f16(q) (round to nearest), 2^11 (p - p1) = f16(q - 2^11 p1): the exact f32 remainder
                // rounded once (v_fma_mix reads the f16 half of the packed pair in place)
                unsigned w1[4], w2[4];
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    const float q0 = s[kt][8 * ks + 2 * jj], q1 = s[kt][8 * ks + 2 * jj + 1];
                    w1[jj] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){q0, q1}, f16x2));
                    w2[jj] = hfa::split_lo_pair(w1[jj], q0, q1, one);
                }
                p1s = __builtin_bit_cast(f16x8, make_uint4(w1[0], w1[1], w1[2], w1[3]));
                p2 = __builtin_bit_cast(f16x8, make_uint4(w2[0], w2[1], w2[2], w2[3]));
                p1 = p1s * (_Float16)kLo;
                const int rb = (32 * kt + 16 * ks) * (DH * 2);
#pragma unroll
                for (int db = 0; db < 2; ++db) {
                    const f16x4 a0 = lds_tr(sV, rb + vofs[db]);
                    const f16x4 a1 = lds_tr(sV, rb + 8 * DH * 2 + vofs[db]);
                    const f16x4 b0 = lds_tr(sV + SPLANE, rb + vofs[db]);
                    const f16x4 b1 = lds_tr(sV + SPLANE, rb + 8 * DH * 2 + vofs[db]);
                    const f16x8 v1 = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
                    const f16x8 v2 = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
                    o[db] = __builtin_amdgcn_mfma_f32_32x32x16_f16(v1, p1s, o[db], 0, 0, 0);
                    o[db] = __builtin_amdgcn_mfma_f32_32x32x16_f16(v1, p2, o[db], 0, 0, 0);
                    o[db] = __builtin_amdgcn_mfma_f32_32x32x16_f16(v2, p1, o[db], 0, 0, 0);
                }
            }
        if (t + 1 < nkb) {
            hfa::wait_vm_barrier<0>();                     // K(t+2), V(t+1) landed; K(t+1), V(t) reads done
        }
    };
    for (int t = 0; t < nkb; t += 2) {
        step(t, sA, sB);
        if (t + 1 < nkb) step(t + 1, sB, sA);
    }

    __syncthreads();
    const float inv = 1.0f / l_run;                        // o and l both carry the 2^11 scale
    float* slab = reinterpret_cast<float*>(smem) + wave * (QW * 33);
#pragma unroll
    for (int db = 0; db < 2; ++db) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int d = (e & 3) + 8 * (e >> 2) + 4 * half;
            slab[r32 * 33 + d] = o[db][e] * inv;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int idx = lane + i * 64;
            const int row = idx >> 3, c4 = (idx & 7) * 4;
            const int qq = q0 + row;
            if (qq < p.L) {                     // rows past this row's length: zeros (padding of a varlen batch)
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


// ---- split-f16 flash attention on v_mfma_f32_16x16x32_f16 (round 6) --------------------------------------------
// The same arithmetic as attn_fwd_split_kernel (one score accumulator k1 q1 + k1 (2^-11 q2) + k2 (2^-11 q1), stale-max
// online softmax in the exp2 domain, P = 2^11 exp2(...) split in registers, O^T += V1 (2^11 P1) + V1 P2 + V2 P1 on one
// accumulator at scale 2^11, software-pipelined K/V rings) with every contraction on the 16x16x32 MFMA: the same
// cycles per FLOP as 32x32x16, but the chip holds a higher clock under it (MI355X_MICROARCH.md: 1.12-1.15x the
// FLOP/s in bare loops; the split GEMMs gained 4-9 %, profiles/r02/split_mf16.txt).
//   * scores S^T[key][q]: 4 key blocks x 2 query blocks of 16 per wave and 64-key tile; lane (g = lane >> 4, i =
//     lane & 15) holds query 16 qb + i, keys 16 kb + 4 g + e -- two queries per lane, each query's 64 keys over the
//     4 lane groups (row max / sum: in-lane, then xor 16 and xor 32);
//   * P^T as the B operand of a 32-key step j straight from the score registers: lane group g supplies keys
//     32 j + 4 g + (0..3) and 32 j + 16 + 4 g + (0..3); the V^T A operand is read in the same key order with two
//     ds_read_b64_tr_b16 per plane (4 keys x 16 d each, rows 32 j + 4 g and 32 j + 16 + 4 g);
//   * K image as the 32x32 kernel's (chunk c of row r at c ^ ((r >> 1) & 7): conflict-free for the 16x16x32 row
//     reads too); V image with chunk c of row r at c ^ (((r >> 1) & 3) << 1): the four 4-row blocks a 32-lane half
//     reads in one transposed read (rows R .. R + 7) take four different chunk pairs, conflict-free.
template <int SNW>
__global__ __launch_bounds__(SNW * 64, 2) void attn_fwd_split16_kernel(const AttnSP p) {
    constexpr int KST = 2 * SPLANE;                      // halves per K (or V) stage, both planes
    constexpr int NW = SNW, PPW = 8 / SNW;               // 1-KiB DMA pieces (8 keys) per plane per wave
    static_assert(SNW == 4 || SNW == 8, "4 or 8 waves");
    __shared__ __attribute__((aligned(16))) _Float16 smem[4 * KST];   // K0, K1, V0, V1

    const int nwg = gridDim.x, orig = blockIdx.x;
    const int xcd = orig & 7, xq = nwg >> 3, xr = nwg & 7;
    const int wgid = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (orig >> 3);
    const int nqb = (p.L + QW * NW - 1) / (QW * NW);
    const int bh = wgid / nqb, qblk = wgid - bh * nqb;
    const int b = bh / p.H, hd = bh - b * p.H;
    const int L = p.key_len ? p.key_len[b] : p.L;
    if (qblk * (QW * NW) >= L) {                         // whole workgroup is padding: zero its O rows, exit
        for (int i = threadIdx.x; i < QW * NW * (DH / 4); i += NW * 64) {
            const int qq = qblk * (QW * NW) + i / (DH / 4), c4 = (i % (DH / 4)) * 4;
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
    const int g = lane >> 4, i16 = lane & 15;
    const int q0 = qblk * (QW * NW) + wave * QW;

    const _Float16* Q = p.q + b * p.q_bs + hd * DH;
    const _Float16* Kp = p.k + b * p.k_bs + hd * DH;
    const _Float16* Vp = p.v + b * p.v_bs + hd * DH;
    const long long kbytes = ((long long)(L - 1) * p.k_ld + DH) * 2, vbytes = ((long long)(L - 1) * p.v_ld + DH) * 2;
    const __amdgpu_buffer_rsrc_t rK1 = hfa::make_rsrc(Kp, kbytes), rK2 = hfa::make_rsrc(Kp + p.k_sp, kbytes);
    const __amdgpu_buffer_rsrc_t rV1 = hfa::make_rsrc(Vp, vbytes), rV2 = hfa::make_rsrc(Vp + p.v_sp, vbytes);

    // Q^T B operands: lane (g, i) holds query q0 + 16 qb + i, d = 32 s + 8 g .. + 7
    f16x8 q1[2][2], q1s[2][2], q2s[2][2];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
        const int qi = q0 + 16 * qb + i16;
#pragma unroll
        for (int sd = 0; sd < 2; ++sd) {
            f16x8 h1, h2;
            if (qi < L) {
                const _Float16* src = Q + (long long)qi * p.q_ld + 32 * sd + 8 * g;
                h1 = *reinterpret_cast<const f16x8*>(src);
                h2 = *reinterpret_cast<const f16x8*>(src + p.q_sp);
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) h1[j] = h2[j] = (_Float16)0.0f;
            }
            q1[qb][sd] = h1;
            q1s[qb][sd] = h1 * (_Float16)kLo;
            q2s[qb][sd] = h2 * (_Float16)kLo;
        }
    }

    int rowd[PPW], kch[PPW], vch[PPW];
#pragma unroll
    for (int d = 0; d < PPW; ++d) {
        rowd[d] = (wave * PPW + d) * 8 + (lane >> 3);
        kch[d] = (lane & 7) ^ ((rowd[d] >> 1) & 7);
        vch[d] = (lane & 7) ^ (((rowd[d] >> 1) & 3) << 1);
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

    // K row reads: row 16 kb + i, chunk 4 sd + g (halves offset within a plane image)
    int kofs[2];
#pragma unroll
    for (int sd = 0; sd < 2; ++sd) kofs[sd] = i16 * DH + (((4 * sd + g) ^ ((i16 >> 1) & 7)) << 3);
    // (row 16 kb + i has the swizzle of i: 16 kb only adds multiples of 8 to r >> 1)
    // V transposed reads: lane 4qq + pp of the group supplies row R + qq, d columns 16 dblk + 4 pp .. + 3, i.e.
    // chunk 2 dblk + (pp >> 1), byte 8 (pp & 1); R = 32 j + 4 g (+ 16): R + qq has (R + qq) >> 1 & 3 = (2 g + (qq >> 1)) & 3
    // for R = 32 j + 4 g, and the same for R + 16
    const int qq = i16 >> 2, pp = i16 & 3;
    const int vfx = ((((4 * g + qq) >> 1) & 3) << 1);
    int vofs[4];                                          // per dblk, bytes from the row R + qq's start
#pragma unroll
    for (int db = 0; db < 4; ++db) vofs[db] = (((2 * db + (pp >> 1)) ^ vfx) << 4) + 8 * (pp & 1);
    const int vrow0 = (4 * g + qq) * (DH * 2);            // bytes: row 4 g + qq of the step

    const float qscale = p.scale * 1.44269504088896340736f;
    auto scores = [&](const _Float16* sK, f32x4 (&sM)[4][2]) {
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
            for (int qb = 0; qb < 2; ++qb) sM[kb][qb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
            for (int sd = 0; sd < 2; ++sd) {
                const f16x8 k1 = *reinterpret_cast<const f16x8*>(sK + kb * 16 * DH + kofs[sd]);
                const f16x8 k2 = *reinterpret_cast<const f16x8*>(sK + SPLANE + kb * 16 * DH + kofs[sd]);
#pragma unroll
                for (int qb = 0; qb < 2; ++qb) {
                    sM[kb][qb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(k1, q1[qb][sd], sM[kb][qb], 0, 0, 0);
                    sM[kb][qb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(k1, q2s[qb][sd], sM[kb][qb], 0, 0, 0);
                    sM[kb][qb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(k2, q1s[qb][sd], sM[kb][qb], 0, 0, 0);
                }
            }
    };
    f32x4 o[4][2];
#pragma unroll
    for (int db = 0; db < 4; ++db) o[db][0] = o[db][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m_run[2] = {-__builtin_inff(), -__builtin_inff()}, l_run[2] = {0.0f, 0.0f};

    const int nkb = (L + SKB - 1) / SKB;
    issueK(0, 0);
    issueV(0, 0);
    if (nkb > 1) issueK(1, SKB);
    hfa::wait_vm_barrier<0>();
    f32x4 sA[4][2], sB[4][2];
    scores(smem, sA);
    __syncthreads();                                       // every wave's K(0) reads done before K(2) lands there
    const float one = 1.0f;
    auto step = [&](int t, f32x4 (&s)[4][2], f32x4 (&nM)[4][2]) {
        const int st = t & 1;
        if (t + 2 < nkb) issueK(st, (t + 2) * SKB);
        if (t + 1 < nkb) issueV(st ^ 1, (t + 1) * SKB);
        if (t + 1 < nkb) scores(smem + (st ^ 1) * KST, nM);
        const int key0 = t * SKB;
        if (key0 + SKB > L) {
#pragma unroll
            for (int kb = 0; kb < 4; ++kb)
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (key0 + 16 * kb + 4 * g + e >= L) s[kb][0][e] = s[kb][1][e] = -__builtin_inff();
        }
        bool move_any = false;
        float m_new[2];
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
            float bq[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) bq[e] = fmaxf(fmaxf(s[0][qb][e], s[1][qb][e]), fmaxf(s[2][qb][e], s[3][qb][e]));
            float bm = fmaxf(fmaxf(bq[0], bq[1]), fmaxf(bq[2], bq[3]));
            bm = fmaxf(bm, __shfl_xor(bm, 16, 64));
            bm = fmaxf(bm, __shfl_xor(bm, 32, 64)) * qscale;
            const float m_cand = fmaxf(m_run[qb], bm);
            const bool move = m_cand > m_run[qb] + kSlack;
            m_new[qb] = move ? m_cand : m_run[qb];
            move_any |= move;
        }
        if (__builtin_amdgcn_ballot_w64(move_any)) {
#pragma unroll
            for (int qb = 0; qb < 2; ++qb) {
                const float alpha = __builtin_amdgcn_exp2f(m_run[qb] - m_new[qb]);
                l_run[qb] *= alpha;
#pragma unroll
                for (int db = 0; db < 4; ++db) o[db][qb] *= alpha;
                m_run[qb] = m_new[qb];
            }
        }
        float ls[2] = {0.0f, 0.0f};
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
            const float nref = 11.0f - (m_run[qb] + kSlack);
#pragma unroll
            for (int kb = 0; kb < 4; ++kb)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    s[kb][qb][e] = __builtin_amdgcn_exp2f(__builtin_fmaf(s[kb][qb][e], qscale, nref));
                    ls[qb] += s[kb][qb][e];
                }
        }
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
            float v = ls[qb];
            v += __shfl_xor(v, 16, 64);
            v += __shfl_xor(v, 32, 64);
            l_run[qb] += v;
        }
        const char* sV = reinterpret_cast<const char*>(smem + (2 + st) * KST);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            // P^T B operands of step j: keys 32 j + 4 g + (0..3) (score block 2 j) then 32 j + 16 + 4 g + (0..3) (2 j + 1)
            f16x8 p1s[2], p1[2], p2[2];
#pragma unroll
            for (int qb = 0; qb < 2; ++qb) {
                unsigned w1[4], w2[4];
#pragma unroll
                for (int h = 0; h < 2; ++h)
#pragma unroll
                    for (int jj = 0; jj < 2; ++jj) {
                        const float x0 = s[2 * j + h][qb][2 * jj], x1 = s[2 * j + h][qb][2 * jj + 1];
                        w1[2 * h + jj] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){x0, x1}, f16x2));
                        w2[2 * h + jj] = hfa::split_lo_pair(w1[2 * h + jj], x0, x1, one);
                    }
                p1s[qb] = __builtin_bit_cast(f16x8, make_uint4(w1[0], w1[1], w1[2], w1[3]));
                p2[qb] = __builtin_bit_cast(f16x8, make_uint4(w2[0], w2[1], w2[2], w2[3]));
                p1[qb] = p1s[qb] * (_Float16)kLo;
            }
            const int rb = 32 * j * (DH * 2) + vrow0;
#pragma unroll
            for (int db = 0; db < 4; ++db) {
                const f16x4 a0 = lds_tr(reinterpret_cast<const _Float16*>(sV), rb + vofs[db]);
                const f16x4 a1 = lds_tr(reinterpret_cast<const _Float16*>(sV), rb + 16 * DH * 2 + vofs[db]);
                const f16x4 b0 = lds_tr(reinterpret_cast<const _Float16*>(sV) + SPLANE, rb + vofs[db]);
                const f16x4 b1 = lds_tr(reinterpret_cast<const _Float16*>(sV) + SPLANE, rb + 16 * DH * 2 + vofs[db]);
                const f16x8 v1 = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
                const f16x8 v2 = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
#pragma unroll
                for (int qb = 0; qb < 2; ++qb) {
                    o[db][qb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(v1, p1s[qb], o[db][qb], 0, 0, 0);
                    o[db][qb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(v1, p2[qb], o[db][qb], 0, 0, 0);
                    o[db][qb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(v2, p1[qb], o[db][qb], 0, 0, 0);
                }
            }
        }
        if (t + 1 < nkb) {
            hfa::wait_vm_barrier<0>();                     // K(t+2), V(t+1) landed; K(t+1), V(t) reads done
        }
    };
    for (int t = 0; t < nkb; t += 2) {
        step(t, sA, sB);
        if (t + 1 < nkb) step(t + 1, sB, sA);
    }

    // O[q][d] = o[db][qb][e] / l at q = 16 qb + i, d = 16 db + 4 g + e; staged per 32-column half through a
    // [32 q][36] f32 slab per wave, then written as split planes with row-contiguous stores
    __syncthreads();
    float inv[2];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) inv[qb] = 1.0f / l_run[qb];            // o and l both carry the 2^11 scale
    float* slab = reinterpret_cast<float*>(smem) + wave * (QW * 36);
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
#pragma unroll
        for (int dd = 0; dd < 2; ++dd)
#pragma unroll
            for (int qb = 0; qb < 2; ++qb)
                *reinterpret_cast<f32x4*>(slab + (16 * qb + i16) * 36 + 16 * dd + 4 * g) = o[2 * hh + dd][qb] * inv[qb];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int idx = lane + it * 64;
            const int row = idx >> 3, c4 = (idx & 7) * 4;
            const int qq2 = q0 + row;
            if (qq2 < p.L) {
                const f32x4 x4 = *reinterpret_cast<const f32x4*>(slab + row * 36 + c4);
                f16x4 h1, h2;
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const float x = qq2 < L ? x4[t] : 0.0f;
                    h1[t] = (_Float16)x;
                    h2[t] = (_Float16)((x - (float)h1[t]) * 2048.0f);
                }
                _Float16* dst = p.o + b * p.o_bs + (long long)qq2 * p.o_ld + hd * DH + hh * 32 + c4;
                *reinterpret_cast<f16x4*>(dst) = h1;
                *reinterpret_cast<f16x4*>(dst + p.o_sp) = h2;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

}  // namespace

namespace {
thread_local int g_attn_waves = 0;   // hfa_attention_split_tuning override (0: automatic)
thread_local int g_attn_form = 0;    // hfa_attention_split_form override (0: automatic, 32: 32x32x16, 16: 16x16x32)
constexpr int kAttnFormDefault = 16; // the form the automatic choice takes
// Waves (x 32 queries) per workgroup of the split attention, by the busiest CU's share of the grid: the B*H*ceil(L /
// 32w) query blocks of w waves spread over the device's CUs (256 on a whole MI355X), so that CU runs ceil(blocks /
// CUs) * w waves' worth of query rows.  The smaller share wins; on a tie 8 waves for long rows (>= 2048 keys: half the K/V staging per query), 4 for
// short ones (per-block prologue and epilogue).  Measured (profiles/r04/attn_waves_rule.txt): at one utterance,
// L = 1 000 ... 18 000, it picks the faster form at every length, where the old rule (8 from L >= 512) was 9-17 %
// slower at L = 6 000-8 000, 11 000-13 000 and 18 000; 4 x 3 000 -8 %; configs 2, 4 and 5 keep their forms.
inline int split_attn_waves(int B, int H, int L) {
    if (g_attn_waves == 4 || g_attn_waves == 8) return g_attn_waves;
    const long long cus = hfa::device_cus();
    auto share = [&](int w) {
        const long long blocks = (long long)B * H * ((L + QW * w - 1) / (QW * w));
        return (blocks + cus - 1) / cus * w;
    };
    const long long s4 = share(4), s8 = share(8);
    return (s8 < s4 || (s8 == s4 && L >= 2048)) ? 8 : 4;
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

int hfa_attention_split(int B, int H, int L, int head_dim, float scale, const uint16_t* q, long long q_sp,
                        long long q_bs, int q_ld, const uint16_t* k, long long k_sp, long long k_bs, int k_ld,
                        const uint16_t* v, long long v_sp, long long v_bs, int v_ld, uint16_t* o, long long o_sp,
                        long long o_bs, int o_ld, const int32_t* key_len, hipStream_t stream) {
    if (head_dim != DH) {
        hfa::set_error("hfa_attention_split: head_dim=%d unsupported (64 only)", head_dim);
        return HFA_EINVAL;
    }
    if (B < 0 || H < 1 || L < 0) {
        hfa::set_error("hfa_attention_split: bad sizes");
        return HFA_EINVAL;
    }
    if (B == 0 || L == 0) return HFA_OK;
    if ((((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)o) & 15) || (q_ld | k_ld | v_ld | o_ld) % 8 ||
        (q_bs | k_bs | v_bs | o_bs | q_sp | k_sp | v_sp | o_sp) % 8) {
        hfa::set_error("hfa_attention_split: planes must be 16-byte aligned with strides multiple of 8 halves");
        return HFA_EINVAL;
    }
    if (((long long)(L - 1) * k_ld + DH) * 2 >= 0x7fffffffLL || ((long long)(L - 1) * v_ld + DH) * 2 >= 0x7fffffffLL) {
        hfa::set_error("hfa_attention_split: K/V span exceeds 31-bit buffer offsets");
        return HFA_EINVAL;
    }
    AttnSP p{B, H, L, scale, (const _Float16*)q, q_sp, q_bs, q_ld, (const _Float16*)k, k_sp, k_bs, k_ld,
             (const _Float16*)v, v_sp, v_bs, v_ld, (_Float16*)o, o_sp, o_bs, o_ld, key_len};
    const int nw = split_attn_waves(B, H, L);
    const long long nblk = (long long)((L + QW * nw - 1) / (QW * nw)) * B * H;
    if (nblk > 0x7fffffffLL) {
        hfa::set_error("hfa_attention_split: grid too large");
        return HFA_EINVAL;
    }
    const int form = g_attn_form ? g_attn_form : kAttnFormDefault;
    if (form == 16) {
        if (nw == 8)
            hipLaunchKernelGGL((attn_fwd_split16_kernel<8>), dim3((unsigned)nblk), dim3(8 * 64), 0, stream, p);
        else
            hipLaunchKernelGGL((attn_fwd_split16_kernel<4>), dim3((unsigned)nblk), dim3(4 * 64), 0, stream, p);
    } else if (nw == 8) {
        hipLaunchKernelGGL((attn_fwd_split_kernel<8>), dim3((unsigned)nblk), dim3(8 * 64), 0, stream, p);
    } else {
        hipLaunchKernelGGL((attn_fwd_split_kernel<4>), dim3((unsigned)nblk), dim3(4 * 64), 0, stream, p);
    }
    return hfa::check_launch("hfa_attention_split");
}

// Waves per workgroup of hfa_attention_split: 4 or 8, 0 = automatic (benchmarks and the 4/8 parity test).
int hfa_attention_split_tuning(int waves) {
    if (waves != 0 && waves != 4 && waves != 8) {
        hfa::set_error("hfa_attention_split_tuning: waves must be 0, 4 or 8");
        return HFA_EINVAL;
    }
    g_attn_waves = waves;
    return HFA_OK;
}

// MFMA form of hfa_attention_split: 16 (v_mfma_f32_16x16x32_f16), 32 (v_mfma_f32_32x32x16_f16), 0 = automatic.
int hfa_attention_split_form(int form) {
    if (form != 0 && form != 16 && form != 32) {
        hfa::set_error("hfa_attention_split_form: form must be 0, 16 or 32");
        return HFA_EINVAL;
    }
    g_attn_form = form;
    return HFA_OK;
}

// The kernel instantiation hfa_attention_split launches for (B, H, L) under the current tuning (probe / profiler
// labels): "attn_fwd_split16_kernel<4>" etc.
const char* hfa_attention_split_kernel_name(int B, int H, int L) {
    static thread_local char buf[64];
    const int nw = split_attn_waves(B, H, L), form = g_attn_form ? g_attn_form : kAttnFormDefault;
    snprintf(buf, sizeof(buf), "%s<%d>", form == 16 ? "attn_fwd_split16_kernel" : "attn_fwd_split_kernel", nw);
    return buf;
}

}  // extern "C"
