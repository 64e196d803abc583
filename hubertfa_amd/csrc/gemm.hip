// gemm.hip — f32 MFMA implicit-GEMM (v_mfma_f32_32x32x2_f32) with fused epilogues, for every dense
// contraction on the path:
//   * nn.Linear / addmm: feature projection, QKV, out-proj, FFN (networks/hubert/model.py:27-33,122;
//     transformers HubertAttention/HubertFeedForward), UNet shortcut + head (resnet_block.py:36-40,
//     forced_alignment.py:53-55)
//   * conv1d as implicit GEMM over a [T, C] (channels-last) activation: extractor conv1..6 (model.py:100-114),
//     grouped positional conv k128/pad64/g16 (model.py:135-147), UNet k3 convs / k2 stride-2 down-sampling /
//     k2 stride-2 transposed up-sampling (resnet_block.py:18-24,27-33, stride_conv.py:23-47)
//   * the polyphase sinc resampler (torchaudio Resample: tools/load_wav.py:7, tools/encoder.py:46-48) as a
//     GEMM over overlapping frames of the padded wave.
//
//   C[z](m, n) = epi( sum_k A[z](m, k) * W[z](n, k) + bias[n] ) + R[z](m, n)
//   A[z](m, k): k = j*Cg + c,  t = m*stride + j - pad,  A(m,k) = (0 <= t < Tin) ? X[zb*sAb + zg*sAg + t*ldx + c] : 0
//   z = zb*G + zg (batch x group), W[z] = W + zg*sWg (row n at n*ldw, K-contiguous = [Cout][k][Cin] im2col order)
//
// f32-in MFMA is bit-for-bit an fmaf chain (exact f32, no TF32 on gfx950), so this is the fp32 parity path.
// Tile BM x BN x 16 with WM x WN waves, each wave (BM/WM) x (BN/WN) = TI x TJ MFMA 32x32 tiles.  A and W
// tiles are staged global -> LDS by buffer_load ... lds (LDS-DMA, 2-3 stages, no VALU in the main loop; the
// default) or register-staged (fallback for unaligned A / spans past 31-bit offsets) into an XOR-swizzled
// [row][16] image read with conflict-free ds_read_b128.  A lane's ds_read_b128 brings 4 consecutive k of its
// row; the 4 MFMAs of a k-octet consume one element each, with the same permutation on the W side, so every k is
// summed exactly once.  Block ids are remapped so consecutive logical tiles (same A rows, adjacent W columns)
// share an XCD's L2.
#include "hfa_common.h"
#include "hfa.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

struct GemmP {
    int M, N, K, G, m_tiles, n_tiles;
    const float* A; long long sAb, sAg; int ldx, stride, pad, Cg, Tin;
    const float* W; long long sWg; int ldw;
    const float* bias; long long sBg;
    const float* R; long long sRb, sRg; int ldr;
    float* C; long long sCb, sCg; int ldc;
    // split-f16 operands (gemm_split_kernel): A / W / output as two f16 planes (hi, lo * 2^11), element strides
    // as above (halves), plane 1 at +sAp / +sWp / +sCp; Ch set = planes out instead of C; oflow = range flag
    const _Float16* Ah; long long sAp;
    const _Float16* Wh; long long sWp;
    _Float16* Ch; long long sCp;
    int* oflow;
    int cvec;      // split f32 output: 16-B row pieces (C rows 16-B aligned); 0: scalar stores (no R, no planes)
    const _Float16* Rh; long long sRp;   // split f32 output: the residual as split planes (strides of R, in halves)
};

enum { EPI_NONE = 0, EPI_GELU = 1 };

// Epilogue shared by both kernels: C/D layout of the 32x32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) +
// 4*(lane>>5).  GELU is hfa::gelu_fast (branch-free, 17 VALU ops).  (A
// separate unguarded interior-tile path with batched residual loads measured slower: it pushed the 128-VGPR tile
// into spills.)
template <int EPI, int TI, int TJ>
__device__ __forceinline__ void store_tile(const GemmP& p, const f32x16 (&acc)[TI][TJ], int zb, int zg, int wrow0,
                                           int wcol0, int lane) {
    float* Cb = p.C + zb * p.sCb + zg * p.sCg;
    const float* Rb = p.R ? p.R + zb * p.sRb + zg * p.sRg : nullptr;
    const float* biasb = p.bias ? p.bias + zg * p.sBg : nullptr;
    const int row0 = wrow0 + 4 * (lane >> 5);
    const int col0 = wcol0 + (lane & 31);
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
        const int col = col0 + j * 32;
        if (col >= p.N) continue;
        const float bv = biasb ? biasb[col] : 0.0f;
#pragma unroll
        for (int i = 0; i < TI; ++i) {
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int row = row0 + i * 32 + (e & 3) + 8 * (e >> 2);
                if (row >= p.M) continue;
                float v = acc[i][j][e] + bv;
                if (EPI == EPI_GELU) v = hfa::gelu_fast(v);
                if (Rb) v += Rb[(long long)row * p.ldr + col];
                Cb[(long long)row * p.ldc + col] = v;
            }
        }
    }
}

// Epilogue through LDS (DMA kernel, 16-B aligned C/R rows): each 32x32 accumulator sub-tile (+bias, GELU) is
// transposed through a per-wave [32][36] slab so that every lane stores (and adds the residual to) 4 consecutive
// columns with one dwordx4: 4 stores + 4 residual loads per sub-tile instead of 16 + 16 scalar ones, each of
// which also cost a 64-bit address computation on the VALU the f32 MFMAs share (measured: the scalar stores
// cost 2-4 % of a GEMM).
template <int EPI, int TI, int TJ>
__device__ __forceinline__ void store_tile_lds(const GemmP& p, const f32x16 (&acc)[TI][TJ], int zb, int zg,
                                               int wrow0, int wcol0, int lane, float* slab, bool check = false) {
    bool bad = false;                                    // check: raise *oflow on a non-finite accumulator
    float* Cb = p.C + zb * p.sCb + zg * p.sCg;
    const float* Rb = p.R ? p.R + zb * p.sRb + zg * p.sRg : nullptr;
    const float* biasb = p.bias ? p.bias + zg * p.sBg : nullptr;
    const int r32 = lane & 31, h = lane >> 5;
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
        const int col0 = wcol0 + j * 32;
        if (col0 >= p.N) continue;                       // wave-uniform
        const float bv = (biasb && col0 + r32 < p.N) ? biasb[col0 + r32] : 0.0f;
#pragma unroll
        for (int i = 0; i < TI; ++i) {
            const int row0 = wrow0 + i * 32;
            if (row0 >= p.M) continue;                   // wave-uniform
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                if (check) bad |= !__builtin_isfinite(acc[i][j][e]);
                float v = acc[i][j][e] + bv;
                if (EPI == EPI_GELU) v = hfa::gelu_fast(v);
                slab[((e & 3) + 8 * (e >> 2) + 4 * h) * 36 + r32] = v;
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int idx = lane + k * 64;
                const int r = idx >> 3, c4 = (idx & 7) * 4;
                const int row = row0 + r, col = col0 + c4;
                if (row < p.M) {
                    f32x4 v = *reinterpret_cast<const f32x4*>(slab + r * 36 + c4);
                    float* dst = Cb + (long long)row * p.ldc + col;
                    if (col + 3 < p.N && p.cvec) {
                        if (Rb) v += *reinterpret_cast<const f32x4*>(Rb + (long long)row * p.ldr + col);
                        *reinterpret_cast<f32x4*>(dst) = v;
                    } else {
#pragma unroll
                        for (int t = 0; t < 4; ++t)
                            if (col + t < p.N) dst[t] = v[t] + (Rb ? Rb[(long long)row * p.ldr + col + t] : 0.0f);
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    if (bad && p.oflow) *p.oflow = 1;
}

template <int EPI, bool VEC_A, int BK, int BM, int BN, int WM, int WN>
// 4-wave tiles are register-capped at 128 (accumulators included) so 4 workgroups fit per CU.
__global__ __launch_bounds__(64 * WM * WN, (WM * WN == 4) ? 4 : 2) void gemm_f32_kernel(const GemmP p) {
    constexpr int NT = 64 * WM * WN;
    // Unpadded BK-float LDS rows with the 16-B chunk index XOR-swizzled by row: chunk' = chunk ^ sw(row).
    // BK=16: sw = (row>>2)&3 makes every ds_read_b128 lane group (rows {0-3,12-15,20-27} / {4-11,16-19,28-31})
    // hit 16 distinct 4-bank slots, and every 8-lane ds_write_b128 group (2 rows x 4 chunks) 32 distinct
    // banks; BK=32: sw = (row>>1)&7 does the same for 128-B rows.  (PMC: the padded layout spent 1/3 of its
    // LDS cycles in write conflicts.)
    constexpr int LDL = BK;
    constexpr int TI = BM / WM / 32, TJ = BN / WN / 32;
    constexpr int CPR = BK / 4;                 // float4 chunks per row per K-step
    constexpr int LA = BM * CPR / NT;           // A float4 loads per thread
    constexpr int LB = BN * CPR / NT;           // W float4 loads per thread
    static_assert(LA * NT == BM * CPR && LB * NT == BN * CPR, "tile/thread mismatch");
    __shared__ __attribute__((aligned(16))) float sA[2][BM * LDL];
    __shared__ __attribute__((aligned(16))) float sB[2][BN * LDL];

    // XCD-aware bijective remap of the tile id (cdna_hip_programming.md §5.5 T1)
    const int nwg = gridDim.x, orig = blockIdx.x;
    const int xcd = orig & 7, q = nwg >> 3, r8 = nwg & 7;
    const int wgid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (orig >> 3);
    const int tm = wgid / p.n_tiles, tn = wgid - tm * p.n_tiles;
    const int zb = blockIdx.z / p.G, zg = blockIdx.z - zb * p.G;

    const float* Ab = p.A + zb * p.sAb + zg * p.sAg;
    const float* Wb = p.W + zg * p.sWg;
    const int tid = threadIdx.x;

    // Per-thread staging rows are fixed for the whole K loop: precompute their base pointers and the input
    // time index of tap 0 once, so a K-step only adds the (wave-uniform) tap/channel offset.
    int a_row[LA], a_c4[LA], b_row[LB], b_c4[LB], a_t0[LA];
    bool b_ok[LB], a_mok[LA];
    const float* a_base[LA];
    const float* b_base[LB];
#pragma unroll
    for (int i = 0; i < LA; ++i) {
        const int idx = tid + i * NT;
        a_row[i] = idx / CPR;
        a_c4[i] = (idx % CPR) * 4;
        const int m = tm * BM + a_row[i];
        a_mok[i] = m < p.M;
        a_t0[i] = m * p.stride - p.pad;
        a_base[i] = Ab + (long long)a_t0[i] * p.ldx + a_c4[i];
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
        const int idx = tid + i * NT;
        b_row[i] = idx / CPR;
        b_c4[i] = (idx % CPR) * 4;
        b_ok[i] = tn * BN + b_row[i] < p.N;
        b_base[i] = Wb + (long long)(tn * BN + b_row[i]) * p.ldw + b_c4[i];
    }
    f32x4 ra[LA], rb[LB];
    auto load_regs = [&](int k0) {
        const int j = k0 / p.Cg;                       // wave-uniform: tap index of this K-step
        const long long aoff = (long long)j * p.ldx + (k0 - j * p.Cg);
#pragma unroll
        for (int i = 0; i < LA; ++i) {
            const int t = a_t0[i] + j;
            const bool ok = a_mok[i] && (t >= 0) && (t < p.Tin);
            // (a guarded load costs an exec-mask branch but fewer VGPRs than a clamped load + select, which
            // spilled at the 128-register cap; measured: the guarded form is 3-25 % faster)
            const float* src = a_base[i] + aoff;
            if (VEC_A) ra[i] = ok ? *reinterpret_cast<const f32x4*>(src) : f32x4{0.f, 0.f, 0.f, 0.f};
            else ra[i] = ok ? f32x4{src[0], src[1], src[2], src[3]} : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int i = 0; i < LB; ++i)
            rb[i] = b_ok[i] ? *reinterpret_cast<const f32x4*>(b_base[i] + k0) : f32x4{0.f, 0.f, 0.f, 0.f};
    };
    auto swz = [](int row, int c4) {   // float offset of logical (row, float c4) in the swizzled image
        constexpr int SH = (CPR == 4) ? 2 : 1;
        return row * LDL + ((((c4 >> 2) ^ (row >> SH)) & (CPR - 1)) << 2);
    };
    auto store_lds = [&](int buf) {
#pragma unroll
        for (int i = 0; i < LA; ++i) *reinterpret_cast<f32x4*>(&sA[buf][swz(a_row[i], a_c4[i])]) = ra[i];
#pragma unroll
        for (int i = 0; i < LB; ++i) *reinterpret_cast<f32x4*>(&sB[buf][swz(b_row[i], b_c4[i])]) = rb[i];
    };

    const int wave = tid >> 6, lane = tid & 63;
    const int wm = wave / WN, wn = wave % WN;
    const int r32 = lane & 31, h = lane >> 5;
    f32x16 acc[TI][TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

    // Read offsets in float4 units: the swizzle depends on row bits that the 32-row sub-tile offsets leave
    // unchanged, so one per-lane offset per k-octet serves every sub-tile (i*32*CPR folds into the immediate).
    // Indexing whole f32x4 elements keeps the 16-B alignment visible, so every read is one ds_read_b128 (byte
    // arithmetic on a float* let the compiler split half of them into ds_read2_b32 pairs: 2x the LDS cycles
    // plus bank conflicts under the 32-bank rule).
    int rdA[BK / 8], rdB[BK / 8];
#pragma unroll
    for (int kk = 0; kk < BK / 8; ++kk) {
        rdA[kk] = swz(wm * (BM / WM) + r32, kk * 8 + h * 4) >> 2;
        rdB[kk] = swz(wn * (BN / WN) + r32, kk * 8 + h * 4) >> 2;
    }

    const int nk = p.K / BK;
    load_regs(0);
    store_lds(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) load_regs((kt + 1) * BK);
        const f32x4* sA4 = reinterpret_cast<const f32x4*>(sA[cur]);
        const f32x4* sB4 = reinterpret_cast<const f32x4*>(sB[cur]);
#pragma unroll
        for (int kk = 0; kk < BK / 8; ++kk) {
            f32x4 a[TI], b[TJ];
#pragma unroll
            for (int i = 0; i < TI; ++i) a[i] = sA4[rdA[kk] + i * 32 * CPR];
#pragma unroll
            for (int j = 0; j < TJ; ++j) b[j] = sB4[rdB[kk] + j * 32 * CPR];
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int i = 0; i < TI; ++i)
#pragma unroll
                    for (int j = 0; j < TJ; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][e], b[j][e], acc[i][j], 0, 0, 0);
        }
        if (kt + 1 < nk) store_lds(cur ^ 1);
        __syncthreads();
    }

    store_tile<EPI, TI, TJ>(p, acc, zb, zg, tm * BM + wm * (BM / WM), tn * BN + wn * (BN / WN), lane);
}

// ---- LDS-DMA pipeline ------------------------------------------------------------------------------------------
// On gfx950 the f32 MFMA runs at the f32 VECTOR rate, so every VALU instruction in the main loop costs MFMA
// cycles (ablation, scripts/gpu_gemm_abl.sh: dropping the register-staged loads + ds_writes alone took conv1 from
// 125 to 143 TFLOP/s).  This kernel stages A and W with buffer_load_dwordx4 ... lds (global -> LDS, no VGPR
// data, no ds_write) from per-lane byte offsets fixed for a whole tap; the K-step advance is a scalar soffset,
// so the main loop is 32 MFMAs + 8 ds_read_b128 + (DA+DB) DMA issues + one counted wait/barrier per K-step, with
// no vector ALU work.  NS LDS stages (NS-1 K-steps in flight across the barrier).  The LDS image is the same
// XOR-swizzled [row][16] image as above: one DMA wave-instruction writes 1 KiB lane-linearly (16 rows x 4
// chunks), so the swizzle is applied on the SOURCE side (lane l loads chunk (l&3) ^ sw(row)).
// Out-of-range conv taps (padding) read through a voffset beyond the buffer's num_records, which the range check
// turns into zeros (scripts/probes/dma_oob.hip); rows past M / N are clamped (their outputs are never stored).

template <int EPI, int BM, int BN, int WM, int WN, int NS, int OCC, bool VEC_C>
__global__ __launch_bounds__(64 * WM * WN, OCC) void gemm_dma_kernel(const GemmP p) {
    constexpr int BK = 16, CPR = 4, NW = WM * WN;
    constexpr int TI = BM / WM / 32, TJ = BN / WN / 32;
    // 1-KiB DMA wave-instructions per K-step: IA = BM/16 for A, IW = BN/16 for W, instruction i on wave i % NW;
    // a wave issues at most DA / DB of them.  Uneven shares (BN = 96 over 4 waves) need NS = 2, whose waits
    // drain to vmcnt(0); the counted waits of NS = 3 assume every wave issues the same number.
    constexpr int IA = BM / 16, IW = BN / 16;
    constexpr int DA = (IA + NW - 1) / NW, DB = (IW + NW - 1) / NW;
    static_assert(IA * 16 == BM && IW * 16 == BN, "tile/DMA mismatch");
    static_assert(NS == 2 || (IA % NW == 0 && IW % NW == 0), "uneven DMA shares need the 2-stage pipeline");
    constexpr int STAGE = (BM + BN) * BK;                     // floats per stage (A image, then W image)
    __shared__ __attribute__((aligned(16))) float smem[NS * STAGE];   // one LDS object (no extra waits)

    const int nwg = gridDim.x, orig = blockIdx.x;
    const int xcd = orig & 7, q = nwg >> 3, r8 = nwg & 7;
    const int wgid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (orig >> 3);
    const int tm = wgid / p.n_tiles, tn = wgid - tm * p.n_tiles;
    const int zb = blockIdx.z / p.G, zg = blockIdx.z - zb * p.G;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    // buffer descriptors over this (batch, group)'s A rows and W rows (host checks both spans fit 31 bits)
    const float* Ab = p.A + zb * p.sAb + zg * p.sAg;
    const float* Wb = p.W + zg * p.sWg;
    const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(
        (void*)Ab, (short)0, (int)(((long long)(p.Tin - 1) * p.ldx + p.Cg) * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc(
        (void*)Wb, (short)0, (int)(((long long)(p.N - 1) * p.ldw + p.K) * 4), 0x00020000);

    // per-lane source: DMA d of this wave fills tile rows (wave*D + d)*16 + lane/4, LDS chunk slot lane&3
    int a_t0[DA], a_c[DA];
    unsigned voffA[DA], voffW[DB];
#pragma unroll
    for (int d = 0; d < DA; ++d) {
        const int row = (wave + d * NW) * 16 + (lane >> 2);
        int m = tm * BM + row;
        m = m < p.M ? m : p.M - 1;
        a_t0[d] = m * p.stride - p.pad;
        a_c[d] = ((lane & 3) ^ ((row >> 2) & 3)) * 4;
    }
#pragma unroll
    for (int d = 0; d < DB; ++d) {
        const int row = (wave + d * NW) * 16 + (lane >> 2);
        int n = tn * BN + row;
        n = n < p.N ? n : p.N - 1;
        voffW[d] = (unsigned)((n * p.ldw + ((lane & 3) ^ ((row >> 2) & 3)) * 4) * 4);
    }
    auto set_tap = [&](int j) {      // once per conv tap (every Cg/16 K-steps)
#pragma unroll
        for (int d = 0; d < DA; ++d) {
            const int t = a_t0[d] + j;
            voffA[d] = (t >= 0 && t < p.Tin) ? (unsigned)((t * p.ldx + a_c[d]) * 4) : hfa::DMA_OOB;
        }
    };
    const unsigned lds0 = hfa::lds_addr(smem);
    // K-step cursor: tap j, channel offset c0 inside the tap, absolute k0
    int cur_j = 0, cur_c0 = 0, cur_k0 = 0;
    set_tap(0);
    auto issue = [&](int stage) {
        const unsigned a_dst = lds0 + stage * STAGE * 4 + wave * 1024;
        const unsigned w_dst = lds0 + (stage * STAGE + BM * BK) * 4 + wave * 1024;
#pragma unroll
        for (int d = 0; d < DA; ++d)
            if (IA % NW == 0 || wave + d * NW < IA)
                hfa::dma16(voffA[d], rA, (unsigned)cur_c0 * 4, a_dst + d * NW * 1024);
#pragma unroll
        for (int d = 0; d < DB; ++d)
            if (IW % NW == 0 || wave + d * NW < IW)
                hfa::dma16(voffW[d], rW, (unsigned)cur_k0 * 4, w_dst + d * NW * 1024);
        cur_k0 += BK;
        cur_c0 += BK;
        if (cur_c0 == p.Cg) {
            cur_c0 = 0;
            set_tap(++cur_j);
        }
    };

    const int wm = wave / WN, wn = wave % WN;
    const int r32 = lane & 31, h = lane >> 5;
    int rdA[2], rdB[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
        const int c = kk * 2 + h;
        rdA[kk] = (wm * (BM / WM) + r32) * CPR + (c ^ ((r32 >> 2) & 3));
        rdB[kk] = BM * CPR + (wn * (BN / WN) + r32) * CPR + (c ^ ((r32 >> 2) & 3));
    }
    f32x16 acc[TI][TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

    const int nk = p.K / BK;
    // prologue: NS-1 K-steps in flight, wait for the first
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
        if (s < nk) issue(s);
    if (nk >= NS - 1) hfa::wait_vm_barrier<(NS - 2) * (DA + DB)>();
    else hfa::wait_vm_barrier<0>();

    const f32x4* s4 = reinterpret_cast<const f32x4*>(smem);
    int stage = 0;
    for (int kt = 0; kt < nk; ++kt) {
        // refill the stage read NS-1 steps ago (every wave passed the barrier after its reads)
        const bool more = kt + NS - 1 < nk;
        if (more) issue(stage == 0 ? NS - 1 : stage - 1);
        const f32x4* st = s4 + stage * (STAGE / 4);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            f32x4 a[TI], b[TJ];
#pragma unroll
            for (int i = 0; i < TI; ++i) a[i] = st[rdA[kk] + i * 32 * CPR];
#pragma unroll
            for (int j = 0; j < TJ; ++j) b[j] = st[rdB[kk] + j * 32 * CPR];
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int i = 0; i < TI; ++i)
#pragma unroll
                    for (int j = 0; j < TJ; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][e], b[j][e], acc[i][j], 0, 0, 0);
        }
        if (kt + 1 < nk) {
            if (more) hfa::wait_vm_barrier<(NS - 2) * (DA + DB)>();   // K-step kt+1 landed, kt+2.. still in flight
            else hfa::wait_vm_barrier<0>();
        }
        stage = stage + 1 == NS ? 0 : stage + 1;
    }
    if constexpr (VEC_C) {
        static_assert(NW * 32 * 36 <= NS * STAGE, "epilogue slabs exceed the staging LDS");
        __syncthreads();                                 // every wave done reading the last stage
        store_tile_lds<EPI, TI, TJ>(p, acc, zb, zg, tm * BM + wm * (BM / WM), tn * BN + wn * (BN / WN), lane,
                                    smem + wave * (32 * 36));
    } else {
        store_tile<EPI, TI, TJ>(p, acc, zb, zg, tm * BM + wm * (BM / WM), tn * BN + wn * (BN / WN), lane);
    }
}

// ---- 48-wide tile on 16x16x4 MFMAs (the grouped positional conv: 48 output channels per group) -------------
// A 64-wide tile wastes a quarter of its MFMAs on N = 48.  Here each of 4 waves owns 32 rows x 48 columns =
// 2 x 3 blocks of v_mfma_f32_16x16x4_f32 (lane l: A[l&15][k=l>>4], B[k=l>>4][l&15]; D: col l&15,
// row 4(l>>4)+r).  A lane's ds_read_b128 brings 4 consecutive k of its row (chunk l>>4 of the 16-k step), and
// MFMA e consumes element e, the same permutation on both operands.  The 16-row read groups need their own
// chunk swizzle: chunk' = chunk ^ F[(row>>2)&3] with F = {0,2,3,1} keeps every ds_read_b128 lane group on 16
// distinct 16-B slots (the 32-row tiles' F = identity does not).  DMA: A 2 x 1 KiB per wave, W 3 x 1 KiB on
// waves 0-2; stages as in gemm_dma_kernel.
constexpr int swz48(int row) { return (0x78 >> (((row >> 2) & 3) * 2)) & 3; }    // F = {0, 2, 3, 1}

template <int EPI, int NS>
__global__ __launch_bounds__(256, 4) void gemm_dma_n48_kernel(const GemmP p) {
    constexpr int BM = 128, BN = 48, BK = 16, NW = 4;
    constexpr int STAGE = (BM + BN) * BK;
    __shared__ __attribute__((aligned(16))) float smem[NS * STAGE];

    const int nwg = gridDim.x, orig = blockIdx.x;
    const int xcd = orig & 7, q = nwg >> 3, r8 = nwg & 7;
    const int wgid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (orig >> 3);
    const int tm = wgid / p.n_tiles, tn = wgid - tm * p.n_tiles;
    const int zb = blockIdx.z / p.G, zg = blockIdx.z - zb * p.G;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    const float* Ab = p.A + zb * p.sAb + zg * p.sAg;
    const float* Wb = p.W + zg * p.sWg;
    const __amdgpu_buffer_rsrc_t rA = hfa::make_rsrc(Ab, ((long long)(p.Tin - 1) * p.ldx + p.Cg) * 4);
    const __amdgpu_buffer_rsrc_t rW = hfa::make_rsrc(Wb, ((long long)(p.N - 1) * p.ldw + p.K) * 4);

    int a_t0[2], a_c[2];
    unsigned voffA[2], voffW = 0;
#pragma unroll
    for (int d = 0; d < 2; ++d) {
        const int row = (wave * 2 + d) * 16 + (lane >> 2);
        int m = tm * BM + row;
        m = m < p.M ? m : p.M - 1;
        a_t0[d] = m * p.stride - p.pad;
        a_c[d] = ((lane & 3) ^ swz48(row)) * 4;
    }
    {
        const int row = wave * 16 + (lane >> 2);          // waves 0-2: W rows 0..47
        int n = tn * BN + row;
        n = n < p.N ? n : p.N - 1;
        voffW = (unsigned)((n * p.ldw + ((lane & 3) ^ swz48(row)) * 4) * 4);
    }
    auto set_tap = [&](int j) {
#pragma unroll
        for (int d = 0; d < 2; ++d) {
            const int t = a_t0[d] + j;
            voffA[d] = (t >= 0 && t < p.Tin) ? (unsigned)((t * p.ldx + a_c[d]) * 4) : hfa::DMA_OOB;
        }
    };
    const unsigned lds0 = hfa::lds_addr(smem);
    int cur_j = 0, cur_c0 = 0, cur_k0 = 0;
    set_tap(0);
    auto issue = [&](int stage) {
        const unsigned a_dst = lds0 + stage * STAGE * 4 + wave * 2 * 1024;
        hfa::dma16(voffA[0], rA, (unsigned)cur_c0 * 4, a_dst);
        hfa::dma16(voffA[1], rA, (unsigned)cur_c0 * 4, a_dst + 1024);
        if (wave < 3) hfa::dma16(voffW, rW, (unsigned)cur_k0 * 4, lds0 + (stage * STAGE + BM * BK) * 4 + wave * 1024);
        cur_k0 += BK;
        cur_c0 += BK;
        if (cur_c0 == p.Cg) {
            cur_c0 = 0;
            set_tap(++cur_j);
        }
    };
    // this wave's DMAs per K-step: 3 (waves 0-2) or 2 (wave 3); the counted wait differs per wave
    auto wait_steps_in_flight = [&](bool keep) {
        if (!keep) hfa::wait_vm_barrier<0>();
        else if (wave < 3) hfa::wait_vm_barrier<(NS - 2) * 3>();
        else hfa::wait_vm_barrier<(NS - 2) * 2>();
    };

    const int r16 = lane & 15, g = lane >> 4;
    int rdA[2], rdB[3];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int row = wave * 32 + i * 16 + r16;
        rdA[i] = row * 4 + (g ^ swz48(row));
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int row = j * 16 + r16;
        rdB[j] = BM * 4 + row * 4 + (g ^ swz48(row));
    }
    f32x4 acc[2][3];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = p.K / BK;
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
        if (s < nk) issue(s);
    wait_steps_in_flight(nk >= NS - 1);
    const f32x4* s4 = reinterpret_cast<const f32x4*>(smem);
    int stage = 0;
    for (int kt = 0; kt < nk; ++kt) {
        const bool more = kt + NS - 1 < nk;
        if (more) issue(stage == 0 ? NS - 1 : stage - 1);
        const f32x4* st = s4 + stage * (STAGE / 4);
        f32x4 a[2], b[3];
#pragma unroll
        for (int i = 0; i < 2; ++i) a[i] = st[rdA[i]];
#pragma unroll
        for (int j = 0; j < 3; ++j) b[j] = st[rdB[j]];
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][e], b[j][e], acc[i][j], 0, 0, 0);
        if (kt + 1 < nk) wait_steps_in_flight(more);
        stage = stage + 1 == NS ? 0 : stage + 1;
    }

    // epilogue: D col = lane&15, row = 4(lane>>4) + r
    float* Cb = p.C + zb * p.sCb + zg * p.sCg;
    const float* Rb = p.R ? p.R + zb * p.sRb + zg * p.sRg : nullptr;
    const float* biasb = p.bias ? p.bias + zg * p.sBg : nullptr;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int col = tn * BN + j * 16 + r16;
        if (col >= p.N) continue;
        const float bv = biasb ? biasb[col] : 0.0f;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = tm * BM + wave * 32 + i * 16 + 4 * g + r;
                if (row >= p.M) continue;
                float v = acc[i][j][r] + bv;
                if (EPI == EPI_GELU) v = hfa::gelu_fast(v);
                if (Rb) v += Rb[(long long)row * p.ldr + col];
                Cb[(long long)row * p.ldc + col] = v;
            }
        }
    }
}

// ---- split-f16 GEMM (f32-class accuracy on the f16 MFMA) ---------------------------------------------------------
// Every f32 operand x is carried as two f16 planes: x1 = f16(x), x2 = f16((x - x1) * 2^11); x1 + 2^-11 x2 keeps 22
// of f32's 24 significand bits (relative error <= 2^-22, absolute 2^-36 below f16's normal range).  The product
// a.w is evaluated as a1.w1 + 2^-11 (a1.w2 + a2.w1): every partial product of two f16 is exact in the MFMA's f32
// accumulator, and the dropped a2.w2 term is 2^-22 relative, so the result is within a few f32 rounding steps of
// the f32-MFMA result (scripts/split_precision_sim.py: per-frame log-probs 2.2e-5 from an f64 evaluation of the
// whole path, the plain f32 path 2.0e-5).  v_mfma_f32_32x32x16_f16 does 16x the FLOP per clock of the f32 MFMA, so
// the 3 products run at 5.3x the f32-MFMA rate.  Two accumulators (main, correction) keep the 2^-11 scale exact.
// Range: |x| must stay below 65504 (f16 max); the producer of a split operand raises *oflow otherwise, and the host
// re-runs the batch on the f32 path (ops.SplitOverflow).
// Tile: the f32 DMA kernel's geometry with 32 halves (64 B) per row per K-step: the same 1-KiB DMA pieces (16 rows
// x 4 chunks), the same XOR-swizzled [row][64 B] image per plane, 4 planes per stage (A1, A2, W1, W2).  A lane's
// ds_read_b128 brings 8 consecutive k of its row = one MFMA operand (lane l: row l&31, k 8(l>>5)..+7 of a 16-k
// sub-step; the same mapping on both operands).
template <int MF> struct AccT;
template <> struct AccT<16> { typedef f32x4 type; };

// The 32x32 output block (i, j) of a wave's tile (units of 32 rows / columns) -> the wave's [32][S] LDS slab, with
// bias and GELU applied, from the 2 x 2 16x16x32 accumulators that cover it (col lane&15, row 4(lane>>4) + e).
// Returns true when an accumulator is not finite.
template <int MF, int NI, int NJ, int S = 36>
__device__ __forceinline__ bool fill_slab(const typename AccT<MF>::type (&acc)[NI][NJ], int i, int j, int epi,
                                          const float* biasb, int col0, int N, int lane, float* slab,
                                          float scale = 1.0f) {
    static_assert(MF == 16, "16x16x32 accumulators");
    bool bad = false;
    const int c16 = lane & 15, g = lane >> 4;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
        const int col = 16 * jj + c16;
        const float bv = (biasb && col0 + col < N) ? biasb[col0 + col] : 0.0f;
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float a = acc[2 * i + ii][2 * j + jj][e];
                bad |= !__builtin_isfinite(a);
                float v = __builtin_fmaf(a, scale, bv);   // scale: the single accumulator's 2^-11 (exact)
                if (epi == EPI_GELU) v = hfa::gelu_fast(v);
                slab[(16 * ii + 4 * g + e) * S + col] = v;
            }
    }
    return bad;
}

// Split-plane epilogue: TI x TJ blocks of 32 x 32 per wave, each through the slab (16-B row pieces out).
template <int MF, int TI, int TJ, int NI, int NJ>
__device__ __forceinline__ void store_split_lds(const GemmP& p, const typename AccT<MF>::type (&acc)[NI][NJ], int EPI_,
                                                int zb, int zg, int wrow0, int wcol0, int lane, float* slab,
                                                float scale = 1.0f) {
    _Float16* Cb = p.Ch + zb * p.sCb + zg * p.sCg;
    const float* biasb = p.bias ? p.bias + zg * p.sBg : nullptr;
    hfa::h2v nanacc = {(_Float16)0.0f, (_Float16)0.0f};
    const float c2048 = 2048.0f;
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
        const int col0 = wcol0 + j * 32;
        if (col0 >= p.N) continue;
#pragma unroll
        for (int i = 0; i < TI; ++i) {
            const int row0 = wrow0 + i * 32;
            if (row0 >= p.M) continue;
            fill_slab<MF>(acc, i, j, EPI_, biasb, col0, p.N, lane, slab, scale);
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int idx = lane + k * 64;
                const int r = idx >> 3, c4 = (idx & 7) * 4;
                const int row = row0 + r, col = col0 + c4;
                if (row < p.M) {
                    const f32x4 v = *reinterpret_cast<const f32x4*>(slab + r * 36 + c4);
                    uint2 u1, u2;   // columns past N hold finite zeros (zero W rows): the range check may see them
                    hfa::split_pair(v[0], v[1], u1.x, u2.x, nanacc, c2048);
                    hfa::split_pair(v[2], v[3], u1.y, u2.y, nanacc, c2048);
                    const f16x4 v1 = __builtin_bit_cast(f16x4, u1), v2 = __builtin_bit_cast(f16x4, u2);
                    _Float16* dst = Cb + (long long)row * p.ldc + col;
                    if (col + 3 < p.N) {
                        *reinterpret_cast<f16x4*>(dst) = v1;
                        *reinterpret_cast<f16x4*>(dst + p.sCp) = v2;
                    } else {
#pragma unroll
                        for (int t = 0; t < 4; ++t)
                            if (col + t < p.N) {
                                dst[t] = v1[t];
                                dst[t + p.sCp] = v2[t];
                            }
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    if (hfa::range_bad(nanacc) && p.oflow) *p.oflow = 1;
}

// Split-plane epilogue over PAIRS of 32 x 32 blocks (TJ even): the two blocks side by side in a [32][68] slab, so a
// store instruction writes 4 rows x 128 B per plane (whole cache lines) instead of 8 rows x 64 B.  Row stride 68:
// the fill's 4 rows of 16 columns land on disjoint banks (68 x 4 = 16 mod 64).  Same values as store_split_lds.
constexpr int kSlab2 = 68;
template <int MF, int TI, int TJ, int NI, int NJ>
__device__ __forceinline__ void store_split_lds2(const GemmP& p, const typename AccT<MF>::type (&acc)[NI][NJ],
                                                 int EPI_, int zb, int zg, int wrow0, int wcol0, int lane,
                                                 float* slab, float scale) {
    static_assert(TJ % 2 == 0, "pairs of column blocks");
    _Float16* Cb = p.Ch + zb * p.sCb + zg * p.sCg;
    const float* biasb = p.bias ? p.bias + zg * p.sBg : nullptr;
    hfa::h2v nanacc = {(_Float16)0.0f, (_Float16)0.0f};
    const float c2048 = 2048.0f;
#pragma unroll
    for (int j = 0; j < TJ; j += 2) {
        const int col0 = wcol0 + j * 32;
        if (col0 >= p.N) continue;
#pragma unroll
        for (int i = 0; i < TI; ++i) {
            const int row0 = wrow0 + i * 32;
            if (row0 >= p.M) continue;
            fill_slab<MF, NI, NJ, kSlab2>(acc, i, j, EPI_, biasb, col0, p.N, lane, slab, scale);
            fill_slab<MF, NI, NJ, kSlab2>(acc, i, j + 1, EPI_, biasb, col0 + 32, p.N, lane, slab + 32, scale);
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int idx = lane + k * 64;
                const int r = idx >> 4, c4 = (idx & 15) * 4;
                const int row = row0 + r, col = col0 + c4;
                if (row < p.M) {
                    const f32x4 v = *reinterpret_cast<const f32x4*>(slab + r * kSlab2 + c4);
                    uint2 u1, u2;   // columns past N hold finite zeros (zero W rows): the range check may see them
                    hfa::split_pair(v[0], v[1], u1.x, u2.x, nanacc, c2048);
                    hfa::split_pair(v[2], v[3], u1.y, u2.y, nanacc, c2048);
                    _Float16* dst = Cb + (long long)row * p.ldc + col;
                    if (col + 3 < p.N) {
                        *reinterpret_cast<uint2*>(dst) = u1;
                        *reinterpret_cast<uint2*>(dst + p.sCp) = u2;
                    } else {
                        const f16x4 v1 = __builtin_bit_cast(f16x4, u1), v2 = __builtin_bit_cast(f16x4, u2);
#pragma unroll
                        for (int t = 0; t < 4; ++t)
                            if (col + t < p.N) {
                                dst[t] = v1[t];
                                dst[t + p.sCp] = v2[t];
                            }
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    if (hfa::range_bad(nanacc) && p.oflow) *p.oflow = 1;
}

// f32 epilogue of the split kernel (+R), through the slab; raises *oflow on a non-finite accumulator.  With p.Ch
// set as well (dual output) the final values also go out as split planes (the next split GEMM's operand, e.g. the
// positional conv's input next to its f32 residual copy), with the planes' range check.
template <int MF, int EPI, int TI, int TJ, int NI, int NJ>
__device__ __forceinline__ void store_f32_lds(const GemmP& p, const typename AccT<MF>::type (&acc)[NI][NJ], int zb,
                                              int zg, int wrow0, int wcol0, int lane, float* slab, bool check,
                                              float scale = 1.0f) {
    bool bad = false;
    hfa::h2v nanacc = {(_Float16)0.0f, (_Float16)0.0f};
    const float c2048 = 2048.0f;
    float* Cb = p.C + zb * p.sCb + zg * p.sCg;
    _Float16* Hb = p.Ch ? p.Ch + zb * p.sCb + zg * p.sCg : nullptr;
    const float* Rb = p.R ? p.R + zb * p.sRb + zg * p.sRg : nullptr;
    const _Float16* Rhb = p.Rh ? p.Rh + zb * p.sRb + zg * p.sRg : nullptr;
    const float* biasb = p.bias ? p.bias + zg * p.sBg : nullptr;
    // The residual planes (out-projection, FFN2: the LayerNorm's planes) are loaded one 32 x 32 block ahead: block
    // b + 1's loads are issued before block b's slab pass, so their latency hides under it instead of stalling every
    // block (the epilogue runs with the matrix pipe idle).  Vector rows only (col + 3 < N, aligned C); the ragged
    // column tail reads its residual directly below.
    constexpr int NB = TI * TJ;
    f16x4 rn1[4], rn2[4];
    auto load_res = [&](int b, f16x4 (&r1)[4], f16x4 (&r2)[4]) {
        const int row0 = wrow0 + (b % TI) * 32, col0 = wcol0 + (b / TI) * 32;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int idx = lane + k * 64;
            const int row = row0 + (idx >> 3), col = col0 + (idx & 7) * 4;
            if (row < p.M && col + 3 < p.N && p.cvec) {
                const _Float16* rh = Rhb + (long long)row * p.ldr + col;
                r1[k] = *reinterpret_cast<const f16x4*>(rh);
                r2[k] = *reinterpret_cast<const f16x4*>(rh + p.sRp);
            }
        }
    };
    if (Rhb) load_res(0, rn1, rn2);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const int i = b % TI, j = b / TI;
        const int col0 = wcol0 + j * 32;
        const int row0 = wrow0 + i * 32;
        f16x4 rc1[4], rc2[4];
        if (Rhb) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                rc1[k] = rn1[k];
                rc2[k] = rn2[k];
            }
            if (b + 1 < NB) load_res(b + 1, rn1, rn2);
        }
        if (col0 >= p.N || row0 >= p.M) continue;
        bad |= fill_slab<MF>(acc, i, j, EPI, biasb, col0, p.N, lane, slab, scale) && check;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int idx = lane + k * 64;
            const int r = idx >> 3, c4 = (idx & 7) * 4;
            const int row = row0 + r, col = col0 + c4;
            if (row < p.M) {
                f32x4 v = *reinterpret_cast<const f32x4*>(slab + r * 36 + c4);
                float* dst = Cb + (long long)row * p.ldc + col;
                if (col + 3 < p.N && p.cvec) {
                    if (Rb) v += *reinterpret_cast<const f32x4*>(Rb + (long long)row * p.ldr + col);
                    if (Rhb) {          // residual planes: hi + 2^-11 lo (exact in f32), one rounding in the add
#pragma unroll
                        for (int t = 0; t < 4; ++t)
                            v[t] += __builtin_fmaf((float)rc2[k][t], 1.0f / 2048.0f, (float)rc1[k][t]);
                    }
                    *reinterpret_cast<f32x4*>(dst) = v;
                } else {
#pragma unroll
                    for (int t = 0; t < 4; ++t)
                        if (col + t < p.N) {
                            v[t] += Rb ? Rb[(long long)row * p.ldr + col + t] : 0.0f;
                            if (Rhb) {
                                const _Float16* rh = Rhb + (long long)row * p.ldr + col + t;
                                v[t] += __builtin_fmaf((float)rh[p.sRp], 1.0f / 2048.0f, (float)rh[0]);
                            }
                            dst[t] = v[t];
                        }
                }
                if (Hb) {
                    uint2 u1, u2;
                    if (col + 3 >= p.N)   // columns past N: no residual was added, keep them out of the check
#pragma unroll
                        for (int t = 0; t < 4; ++t)
                            if (col + t >= p.N) v[t] = 0.0f;
                    hfa::split_pair(v[0], v[1], u1.x, u2.x, nanacc, c2048);
                    hfa::split_pair(v[2], v[3], u1.y, u2.y, nanacc, c2048);
                    const f16x4 v1 = __builtin_bit_cast(f16x4, u1), v2 = __builtin_bit_cast(f16x4, u2);
                    _Float16* hd = Hb + (long long)row * p.ldc + col;
                    if (col + 3 < p.N) {
                        *reinterpret_cast<f16x4*>(hd) = v1;
                        *reinterpret_cast<f16x4*>(hd + p.sCp) = v2;
                    } else {
#pragma unroll
                        for (int t = 0; t < 4; ++t)
                            if (col + t < p.N) {
                                hd[t] = v1[t];
                                hd[t + p.sCp] = v2[t];
                            }
                    }
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    if ((bad || hfa::range_bad(nanacc)) && p.oflow) *p.oflow = 1;
}

// GT (general taps): Cg a multiple of 8 but not of 32 (the grouped positional conv, Cg = 48): a K-step's four
// 16-B chunks can straddle a tap boundary, so every lane tracks its own chunk's (tap, channel) instead of the
// workgroup-uniform tap + scalar channel offset.
// ONE (single accumulator): the three products share one accumulator at scale 2^11 -- a1 (2^11 w1) + a1 w2 + a2 w1,
// with 2^11 w1 formed exactly in registers (v_pk_mul_f16; needs |w| < 32, an overflow shows as a non-finite
// output, which the epilogue flags) -- and the result is scaled by 2^-11 at the end.  Half the accumulator
// registers, so a wave can own a 128 x 64 tile: 0.5 LDS fragment reads per MFMA instead of 0.67 (the LDS, shared
// by the DMA fills and the fragment reads, is what bounds the 64 x 64-per-wave kernel: scripts/gpu_split_abl.sh).
// BK (halves per row per K-step) 32: [row][4 x 16 B] images.  MF 16: v_mfma_f32_16x16x32_f16, one MFMA per 32-deep
// K-step per 16 x 16 block; chunk c of row r sits at c ^ {0, 2, 3, 1}[(r >> 2) & 3] (conflict-free for the lane map
// row lane&15, chunk lane>>4).  Measured on the workload's shapes (profiles/r02/split_mf16.txt): 4-9 % faster than
// the 32x32x16 form (retired in round 5 with the two-accumulator and 16-deep-K-step tuning tiles); the chip holds a
// higher clock under it (1.96-2.04 vs 1.73-1.85 GHz, same MFMA busy).  The next stage's DMA pieces go out two per A
// block over the first blocks of a K-step instead of all at its top (+2-6 %), so the two waves of a SIMD do not both
// stall on DMA issue while the matrix pipe idles.
// F16 (opt-in fast mode, MF 16 tiles only): the operands' high planes alone, one product a1 w1 per MAC -- f16-class
// accuracy (inputs rounded to 11 significand bits, f32 accumulation); the low planes are neither fetched nor read.
// One output tile of gemm_split_kernel (wgid: the tile, z: the launch's blockIdx.z); smem: the kernel's NS * STAGE
// halves of LDS.  (A function of its own since round 6: the same arithmetic, and 2 % off FFN2's 192 x 256 tile in
// the layer microbenchmark, profiles/r06/gemm_tile_fn_ab.txt.)
template <int EPI, int BM, int BN, int WM, int WN, int NS, int OCC, bool OUT_SPLIT, bool GT, bool ONE, int BK,
          int MF, bool F16>
__device__ __forceinline__ void gemm_split_tile(const GemmP p, int wgid, int z, _Float16* smem) {
    static_assert(MF == 16 && ONE && BK == 32, "the built tiles: 16x16x32 MFMA, single accumulator, BK 32");
    static_assert(!F16 || (MF == 16 && NS == 2 && !GT), "the one-product mode runs on the 2-stage 16x16x32 tiles");
    constexpr int CPR = BK / 8, NW = WM * WN;                // 16-B chunks per row per plane
    constexpr int RPP = 64 / CPR;                             // rows per 1-KiB DMA piece
    constexpr int IA = BM / RPP, IW = BN / RPP;               // 1-KiB DMA pieces per plane per K-step
    constexpr int DA = (IA + NW - 1) / NW, DB = (IW + NW - 1) / NW;   // uneven shares: wave + d*NW < IA only
    static_assert(NS == 2 || (IA % NW == 0 && IW % NW == 0), "counted vmcnt waits need even DMA shares");
    constexpr int PA = BM * BK, PW = BN * BK;                 // halves per plane image
    constexpr int STAGE = 2 * PA + 2 * PW;                    // halves per stage: A1, A2, W1, W2

    const int tm = wgid / p.n_tiles, tn = wgid - tm * p.n_tiles;
    const int zb = z / p.G, zg = z - zb * p.G;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    const _Float16* Ab = p.Ah + zb * p.sAb + zg * p.sAg;
    const _Float16* Wb = p.Wh + zg * p.sWg;
    const long long a_bytes = ((long long)(p.Tin - 1) * p.ldx + p.Cg) * 2;
    const long long w_bytes = ((long long)(p.N - 1) * p.ldw + p.K) * 2;
    const __amdgpu_buffer_rsrc_t rA1 = hfa::make_rsrc(Ab, a_bytes);
    const __amdgpu_buffer_rsrc_t rA2 = hfa::make_rsrc(Ab + p.sAp, a_bytes);
    const __amdgpu_buffer_rsrc_t rW1 = hfa::make_rsrc(Wb, w_bytes);
    const __amdgpu_buffer_rsrc_t rW2 = hfa::make_rsrc(Wb + p.sWp, w_bytes);

    // DMA d of this wave fills rows (wave + d*NW)*RPP + lane/CPR of each plane, chunk slot lane%CPR (swizzled source)
    auto swz = [](int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; };      // {0, 2, 3, 1}[(r >> 2) & 3]
    int a_t0[DA], a_c[DA], a_tap[DA];
    unsigned voffA[DA], voffW[DB];
#pragma unroll
    for (int d = 0; d < DA; ++d) {
        const int row = (wave + d * NW) * RPP + lane / CPR;
        int m = tm * BM + row;
        m = m < p.M ? m : p.M - 1;
        a_t0[d] = m * p.stride - p.pad;
        a_c[d] = ((lane % CPR) ^ swz(row)) * 8;             // GT: the chunk's channel within its current tap
        a_tap[d] = 0;
    }
#pragma unroll
    for (int d = 0; d < DB; ++d) {
        const int row = (wave + d * NW) * RPP + lane / CPR;
        int n = tn * BN + row;
        n = n < p.N ? n : p.N - 1;
        voffW[d] = (unsigned)((n * p.ldw + ((lane % CPR) ^ swz(row)) * 8) * 2);
    }
    auto set_tap = [&](int j) {
#pragma unroll
        for (int d = 0; d < DA; ++d) {
            const int t = a_t0[d] + j;
            voffA[d] = (t >= 0 && t < p.Tin) ? (unsigned)((t * p.ldx + a_c[d]) * 2) : hfa::DMA_OOB;
        }
    };
    const unsigned lds0 = hfa::lds_addr(smem);
    int cur_j = 0, cur_c0 = 0, cur_k0 = 0;
    if constexpr (!GT) set_tap(0);
    auto issueA = [&](int stage) {
        const unsigned base = lds0 + stage * STAGE * 2 + wave * 1024;
#pragma unroll
        for (int d = 0; d < DA; ++d) {
            if (IA % NW != 0 && wave + d * NW >= IA) continue;   // wave-uniform
            if constexpr (GT) {
                const int t = a_t0[d] + a_tap[d];
                const unsigned vo = (t >= 0 && t < p.Tin) ? (unsigned)((t * p.ldx + a_c[d]) * 2) : hfa::DMA_OOB;
                hfa::dma16(vo, rA1, 0u, base + d * NW * 1024);
                if constexpr (!F16) hfa::dma16(vo, rA2, 0u, base + PA * 2 + d * NW * 1024);
                a_c[d] += BK;
                if (a_c[d] >= p.Cg) {                     // Cg >= BK: at most one tap boundary per K-step
                    a_c[d] -= p.Cg;
                    ++a_tap[d];
                }
            } else {
                hfa::dma16(voffA[d], rA1, (unsigned)cur_c0 * 2, base + d * NW * 1024);
                if constexpr (!F16) hfa::dma16(voffA[d], rA2, (unsigned)cur_c0 * 2, base + PA * 2 + d * NW * 1024);
            }
        }
    };
    auto issueW = [&](int stage) {
        const unsigned base = lds0 + stage * STAGE * 2 + wave * 1024;
#pragma unroll
        for (int d = 0; d < DB; ++d) {
            if (IW % NW != 0 && wave + d * NW >= IW) continue;
            hfa::dma16(voffW[d], rW1, (unsigned)cur_k0 * 2, base + 2 * PA * 2 + d * NW * 1024);
            if constexpr (!F16) hfa::dma16(voffW[d], rW2, (unsigned)cur_k0 * 2, base + (2 * PA + PW) * 2 + d * NW * 1024);
        }
    };
    auto advance = [&]() {
        cur_k0 += BK;
        if constexpr (!GT) {
            cur_c0 += BK;
            if (cur_c0 == p.Cg) {
                cur_c0 = 0;
                set_tap(++cur_j);
            }
        }
    };
    auto issue = [&](int stage) {
        issueA(stage);
        issueW(stage);
        advance();
    };
    constexpr int DN = 2 * (DA + DB);                       // DMA issues per wave per K-step
    // one DMA piece q of this wave's share (q < 2 DA: A plane q & 1 of piece q >> 1; else W), in issue order;
    // advance() after the last
    auto issue_piece = [&](int stage, int q) {
        const unsigned base = lds0 + stage * STAGE * 2 + wave * 1024;
        if (F16 && (q & 1)) {                                     // low planes: not used
            if (GT && q < 2 * DA) {
                const int d = q >> 1;
                a_c[d] += BK;
                if (a_c[d] >= p.Cg) {
                    a_c[d] -= p.Cg;
                    ++a_tap[d];
                }
            }
            return;
        }
        if (q < 2 * DA) {
            const int d = q >> 1, pl = q & 1;
            if (IA % NW != 0 && wave + d * NW >= IA) return;
            if constexpr (GT) {
                const int t = a_t0[d] + a_tap[d];
                const unsigned vo = (t >= 0 && t < p.Tin) ? (unsigned)((t * p.ldx + a_c[d]) * 2) : hfa::DMA_OOB;
                hfa::dma16(vo, pl ? rA2 : rA1, 0u, base + pl * PA * 2 + d * NW * 1024);
                if (pl) {
                    a_c[d] += BK;
                    if (a_c[d] >= p.Cg) {
                        a_c[d] -= p.Cg;
                        ++a_tap[d];
                    }
                }
            } else {
                hfa::dma16(voffA[d], pl ? rA2 : rA1, (unsigned)cur_c0 * 2, base + pl * PA * 2 + d * NW * 1024);
            }
        } else {
            const int d = (q - 2 * DA) >> 1, pl = q & 1;
            if (IW % NW != 0 && wave + d * NW >= IW) return;
            hfa::dma16(voffW[d], pl ? rW2 : rW1, (unsigned)cur_k0 * 2, base + (2 * PA + pl * PW) * 2 + d * NW * 1024);
        }
    };

    const int wm = wave / WN, wn = wave % WN;
    {
        constexpr int NI = BM / WM / 16, NJ = BN / WN / 16;       // 16 x 16 blocks per wave

        const int r16 = lane & 15, c = lane >> 4;
        const int rdA = (wm * (BM / WM) + r16) * CPR + (c ^ swz(r16));
        const int rdB = 2 * PA / 8 + (wn * (BN / WN) + r16) * CPR + (c ^ swz(r16));
        f32x4 acc[NI][NJ];
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        const int nk = p.K / BK;
#pragma unroll
        for (int s = 0; s < NS - 1; ++s)
            if (s < nk) issue(s);
        if (nk >= NS - 1) hfa::wait_vm_barrier<(NS - 2) * DN>();
        else hfa::wait_vm_barrier<0>();
        const f16x8* s8 = reinterpret_cast<const f16x8*>(smem);
        int stage = 0;
        for (int kt = 0; kt < nk; ++kt) {
            const bool more = kt + NS - 1 < nk;
            const int nstage = stage == 0 ? NS - 1 : stage - 1;

            const f16x8* st = s8 + stage * (STAGE / 8);
            f16x8 w1[NJ], w2[NJ], w1s[NJ];
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                w1[j] = st[rdB + j * 16 * CPR];
                if constexpr (!F16) {
                    w2[j] = st[rdB + PW / 8 + j * 16 * CPR];
                    w1s[j] = w1[j] * (_Float16)2048.0f;
                }
            }
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                if (more) {                  // the next stage's DMA, two pieces per A block from the first
#pragma unroll
                    for (int q = 0; q < DN; ++q)
                        if ((q / 2 < NI ? q / 2 : NI - 1) == i) issue_piece(nstage, q);
                }
                const f16x8 a1 = st[rdA + i * 16 * CPR];
                if constexpr (F16) {
#pragma unroll
                    for (int j = 0; j < NJ; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, w1[j], acc[i][j], 0, 0, 0);
                } else {
                    const f16x8 a2 = st[rdA + PA / 8 + i * 16 * CPR];
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, w1s[j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, w2[j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2, w1[j], acc[i][j], 0, 0, 0);
                    }
                }
            }
            if (more) advance();
            if (kt + 1 < nk) {
                if (more) hfa::wait_vm_barrier<(NS - 2) * DN>();
                else hfa::wait_vm_barrier<0>();
            }
            stage = stage + 1 == NS ? 0 : stage + 1;
        }
        // the single accumulator's 2^-11 goes into the epilogue's bias fma (exact scaling: the same bits as a
        // separate multiply, one VALU op per output fewer)
        constexpr float kScale = F16 ? 1.0f : 1.0f / 2048.0f;
        constexpr int TI = BM / WM / 32, TJ = BN / WN / 32;
        constexpr bool PAIRS = OUT_SPLIT && TJ % 2 == 0;   // 128-B row segments (store_split_lds2)
        constexpr int SLAB = PAIRS ? 32 * kSlab2 : 32 * 36;
        static_assert(NW * SLAB * 4 <= NS * STAGE * 2, "epilogue slabs exceed the staging LDS");
        __syncthreads();
        float* slab = reinterpret_cast<float*>(smem) + wave * SLAB;
        if constexpr (PAIRS)
            store_split_lds2<16, TI, TJ>(p, acc, EPI, zb, zg, tm * BM + wm * (BM / WM), tn * BN + wn * (BN / WN),
                                         lane, slab, kScale);
        else if constexpr (OUT_SPLIT)
            store_split_lds<16, TI, TJ>(p, acc, EPI, zb, zg, tm * BM + wm * (BM / WM), tn * BN + wn * (BN / WN), lane,
                                        slab, kScale);
        else
            store_f32_lds<16, EPI, TI, TJ>(p, acc, zb, zg, tm * BM + wm * (BM / WM), tn * BN + wn * (BN / WN), lane,
                                           slab, true, kScale);
    }
}

template <int EPI, int BM, int BN, int WM, int WN, int NS, int OCC, bool OUT_SPLIT, bool GT, bool ONE, int BK,
          int MF = 32, bool F16 = false>
__global__ __launch_bounds__(64 * WM * WN, OCC) void gemm_split_kernel(const GemmP p) {
    __shared__ __attribute__((aligned(16))) _Float16 smem[NS * (2 * BM * BK + 2 * BN * BK)];
    // XCD-aware bijective remap: consecutive tile ids (the column tiles of one row panel) share an XCD's L2
    const int nwg = gridDim.x, orig = blockIdx.x;
    const int xcd = orig & 7, q = nwg >> 3, r8 = nwg & 7;
    const int wgid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (orig >> 3);
    gemm_split_tile<EPI, BM, BN, WM, WN, NS, OCC, OUT_SPLIT, GT, ONE, BK, MF, F16>(p, wgid, blockIdx.z, smem);
}

// f32 -> (hi, lo * 2^11) f16 planes, row-wise with 4-element vectors where aligned; raises *oflow for |x| >= 65504
// or a non-finite x.  Rows blockIdx.y, + gridDim.y, ... (a capped grid, hfa::grid_cap).
__global__ __launch_bounds__(256) void split_f16_kernel(int rows, int cols, const float* __restrict__ x, long long ldx,
                                                        _Float16* __restrict__ y, long long ldy, long long sp,
                                                        int* __restrict__ oflow) {
    const int c4 = (blockIdx.x * 256 + threadIdx.x) * 4;
    if (c4 >= cols) return;
    const bool vec = c4 + 3 < cols && ((ldx | ldy | sp) & 3) == 0 && (((uintptr_t)x | (uintptr_t)y) & 15) == 0;
    bool bad = false;
    for (int r = blockIdx.y; r < rows; r += gridDim.y) {
        const float* src = x + (long long)r * ldx + c4;
        _Float16* dst = y + (long long)r * ldy + c4;
        if (vec) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(src);
            f16x4 v1, v2;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                bad |= !(__builtin_fabsf(v[t]) < 65504.0f);
                v1[t] = (_Float16)v[t];
                v2[t] = (_Float16)((v[t] - (float)v1[t]) * 2048.0f);
            }
            *reinterpret_cast<f16x4*>(dst) = v1;
            *reinterpret_cast<f16x4*>(dst + sp) = v2;
        } else {
            for (int t = 0; t < 4 && c4 + t < cols; ++t) {
                const float v = src[t];
                bad |= !(__builtin_fabsf(v) < 65504.0f);
                const _Float16 v1 = (_Float16)v;
                dst[t] = v1;
                dst[t + sp] = (_Float16)((v - (float)v1) * 2048.0f);
            }
        }
    }
    if (bad && oflow) *oflow = 1;
}

// Tile configurations (BM x BN, WM x WN waves); scripts/gemm_bench.py measures each on the workload's shapes.
enum { CFG_AUTO = 0, CFG_128x128 = 1, CFG_128x64 = 2, CFG_256x128 = 3, CFG_128x256 = 4, CFG_256x128_W4 = 5,
       CFG_128x256_W4 = 6, CFG_256x256 = 7, CFG_128x48 = 8, CFG_128x96 = 9, CFG_COUNT = 10 };
// Pipelines: register-staged BK 16 / 32, LDS-DMA with 2 or 3 stages.
enum { PIPE_AUTO = 0, PIPE_REG16 = 16, PIPE_REG32 = 32, PIPE_DMA2 = 102, PIPE_DMA3 = 103 };
thread_local int g_force_pipe = 0, g_force_cfg = 0;   // tuning overrides (hfa_gemm_tuning), 0 = automatic

// workgroups per CU a DMA instantiation is register-capped for: 128x128 3-stage (48 KiB LDS) -> 3, 2-stage and
// 128x64 -> 4 (a 5th 2-stage workgroup measured no faster), 8-wave 128x256 -> 2 (64 accumulators per lane)
// (4-wave 256x128 / 128x256 tiles, 64x128 per wave at 3 workgroups/CU, measured no faster on any workload shape
// and 20-25 % slower on the 768-wide Linear ones)
constexpr int dma_occ(int BN, int NW, int NS) {
    return NW == 4 ? (NS == 3 && BN == 128 ? 3 : 4) : 2;
}

struct Plan {
    int pipe, cfg;
    bool vec_a, vec_c;   // 16-B aligned A rows (DMA-able) / C and R rows (dwordx4 epilogue)
};

inline bool al16(const void* ptr) { return ((uintptr_t)ptr & 15) == 0; }

// LDS-DMA eligibility: 16-B aligned A rows, and both buffer spans addressable by a 31-bit byte offset.
inline bool dma_ok(const GemmP& p, bool vec_a) {
    const long long a_span = ((long long)(p.Tin - 1) * p.ldx + p.Cg) * 4;
    const long long w_span = ((long long)(p.N - 1) * p.ldw + p.K) * 4;
    return vec_a && p.Tin >= 1 && a_span < 0x7fffffffLL && w_span < 0x7fffffffLL;
}

inline Plan make_plan(const GemmP& p, int Z, bool vec_a) {
    // measured (scripts/gemm_bench.py, scripts/gpu_gemm_abl.sh): the LDS-DMA pipeline beats register staging by
    // 8-12 % on every workload shape; 2 stages at 4 workgroups/CU beat 3 stages at 3 for the 128x128 tile; the
    // 64-wide N tile (3 stages) wins for N <= 64 (grouped positional conv: 2x the 128-wide tile) and for grids
    // too small to fill 256 CUs twice (UNet: +33 %); the 8-wave 128x256 tile no longer wins anywhere.
    Plan pl;
    pl.vec_a = vec_a;
    pl.vec_c = al16(p.C) && p.ldc % 4 == 0 && p.sCb % 4 == 0 && p.sCg % 4 == 0 &&
               (!p.R || (al16(p.R) && p.ldr % 4 == 0 && p.sRb % 4 == 0 && p.sRg % 4 == 0));
    const long long blocks128 = (long long)((p.M + 127) / 128) * ((p.N + 127) / 128) * Z;
    pl.cfg = (p.N <= 64 || blocks128 < 512) ? CFG_128x64 : CFG_128x128;
    if (p.N > 32 && p.N <= 48 && dma_ok(p, vec_a)) pl.cfg = CFG_128x48;
    if (g_force_cfg > 0 && g_force_cfg < CFG_COUNT) pl.cfg = g_force_cfg;
    if (pl.cfg == CFG_128x48 && (p.N > 48 || !dma_ok(p, vec_a))) pl.cfg = CFG_128x64;
    const bool dma_cfg = pl.cfg == CFG_128x128 || pl.cfg == CFG_128x64 || pl.cfg == CFG_128x256 ||
                         pl.cfg == CFG_128x48 || pl.cfg == CFG_128x96;
    pl.pipe = PIPE_REG16;
    if (dma_cfg && dma_ok(p, vec_a)) pl.pipe = (pl.cfg == CFG_128x64 || pl.cfg == CFG_128x48) ? PIPE_DMA3 : PIPE_DMA2;
    if (pl.cfg == CFG_128x48) return pl;        // DMA-only tiles
    if (pl.cfg == CFG_128x96) {
        if (pl.pipe != PIPE_REG16) {
            pl.pipe = PIPE_DMA2;
            return pl;
        }
        pl.cfg = CFG_128x128;
    }
    if (g_force_pipe == PIPE_REG16) pl.pipe = PIPE_REG16;
    if (g_force_pipe == PIPE_REG32 && p.K % 32 == 0 && p.Cg % 32 == 0) pl.pipe = PIPE_REG32;
    if ((g_force_pipe == PIPE_DMA2 || g_force_pipe == PIPE_DMA3) && dma_cfg && dma_ok(p, vec_a))
        pl.pipe = g_force_pipe;
    return pl;
}

inline void cfg_shape(int cfg, int& BM, int& BN, int& WM, int& WN) {
    switch (cfg) {
        case CFG_128x64: BM = 128; BN = 64; WM = 2; WN = 2; break;
        case CFG_256x128: BM = 256; BN = 128; WM = 4; WN = 2; break;
        case CFG_128x256: BM = 128; BN = 256; WM = 2; WN = 4; break;
        case CFG_256x128_W4: BM = 256; BN = 128; WM = 2; WN = 2; break;
        case CFG_128x256_W4: BM = 128; BN = 256; WM = 2; WN = 2; break;
        case CFG_256x256: BM = 256; BN = 256; WM = 4; WN = 2; break;
        case CFG_128x48: BM = 128; BN = 48; WM = 4; WN = 1; break;
        case CFG_128x96: BM = 128; BN = 96; WM = 4; WN = 1; break;
        default: BM = 128; BN = 128; WM = 2; WN = 2; break;
    }
}

// rocprof symbol stem of the instantiation a plan launches (bench.py's probe keys on it)
inline void plan_name(const Plan& pl, int epi, char* buf, int len) {
    int BM, BN, WM, WN;
    cfg_shape(pl.cfg, BM, BN, WM, WN);
    if (pl.cfg == CFG_128x48) {
        snprintf(buf, len, "gemm_dma_n48_kernel<%d, %d>", epi, pl.pipe - 100);
    } else if (pl.pipe == PIPE_DMA2 || pl.pipe == PIPE_DMA3) {
        const int ns = pl.pipe - 100, occ = dma_occ(BN, WM * WN, ns);
        snprintf(buf, len, "gemm_dma_kernel<%d, %d, %d, %d, %d, %d, %d, %s>", epi, BM, BN, WM, WN, ns, occ,
                 pl.vec_c ? "true" : "false");
    } else {
        snprintf(buf, len, "gemm_f32_kernel<%d, %s, %d, %d, %d, %d, %d>", epi, pl.vec_a ? "true" : "false",
                 pl.pipe == PIPE_REG32 ? 32 : 16, BM, BN, WM, WN);
    }
}

inline int set_grid(GemmP& p, int BM, int BN, dim3& grid, int Z) {
    p.m_tiles = (p.M + BM - 1) / BM;
    p.n_tiles = (p.N + BN - 1) / BN;
    const long long tiles = (long long)p.m_tiles * p.n_tiles;
    if (tiles > 0x7fffffffLL) {
        hfa::set_error("hfa_conv_gemm_f32: grid too large");
        return HFA_EINVAL;
    }
    grid = dim3((unsigned)tiles, 1, Z);
    return HFA_OK;
}

// ---- split-f16 GEMM for N = 48 (the grouped positional conv at Hubert-base: 16 groups of Cg = 48) ---------------
// 48 output columns fit neither the 32x32 MFMA tiles (a 64-wide tile wastes a quarter of its products) nor
// any 32-multiple, so this kernel uses v_mfma_f32_16x16x32_f16: 48 = 3 x 16.  Tile 128 x 48, 4 waves of 32 x 48
// (2 x 3 blocks of 16 x 16), the same split-f16 single-accumulator arithmetic, operand planes staged by LDS-DMA
// into [row][4 x 16 B] images whose chunk swizzle {0, 2, 3, 1}[(row >> 2) & 3] keeps the 16x16x32 operand reads (lane:
// row lane&15, chunk lane>>4) conflict-free; per-lane tap tracking as GT (Cg % 32 != 0).
template <int EPI>
__global__ __launch_bounds__(256, 2) void gemm_split48_kernel(const GemmP p) {
    constexpr int BM = 128, BN = 48, BK = 32, NW = 4, NS = 2, DA = 2;
    constexpr int PA = BM * BK, PW = BN * BK;                  // halves per plane image
    constexpr int STAGE = 2 * PA + 2 * PW;
    __shared__ __attribute__((aligned(16))) _Float16 smem[NS * STAGE];

    const int nwg = gridDim.x, orig = blockIdx.x;
    const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int tm = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
    const int zb = blockIdx.z / p.G, zg = blockIdx.z - zb * p.G;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    auto swz = [](int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; };   // {0, 2, 3, 1}[(r >> 2) & 3]

    const _Float16* Ab = p.Ah + zb * p.sAb + zg * p.sAg;
    const _Float16* Wb = p.Wh + zg * p.sWg;
    const long long a_bytes = ((long long)(p.Tin - 1) * p.ldx + p.Cg) * 2;
    const long long w_bytes = ((long long)(BN - 1) * p.ldw + p.K) * 2;
    const __amdgpu_buffer_rsrc_t rA1 = hfa::make_rsrc(Ab, a_bytes), rA2 = hfa::make_rsrc(Ab + p.sAp, a_bytes);
    const __amdgpu_buffer_rsrc_t rW1 = hfa::make_rsrc(Wb, w_bytes), rW2 = hfa::make_rsrc(Wb + p.sWp, w_bytes);

    // A: pieces wave + 4d (16 rows x 4 chunks each), per-lane (tap, channel) tracking; W: piece = wave (< 3)
    int a_t0[DA], a_c[DA], a_tap[DA];
#pragma unroll
    for (int d = 0; d < DA; ++d) {
        const int row = (wave + d * NW) * 16 + (lane >> 2);
        int m = tm * BM + row;
        m = m < p.M ? m : p.M - 1;
        a_t0[d] = m * p.stride - p.pad;
        a_c[d] = ((lane & 3) ^ swz(row)) * 8;
        a_tap[d] = 0;
    }
    const int wrow = wave * 16 + (lane >> 2);
    const unsigned voffW = (unsigned)(((wrow < BN ? wrow : BN - 1) * p.ldw + ((lane & 3) ^ swz(wrow)) * 8) * 2);
    const unsigned lds0 = hfa::lds_addr(smem);
    int cur_k0 = 0;
    auto issue = [&](int stage) {
        const unsigned base = lds0 + stage * STAGE * 2 + wave * 1024;
#pragma unroll
        for (int d = 0; d < DA; ++d) {
            const int t = a_t0[d] + a_tap[d];
            const unsigned vo = (t >= 0 && t < p.Tin) ? (unsigned)((t * p.ldx + a_c[d]) * 2) : hfa::DMA_OOB;
            hfa::dma16(vo, rA1, 0u, base + d * NW * 1024);
            hfa::dma16(vo, rA2, 0u, base + PA * 2 + d * NW * 1024);
            a_c[d] += BK;
            if (a_c[d] >= p.Cg) {                         // Cg >= BK: at most one tap boundary per K-step
                a_c[d] -= p.Cg;
                ++a_tap[d];
            }
        }
        if (wave < BN / 16) {
            hfa::dma16(voffW, rW1, (unsigned)cur_k0 * 2, base + 2 * PA * 2);
            hfa::dma16(voffW, rW2, (unsigned)cur_k0 * 2, base + (2 * PA + PW) * 2);
        }
        cur_k0 += BK;
    };

    // operand reads (f16x8 units): lane row r16, chunk q = lane >> 4 (k 8q .. 8q + 7 of the 32-deep step)
    const int r16 = lane & 15, q = lane >> 4;
    const int sl = q ^ swz(r16);
    const int rdA = (wave * 32 + r16) * 4 + sl;              // + rb * 64 per 16-row block
    const int rdW = 2 * PA / 8 + r16 * 4 + sl;              // + cb * 64 per 16-column block
    f32x4 acc[2][3];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = p.K / BK;
    issue(0);
    hfa::wait_vm_barrier<0>();
    const f16x8* s8 = reinterpret_cast<const f16x8*>(smem);
    int stage = 0;
    for (int kt = 0; kt < nk; ++kt) {
        const bool more = kt + 1 < nk;
        if (more) issue(stage ^ 1);
        const f16x8* st = s8 + stage * (STAGE / 8);
        f16x8 a1[2], a2[2], w1[3], w2[3], w1s[3];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            a1[i] = st[rdA + i * 64];
            a2[i] = st[rdA + i * 64 + PA / 8];
        }
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            w1[j] = st[rdW + j * 64];
            w2[j] = st[rdW + j * 64 + PW / 8];
            w1s[j] = w1[j] * (_Float16)2048.0f;
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[i], w1s[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[i], w2[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2[i], w1[j], acc[i][j], 0, 0, 0);
            }
        if (more) hfa::wait_vm_barrier<0>();
        stage ^= 1;
    }

    // epilogue: C/D of the 16x16 MFMA: column lane & 15, rows 4 (lane >> 4) + e
    float* Cb = p.C + zb * p.sCb + zg * p.sCg;
    const float* Rb = p.R ? p.R + zb * p.sRb + zg * p.sRg : nullptr;
    const float* biasb = p.bias ? p.bias + zg * p.sBg : nullptr;
    bool bad = false;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int col = j * 16 + r16;
        const float bv = biasb ? biasb[col] : 0.0f;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int row = tm * BM + wave * 32 + i * 16 + 4 * q + e;
                const float a = acc[i][j][e] * (1.0f / 2048.0f);
                bad |= !__builtin_isfinite(a);
                if (row < p.M) {
                    float v = a + bv;
                    if (EPI == EPI_GELU) v = hfa::gelu_fast(v);
                    if (Rb) v += Rb[(long long)row * p.ldr + col];
                    Cb[(long long)row * p.ldc + col] = v;
                }
            }
    }
    if (bad && p.oflow) *p.oflow = 1;
}

// ---- grouped positional conv with an LDS-resident input window ------------------------------------------------
// The implicit GEMM re-fetches the A rows of every tap from L2 (128 taps x 48 channels: ~56 B of DMA per kFLOP for
// the N = 48 tile), so for the positional conv (stride 1, k = 128, Cg = 48, N = Cg) a workgroup instead stages its
// whole input window once -- the 256 + k - 1 input rows its 256 output rows read, both planes, zero rows outside
// [0, Tin) (the conv's padding) -- and streams only W through a 3-stage ring (6 KiB per 32-deep K-step): ~8 B of
// DMA per kFLOP.  The window is chunk-major ([plane][8-channel chunk][row], 16 B per cell), so a 16x16x32 operand
// read (16 consecutive rows of one chunk per 16 lanes) covers all 64 banks once; the K index is the flattened
// (tap, channel) of the im2col weight rows, each lane's 8-wide chunk mapping to its own (tap, chunk) pair.
// 8 waves x (16 RB rows x 16 NB columns) on v_mfma_f32_16x16x32_f16, split-f16 single-accumulator arithmetic.
// RB (row blocks of 16 per wave): 2 -> 256-row tiles; 4 -> 512-row tiles (Cg = 48, round 4): a wave then reads 8 A
// and 6 W operands per 36 MFMAs instead of 4 and 6 per 18 -- the LDS operand reads, not the MFMAs, bounded the
// 256-row form (~140 B of LDS reads per cycle per CU wanted against 128) -- and one tile covers a 10 s utterance's
// 499 frames (one window load per (batch, group) instead of two overlapping ones).
constexpr int win_rows(int RB) { return RB == 4 ? 640 : 384; }  // 128 RB + k - 1 (k <= 128), 64-row pieces

template <int EPI, int NB, int RB = 2>
__global__ __launch_bounds__(512, 1) void posconv_split_kernel(const GemmP p) {
    constexpr int BM = 128 * RB, BN = 16 * NB, BK = 32, NW = 8, NS = 3;   // NB = 3 (Cg 48) or 4 (Cg 64)
    constexpr int kWinRows = win_rows(RB);
    constexpr int PW = BN * BK;                                  // halves per W plane image
    constexpr int WSTAGE = 2 * PW;
    const int CC = p.Cg / 8;                                     // 8-channel chunks per row (<= 2 NB)
    __shared__ __attribute__((aligned(16))) _Float16 dsm[2 * 2 * NB * kWinRows * 8 + NS * WSTAGE];
    _Float16* win = dsm;                                         // [2][CC][kWinRows] x 8 halves
    _Float16* wst = dsm + 2 * 2 * NB * kWinRows * 8;             // NS stages of [2][BN][32]

    const int nwg = gridDim.x, orig = blockIdx.x;
    const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int tm = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
    const int zb = blockIdx.z / p.G, zg = blockIdx.z - zb * p.G;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    auto swz = [](int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; };   // {0, 2, 3, 1}[(r >> 2) & 3]

    const _Float16* Ab = p.Ah + zb * p.sAb + zg * p.sAg;
    const _Float16* Wb = p.Wh + zg * p.sWg;
    const long long a_bytes = ((long long)(p.Tin - 1) * p.ldx + p.Cg) * 2;
    const long long w_bytes = ((long long)(BN - 1) * p.ldw + p.K) * 2;
    const __amdgpu_buffer_rsrc_t rA1 = hfa::make_rsrc(Ab, a_bytes), rA2 = hfa::make_rsrc(Ab + p.sAp, a_bytes);
    const __amdgpu_buffer_rsrc_t rW1 = hfa::make_rsrc(Wb, w_bytes), rW2 = hfa::make_rsrc(Wb + p.sWp, w_bytes);
    const unsigned lds_win = hfa::lds_addr(win), lds_w = hfa::lds_addr(wst);

    // input window: pieces of 64 rows of one (plane, chunk); window row r <-> input row t0 + r
    const int t0 = tm * BM - p.pad;
    constexpr int GP = kWinRows / 64;                            // 64-row pieces per (plane, chunk)
    const int npieces = 2 * CC * GP;
    for (int pc = wave; pc < npieces; pc += NW) {
        const int plane = pc / (CC * GP), rest = pc - plane * CC * GP, c = rest / GP, g = rest - c * GP;
        const int t = t0 + g * 64 + lane;
        const unsigned vo = (t >= 0 && t < p.Tin) ? (unsigned)((t * p.ldx + c * 8) * 2) : hfa::DMA_OOB;
        hfa::dma16(vo, plane ? rA2 : rA1, 0u, lds_win + ((plane * CC + c) * kWinRows + g * 64) * 16);
    }
    // W ring: waves 0 .. 2 NB - 1 each own one 1-KiB piece (plane w / NB, rows 16 (w % NB) + lane / 4) of a K-step
    const int wrow = (wave % NB) * 16 + (lane >> 2);
    const unsigned voffW = (unsigned)((wrow * p.ldw + ((lane & 3) ^ swz(wrow)) * 8) * 2);
    const bool wdma = wave < 2 * NB;
    auto issueW = [&](int stage, int s) {
        if (wdma)
            hfa::dma16(voffW, wave < NB ? rW1 : rW2, (unsigned)(s * BK * 2),
                       lds_w + (stage * WSTAGE + (wave < NB ? 0 : PW)) * 2 + (wave % NB) * 1024);
    };
    const int nk = p.K / BK;
    issueW(0, 0);
    if (nk > 1) issueW(1, 1);
    hfa::wait_vm_barrier<0>();                                   // window and steps 0, 1 landed

    // per-lane operand addressing: output row l = 16 RB wave + 16 b + r16, chunk q = lane >> 4 (k 8q..8q+7 of a step)
    const int r16 = lane & 15, q = lane >> 4;
    int tap = 0, ch = q;                                         // (tap, 8-channel chunk) of this lane's k
    while (ch >= CC) { ch -= CC; ++tap; }
    const f16x8* w8 = reinterpret_cast<const f16x8*>(wst);
    const f16x8* a8 = reinterpret_cast<const f16x8*>(win);
    const int rdW = (r16 * 4) + (q ^ swz(r16));                  // + cb * 64, + plane * PW / 8, + stage * WSTAGE / 8
    const int lrow = 16 * RB * wave + r16;
    f32x4 acc[RB][NB];
#pragma unroll
    for (int i = 0; i < RB; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    int stage = 0;
    for (int s = 0; s < nk; ++s) {
        if (s + 2 < nk) issueW(stage == 0 ? 2 : stage - 1, s + 2);    // into the stage read at step s - 1
        const f16x8* st = w8 + stage * (WSTAGE / 8);
        f16x8 a1[RB], a2[RB], w1[NB], w2[NB], w1s[NB];
#pragma unroll
        for (int b = 0; b < RB; ++b) {
            const int cell = ch * kWinRows + lrow + 16 * b + tap;
            a1[b] = a8[cell];
            a2[b] = a8[CC * kWinRows + cell];
        }
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            w1[j] = st[rdW + j * 64];
            w2[j] = st[rdW + j * 64 + PW / 8];
            w1s[j] = w1[j] * (_Float16)2048.0f;
        }
#pragma unroll
        for (int i = 0; i < RB; ++i)
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[i], w1s[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[i], w2[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2[i], w1[j], acc[i][j], 0, 0, 0);
            }
        ch += 4;                                                 // next step: k + 32 = 4 chunks on
        if (ch >= CC) { ch -= CC; ++tap; }
        if (s + 1 < nk) {                                        // step s + 1 landed; every wave done with s - 1
            if (s + 2 < nk) hfa::wait_vm_barrier<1>();
            else hfa::wait_vm_barrier<0>();
        }
        stage = stage == NS - 1 ? 0 : stage + 1;
    }

    float* Cb = p.C + zb * p.sCb + zg * p.sCg;
    const float* Rb = p.R ? p.R + zb * p.sRb + zg * p.sRg : nullptr;
    const float* biasb = p.bias ? p.bias + zg * p.sBg : nullptr;
    bool bad = false;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        const int col = j * 16 + r16;
        const float bv = biasb ? biasb[col] : 0.0f;
#pragma unroll
        for (int i = 0; i < RB; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int row = tm * BM + 16 * RB * wave + i * 16 + 4 * q + e;
                const float a = acc[i][j][e] * (1.0f / 2048.0f);
                bad |= !__builtin_isfinite(a);
                if (row < p.M) {
                    float v = a + bv;
                    if (EPI == EPI_GELU) v = hfa::gelu_fast(v);
                    if (Rb) v += Rb[(long long)row * p.ldr + col];
                    Cb[(long long)row * p.ldc + col] = v;
                }
            }
    }
    if (bad && p.oflow) *p.oflow = 1;
}

// ---- split-f16 dispatch --------------------------------------------------------------------------------------
// Tile ids (hfa_gemm_split_tuning): only the tiles the automatic choice can return are built.  The ids are the ones
// earlier rounds' measurements name (profiles/r0*/): 1-14, 21, 22 and 26 were tuning-only tiles (the 32x32x16
// two-accumulator forms, 16-deep K-steps, 3/4-stage rings, 192 x 128) and are retired (git history keeps them).
enum { SCFG_AUTO = 0, SCFG_N48 = 15, SCFG_WIN = 16, SCFG_256x256_M16 = 17, SCFG_128x128_M16 = 18,
       SCFG_128x64_M16 = 19, SCFG_256x64_M16 = 20, SCFG_256x192_M16 = 23, SCFG_192x256_M16 = 24,
       SCFG_128x192_M16 = 25 };
struct SplitGeom { int BM, BN, WM, WN, NS, OCC; };
inline bool split_cfg_valid(int cfg) {
    return cfg == SCFG_AUTO || (cfg >= SCFG_N48 && cfg <= SCFG_256x64_M16) || (cfg >= SCFG_256x192_M16 &&
                                                                                  cfg <= SCFG_128x192_M16);
}
// every gemm_split_kernel tile: single accumulator, v_mfma_f32_16x16x32_f16, 32-deep K-steps
constexpr SplitGeom split_geom(int cfg) {
    switch (cfg) {
        case SCFG_N48: return {128, 48, 4, 1, 2, 2};    // gemm_split48_kernel (16x16x32 MFMA), not gemm_split_kernel
        case SCFG_WIN: return {256, 48, 8, 1, 3, 1};    // posconv_split_kernel (LDS-resident input window)
        case SCFG_256x256_M16: return {256, 256, 2, 4, 2, 1};
        case SCFG_128x64_M16: return {128, 64, 2, 2, 2, 2};
        case SCFG_256x64_M16: return {256, 64, 4, 1, 2, 2};
        case SCFG_256x192_M16: return {256, 192, 4, 2, 2, 1};
        case SCFG_192x256_M16: return {192, 256, 2, 4, 2, 1};
        // two workgroups per CU (2 x 80 KiB of LDS): 500 tiles fill the 512 slots of an N = 768 grid at B*L = 15968
        // rows in one balanced round (the 256 x 256 tile: 189 tiles on 256 CUs)
        case SCFG_128x192_M16: return {128, 192, 2, 2, 2, 2};
        default: return {128, 128, 2, 2, 2, 2};         // SCFG_128x128_M16
    }
}
thread_local int g_split_cfg = 0;   // tuning override (hfa_gemm_split_tuning)
thread_local int g_win_nb = 3;   // column blocks of the window kernel the name query reports (N / 16)
thread_local int g_win_rb = 2;   // and its row blocks per wave

// Measured on the workload's shapes (scripts/split_gemm_bench.py, profiles/r01/split_gemm_cfgs.txt): the 256 x 256
// single-accumulator tile is 7-15 % faster than 128 x 128 on the extractor convs, FFN and out-projection (even at
// 189 tiles for N = 768) and within 3 % on the QKV projection; small grids keep the narrower tiles.  Every
// tile is a single-accumulator tile: each output element then sees the same MFMA sequence (same k-blocks, same three
// products in the same order) whatever the tile, so a row's result does not depend on the batch it is in
// (variable-length batches stay bit-identical to the reference's B = 1 runs).  Since round 2 every tile is a
// 16x16x32 (MF 16) tile (4-9 % over the 32x32x16 form, profiles/r02/split_mf16.txt).
inline bool win_ok(const GemmP& p) {   // posconv_split_kernel: stride 1, N 48 or 64, Cg % 8, Cg <= 64, window fits
    return (p.N == 48 || p.N == 64) && p.Ch == nullptr && p.stride == 1 && p.Cg % 8 == 0 && p.Cg >= 32 &&
           p.Cg <= 2 * (p.N / 16) * 8 && p.K % p.Cg == 0 && 256 + p.K / p.Cg - 1 <= win_rows(2);
}
// 512-row tiles (RB 4) for N = 48 when the rows fill more than one 256-row tile and the 640-row window holds the taps
inline bool win_rb4(const GemmP& p) { return p.N == 48 && p.M > 256 && 512 + p.K / p.Cg - 1 <= win_rows(4); }

inline int split_cfg(const GemmP& p, int Z) {
    const bool n48 = p.N == 48 && p.Ch == nullptr && p.Cg % 8 == 0 && p.Cg >= 32;
    if (g_split_cfg != SCFG_AUTO) {
        if (g_split_cfg == SCFG_N48 && !n48) return SCFG_128x64_M16;
        if (g_split_cfg == SCFG_WIN && !win_ok(p)) return SCFG_128x64_M16;
        return g_split_cfg;
    }
    if (win_ok(p)) return SCFG_WIN;
    if (n48) return SCFG_N48;
    // the rules below were measured on a whole MI355X (256 CUs); a partitioned device scales them with its CU count
    const long long cus = hfa::device_cus();
    const long long blocks128 = (long long)((p.M + 127) / 128) * ((p.N + 127) / 128) * Z;
    const long long blocks256 = (long long)((p.M + 255) / 256) * ((p.N + 255) / 256) * Z;
    if (p.N == 64 && p.Cg % 32 == 0 && (long long)((p.M + 255) / 256) * Z >= cus)
        return SCFG_256x64_M16;            // grouped positional conv at Cg = 64 (Hubert-large): 1.26x the 128x64 tile
    if (p.N <= 64 || blocks128 < cus) return SCFG_128x64_M16;
    // (a half-filled single round of big tiles loses to 128 x 128: extractor conv6, 128 big tiles, 227 vs 288 TF/s;
    // at 189 big tiles -- the N = 768 projections -- 256 x 256 still wins, 300 vs 275, profiles/r03/conv6_tiles.txt)
    if (2 * blocks256 <= cus || p.N < 512) {
        // narrow N that 128-wide column tiles would pad (profiles/r05/side_tiles.txt): N = 192 at K <= 1152 (the
        // UNet's 192-channel convs and linears) on exact 64-wide tiles, 5-20 % faster; 128 < N < 192 (the
        // 44.1 k -> 16 k resampler, N = 160) on one 192-wide column tile, 14 % faster.  Only the measured widths:
        // other N % 128 != 0 shapes (320, 448, ...) keep 128 x 128 until measured.
        if (p.N == 192 && p.K <= 1152) return SCFG_128x64_M16;
        if (p.N > 128 && p.N < 192) return SCFG_128x192_M16;
        return SCFG_128x128_M16;
    }
    // Large grids: the 256 x 256 tile unless a 192-wide tile fills the last round of CUs much better.  Score =
    // fill of the rounds (tiles / (rounds x 256 CUs)) x the tile's per-FLOP speed (192-wide tiles 0.92 of 256 x 256),
    // ties to 256 x 256.  Measured (scripts/split_gemm_bench.py, profiles/r03/split_tiles_c5.txt): QKV at M = 15 968
    // (567 big tiles = 2.2 rounds) 192 x 256 347 / 256 x 192 339 / 256 x 256 300 / 128 x 128 297 TF/s; at
    // M = 17 924 (config 5 windows: 639 tiles = 2.5 rounds) 256 x 256 340 / 128 x 128 318; FFN1 at M = 17 924 (852
    // tiles = 3.3 rounds) 256 x 256 308 / 192 x 256 304 / 128 x 128 276 — a thin last round costs less than its
    // share (fewer busy CUs hold a higher clock), so the 128 x 128 tile is never the better large-grid choice.
    auto fill = [cus](long long b) { return (double)b / (double)(((b + cus - 1) / cus) * cus); };
    const long long blocks192n = (long long)((p.M + 255) / 256) * ((p.N + 191) / 192) * Z;   // 256 x 192
    const long long blocks192m = (long long)((p.M + 191) / 192) * ((p.N + 255) / 256) * Z;   // 192 x 256
    // One-round grids: the 192 x 256 tile when it still makes one round and busies more CUs -- the N = 768 family
    // at B*L = 15968 rows, 252 instead of 189 tiles on 256 CUs: FFN2 228 -> 208 us, the out-projection 77 -> 69 us,
    // measured as hubert.py launches them (profiles/r04/layer_tiles.txt; round 2's per-utterance Z-batched
    // microbenchmark had not shown it).
    double best = fill(blocks256);
    int cfg = SCFG_256x256_M16;
    if (blocks256 <= cus) {
        // Short K (the out-projection and the feature projection, K <= 1024): two 128 x 192 workgroups per CU when
        // they still make one round of the 512 slots, so one tile's epilogue runs beside the other's main loop
        // (out-projection 70-72 -> 69-70 us, three interleaved pairs, profiles/r04/attn_persistent_ab.txt; FFN2's
        // K = 3072 stays on 192 x 256: 208 vs 219 us, profiles/r04/layer_tiles.txt)
        const long long blocks128x192 = (long long)((p.M + 127) / 128) * ((p.N + 191) / 192) * Z;
        if (p.K <= 1024 && blocks128x192 <= 2 * cus && blocks128x192 > 2 * blocks256) return SCFG_128x192_M16;
        return (blocks192m <= cus && blocks192m > blocks256) ? SCFG_192x256_M16 : cfg;
    }
    if (0.92 * fill(blocks192m) > best + 0.05) {
        best = 0.92 * fill(blocks192m);
        cfg = SCFG_192x256_M16;
    }
    if (p.N % 192 == 0 && 0.92 * fill(blocks192n) > best + 0.05) cfg = SCFG_256x192_M16;
    return cfg;
}

// general taps (Cg % 32 != 0, the grouped positional conv off the window kernel): the tiles with a GT instantiation
inline int gt_cfg(int cfg) {
    if (cfg == SCFG_256x64_M16) return SCFG_256x64_M16;
    return split_geom(cfg).BN == 64 ? SCFG_128x64_M16 : SCFG_128x128_M16;
}

inline void split_name(int cfg, int epi, bool outs, bool gt, bool f16, char* buf, int len) {
    if (cfg == SCFG_N48) {
        snprintf(buf, len, "gemm_split48_kernel<%d>", epi);
        return;
    }
    if (cfg == SCFG_WIN) {
        if (g_win_rb == 4) snprintf(buf, len, "posconv_split_kernel<%d, %d, 4>", epi, g_win_nb);
        else snprintf(buf, len, "posconv_split_kernel<%d, %d, 2>", epi, g_win_nb);
        return;
    }
    if (gt) cfg = gt_cfg(cfg);
    const SplitGeom g = split_geom(cfg);
    snprintf(buf, len, "gemm_split_kernel<%d, %d, %d, %d, %d, %d, %d, %s, %s, true, 32, 16, %s>", epi, g.BM, g.BN,
             g.WM, g.WN, g.NS, g.OCC, outs ? "true" : "false", gt ? "true" : "false", f16 ? "true" : "false");
}

template <int EPI, bool OUTS, int CFG, bool GT = false, bool F16 = false>
int launch_split_cfg(GemmP p, int Z, hipStream_t st) {
    constexpr SplitGeom g = split_geom(CFG);
    dim3 grid;
    if (int rc = set_grid(p, g.BM, g.BN, grid, Z)) return rc;
    hipLaunchKernelGGL((gemm_split_kernel<EPI, g.BM, g.BN, g.WM, g.WN, g.NS, g.OCC, OUTS, GT, true, 32, 16, F16>),
                       grid, dim3(64 * g.WM * g.WN), 0, st, p);
    return hfa::check_launch("hfa_conv_gemm_split");
}

// the one-product fast mode (HFA_GEMM_F16): the 256 x 256 / 256 x 192 / 128 x 128 / 128 x 64 / 256 x 64 tiles; the
// 192-row tiles map to 256 x 256
inline int f16_cfg(int cfg) {
    switch (cfg) {
        case SCFG_256x256_M16: case SCFG_128x128_M16: case SCFG_128x64_M16: case SCFG_256x64_M16:
        case SCFG_256x192_M16: return cfg;
        case SCFG_192x256_M16: return SCFG_256x256_M16;
        default: return split_geom(cfg).BN == 64 ? SCFG_128x64_M16 : SCFG_128x128_M16;
    }
}

template <int EPI, bool OUTS>
int launch_split_f16(GemmP p, int Z, int cfg, hipStream_t st) {
    switch (f16_cfg(cfg)) {
        case SCFG_256x256_M16: return launch_split_cfg<EPI, OUTS, SCFG_256x256_M16, false, true>(p, Z, st);
        case SCFG_128x64_M16: return launch_split_cfg<EPI, OUTS, SCFG_128x64_M16, false, true>(p, Z, st);
        case SCFG_256x64_M16: return launch_split_cfg<EPI, OUTS, SCFG_256x64_M16, false, true>(p, Z, st);
        case SCFG_256x192_M16: return launch_split_cfg<EPI, OUTS, SCFG_256x192_M16, false, true>(p, Z, st);
        default: return launch_split_cfg<EPI, OUTS, SCFG_128x128_M16, false, true>(p, Z, st);
    }
}

template <int EPI, bool OUTS>
int launch_split(GemmP p, int Z, int cfg, hipStream_t st, bool f16) {
    if (f16 && p.Cg % 32 == 0) return launch_split_f16<EPI, OUTS>(p, Z, cfg, st);
    if (p.Cg % 32) {                          // general taps (Cg % 8 == 0): the two common tiles only
        if constexpr (OUTS) {
            hfa::set_error("hfa_conv_gemm_split: Cg %% 32 != 0 takes no split output");
            return HFA_EINVAL;
        } else {
            switch (gt_cfg(cfg)) {
                case SCFG_256x64_M16: return launch_split_cfg<EPI, false, SCFG_256x64_M16, true>(p, Z, st);
                case SCFG_128x64_M16: return launch_split_cfg<EPI, false, SCFG_128x64_M16, true>(p, Z, st);
                default: return launch_split_cfg<EPI, false, SCFG_128x128_M16, true>(p, Z, st);
            }
        }
    }
    switch (cfg) {
        case SCFG_256x256_M16: return launch_split_cfg<EPI, OUTS, SCFG_256x256_M16>(p, Z, st);
        case SCFG_128x64_M16: return launch_split_cfg<EPI, OUTS, SCFG_128x64_M16>(p, Z, st);
        case SCFG_256x64_M16: return launch_split_cfg<EPI, OUTS, SCFG_256x64_M16>(p, Z, st);
        case SCFG_256x192_M16: return launch_split_cfg<EPI, OUTS, SCFG_256x192_M16>(p, Z, st);
        case SCFG_192x256_M16: return launch_split_cfg<EPI, OUTS, SCFG_192x256_M16>(p, Z, st);
        case SCFG_128x192_M16: return launch_split_cfg<EPI, OUTS, SCFG_128x192_M16>(p, Z, st);
        default: return launch_split_cfg<EPI, OUTS, SCFG_128x128_M16>(p, Z, st);
    }
}

template <int EPI, int BK, int BM, int BN, int WM, int WN>
int launch_reg(GemmP p, int Z, bool vec_a, hipStream_t st) {
    dim3 grid;
    if (int rc = set_grid(p, BM, BN, grid, Z)) return rc;
    if (vec_a) hipLaunchKernelGGL((gemm_f32_kernel<EPI, true, BK, BM, BN, WM, WN>), grid, dim3(64 * WM * WN), 0, st, p);
    else hipLaunchKernelGGL((gemm_f32_kernel<EPI, false, BK, BM, BN, WM, WN>), grid, dim3(64 * WM * WN), 0, st, p);
    return hfa::check_launch("hfa_conv_gemm_f32");
}

template <int EPI, int BM, int BN, int WM, int WN, int NS>
int launch_dma(GemmP p, int Z, bool vec_c, hipStream_t st) {
    constexpr int OCC = dma_occ(BN, WM * WN, NS);
    dim3 grid;
    if (int rc = set_grid(p, BM, BN, grid, Z)) return rc;
    if (vec_c) hipLaunchKernelGGL((gemm_dma_kernel<EPI, BM, BN, WM, WN, NS, OCC, true>), grid, dim3(64 * WM * WN), 0, st, p);
    else hipLaunchKernelGGL((gemm_dma_kernel<EPI, BM, BN, WM, WN, NS, OCC, false>), grid, dim3(64 * WM * WN), 0, st, p);
    return hfa::check_launch("hfa_conv_gemm_f32");
}

template <int EPI, int BK>
int launch_reg_cfg(int cfg, const GemmP& p, int Z, bool vec_a, hipStream_t st) {
    switch (cfg) {
        case CFG_128x64: return launch_reg<EPI, BK, 128, 64, 2, 2>(p, Z, vec_a, st);
        case CFG_256x128: return launch_reg<EPI, BK, 256, 128, 4, 2>(p, Z, vec_a, st);
        case CFG_128x256: return launch_reg<EPI, BK, 128, 256, 2, 4>(p, Z, vec_a, st);
        case CFG_256x128_W4: return launch_reg<EPI, BK, 256, 128, 2, 2>(p, Z, vec_a, st);
        case CFG_128x256_W4: return launch_reg<EPI, BK, 128, 256, 2, 2>(p, Z, vec_a, st);
        case CFG_256x256: return launch_reg<EPI, BK, 256, 256, 4, 2>(p, Z, vec_a, st);
        default: return launch_reg<EPI, BK, 128, 128, 2, 2>(p, Z, vec_a, st);
    }
}

template <int EPI, int NS>
int launch_n48(GemmP p, int Z, hipStream_t st) {
    dim3 grid;
    if (int rc = set_grid(p, 128, 48, grid, Z)) return rc;
    hipLaunchKernelGGL((gemm_dma_n48_kernel<EPI, NS>), grid, dim3(256), 0, st, p);
    return hfa::check_launch("hfa_conv_gemm_f32");
}

template <int EPI, int NS>
int launch_dma_cfg(int cfg, const GemmP& p, int Z, bool vec_c, hipStream_t st) {
    switch (cfg) {
        case CFG_128x48: return launch_n48<EPI, NS>(p, Z, st);
        case CFG_128x64: return launch_dma<EPI, 128, 64, 2, 2, NS>(p, Z, vec_c, st);
        case CFG_128x256: return launch_dma<EPI, 128, 256, 2, 4, NS>(p, Z, vec_c, st);
        case CFG_128x96: return launch_dma<EPI, 128, 96, 4, 1, 2>(p, Z, vec_c, st);     // uneven W DMA: 2 stages
        default: return launch_dma<EPI, 128, 128, 2, 2, NS>(p, Z, vec_c, st);
    }
}

template <int EPI>
int launch(const GemmP& p, int Z, const Plan& pl, hipStream_t st) {
    switch (pl.pipe) {
        case PIPE_DMA3: return launch_dma_cfg<EPI, 3>(pl.cfg, p, Z, pl.vec_c, st);
        case PIPE_DMA2: return launch_dma_cfg<EPI, 2>(pl.cfg, p, Z, pl.vec_c, st);
        case PIPE_REG32: return launch_reg_cfg<EPI, 32>(pl.cfg, p, Z, pl.vec_a, st);
        default: return launch_reg_cfg<EPI, 16>(pl.cfg, p, Z, pl.vec_a, st);
    }
}

int check_args(int M, int N, int K, int Zb, int G, const float* A, long long sAb, long long sAg, int ldx,
               int stride, int Cg, const float* W, long long sWg, int ldw, const float* C, int epilogue) {
    if (M < 0 || N < 0 || K < 0 || Zb < 0 || G < 1 || stride < 1 || Cg < 1) {
        hfa::set_error("hfa_conv_gemm_f32: bad sizes M=%d N=%d K=%d Zb=%d G=%d", M, N, K, Zb, G);
        return HFA_EINVAL;
    }
    if (M == 0 || N == 0 || Zb == 0) return HFA_OK;
    if (!A || !W || !C || K == 0) {
        hfa::set_error("hfa_conv_gemm_f32: null operand or K=0");
        return HFA_EINVAL;
    }
    if (K % 16 || Cg % 16 || K % Cg) {
        hfa::set_error("hfa_conv_gemm_f32: K=%d and Cg=%d must be multiples of 16 with Cg | K", K, Cg);
        return HFA_EINVAL;
    }
    if (!al16(W) || ldw % 4 || sWg % 4) {
        hfa::set_error("hfa_conv_gemm_f32: W must be 16-byte aligned with ldw, sWg multiples of 4");
        return HFA_EINVAL;
    }
    if (epilogue != EPI_NONE && epilogue != EPI_GELU) {
        hfa::set_error("hfa_conv_gemm_f32: unknown epilogue %d", epilogue);
        return HFA_EINVAL;
    }
    if ((long long)Zb * G > 65535) {
        hfa::set_error("hfa_conv_gemm_f32: Zb*G=%lld exceeds the grid z limit", (long long)Zb * G);
        return HFA_EINVAL;
    }
    return HFA_OK;
}

GemmP make_params(int M, int N, int K, int G, const float* A, long long sAb, long long sAg, int ldx, int stride,
                  int pad, int Cg, int Tin, const float* W, long long sWg, int ldw) {
    GemmP p;
    p.M = M; p.N = N; p.K = K; p.G = G;
    p.m_tiles = p.n_tiles = 0;   // set per tile configuration at launch
    p.A = A; p.sAb = sAb; p.sAg = sAg; p.ldx = ldx; p.stride = stride; p.pad = pad; p.Cg = Cg; p.Tin = Tin;
    p.W = W; p.sWg = sWg; p.ldw = ldw;
    p.bias = nullptr; p.sBg = 0;
    p.R = nullptr; p.sRb = p.sRg = 0; p.ldr = 0;
    p.C = nullptr; p.sCb = p.sCg = 0; p.ldc = 0;
    p.Ah = nullptr; p.sAp = 0; p.Wh = nullptr; p.sWp = 0; p.Ch = nullptr; p.sCp = 0; p.oflow = nullptr;
    p.cvec = 1;
    p.Rh = nullptr; p.sRp = 0;
    return p;
}

inline bool vec_a_of(const float* A, int ldx, long long sAb, long long sAg) {
    return al16(A) && ldx % 4 == 0 && sAb % 4 == 0 && sAg % 4 == 0;
}

thread_local char g_name[128];

}  // namespace

extern "C" {

int hfa_conv_gemm_f32(int M, int N, int K, int Zb, int G, const float* A, long long sAb, long long sAg, int ldx,
                      int stride, int pad, int Cg, int Tin, const float* W, long long sWg, int ldw,
                      const float* bias, long long sBg, const float* R, long long sRb, long long sRg, int ldr,
                      float* C, long long sCb, long long sCg, int ldc, int epilogue, hipStream_t stream) {
    if (int rc = check_args(M, N, K, Zb, G, A, sAb, sAg, ldx, stride, Cg, W, sWg, ldw, C, epilogue)) return rc;
    if (M == 0 || N == 0 || Zb == 0) return HFA_OK;
    GemmP p = make_params(M, N, K, G, A, sAb, sAg, ldx, stride, pad, Cg, Tin, W, sWg, ldw);
    p.bias = bias; p.sBg = sBg;
    p.R = R; p.sRb = sRb; p.sRg = sRg; p.ldr = ldr;
    p.C = C; p.sCb = sCb; p.sCg = sCg; p.ldc = ldc;
    const int Z = Zb * G;
    const Plan pl = make_plan(p, Z, vec_a_of(A, ldx, sAb, sAg));
    return epilogue == EPI_GELU ? launch<EPI_GELU>(p, Z, pl, stream) : launch<EPI_NONE>(p, Z, pl, stream);
}

const char* hfa_gemm_kernel_name(int M, int N, int K, int Zb, int G, const float* A, long long sAb, long long sAg,
                                 int ldx, int stride, int pad, int Cg, int Tin, const float* W, long long sWg, int ldw,
                                 const float* bias, long long sBg, const float* R, long long sRb, long long sRg,
                                 int ldr, float* C, long long sCb, long long sCg, int ldc, int epilogue) {
    GemmP p = make_params(M, N, K, G, A, sAb, sAg, ldx, stride, pad, Cg, Tin, W, sWg, ldw);
    p.bias = bias; p.sBg = sBg;
    p.R = R; p.sRb = sRb; p.sRg = sRg; p.ldr = ldr;
    p.C = C; p.sCb = sCb; p.sCg = sCg; p.ldc = ldc;
    const Plan pl = make_plan(p, Zb * G, vec_a_of(A, ldx, sAb, sAg));
    plan_name(pl, epilogue, g_name, sizeof(g_name));
    return g_name;
}

int hfa_gemm_tuning(int force_pipe, int force_cfg) {
    g_force_pipe = force_pipe;
    g_force_cfg = force_cfg;
    return HFA_OK;
}

int hfa_gemm_f32(int M, int N, int K, const float* A, int lda, const float* W, int ldw, const float* bias,
                 const float* R, int ldr, float* C, int ldc, int epilogue, hipStream_t stream) {
    return hfa_conv_gemm_f32(M, N, K, 1, 1, A, 0, 0, lda, 1, 0, K, M, W, 0, ldw, bias, 0, R, 0, 0, ldr, C, 0, 0,
                             ldc, epilogue, stream);
}

// Split-f16 implicit GEMM (gemm_split_kernel): A, W as f16 plane pairs (plane 1 at +sAp / +sWp halves), element
// strides in halves; output either f32 C (+R) or, with Cs, f16 planes (plane 1 at +sCp; bias/GELU only, no R).
int hfa_conv_gemm_split(int M, int N, int K, int Zb, int G, const uint16_t* A, long long sAp, long long sAb,
                        long long sAg, int ldx, int stride, int pad, int Cg, int Tin, const uint16_t* W,
                        long long sWp, long long sWg, int ldw, const float* bias, long long sBg, const float* R,
                        long long sRb, long long sRg, int ldr, const uint16_t* Rs, long long sRp, float* C,
                        uint16_t* Cs, long long sCp, long long sCb, long long sCg, int ldc, int epilogue, int* oflow,
                        hipStream_t stream) {
    if (M < 0 || N < 0 || K < 0 || Zb < 0 || G < 1 || stride < 1 || Cg < 1 || Tin < 1) {
        hfa::set_error("hfa_conv_gemm_split: bad sizes M=%d N=%d K=%d Zb=%d G=%d", M, N, K, Zb, G);
        return HFA_EINVAL;
    }
    if (M == 0 || N == 0 || Zb == 0) return HFA_OK;
    if (!A || !W || (!C && !Cs) || K == 0 || (Cs && !C && R)) {
        hfa::set_error("hfa_conv_gemm_split: need A, W and C and / or Cs (Cs alone takes no residual)");
        return HFA_EINVAL;
    }
    if (K % 32 || Cg % 8 || (Cg % 32 && Cg < 32) || K % Cg) {
        hfa::set_error("hfa_conv_gemm_split: K=%d must be a multiple of 32 and Cg=%d a multiple of 32 (or of 8 and "
                       ">= 32), with Cg | K", K, Cg);
        return HFA_EINVAL;
    }
    if (!al16(A) || !al16(W) || (ldx | ldw) % 8 || (sAp | sAb | sAg | sWp | sWg) % 8) {
        hfa::set_error("hfa_conv_gemm_split: A/W planes must be 16-byte aligned with strides multiple of 8 halves");
        return HFA_EINVAL;
    }
    const long long a_span = ((long long)(Tin - 1) * ldx + Cg) * 2, w_span = ((long long)(N - 1) * ldw + K) * 2;
    if (a_span >= 0x7fffffffLL || w_span >= 0x7fffffffLL) {
        hfa::set_error("hfa_conv_gemm_split: operand span past 31-bit buffer offsets");
        return HFA_EINVAL;
    }
    if (Rs && (R || !C || Cs || ((uintptr_t)Rs & 7) || (ldr | sRb | sRg | sRp) % 4)) {
        hfa::set_error("hfa_conv_gemm_split: a split-plane residual Rs goes with an f32 C alone (no R, no Cs), 8-B "
                       "aligned with strides multiple of 4 halves");
        return HFA_EINVAL;
    }
    const bool c_al = C && al16(C) && ldc % 4 == 0 && sCb % 4 == 0 && sCg % 4 == 0;
    const bool vc = (!C || (c_al && (!R || (al16(R) && ldr % 4 == 0 && sRb % 4 == 0 && sRg % 4 == 0))) ||
                     (!R && !Cs && ((uintptr_t)C & 3) == 0)) &&         // unaligned f32 C alone: scalar stores
                    (!Cs || (((uintptr_t)Cs & 7) == 0 && ldc % 4 == 0 && (sCp | sCb | sCg) % 4 == 0));
    if (!vc) {
        hfa::set_error("hfa_conv_gemm_split: C/R (or Cs) rows must be 16-B (8-B) aligned (an f32 C without R and "
                       "planes may be unaligned)");
        return HFA_EINVAL;
    }
    const bool f16 = (epilogue & HFA_GEMM_F16) != 0;
    epilogue &= ~HFA_GEMM_F16;
    if (epilogue != EPI_NONE && epilogue != EPI_GELU) {
        hfa::set_error("hfa_conv_gemm_split: unknown epilogue %d", epilogue);
        return HFA_EINVAL;
    }
    if ((long long)Zb * G > 65535) {
        hfa::set_error("hfa_conv_gemm_split: Zb*G exceeds the grid z limit");
        return HFA_EINVAL;
    }
    GemmP p = make_params(M, N, K, G, nullptr, sAb, sAg, ldx, stride, pad, Cg, Tin, nullptr, sWg, ldw);
    p.Ah = reinterpret_cast<const _Float16*>(A); p.sAp = sAp;
    p.Wh = reinterpret_cast<const _Float16*>(W); p.sWp = sWp;
    p.bias = bias; p.sBg = sBg;
    p.R = R; p.sRb = sRb; p.sRg = sRg; p.ldr = ldr;
    p.C = C; p.Ch = reinterpret_cast<_Float16*>(Cs); p.sCp = sCp; p.sCb = sCb; p.sCg = sCg; p.ldc = ldc;
    p.oflow = oflow;
    p.cvec = !C || c_al;
    p.Rh = reinterpret_cast<const _Float16*>(Rs); p.sRp = sRp;
    if (Rs && !p.cvec) {
        hfa::set_error("hfa_conv_gemm_split: a split-plane residual needs 16-B aligned C rows");
        return HFA_EINVAL;
    }
    const int Z = Zb * G, cfg = split_cfg(p, Z);
    if ((cfg == SCFG_WIN || cfg == SCFG_N48) && (!p.cvec || Rs)) {
        hfa::set_error("hfa_conv_gemm_split: the grouped positional conv kernels need 16-B aligned C rows and an f32 "
                       "residual");
        return HFA_EINVAL;
    }
    if (cfg == SCFG_WIN) {                     // grouped positional conv: LDS-resident input window
        const bool rb4 = win_rb4(p);
        dim3 grid((unsigned)((M + (rb4 ? 511 : 255)) / (rb4 ? 512 : 256)), 1, Z);
        if (rb4 && epilogue == EPI_GELU)
            hipLaunchKernelGGL((posconv_split_kernel<EPI_GELU, 3, 4>), grid, dim3(512), 0, stream, p);
        else if (rb4)
            hipLaunchKernelGGL((posconv_split_kernel<EPI_NONE, 3, 4>), grid, dim3(512), 0, stream, p);
        else if (N == 48 && epilogue == EPI_GELU)
            hipLaunchKernelGGL((posconv_split_kernel<EPI_GELU, 3>), grid, dim3(512), 0, stream, p);
        else if (N == 48)
            hipLaunchKernelGGL((posconv_split_kernel<EPI_NONE, 3>), grid, dim3(512), 0, stream, p);
        else if (epilogue == EPI_GELU)
            hipLaunchKernelGGL((posconv_split_kernel<EPI_GELU, 4>), grid, dim3(512), 0, stream, p);
        else
            hipLaunchKernelGGL((posconv_split_kernel<EPI_NONE, 4>), grid, dim3(512), 0, stream, p);
        return hfa::check_launch("hfa_conv_gemm_split");
    }
    if (cfg == SCFG_N48) {                     // N = 48, f32 output: the 16x16x32 kernel
        dim3 grid((unsigned)((M + 127) / 128), 1, Z);
        if (epilogue == EPI_GELU) hipLaunchKernelGGL(gemm_split48_kernel<EPI_GELU>, grid, dim3(256), 0, stream, p);
        else hipLaunchKernelGGL(gemm_split48_kernel<EPI_NONE>, grid, dim3(256), 0, stream, p);
        return hfa::check_launch("hfa_conv_gemm_split");
    }
    if (Cs && !C) return epilogue == EPI_GELU ? launch_split<EPI_GELU, true>(p, Z, cfg, stream, f16)
                                              : launch_split<EPI_NONE, true>(p, Z, cfg, stream, f16);
    return epilogue == EPI_GELU ? launch_split<EPI_GELU, false>(p, Z, cfg, stream, f16)
                                : launch_split<EPI_NONE, false>(p, Z, cfg, stream, f16);
}

const char* hfa_gemm_split_kernel_name(int M, int N, int K, int Z, int out_split, int epilogue, int Cg) {
    GemmP p = make_params(M, N, K, 1, nullptr, 0, 0, 0, 1, 0, Cg, 1, nullptr, 0, 0);
    p.Ch = out_split ? reinterpret_cast<_Float16*>(g_name) : nullptr;    // only its null-ness is read
    g_win_nb = N / 16;
    g_win_rb = win_rb4(p) ? 4 : 2;
    const bool f16 = (epilogue & HFA_GEMM_F16) != 0 && Cg % 32 == 0;
    int cfg = split_cfg(p, Z);
    if (f16 && cfg != SCFG_WIN && cfg != SCFG_N48) cfg = f16_cfg(cfg);
    split_name(cfg, epilogue & ~HFA_GEMM_F16, out_split != 0, Cg % 32 != 0, f16, g_name, sizeof(g_name));
    return g_name;
}

int hfa_gemm_split_tuning(int cfg) {
    if (!split_cfg_valid(cfg)) {
        hfa::set_error("hfa_gemm_split_tuning: tile %d is not built (0 auto, 15-20, 23-25)", cfg);
        return HFA_EINVAL;
    }
    g_split_cfg = cfg;
    return HFA_OK;
}

// x [rows, cols] f32 (row stride ldx) -> planes y (row stride ldy halves, plane 1 at +sp): y1 = f16(x),
// y2 = f16((x - y1) * 2^11).  Sets *oflow (when given) if any |x| >= 65504 or x is not finite.
int hfa_split_f16(int rows, int cols, const float* x, long long ldx, uint16_t* y, long long ldy, long long sp,
                  int* oflow, hipStream_t stream) {
    if (rows < 0 || cols < 0 || (rows && cols && (!x || !y))) {
        hfa::set_error("hfa_split_f16: bad arguments");
        return HFA_EINVAL;
    }
    if (!rows || !cols) return HFA_OK;
    if (rows > 65535 * 64) {
        hfa::set_error("hfa_split_f16: too many rows");
        return HFA_EINVAL;
    }
    const int cb = (cols + 1023) / 1024;
    const int gy = hfa::capped((long long)rows * cb) / cb;
    dim3 grid(cb, gy > 0 ? gy : 1);
    hipLaunchKernelGGL(split_f16_kernel, grid, dim3(256), 0, stream, rows, cols, x, ldx,
                       reinterpret_cast<_Float16*>(y), ldy, sp, oflow);
    return hfa::check_launch("hfa_split_f16");
}

}  // extern "C"
