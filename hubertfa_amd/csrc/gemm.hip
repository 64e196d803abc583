// gemm.hip — f32 MFMA implicit-GEMM (v_mfma_f32_32x32x2_f32) with fused epilogues, for every dense
// contraction on the path:
//   * nn.Linear / addmm: feature projection, QKV, out-proj, FFN (networks/hubert/model.py:27-33,122;
//     transformers HubertAttention/HubertFeedForward), UNet shortcut + head (resnet_block.py:164-168,
//     forced_alignment.py:53-55)
//   * conv1d as implicit GEMM over a [T, C] (channels-last) activation: extractor conv1..6 (model.py:100-114),
//     grouped positional conv k128/pad64/g16 (model.py:135-147), UNet k3 convs / k2 stride-2 down-sampling /
//     k2 stride-2 transposed up-sampling (resnet_block.py:145-162, stride_conv.py:23-47)
//   * the polyphase sinc resampler (torchaudio Resample: tools/load_wav.py:7, tools/encoder.py:46-48) as a
//     GEMM over overlapping frames of the padded wave.
//
//   C[z](m, n) = epi( sum_k A[z](m, k) * W[z](n, k) + bias[n] ) + R[z](m, n)
//   A[z](m, k): k = j*Cg + c,  t = m*stride + j - pad,  A(m,k) = (0 <= t < Tin) ? X[zb*sAb + zg*sAg + t*ldx + c] : 0
//   z = zb*G + zg (batch x group), W[z] = W + zg*sWg (row n at n*ldw, K-contiguous = [Cout][k][Cin] im2col order)
//
// f32-in MFMA is bit-for-bit an fmaf chain (exact f32, no TF32 on gfx950), so this is the fp32 parity path.
// Tile BM x BN x BK with WM x WN waves, each wave (BM/WM) x (BN/WN) = TI x TJ MFMA 32x32 tiles; A and W tiles
// are register-staged into double-buffered LDS whose rows are padded to BK+4 floats (ds_read_b128
// conflict-free).  A lane's ds_read_b128 brings 4 consecutive k of its row; the 4 MFMAs of a k-octet consume
// one element each, with the same permutation on the W side, so every k is summed exactly once.
// Block ids are remapped so consecutive logical tiles (same A rows, adjacent W columns) share an XCD's L2.
#include "hfa_common.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

struct GemmP {
    int M, N, K, G, m_tiles, n_tiles;
    const float* A; long long sAb, sAg; int ldx, stride, pad, Cg, Tin;
    const float* W; long long sWg; int ldw;
    const float* bias; long long sBg;
    const float* R; long long sRb, sRg; int ldr;
    float* C; long long sCb, sCg; int ldc;
};

enum { EPI_NONE = 0, EPI_GELU = 1 };

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

    const int nk = p.K / BK;
    load_regs(0);
    store_lds(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) load_regs((kt + 1) * BK);
#pragma unroll
        for (int kk = 0; kk < BK / 8; ++kk) {
            f32x4 a[TI], b[TJ];
#pragma unroll
            for (int i = 0; i < TI; ++i)
                a[i] = *reinterpret_cast<const f32x4*>(&sA[cur][swz(wm * (BM / WM) + i * 32 + r32, kk * 8 + h * 4)]);
#pragma unroll
            for (int j = 0; j < TJ; ++j)
                b[j] = *reinterpret_cast<const f32x4*>(&sB[cur][swz(wn * (BN / WN) + j * 32 + r32, kk * 8 + h * 4)]);
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

    // epilogue: C/D layout of 32x32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
    // GELU uses the branch-free erf (hfa::erf_nb), so lanes in different erf ranges never split.  (A separate
    // unguarded interior-tile path with batched residual loads measured slower: it pushed the 128-VGPR tile
    // into spills.)
    float* Cb = p.C + zb * p.sCb + zg * p.sCg;
    const float* Rb = p.R ? p.R + zb * p.sRb + zg * p.sRg : nullptr;
    const float* biasb = p.bias ? p.bias + zg * p.sBg : nullptr;
    const int row0 = tm * BM + wm * (BM / WM) + 4 * h;
    const int col0 = tn * BN + wn * (BN / WN) + r32;
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
                if (EPI == EPI_GELU) v = hfa::gelu_erf(v);
                if (Rb) v += Rb[(long long)row * p.ldr + col];
                Cb[(long long)row * p.ldc + col] = v;
            }
        }
    }
}

// Tile configurations (BM x BN, WM x WN waves); scripts/gemm_bench.py measures each on the workload's shapes.
enum { CFG_AUTO = 0, CFG_128x128 = 1, CFG_128x64 = 2, CFG_256x128 = 3, CFG_128x256 = 4, CFG_256x128_W4 = 5,
       CFG_128x256_W4 = 6, CFG_256x256 = 7, CFG_COUNT = 8 };
int g_force_bk = 0, g_force_cfg = 0;   // tuning overrides (hfa_gemm_tuning), 0 = automatic

template <int EPI, int BK, int BM, int BN, int WM, int WN>
int launch_cfg(GemmP p, int Z, bool vec_a, hipStream_t st) {
    p.m_tiles = (p.M + BM - 1) / BM;
    p.n_tiles = (p.N + BN - 1) / BN;
    const long long tiles = (long long)p.m_tiles * p.n_tiles;
    if (tiles > 0x7fffffffLL) {
        hfa::set_error("hfa_conv_gemm_f32: grid too large");
        return HFA_EINVAL;
    }
    dim3 grid((unsigned)tiles, 1, Z);
    if (vec_a) hipLaunchKernelGGL((gemm_f32_kernel<EPI, true, BK, BM, BN, WM, WN>), grid, dim3(64 * WM * WN), 0, st, p);
    else hipLaunchKernelGGL((gemm_f32_kernel<EPI, false, BK, BM, BN, WM, WN>), grid, dim3(64 * WM * WN), 0, st, p);
    return hfa::check_launch("hfa_conv_gemm_f32");
}

template <int EPI, int BK>
int launch_bk(int cfg, const GemmP& p, int Z, bool vec_a, hipStream_t st) {
    switch (cfg) {
        case CFG_128x64: return launch_cfg<EPI, BK, 128, 64, 2, 2>(p, Z, vec_a, st);
        case CFG_256x128: return launch_cfg<EPI, BK, 256, 128, 4, 2>(p, Z, vec_a, st);
        case CFG_128x256: return launch_cfg<EPI, BK, 128, 256, 2, 4>(p, Z, vec_a, st);
        case CFG_256x128_W4: return launch_cfg<EPI, BK, 256, 128, 2, 2>(p, Z, vec_a, st);
        case CFG_128x256_W4: return launch_cfg<EPI, BK, 128, 256, 2, 2>(p, Z, vec_a, st);
        case CFG_256x256: return launch_cfg<EPI, BK, 256, 256, 4, 2>(p, Z, vec_a, st);
        default: return launch_cfg<EPI, BK, 128, 128, 2, 2>(p, Z, vec_a, st);
    }
}

template <int EPI>
int launch(const GemmP& p, int Z, bool vec_a, hipStream_t st) {
    // measured (scripts/gemm_bench.py): BK=16 keeps 3 blocks/CU and wins on every workload shape; the 64-wide
    // N tile wins for N <= 64 (grouped positional conv) and for grids too small to fill 256 CUs twice (UNet).
    // The 8-wave 128x256 tile wins on the extractor convs (long K over overlapping rows, M*Z >= 30k rows:
    // +3..29 %) and loses on the transformer's Linear shapes (-5..-20 %).
    const long long blocks128 = (long long)((p.M + 127) / 128) * ((p.N + 127) / 128) * Z;
    int cfg = (p.N <= 64 || blocks128 < 512) ? CFG_128x64 : CFG_128x128;
    if (cfg == CFG_128x128 && p.N >= 512 && p.K >= 1024 && (long long)p.M * Z >= 30000 && p.stride > 1)
        cfg = CFG_128x256;
    if (g_force_cfg > 0 && g_force_cfg < CFG_COUNT) cfg = g_force_cfg;
    const bool bk32_ok = p.K % 32 == 0 && p.Cg % 32 == 0;
    if (g_force_bk == 32 && bk32_ok) return launch_bk<EPI, 32>(cfg, p, Z, vec_a, st);
    return launch_bk<EPI, 16>(cfg, p, Z, vec_a, st);
}

inline bool al16(const void* ptr) { return ((uintptr_t)ptr & 15) == 0; }

}  // namespace

extern "C" {

int hfa_conv_gemm_f32(int M, int N, int K, int Zb, int G, const float* A, long long sAb, long long sAg, int ldx,
                      int stride, int pad, int Cg, int Tin, const float* W, long long sWg, int ldw,
                      const float* bias, long long sBg, const float* R, long long sRb, long long sRg, int ldr,
                      float* C, long long sCb, long long sCg, int ldc, int epilogue, hipStream_t stream) {
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
    const bool vec_a = al16(A) && ldx % 4 == 0 && sAb % 4 == 0 && sAg % 4 == 0;
    GemmP p;
    p.M = M; p.N = N; p.K = K; p.G = G;
    p.m_tiles = p.n_tiles = 0;   // set per tile configuration in launch_cfg
    p.A = A; p.sAb = sAb; p.sAg = sAg; p.ldx = ldx; p.stride = stride; p.pad = pad; p.Cg = Cg; p.Tin = Tin;
    p.W = W; p.sWg = sWg; p.ldw = ldw;
    p.bias = bias; p.sBg = sBg;
    p.R = R; p.sRb = sRb; p.sRg = sRg; p.ldr = ldr;
    p.C = C; p.sCb = sCb; p.sCg = sCg; p.ldc = ldc;
    const int Z = Zb * G;
    return epilogue == EPI_GELU ? launch<EPI_GELU>(p, Z, vec_a, stream) : launch<EPI_NONE>(p, Z, vec_a, stream);
}

int hfa_gemm_tuning(int force_bk, int force_cfg) {
    g_force_bk = force_bk;
    g_force_cfg = force_cfg;
    return HFA_OK;
}

int hfa_gemm_f32(int M, int N, int K, const float* A, int lda, const float* W, int ldw, const float* bias,
                 const float* R, int ldr, float* C, int ldc, int epilogue, hipStream_t stream) {
    return hfa_conv_gemm_f32(M, N, K, 1, 1, A, 0, 0, lda, 1, 0, K, M, W, 0, ldw, bias, 0, R, 0, 0, ldr, C, 0, 0,
                             ldc, epilogue, stream);
}

}  // extern "C"
