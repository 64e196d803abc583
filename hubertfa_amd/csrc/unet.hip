// unet.hip — the lattice producer of LitForcedAlignmentTask (UNetBackbone + head) as ONE kernel per batch:
// one workgroup per utterance runs the whole layer chain on its own rows.
//
// Reference: networks/layer/backbone/unet.py:100-119 (UNetBackbone.forward), networks/layer/block/resnet_block.py:
// 17-50 (ResidualBasicBlock: conv k3 -> GroupNorm(16) -> Hardswish -> conv k3, + shortcut, -> LayerNorm ->
// Hardswish), networks/layer/scaling/stride_conv.py:23-47 (DownSampling k2 s2 conv, UpSampling k2 s2 transposed
// conv), networks/task/forced_alignment.py:53-55,284-292 (head).
//
// Why one workgroup per utterance: at config 2 (B = 32, T = 864, 192 / 384 channels) the UNet is 84 GFLOP in ~30
// small GEMMs plus their norms.  As chip-wide launches on the side stream (tiles of a few hundred workgroups, 74
// kernels with the lattice and DP) it cost the encoder beside it 1.55 ms of a 16.6 ms step (bench.py
// step_breakdown) — about as much as running it alone.  Here every layer of one utterance stays inside one CU: no
// launch or grid-wide dependency between layers, GroupNorm's statistics over the utterance's T are a reduction
// inside the workgroup, LayerNorm's row statistics are a reduction across the workgroup's waves (every workgroup
// computes all output channels of its rows), the GroupNorm + Hardswish of the second conv is applied while its
// operand is staged (no pass over memory), and the activations live in a per-utterance scratch that stays in L2 /
// the Infinity Cache.  B utterances occupy B CUs for ~2 ms; the encoder keeps the rest.  Each utterance's result
// depends on that utterance alone (never on the batch it runs in), as the reference's one-utterance runs require.
//
// Arithmetic: split-f16 (gemm.hip gemm_split_kernel): activations are split into (hi, lo * 2^11) f16 planes while
// they are staged into LDS, weights are split once at load; every MAC is a1 (2^11 w1) + a1 w2 + a2 w1 on
// v_mfma_f32_16x16x32_f16 (one accumulator at scale 2^11, |w| < 16).  Norm statistics: GroupNorm in f64 sums,
// LayerNorm two-pass in f32 (norm.hip's formulas).  A staged value outside f16 range raises *oflow (the caller
// re-runs on the f32 path).
//
// Tile: 8 waves; a row block of BM = 128 output rows x all N output columns (N <= 384): waves 2 (rows) x 4 (columns),
// a wave owns 64 x N/4 (4 x NJ blocks of 16 x 16).  K runs in steps of 32 channels of one tap: the operand window
// (BM + taps - 1 rows x 32 channels) is loaded once per channel chunk through registers (transform + split), W's
// planes for each (tap, chunk) step go global -> LDS by LDS-DMA one step ahead, two stages each.
#include "hfa_common.h"
#include "hfa.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr int NT = 512, NWV = 8, BM = 128, KS = 32;
constexpr int WIN_MAX = BM + 2;                          // k3 conv window rows
constexpr int A_PLANE = WIN_MAX * 64;                    // bytes of one plane image of the operand window
constexpr int A_STAGE = 2 * A_PLANE;
constexpr int N_MAX = 384;
constexpr int W_PLANE_MAX = N_MAX * 64;
constexpr int W_STAGE_MAX = 2 * W_PLANE_MAX;
constexpr int LDS_A = 2 * A_STAGE, LDS_W = 2 * W_STAGE_MAX;

enum { U_CONV1 = 0, U_CONV2 = 1, U_DOWN = 2, U_UP = 3, U_HEAD = 4 };

// chunk c (16 B) of image row r sits at slot c ^ swz(r): conflict-free ds_read_b128 for the 16x16x32 operand map
// (lane: row lane & 15, chunk lane >> 4), as gemm.hip's MF 16 images
__device__ __forceinline__ int swz(int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; }

struct Stage {       // one K-segment of an op: A source (f32 rows), taps, weights
    const float* src;      // row t of the source at src + t * ld (f32)
    int ld, cin, taps, pad, rows;  // channels per row read, taps (1 or 3), rows before the window, source rows
    bool gn;               // apply the block's GroupNorm + Hardswish while staging
    const _Float16* w;     // weight planes [2][N][K] (plane stride wp halves), K = taps * cin, tap-major
    long long wp;
    int ldw;
};

struct Shared {
    unsigned char a[LDS_A];
    unsigned char w[LDS_W];
    float red[2][64][4];          // LayerNorm row partials [row half][row][column wave]
    double colsum[2][N_MAX][2];   // GroupNorm column partials [row half][column][sum, sum of squares]
    float gstat[64][2];           // GroupNorm mean, rstd per group
};

// ---- staging -------------------------------------------------------------------------------------------------
// Operand window of chunk c0 (32 channels) for output rows [m0, m0 + BM): source rows m0 - pad .. m0 - pad + win - 1
// -> split planes in LDS image `abuf` (row w at 64 B per plane; chunk slots swizzled).  GroupNorm + Hardswish
// (gn) with the block's statistics; rows outside [0, rows) are the conv's zero padding (of the transformed value).
struct ARegs {
    f32x4 v[3];
};

__device__ __forceinline__ void load_a(const Stage& s, int m0, int c0, int win, ARegs& r) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int it = 0; it < 3; ++it) {
        const int idx = tid + it * NT;
        const int w = idx >> 3, q = idx & 7;
        const int t = m0 - s.pad + w;
        r.v[it] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (w < win && t >= 0 && t < s.rows)
            r.v[it] = *reinterpret_cast<const f32x4*>(s.src + (long long)t * s.ld + c0 + q * 4);
    }
}

__device__ __forceinline__ void store_a(const Stage& s, int m0, int c0, int win, const ARegs& r, unsigned char* abuf,
                                        const float* gamma, const float* beta, const Shared& sh, int G, bool& bad) {
    const int cg = s.gn ? s.cin / G : 1;                  // channels per GroupNorm group of the staged tensor
    const int tid = threadIdx.x;
#pragma unroll
    for (int it = 0; it < 3; ++it) {
        const int idx = tid + it * NT;
        const int w = idx >> 3, q = idx & 7;
        if (w >= win) continue;
        const int t = m0 - s.pad + w;
        f32x4 v = r.v[it];
        if (s.gn) {
            const int c = c0 + q * 4;
            const f32x4 g = *reinterpret_cast<const f32x4*>(gamma + c);
            const f32x4 b = *reinterpret_cast<const f32x4*>(beta + c);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int grp = (c + e) / cg;
                const float o = hfa::hardswish((v[e] - sh.gstat[grp][0]) * sh.gstat[grp][1] * g[e] + b[e]);
                v[e] = (t >= 0 && t < s.rows) ? o : 0.0f;
            }
        }
        f16x4 h1, h2;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            bad |= !(__builtin_fabsf(v[e]) < 65504.0f);
            h1[e] = (_Float16)v[e];
            h2[e] = (_Float16)((v[e] - (float)h1[e]) * 2048.0f);
        }
        const int off = w * 64 + (((q >> 1) ^ swz(w)) << 4) + (q & 1) * 8;
        *reinterpret_cast<f16x4*>(abuf + off) = h1;
        *reinterpret_cast<f16x4*>(abuf + A_PLANE + off) = h2;
    }
}

// W planes of one (tap, chunk) step: N rows x 64 B per plane, by LDS-DMA (one 1-KiB piece = 16 rows of a plane)
__device__ __forceinline__ void issue_w(const Stage& s, int N, int k0, unsigned wlds, int wave, int lane) {
    const int pieces = 2 * ((N + 15) / 16);
    const int per_plane = pieces / 2;
    const unsigned plane_bytes = (unsigned)((N + 15) / 16) * 1024u;
    // the descriptor, the LDS address and the offset go in SGPRs: make their (wave-uniform) values explicit
    const int wbytes = __builtin_amdgcn_readfirstlane(N * s.ldw * 2);
    auto uptr = [](const _Float16* p) {
        const unsigned long long v = reinterpret_cast<unsigned long long>(p);
        const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
        const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
        return reinterpret_cast<const _Float16*>(((unsigned long long)hi << 32) | lo);
    };
    const __amdgpu_buffer_rsrc_t r1 = hfa::make_rsrc(uptr(s.w), wbytes);
    const __amdgpu_buffer_rsrc_t r2 = hfa::make_rsrc(uptr(s.w + s.wp), wbytes);
    for (int p = wave; p < pieces; p += NWV) {
        const int pl = p / per_plane, rg = p - pl * per_plane;
        const int n = rg * 16 + (lane >> 2);
        const unsigned voff = n < N ? (unsigned)((n * s.ldw + k0 + (((lane & 3) ^ swz(n)) * 8)) * 2) : hfa::DMA_OOB;
        const unsigned lds = __builtin_amdgcn_readfirstlane(wlds + pl * plane_bytes + rg * 1024u);
        if (pl) hfa::dma16(voff, r2, 0u, lds);
        else hfa::dma16(voff, r1, 0u, lds);
    }
}

__device__ __forceinline__ void wait_all_barrier() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ---- one op: all row blocks of one GEMM with its epilogue ---------------------------------------------------------
struct OpArgs {
    int kind, rows_out, N;       // output rows (UP: input rows; each writes 2), output columns
    Stage st[2];                 // K segments (CONV2 + shortcut: 2)
    int nst;
    const float* bias;
    const float* gamma;          // CONV2: the GroupNorm's (staging); LN's below
    const float* beta;
    const float* ln_g;
    const float* ln_b;
    const float* res;            // CONV2: identity residual (f32 rows, ld = N); UP: skip (rows of 2N... see below)
    float* dst;                  // f32 output rows (row stride ldd; UP: N = 2 cout columns over input rows)
    int ldd;
    int G;                       // GroupNorm groups (CONV1 statistics / CONV2 staging)
};

// NI x NJ blocks of 16 x 16 per wave: a row block of 32 NI rows (2 row waves) x 64 NJ columns (4 column waves);
// NI NJ <= 12 keeps the accumulators at 48 VGPRs
template <int NI, int NJ>
__device__ void run_op(const OpArgs& o, Shared& sh, bool& bad) {
    constexpr int BMO = 32 * NI;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;                // 2 x 4 waves
    const int N = o.N;
    const int cg = o.G > 0 ? N / o.G : 1;                  // CONV1: channels per group of its output
    const unsigned lds_w = hfa::lds_addr(sh.w);
    const unsigned wstage = (unsigned)((N + 15) / 16) * 2048u;   // bytes per W stage (2 planes)
    const f16x8* abase = reinterpret_cast<const f16x8*>(sh.a);
    const f16x8* wbase = reinterpret_cast<const f16x8*>(sh.w);

    if (o.kind == U_CONV1) {                                // GroupNorm column sums, accumulated block by block
        for (int i = tid; i < 2 * N_MAX * 2; i += NT) (&sh.colsum[0][0][0])[i] = 0.0;
    }
    const int nblk = (o.rows_out + BMO - 1) / BMO;
    for (int blk = 0; blk < nblk; ++blk) {
        const int m0 = blk * BMO;
        f32x4 acc[NI][NJ];
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

        // step list: for each segment, for each 32-channel chunk, for each tap
        int seg = 0, c0 = 0, tap = 0, step = 0, chunk = 0;
        ARegs ar;
        {
            const Stage& s = o.st[0];
            wait_all_barrier();            // every wave is done reading the previous block's / op's LDS images
            issue_w(s, N, 0, lds_w, wave, lane);
            load_a(s, m0, 0, BMO + s.taps - 1, ar);
            wait_all_barrier();
            store_a(s, m0, 0, BMO + s.taps - 1, ar, sh.a, o.gamma, o.beta, sh, o.G, bad);
            wait_all_barrier();
        }
        while (true) {
            const Stage s = seg ? o.st[1] : o.st[0];     // (no dynamic index: the stages stay in registers)
            // next step
            int nseg = seg, nc0 = c0, ntap = tap + 1;
            if (ntap == s.taps) {
                ntap = 0;
                nc0 = c0 + KS;
                if (nc0 >= s.cin) {
                    nc0 = 0;
                    ++nseg;
                }
            }
            const bool has_next = nseg < o.nst;
            const bool new_chunk = has_next && ntap == 0;
            if (has_next) {
                const Stage ns = nseg ? o.st[1] : o.st[0];
                issue_w(ns, N, ntap * ns.cin + nc0, lds_w + ((step + 1) & 1) * wstage, wave, lane);
                if (new_chunk) load_a(ns, m0, nc0, BMO + ns.taps - 1, ar);
            }
            // MFMAs of this step: A rows (window row r + tap), W rows of this wave's columns
            const f16x8* ab = abase + (chunk & 1) * (A_STAGE / 16);
            const f16x8* wb = wbase + (step & 1) * (wstage / 16);
            f16x8 a1[NI], a2[NI];
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                const int w = wm * (BMO / 2) + i * 16 + (lane & 15) + tap;
                const int slot = w * 4 + ((lane >> 4) ^ swz(w));
                a1[i] = ab[slot];
                a2[i] = ab[A_PLANE / 16 + slot];
            }
            const int wplane = ((N + 15) / 16) * 1024 / 16;      // f16x8 units per W plane
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int n = wn * (NJ * 16) + j * 16 + (lane & 15);
                const int slot = n * 4 + ((lane >> 4) ^ swz(n));
                const f16x8 w1 = wb[slot];
                const f16x8 w2 = wb[wplane + slot];
                const f16x8 w1s = w1 * (_Float16)2048.0f;
#pragma unroll
                for (int i = 0; i < NI; ++i) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[i], w1s, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[i], w2, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2[i], w1, acc[i][j], 0, 0, 0);
                }
            }
            if (!has_next) break;
            if (new_chunk) {                 // the next chunk's window into the other A image
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const Stage ns = nseg ? o.st[1] : o.st[0];
                store_a(ns, m0, nc0, BMO + ns.taps - 1, ar, sh.a + ((chunk + 1) & 1) * A_STAGE, o.gamma, o.beta, sh, o.G,
                        bad);
                ++chunk;
            }
            wait_all_barrier();
            seg = nseg;
            c0 = nc0;
            tap = ntap;
            ++step;
        }

        // ---- epilogue: rows m0 + wm*64 + 16 i + 4 (lane >> 4) + e, column wn*NJ*16 + 16 j + (lane & 15) -----------
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[i][j] *= 1.0f / 2048.0f;
        const int col_base = wn * (NJ * 16) + (lane & 15);
        const int row_base = m0 + wm * (BMO / 2) + 4 * (lane >> 4);
        if (o.kind == U_CONV1) {
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int row = row_base + 16 * i + e;
                    if (row >= o.rows_out) continue;
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        const int col = col_base + 16 * j;
                        if (col >= N) continue;
                        const float v = acc[i][j][e];
                        bad |= !__builtin_isfinite(v);
                        o.dst[(long long)row * o.ldd + col] = v;
                    }
                }
            // this block's column sums (valid rows): the lane's rows, then the lanes of a column (bits 4, 5), added
            // to the workgroup's partials in block order (deterministic)
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                double s = 0.0, ss = 0.0;
#pragma unroll
                for (int i = 0; i < NI; ++i)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int row = row_base + 16 * i + e;
                        if (row < o.rows_out) {
                            const double v = (double)acc[i][j][e];
                            s += v;
                            ss += v * v;
                        }
                    }
                s += __shfl_xor(s, 16, 64);
                ss += __shfl_xor(ss, 16, 64);
                s += __shfl_xor(s, 32, 64);
                ss += __shfl_xor(ss, 32, 64);
                const int col = col_base + 16 * j;
                if (lane < 16 && col < N) {
                    sh.colsum[wm][col][0] += s;
                    sh.colsum[wm][col][1] += ss;
                }
            }
        } else if (o.kind == U_CONV2) {
            // + identity residual, then LayerNorm over the row's N columns (4 column waves) + Hardswish
            float rs[NI][4];
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int row = row_base + 16 * i + e;
                    float s = 0.f;
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        const int col = col_base + 16 * j;
                        if (o.res && row < o.rows_out && col < N) acc[i][j][e] += o.res[(long long)row * N + col];
                        if (col < N) s += acc[i][j][e];
                    }
                    rs[i][e] = s;
                }
            // row sums: over the 16 lanes of a row group, then over the 4 column waves through LDS
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float s = rs[i][e];
                    s += __shfl_xor(s, 1, 64);
                    s += __shfl_xor(s, 2, 64);
                    s += __shfl_xor(s, 4, 64);
                    s += __shfl_xor(s, 8, 64);
                    rs[i][e] = s;
                }
            if ((lane & 15) == 0) {
#pragma unroll
                for (int i = 0; i < NI; ++i)
#pragma unroll
                    for (int e = 0; e < 4; ++e) sh.red[wm][16 * i + 4 * (lane >> 4) + e][wn] = rs[i][e];
            }
            __syncthreads();
            float (&mean)[NI][4] = rs;       // the row means replace the partial sums
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int r = 16 * i + 4 * (lane >> 4) + e;
                    mean[i][e] = ((sh.red[wm][r][0] + sh.red[wm][r][1]) + (sh.red[wm][r][2] + sh.red[wm][r][3])) /
                                 (float)N;
                }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float s = 0.f;
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        const int col = col_base + 16 * j;
                        if (col < N) {
                            const float d = acc[i][j][e] - mean[i][e];
                            s += d * d;
                        }
                    }
                    s += __shfl_xor(s, 1, 64);
                    s += __shfl_xor(s, 2, 64);
                    s += __shfl_xor(s, 4, 64);
                    s += __shfl_xor(s, 8, 64);
                    if ((lane & 15) == 0) sh.red[wm][16 * i + 4 * (lane >> 4) + e][wn] = s;
                }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int r = 16 * i + 4 * (lane >> 4) + e;
                    const int row = row_base + 16 * i + e;
                    const float var = ((sh.red[wm][r][0] + sh.red[wm][r][1]) + (sh.red[wm][r][2] + sh.red[wm][r][3])) /
                                      (float)N;
                    const float rstd = 1.0f / sqrtf(var + 1e-5f);
                    if (row >= o.rows_out) continue;
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        const int col = col_base + 16 * j;
                        if (col >= N) continue;
                        const float v = hfa::hardswish((acc[i][j][e] - mean[i][e]) * rstd * o.ln_g[col] + o.ln_b[col]);
                        bad |= !__builtin_isfinite(v);
                        o.dst[(long long)row * o.ldd + col] = v;
                    }
                }
            __syncthreads();                 // sh.red reused by the next block
        } else {
            // DOWN / HEAD: + bias; UP: + bias + skip (output [T, N] is bit-for-bit the [2T, N/2] rows)
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int row = row_base + 16 * i + e;
                    if (row >= o.rows_out) continue;
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        const int col = col_base + 16 * j;
                        if (col >= N) continue;
                        float v = acc[i][j][e] + o.bias[col];
                        if (o.res) v += o.res[(long long)row * N + col];
                        bad |= !__builtin_isfinite(v);
                        o.dst[(long long)row * o.ldd + col] = v;
                    }
                }
        }
    }

    if (o.kind == U_CONV1) {
        // GroupNorm statistics over the utterance: the two row halves and the group's columns in a fixed order
        __syncthreads();
        if (tid < o.G) {
            double S = 0.0, SS = 0.0;
            for (int c = tid * cg; c < (tid + 1) * cg; ++c) {
                S += sh.colsum[0][c][0] + sh.colsum[1][c][0];
                SS += sh.colsum[0][c][1] + sh.colsum[1][c][1];
            }
            const double n = (double)o.rows_out * cg;
            const double mean_d = o.rows_out > 0 ? S / n : 0.0;
            double var_d = o.rows_out > 0 ? SS / n - mean_d * mean_d : 0.0;
            if (var_d < 0) var_d = 0;
            sh.gstat[tid][0] = (float)mean_d;
            sh.gstat[tid][1] = (float)(1.0 / sqrt(var_d + 1e-5));
        }
    }
    __syncthreads();
}

// ---- the kernel: one workgroup per utterance walks the op table ---------------------------------------------------
struct UnetArgs {
    const hfa_unet_op* ops;
    int nops;
    const float* feats;       // [B, Tmax, Cin] rows (row stride f_ld, batch stride f_bs)
    long long f_bs;
    int f_ld;
    float* logits;            // [B, Tmax, V + 2] (row stride l_ld, batch stride l_bs)
    long long l_bs;
    int l_ld;
    const int32_t* t_pad;     // [B] each utterance's padded length (a multiple of 2^levels), 0 = skip
    float* ws;                // per-utterance scratch, ws_bs floats apart
    long long ws_bs;
    int Tmax;
    int* oflow;
};

__device__ __forceinline__ const float* slot_ptr(const UnetArgs& a, float* wsb, int slot, long long off) {
    if (slot == HFA_UNET_INPUT) return a.feats + blockIdx.x * a.f_bs;
    return wsb + off * a.Tmax;
}

__global__ __launch_bounds__(NT, 1) void unet_head_kernel(const UnetArgs a) {
    __shared__ Shared sh;
    const int b = blockIdx.x;
    const int T0 = a.t_pad[b];
    if (T0 <= 0) return;
    float* wsb = a.ws + b * a.ws_bs;
    bool bad = false;
    for (int k = 0; k < a.nops; ++k) {
        const hfa_unet_op& u = a.ops[k];
        OpArgs o;
        o.kind = u.kind;
        o.N = u.n;
        o.G = u.groups;
        o.nst = u.nseg;
        const int T = T0 >> u.level;                        // rows of this op's output level (UP: its input level)
        o.rows_out = T;
        for (int s = 0; s < 2; ++s) {
            Stage& st = o.st[s];
            const int slot = u.src[s];
            st.src = slot == HFA_UNET_NONE ? nullptr : slot_ptr(a, wsb, slot, u.src_off[s]);
            st.ld = slot == HFA_UNET_INPUT ? a.f_ld : u.src_ld[s];
            st.cin = u.cin[s];
            st.taps = u.taps[s];
            st.pad = st.taps / 2;
            st.rows = T;
            st.gn = u.gn[s] != 0;
            st.w = reinterpret_cast<const _Float16*>(u.w[s]);
            st.wp = u.wp[s];
            st.ldw = u.ldw[s];
        }
        o.bias = u.bias;
        o.gamma = u.gn_gamma;
        o.beta = u.gn_beta;
        o.ln_g = u.ln_gamma;
        o.ln_b = u.ln_beta;
        o.res = u.res == HFA_UNET_NONE ? nullptr : slot_ptr(a, wsb, u.res, u.res_off);
        if (u.dst == HFA_UNET_OUTPUT) {
            o.dst = a.logits + b * a.l_bs;
            o.ldd = a.l_ld;
        } else {
            o.dst = wsb + u.dst_off * a.Tmax;
            o.ldd = u.n;
        }
        if (o.N <= 128) run_op<4, 2>(o, sh, bad);
        else if (o.N <= 192) run_op<4, 3>(o, sh, bad);
        else if (o.N <= 256) run_op<2, 4>(o, sh, bad);
        else run_op<2, 6>(o, sh, bad);
    }
    if (bad && a.oflow) *a.oflow = 1;
}

}  // namespace

extern "C" {

long long hfa_unet_lds_bytes(void) { return (long long)sizeof(Shared); }

int hfa_unet_head(int B, int Tmax, const hfa_unet_op* ops, int nops, const float* feats, long long f_bs, int f_ld,
                  float* logits, long long l_bs, int l_ld, const int32_t* t_pad, float* workspace, long long ws_bs,
                  int* oflow, hipStream_t stream) {
    if (B < 0 || Tmax < 0 || nops < 1 || nops > 256 || !ops || !feats || !logits || !t_pad || !workspace ||
        f_ld % 4 || l_ld < 1 || ws_bs < 0 || (reinterpret_cast<uintptr_t>(feats) & 15) || (f_bs % 4)) {
        hfa::set_error("hfa_unet_head: bad arguments (B=%d Tmax=%d nops=%d f_ld=%d l_ld=%d)", B, Tmax, nops, f_ld,
                       l_ld);
        return HFA_EINVAL;
    }
    if (B == 0) return HFA_OK;
    UnetArgs a{ops, nops, feats, f_bs, f_ld, logits, l_bs, l_ld, t_pad, workspace, ws_bs, Tmax, oflow};
    hipLaunchKernelGGL(unet_head_kernel, dim3(B), dim3(NT), 0, stream, a);
    return hfa::check_launch("hfa_unet_head");
}

}  // extern "C"
