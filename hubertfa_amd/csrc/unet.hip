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
// Tile: 8 waves; a row block of 32 NI output rows x all N output columns (N <= 384): waves 2 (rows) x 4 (columns), a
// wave owns 16 NI x 16 NJ (NI x NJ blocks of 16 x 16, NI NJ <= 12).  K runs in steps of 32 channels of one tap: the
// operand window (rows + taps - 1 x 32 channels) is loaded once per channel chunk through registers (transform +
// split) into one of two LDS images, one barrier per chunk; each step's W fragments come from L2 straight into
// registers one step ahead (the two row waves of a column read the same W; no LDS stage for it, so the k3 convs
// run 3 steps per barrier).
#include "hfa_common.h"
#include "hfa.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
// pointers that came through the op table are generic; these make their loads / stores global_* instructions
typedef const __attribute__((address_space(1))) f16x8 GF16x8;
typedef const __attribute__((address_space(1))) f32x4 GF32x4;
typedef const __attribute__((address_space(1))) float GF32;
typedef __attribute__((address_space(1))) float GF32w;
typedef __attribute__((address_space(1))) f32x4 GF32x4w;

constexpr int NT = 512, BM = 128, KS = 32;
constexpr int WIN_MAX = BM + 2;                          // k3 conv window rows
constexpr int A_PLANE = WIN_MAX * 64;                    // bytes of one plane image of the operand window
constexpr int A_STAGE = 2 * A_PLANE;
constexpr int N_MAX = 384;
constexpr int LDS_A = 2 * A_STAGE;

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

constexpr int TILE_FLOATS = 128 * (192 + 16);         // the largest C tile: 128 x 192 (NI 4, NJ 3); 64 x 384 fits

struct Shared {
    unsigned char a[LDS_A];
    float tile[TILE_FLOATS];      // the row block's outputs for the row-wise epilogue (row stride 64 NJ + 16 floats);
                                  // at the end of a first conv: the waves' GroupNorm column partials (f64)
    float gstat[64][2];           // GroupNorm mean, rstd per group
};
static_assert(8 * N_MAX * 2 * sizeof(double) <= TILE_FLOATS * sizeof(float), "GroupNorm partials fit the tile");

// ---- staging -------------------------------------------------------------------------------------------------
// Operand window of one 32-channel chunk for output rows [m0, m0 + rows_blk): source rows m0 - pad .. m0 - pad + win - 1
// -> split planes in an LDS image (row w at 64 B per plane; chunk slots swizzled).  GN: the block's GroupNorm +
// Hardswish on the way in; rows outside [0, rows) are the conv's zero padding (of the transformed value).  A thread
// always handles the same channel quad (tid & 7) of the chunk, at rows tid/8 + 64 it.  Loads are branch-free (a
// clamped row is read; store_a zeroes it), and nothing touches the loaded registers before store_a, so the loads
// stay in flight under the chunk's MFMAs.
struct ARegs {
    f32x4 v[3];
};

__device__ __forceinline__ void load_a(const Stage& s, int m0, int c0, int win, ARegs& r) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int it = 0; it < 3; ++it) {
        const int w = (tid >> 3) + it * (NT / 8), q = tid & 7;
        const int t = m0 - s.pad + w;
        const int tc = t < 0 ? 0 : (t >= s.rows ? s.rows - 1 : t);
        r.v[it] = *(const GF32x4*)(s.src + (long long)tc * s.ld + c0 + q * 4);
    }
}

// GroupNorm + Hardswish of the thread's 4 channels (c0 + 4 (tid & 7) ..): y = x * scale + shift, per channel
struct GnCoef {
    f32x4 scale, shift;
};

__device__ __forceinline__ GnCoef gn_coef(const Shared& sh, const float* gamma, int c0, int cg) {
    const int c = c0 + (threadIdx.x & 7) * 4;
    const f32x4 g = *(const GF32x4*)(gamma + c);
    GnCoef k;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int grp = (c + e) / cg;
        k.shift[e] = sh.gstat[grp][0];            // (x - mean) * (rstd * gamma) + beta
        k.scale[e] = sh.gstat[grp][1] * g[e];
    }
    return k;
}

template <bool GN>
__device__ __forceinline__ void store_a(const Stage& s, int m0, int c0, int win, const ARegs& r, unsigned char* abuf,
                                        const float* beta, const GnCoef& k, bool& bad) {
    const int tid = threadIdx.x, q = tid & 7;
    f32x4 b{0.f, 0.f, 0.f, 0.f};
    if constexpr (GN) b = *(const GF32x4*)(beta + c0 + q * 4);
#pragma unroll
    for (int it = 0; it < 3; ++it) {
        const int w = (tid >> 3) + it * (NT / 8);
        if (w >= win) continue;
        const int t = m0 - s.pad + w;
        const bool ok = t >= 0 && t < s.rows;
        f32x4 v = r.v[it];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float o = v[e];
            if constexpr (GN) o = hfa::hardswish((o - k.shift[e]) * k.scale[e] + b[e]);
            v[e] = ok ? o : 0.0f;
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

// W fragments of one step for a wave's NJ column blocks, straight from global (L2) into registers in the 16x16x32
// operand map: lane l holds row n = 16 nb + (l & 15), k = k0 + 8 (l >> 4) .. +7, both planes.  The weights are stored
// in exactly that order (fragment layout, built at load: [plane][k / 32][n / 16][lane][8 halves]), so a fragment is
// one contiguous 1 KiB load per wave.  Column blocks past the last read the last one (never stored).
template <int NJ>
struct WFr {
    f16x8 w1[NJ], w2[NJ];
};

template <int NJ>
__device__ __forceinline__ void load_wf(const Stage& s, int N, int k0, int wn, int lane, WFr<NJ>& f) {
    const int NB = (N + 15) >> 4;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        int nb = wn * NJ + j;
        nb = nb < NB ? nb : NB - 1;
        const _Float16* p = s.w + ((long long)((k0 >> 5) * NB + nb) * 64 + lane) * 8;
        f.w1[j] = *(const GF16x8*)(p);      // global, not flat: a flat load would also count in
        f.w2[j] = *(const GF16x8*)(p + s.wp);   // lgkmcnt and every LDS wait would wait for it
    }
}

__device__ __forceinline__ void wait_all_barrier() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// One K-step: the wave's NI x NJ blocks += A(window rows + tap) . W(cur), three split products each.
template <int NI, int NJ>
__device__ __forceinline__ void mfma_step(f32x4 (&acc)[NI][NJ], const f16x8* ab, const WFr<NJ>& cur, int wrow, int tap,
                                          int lane) {
    f16x8 w1s[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) w1s[j] = cur.w1[j] * (_Float16)2048.0f;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int w = wrow + i * 16 + (lane & 15) + tap;
        const int slot = w * 4 + ((lane >> 4) ^ swz(w));
        const f16x8 a1 = ab[slot];
        const f16x8 a2 = ab[A_PLANE / 16 + slot];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, w1s[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, cur.w2[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2, cur.w1[j], acc[i][j], 0, 0, 0);
        }
    }
}

// All K-steps of one segment (TAPS taps x cin/32 chunks) for the row block at m0.  The window of chunk q + 1 and the
// W fragments of the next step are loaded while step q's MFMAs run (every load unconditional: the last chunk
// re-reads itself); W alternates between two register sets, so chunks are walked in pairs (TAPS odd flips the
// parity each chunk).  One barrier per chunk.  On entry the caller has the LDS images free (a barrier behind it).
template <int NI, int NJ, int TAPS, bool GN>
__device__ __forceinline__ void kloop(const Stage& s, int N, int m0, f32x4 (&acc)[NI][NJ], Shared& sh,
                                      const float* gamma, const float* beta, int G, int wm, int wn, int lane,
                                      bool& bad) {
    constexpr int BMO = 32 * NI, WIN = BMO + TAPS - 1;
    const int nch = s.cin / KS;
    const int cg = GN ? s.cin / G : 1;
    const f16x8* abase = reinterpret_cast<const f16x8*>(sh.a);
    const int wrow = wm * (BMO / 2);
    ARegs ar;
    WFr<NJ> wa, wb;
    load_a(s, m0, 0, WIN, ar);
    load_wf<NJ>(s, N, 0, wn, lane, wa);
    GnCoef k{};
    if constexpr (GN) k = gn_coef(sh, gamma, 0, cg);
    store_a<GN>(s, m0, 0, WIN, ar, sh.a, beta, k, bad);
    wait_all_barrier();
    // chunk q with its first W set in X: taps alternate X, Y, X, ...; the next chunk's first set lands in the
    // other one (Y for TAPS odd)
    auto chunk = [&](int q, WFr<NJ>& X, WFr<NJ>& Y) {
        const int qn = q + 1 < nch ? q + 1 : q;
        const f16x8* ab = abase + (q & 1) * (A_STAGE / 16);
        load_a(s, m0, qn * KS, WIN, ar);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int tp = 0; tp < TAPS; ++tp) {
            WFr<NJ>& cur = (tp & 1) ? Y : X;
            WFr<NJ>& nxt = (tp & 1) ? X : Y;
            if (tp + 1 < TAPS) load_wf<NJ>(s, N, (tp + 1) * s.cin + q * KS, wn, lane, nxt);
            else load_wf<NJ>(s, N, qn * KS, wn, lane, nxt);
            __builtin_amdgcn_sched_barrier(0);          // the prefetch stays ahead of this step's MFMAs
            mfma_step<NI, NJ>(acc, ab, cur, wrow, tp, lane);
        }
        if (q + 1 < nch) {
            if constexpr (GN) k = gn_coef(sh, gamma, qn * KS, cg);
            store_a<GN>(s, m0, qn * KS, WIN, ar, sh.a + ((q + 1) & 1) * A_STAGE, beta, k, bad);
            wait_all_barrier();
        }
    };
    static_assert(TAPS == 1 || TAPS == 3, "taps 1 or 3");
    for (int q = 0; q < nch; q += 2) {
        chunk(q, wa, wb);                       // TAPS odd: its last step prefetched chunk q + 1's first set into wb
        if (q + 1 < nch) chunk(q + 1, wb, wa);
    }
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
// Not inlined: each (NI, NJ) instance gets its own register allocation (inlined into one kernel body, the union of
// the four instances' live ranges spilled inside the MFMA loops).  Returns whether a value left f16 range.
// Row blocks [blk0, blk1) of the op (the fused kernel: all of them).  gn_out (tiled CONV1 only): this workgroup's
// GroupNorm partial sums per group (f64 sum, sum of squares) go to gn_out[G][2] instead of becoming the statistics.
template <int NI, int NJ>
__device__ __attribute__((noinline)) bool run_op(const OpArgs& o, Shared& sh, int blk0, int blk1, double* gn_out) {
    bool bad = false;
    constexpr int BMO = 32 * NI;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;                // 2 x 4 waves
    const int N = o.N;
    const int cg = o.G > 0 ? N / o.G : 1;                  // CONV1: channels per group of its output

    // Row-wise epilogue geometry: a lane owns the float4 columns 4 lane + 256 k (k < C4; N % 4 == 0)
    constexpr int C4 = (NJ * 64 + 255) / 256;
    constexpr int LDT = NJ * 64 + 16;                       // tile row stride (floats): 64 B off a bank row
    static_assert(BMO * LDT <= TILE_FLOATS, "tile");
    // per-column parameters, loaded once per op
    f32x4 pb[C4], pg[C4], pbt[C4];
#pragma unroll
    for (int k = 0; k < C4; ++k) {
        const int c = 4 * lane + 256 * k;
        const int cc = c < N ? c : 0;                           // (branch-free: a valid address, value unused)
        pb[k] = o.bias ? *(const GF32x4*)(o.bias + cc) : f32x4{0.f, 0.f, 0.f, 0.f};
        pg[k] = o.ln_g ? *(const GF32x4*)(o.ln_g + cc) : f32x4{0.f, 0.f, 0.f, 0.f};
        pbt[k] = o.ln_b ? *(const GF32x4*)(o.ln_b + cc) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // CONV1: this wave's GroupNorm column partials (its rows, its lane's columns), f64
    double gs[C4][4], gss[C4][4];
#pragma unroll
    for (int k = 0; k < C4; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) gs[k][e] = gss[k][e] = 0.0;
    const int nblk = min((o.rows_out + BMO - 1) / BMO, blk1);
    for (int blk = blk0; blk < nblk; ++blk) {
        const int m0 = blk * BMO;
        f32x4 acc[NI][NJ];
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

        // K: segment 0 (the op's operand), then the shortcut segment of a block's second conv
        wait_all_barrier();                // every wave is done with the previous block's LDS images and tile
        if (o.kind == U_CONV1)
            kloop<NI, NJ, 3, false>(o.st[0], N, m0, acc, sh, o.gamma, o.beta, o.G, wm, wn, lane, bad);
        else if (o.kind == U_CONV2)
            kloop<NI, NJ, 3, true>(o.st[0], N, m0, acc, sh, o.gamma, o.beta, o.G, wm, wn, lane, bad);
        else
            kloop<NI, NJ, 1, false>(o.st[0], N, m0, acc, sh, o.gamma, o.beta, o.G, wm, wn, lane, bad);
        if (o.nst > 1) {
            wait_all_barrier();
            kloop<NI, NJ, 1, false>(o.st[1], N, m0, acc, sh, o.gamma, o.beta, o.G, wm, wn, lane, bad);
        }

        // ---- epilogue, 1: the accumulators (scaled back by 2^-11) into the tile: row 16 i + 4 (lane >> 4) + e of
        // the wave's rows, column 16 j + (lane & 15) of its columns
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int r = wm * (BMO / 2) + 16 * i + 4 * (lane >> 4) + e;
                    const int c = wn * (NJ * 16) + 16 * j + (lane & 15);
                    sh.tile[r * LDT + c] = acc[i][j][e] * (1.0f / 2048.0f);
                }
        __syncthreads();
        // ---- 2: row-wise, one wave per row (rows wave, wave + 8, ...), two rows at a time: a lane handles the
        // float4 columns 4 lane + 256 k, so every global access is a contiguous row segment of 16-B pieces, the
        // residual loads of both rows are in flight together, and LayerNorm's statistics are wave reductions
        const int rows_here = o.rows_out - m0 < BMO ? o.rows_out - m0 : BMO;
        for (int r0 = wave; r0 < rows_here; r0 += 16) {
            f32x4 v[2][C4], rr[2][C4];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int r = r0 + 8 * h;
                const int rc = r < rows_here ? r : r0;             // (the second row may not exist: reread the first)
#pragma unroll
                for (int k = 0; k < C4; ++k) {
                    const int c = 4 * lane + 256 * k;
                    const int cc = c < N ? c : 0;
                    v[h][k] = *reinterpret_cast<const f32x4*>(&sh.tile[rc * LDT + cc]);
                    rr[h][k] = o.res ? *(const GF32x4*)(o.res + (long long)(m0 + rc) * N + cc)
                                     : f32x4{0.f, 0.f, 0.f, 0.f};
                }
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int r = r0 + 8 * h;
                if (r >= rows_here) break;                         // (wave-uniform)
                const int row = m0 + r;
                if (o.kind == U_CONV1) {
#pragma unroll
                    for (int k = 0; k < C4; ++k) {
                        const int c = 4 * lane + 256 * k;
                        if (c < N) {
#pragma unroll
                            for (int e = 0; e < 4; ++e) {
                                bad |= !__builtin_isfinite(v[h][k][e]);
                                gs[k][e] += (double)v[h][k][e];
                                gss[k][e] += (double)v[h][k][e] * (double)v[h][k][e];
                            }
                            *(GF32x4w*)(o.dst + (long long)row * o.ldd + c) = v[h][k];
                        }
                    }
                } else if (o.kind == U_CONV2) {
                    // + identity residual, LayerNorm over the row's N columns (two-pass, f32) + Hardswish
                    float s = 0.f;
#pragma unroll
                    for (int k = 0; k < C4; ++k) {
                        const int c = 4 * lane + 256 * k;
                        if (c < N) {
                            v[h][k] += rr[h][k];
                            s += (v[h][k][0] + v[h][k][1]) + (v[h][k][2] + v[h][k][3]);
                        }
                    }
                    const float mean = hfa::wave_sum(s) / (float)N;
                    float ss = 0.f;
#pragma unroll
                    for (int k = 0; k < C4; ++k) {
                        const int c = 4 * lane + 256 * k;
                        if (c < N) {
#pragma unroll
                            for (int e = 0; e < 4; ++e) {
                                const float d = v[h][k][e] - mean;
                                ss += d * d;
                            }
                        }
                    }
                    const float rstd = 1.0f / sqrtf(hfa::wave_sum(ss) / (float)N + 1e-5f);
#pragma unroll
                    for (int k = 0; k < C4; ++k) {
                        const int c = 4 * lane + 256 * k;
                        if (c < N) {
                            f32x4 y;
#pragma unroll
                            for (int e = 0; e < 4; ++e) {
                                y[e] = hfa::hardswish((v[h][k][e] - mean) * rstd * pg[k][e] + pbt[k][e]);
                                bad |= !__builtin_isfinite(y[e]);
                            }
                            *(GF32x4w*)(o.dst + (long long)row * o.ldd + c) = y;
                        }
                    }
                } else {
                    // DOWN / HEAD: + bias; UP: + bias + skip (its [T, N] rows are bit-for-bit the [2T, N/2] rows)
#pragma unroll
                    for (int k = 0; k < C4; ++k) {
                        const int c = 4 * lane + 256 * k;
                        if (c < N) {
                            f32x4 y = v[h][k] + pb[k] + rr[h][k];
#pragma unroll
                            for (int e = 0; e < 4; ++e) bad |= !__builtin_isfinite(y[e]);
                            *(GF32x4w*)(o.dst + (long long)row * o.ldd + c) = y;
                        }
                    }
                }
            }
        }
    }

    if (o.kind == U_CONV1) {
        // GroupNorm statistics over the utterance: every wave's column partials into the tile space, then per group
        // the waves and the group's columns in a fixed order (deterministic)
        __syncthreads();
        double* part = reinterpret_cast<double*>(sh.tile);         // [8 waves][N][2]
#pragma unroll
        for (int k = 0; k < C4; ++k)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int c = 4 * lane + 256 * k + e;
                if (c < N) {
                    part[(wave * N + c) * 2] = gs[k][e];
                    part[(wave * N + c) * 2 + 1] = gss[k][e];
                }
            }
        __syncthreads();
        if (tid < o.G) {
            double S = 0.0, SS = 0.0;
            for (int c = tid * cg; c < (tid + 1) * cg; ++c)
                for (int w = 0; w < 8; ++w) {
                    S += part[(w * N + c) * 2];
                    SS += part[(w * N + c) * 2 + 1];
                }
            if (gn_out) {                                          // tiled: the partials of this row block
                *(__attribute__((address_space(1))) double*)(gn_out + 2 * tid) = S;
                *(__attribute__((address_space(1))) double*)(gn_out + 2 * tid + 1) = SS;
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
    return bad;
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
    long long* prof;          // optional (hfa_unet_profile): workgroup 0's s_memrealtime at every op boundary
};

__device__ __forceinline__ const float* slot_ptr(const UnetArgs& a, int b, float* wsb, int slot, long long off) {
    if (slot == HFA_UNET_INPUT) return a.feats + b * a.f_bs;
    return wsb + off * a.Tmax;
}

// table entry u -> the op's arguments for utterance b (T0 padded rows, scratch wsb)
__device__ __forceinline__ void make_op(const UnetArgs& a, const hfa_unet_op& u, int b, int T0, float* wsb, OpArgs& o) {
    o.kind = u.kind;
    o.N = u.n;
    o.G = u.groups;
    o.nst = u.nseg;
    const int T = T0 >> u.level;                            // rows of this op's output level (UP: its input level)
    o.rows_out = T;
    for (int s = 0; s < 2; ++s) {
        Stage& st = o.st[s];
        const int slot = u.src[s];
        st.src = slot == HFA_UNET_NONE ? nullptr : slot_ptr(a, b, wsb, slot, u.src_off[s]);
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
    o.res = u.res == HFA_UNET_NONE ? nullptr : slot_ptr(a, b, wsb, u.res, u.res_off);
    if (u.dst == HFA_UNET_OUTPUT) {
        o.dst = a.logits + b * a.l_bs;
        o.ldd = a.l_ld;
    } else {
        o.dst = wsb + u.dst_off * a.Tmax;
        o.ldd = u.n;
    }
}

// rows per row block of an op with N output columns (run_op's NI): the dispatch below and the host's grid agree on it
__host__ __device__ constexpr int op_block_rows(int N) { return N <= 192 ? 128 : 64; }

__device__ __forceinline__ bool dispatch_op(const OpArgs& o, Shared& sh, int blk0, int blk1, double* gn_out) {
    if (o.N <= 128) return run_op<4, 2>(o, sh, blk0, blk1, gn_out);
    if (o.N <= 192) return run_op<4, 3>(o, sh, blk0, blk1, gn_out);
    if (o.N <= 256) return run_op<2, 4>(o, sh, blk0, blk1, gn_out);
    return run_op<2, 6>(o, sh, blk0, blk1, gn_out);
}

__global__ __launch_bounds__(NT, 1) void unet_head_kernel(const UnetArgs a) {
    __shared__ Shared sh;
    const int b = blockIdx.x;
    const int T0 = a.t_pad[b];
    if (T0 <= 0 || T0 > a.Tmax) return;
    float* wsb = a.ws + b * a.ws_bs;
    bool bad = false;
    for (int k = 0; k < a.nops; ++k) {
        if (a.prof && b == 0 && threadIdx.x == 0) a.prof[k] = (long long)__builtin_amdgcn_s_memrealtime();
        OpArgs o;
        make_op(a, a.ops[k], b, T0, wsb, o);
        bad |= dispatch_op(o, sh, 0, 1 << 30, nullptr);
    }
    if (a.prof && b == 0 && threadIdx.x == 0) a.prof[a.nops] = (long long)__builtin_amdgcn_s_memrealtime();
    if (bad && a.oflow) *a.oflow = 1;
}

// Tiled form: ONE op per launch, one workgroup per (row block, utterance) — the same op engine, spread over the
// chip in short-lived workgroups instead of one long-lived workgroup per utterance.  A first conv writes its row
// block's GroupNorm partials to gn[b][blk][G][2]; the block's second conv sums its utterance's nblk_gn partials in
// block order (deterministic, independent of the batch) before staging.
__global__ __launch_bounds__(NT, 1) void unet_op_kernel(const UnetArgs a, int k, double* gn, long long gn_bs,
                                                        int nblk_gn) {
    __shared__ Shared sh;
    const int b = blockIdx.y, blk = blockIdx.x;
    const int T0 = a.t_pad[b];
    if (T0 <= 0 || T0 > a.Tmax) return;
    const hfa_unet_op& u = a.ops[k];
    if (blk * op_block_rows(u.n) >= (T0 >> u.level)) return;      // this utterance has fewer rows
    float* wsb = a.ws + b * a.ws_bs;
    OpArgs o;
    make_op(a, u, b, T0, wsb, o);
    double* gnb = gn + b * gn_bs;
    if (o.kind == U_CONV2) {
        const int rows1 = T0 >> u.level, cg = o.st[0].cin / o.G;
        const int nb = min(nblk_gn, (rows1 + op_block_rows(o.st[0].cin) - 1) / op_block_rows(o.st[0].cin));
        if ((int)threadIdx.x < o.G) {
            double S = 0.0, SS = 0.0;
            for (int i = 0; i < nb; ++i) {
                S += gnb[(i * 64 + threadIdx.x) * 2];
                SS += gnb[(i * 64 + threadIdx.x) * 2 + 1];
            }
            const double n = (double)rows1 * cg;
            const double mean_d = rows1 > 0 ? S / n : 0.0;
            double var_d = rows1 > 0 ? SS / n - mean_d * mean_d : 0.0;
            if (var_d < 0) var_d = 0;
            sh.gstat[threadIdx.x][0] = (float)mean_d;
            sh.gstat[threadIdx.x][1] = (float)(1.0 / sqrt(var_d + 1e-5));
        }
        __syncthreads();
    }
    const bool bad = dispatch_op(o, sh, blk, blk + 1, o.kind == U_CONV1 ? gnb + blk * 64 * 2 : nullptr);
    if (bad && a.oflow) *a.oflow = 1;
}

thread_local long long* g_prof = nullptr;

}  // namespace

extern "C" {

long long hfa_unet_lds_bytes(void) { return (long long)sizeof(Shared); }

int hfa_unet_validate(const hfa_unet_op* ops, int nops, long long wpr, int l_ld) {
    if (!ops || nops < 1 || nops > 256 || wpr < 0) {
        hfa::set_error("hfa_unet_validate: bad table (nops=%d)", nops);
        return HFA_EINVAL;
    }
    // floats per Tmax row a level-`lv` tensor of row width `ld` at slot offset `off` reaches
    auto inside = [&](long long off, int ld, int lv) { return off >= 0 && off + ((long long)ld + (1LL << lv) - 1) / (1LL << lv) <= wpr; };
    for (int k = 0; k < nops; ++k) {
        const hfa_unet_op& u = ops[k];
        const char* why = nullptr;
        const bool head = u.kind == U_HEAD;
        if (u.kind < U_CONV1 || u.kind > U_HEAD) why = "kind";
        else if (u.level < 0 || u.level > 12) why = "level";
        else if (u.n < 4 || u.n > 384 || u.n % 4) why = "n (4..384, a multiple of 4)";
        else if (u.nseg < 1 || u.nseg > (u.kind == U_CONV2 ? 2 : 1)) why = "nseg";
        else if (u.kind == U_CONV1 && (u.groups < 1 || u.n % u.groups)) why = "groups";
        else if (u.kind == U_CONV2 && (!u.gn_gamma || !u.gn_beta || !u.ln_gamma || !u.ln_beta)) why = "norm parameters";
        else if (u.kind == U_CONV2 && (k == 0 || ops[k - 1].kind != U_CONV1 || ops[k - 1].n != u.cin[0] ||
                                       !u.gn[0] || u.groups != ops[k - 1].groups))
            why = "conv2 without its conv1 (GroupNorm statistics)";
        else if (head != (u.dst == HFA_UNET_OUTPUT)) why = "dst (HFA_UNET_OUTPUT is the head's only)";
        else if (head && u.n > l_ld) why = "head n > l_ld";
        else if (!head && (u.dst < 0 || !inside(u.dst_off, u.n, u.level))) why = "dst slot outside the workspace";
        else if (u.res != HFA_UNET_NONE && u.res != HFA_UNET_INPUT &&
                 (u.res < 0 || !inside(u.res_off, u.n, u.level)))
            why = "res slot outside the workspace";
        for (int s = 0; s < u.nseg && !why; ++s) {
            if (u.cin[s] < 32 || u.cin[s] % 32) why = "cin (a multiple of 32)";
            else if (u.taps[s] != 1 && u.taps[s] != 3) why = "taps (1 or 3)";
            else if (u.ldw[s] != u.taps[s] * u.cin[s]) why = "ldw != taps * cin";
            else if (!u.w[s] || (reinterpret_cast<uintptr_t>(u.w[s]) & 15) || u.wp[s] % 8 ||
                     u.wp[s] < (long long)u.ldw[s] / 32 * ((u.n + 15) / 16) * 512)
                why = "weight planes";
            else if (u.gn[s] && (s != 0 || u.kind != U_CONV2)) why = "gn outside conv2's first segment";
            else if (u.src[s] == HFA_UNET_INPUT) {
                if (u.level != 0) why = "INPUT read off level 0";
            } else if (u.src[s] < 0 || u.src_ld[s] < u.cin[s] || u.src_ld[s] % 4 ||
                       !inside(u.src_off[s], u.src_ld[s], u.level))
                why = "src slot outside the workspace";
        }
        if (why) {
            hfa::set_error("hfa_unet_validate: op %d: %s", k, why);
            return HFA_EINVAL;
        }
    }
    return HFA_OK;
}

int hfa_unet_profile(long long* buf) {
    g_prof = buf;
    return HFA_OK;
}

int hfa_unet_head(int B, int Tmax, const hfa_unet_op* ops, int nops, const float* feats, long long f_bs, int f_ld,
                  float* logits, long long l_bs, int l_ld, const int32_t* t_pad, float* workspace, long long ws_bs,
                  int* oflow, hipStream_t stream) {
    if (B < 0 || Tmax < 0 || nops < 1 || nops > 256 || !ops || !feats || !logits || !t_pad || !workspace ||
        f_ld % 4 || l_ld < 1 || l_ld % 4 || l_bs % 4 || ws_bs < 0 || ws_bs % 4 || (reinterpret_cast<uintptr_t>(feats) & 15) ||
        (reinterpret_cast<uintptr_t>(logits) & 15) || (reinterpret_cast<uintptr_t>(workspace) & 15) || (f_bs % 4)) {
        hfa::set_error("hfa_unet_head: bad arguments (B=%d Tmax=%d nops=%d f_ld=%d l_ld=%d)", B, Tmax, nops, f_ld,
                       l_ld);
        return HFA_EINVAL;
    }
    if (B == 0) return HFA_OK;
    UnetArgs a{ops, nops, feats, f_bs, f_ld, logits, l_bs, l_ld, t_pad, workspace, ws_bs, Tmax, oflow, g_prof};
    g_prof = nullptr;
    hipLaunchKernelGGL(unet_head_kernel, dim3(B), dim3(NT), 0, stream, a);
    return hfa::check_launch("hfa_unet_head");
}

long long hfa_unet_gn_doubles(int Tmax) {
    return (long long)((Tmax + 63) / 64) * 64 * 2;            // row blocks of >= 64 rows, 64 groups, (sum, sumsq)
}

int hfa_unet_head_tiled(int B, int Tmax, const hfa_unet_op* host_ops, const hfa_unet_op* ops, int nops,
                        const float* feats, long long f_bs, int f_ld, float* logits, long long l_bs, int l_ld,
                        const int32_t* t_pad, float* workspace, long long ws_bs, double* gn_ws, long long gn_bs,
                        int* oflow, hipStream_t stream) {
    if (B < 0 || Tmax < 0 || nops < 1 || nops > 256 || !host_ops || !ops || !feats || !logits || !t_pad ||
        !workspace || !gn_ws || gn_bs < hfa_unet_gn_doubles(Tmax) || f_ld % 4 || l_ld < 1 || l_ld % 4 ||
        l_bs % 4 || ws_bs < 0 || ws_bs % 4 || (reinterpret_cast<uintptr_t>(feats) & 15) ||
        (reinterpret_cast<uintptr_t>(logits) & 15) || (reinterpret_cast<uintptr_t>(workspace) & 15) || (f_bs % 4) ||
        B > 65535) {
        hfa::set_error("hfa_unet_head_tiled: bad arguments (B=%d Tmax=%d nops=%d f_ld=%d l_ld=%d gn_bs=%lld)", B,
                       Tmax, nops, f_ld, l_ld, gn_bs);
        return HFA_EINVAL;
    }
    if (B == 0 || Tmax == 0) return HFA_OK;
    UnetArgs a{ops, nops, feats, f_bs, f_ld, logits, l_bs, l_ld, t_pad, workspace, ws_bs, Tmax, oflow, nullptr};
    for (int k = 0; k < nops; ++k) {
        const hfa_unet_op& u = host_ops[k];
        const int rows = Tmax >> u.level;
        const int nblk = (rows + op_block_rows(u.n) - 1) / op_block_rows(u.n);
        const int nblk_gn = u.kind == U_CONV2 ? (rows + op_block_rows(u.cin[0]) - 1) / op_block_rows(u.cin[0]) : 0;
        if (nblk < 1) continue;
        hipLaunchKernelGGL(unet_op_kernel, dim3(nblk, B), dim3(NT), 0, stream, a, k, gn_ws, gn_bs, nblk_gn);
        if (int rc = hfa::check_launch("hfa_unet_head_tiled")) return rc;
    }
    return HFA_OK;
}

}  // extern "C"
