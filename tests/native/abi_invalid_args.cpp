// Host-side sanitizer driver (ASan/UBSan on the host code): links the AddressSanitizer /
// UndefinedBehaviorSanitizer build of libhfa's host code (hubertfa_amd/_build_asan/libhfa.so, device code as
// shipped) and drives every entry point of include/hfa.h through its argument validation with bad arguments —
// negative sizes, NULL operands, misaligned pointers and strides, out-of-range options — plus the pure host
// queries (workspace sizes, kernel-name queries, tuning hooks, error strings).  No call reaches a kernel launch,
// so it runs without a GPU.  Exit 0 = every call returned its error code with a message and no sanitizer fired.
#include <hfa.h>

#include <cstdio>
#include <cstring>

static int g_fail = 0, g_n = 0;

// Every check is armed first: a known error (hfa_viterbi_tuning's) goes into the thread's message slot, so a call
// that fails without writing its own message is caught (its rc < 0 but the message is still the sentinel's).
static char g_sentinel[256];
#define CHECK(call, what)                                                                               \
    do {                                                                                               \
        hfa_viterbi_tuning(3);                                                                         \
        std::snprintf(g_sentinel, sizeof(g_sentinel), "%s", hfa_last_error());                         \
        expect_err((call), what);                                                                      \
    } while (0)

static void expect_err(int rc, const char* what) {
    ++g_n;
    const char* msg = hfa_last_error();
    if (rc >= 0 || !msg || !*msg || std::strcmp(msg, g_sentinel) == 0) {
        std::printf("FAIL %s: rc=%d msg=%s\n", what, rc, msg ? msg : "(null)");
        ++g_fail;
    }
}

int main() {
    hipStream_t st = nullptr;
    float* fp = reinterpret_cast<float*>(0x100000);          // never dereferenced: validation rejects first
    float* fmis = reinterpret_cast<float*>(0x100004);        // 4-B aligned, not 16-B
    uint16_t* hp = reinterpret_cast<uint16_t*>(0x100000);
    uint16_t* hmis = reinterpret_cast<uint16_t*>(0x100002);
    const int32_t* ip = reinterpret_cast<const int32_t*>(0x100000);
    double* dp = reinterpret_cast<double*>(0x100000);
    int8_t* bp = reinterpret_cast<int8_t*>(0x100000);
    int* op = reinterpret_cast<int*>(0x100000);
    void* ws = reinterpret_cast<void*>(0x100000);

    if (hfa_abi_version() <= 0 || !hfa_build_arch() || std::strcmp(hfa_build_arch(), "gfx950") != 0) {
        std::printf("FAIL abi version / arch\n");
        ++g_fail;
    }
    // alignment decoder
    CHECK(hfa_viterbi_forward(-1, 10, 8, ip, ip, nullptr, fp, fp, fp, dp, fp, bp, ip, st), "viterbi B<0");
    CHECK(hfa_viterbi_forward(2, 10, 9000, ip, ip, nullptr, fp, fp, fp, dp, fp, bp, ip, st), "viterbi Smax");
    CHECK(hfa_viterbi_forward(2, 10, 8, nullptr, ip, nullptr, fp, fp, fp, dp, fp, bp, ip, st), "viterbi NULL T");
    CHECK(hfa_viterbi_forward_steps(2, 10, 8, ip, ip, nullptr, fp, fp, fp, dp, fp, bp, ip, 0, 5, st),
          "viterbi steps t_begin 0");
    CHECK(hfa_viterbi_forward_steps(2, 10, 8, ip, ip, nullptr, fp, fp, fp, dp, fp, bp, ip, 6, 5, st),
          "viterbi steps reversed");
    CHECK(hfa_viterbi_forward_steps(2, 10, 9000, ip, ip, nullptr, fp, fp, fp, dp, fp, bp, ip, 2, 5, st),
          "viterbi steps wide partial");
    g_sentinel[0] = 0;
    expect_err(hfa_viterbi_tuning(3), "viterbi tuning k=3");   // the sentinel call itself
    CHECK(hfa_viterbi_backtrack(2, 70000, 8, ip, ip, fp, bp, ip, nullptr, nullptr, nullptr, fp, st),
               "backtrack NULL out");
    CHECK(hfa_viterbi_backtrack(-3, 10, 8, ip, ip, fp, bp, ip, op, op, op, fp, st), "backtrack B<0");
    CHECK(hfa_lattice_prologue(-1, 10, 60, 8, ip, ip, fp, 60, 600, fp, 1, 10, ip, fp, fp, fp, fp, fp, fp, dp,
                               nullptr, nullptr, st), "prologue B<0");
    CHECK(hfa_lattice_prologue(1, 10, 60, 8, ip, ip, nullptr, 60, 600, fp, 1, 10, ip, fp, fp, fp, fp, fp, fp,
                               dp, nullptr, nullptr, st), "prologue NULL logits");
    CHECK(hfa_lattice_prologue(1, 10, 60, 8, ip, ip, fp, 60, 600, fp, 1, 10, ip, fp, fp, fp, fp, fp, fp, dp, fp,
                               nullptr, st), "prologue dp without curr");
    CHECK(hfa_viterbi_init(-1, 10, 8, ip, ip, fp, ip, fp, dp, st), "viterbi_init B<0");
    CHECK(hfa_viterbi_init(1, 10, 8, ip, ip, fp, ip, nullptr, dp, st), "viterbi_init NULL dp");
    // GEMMs
    CHECK(hfa_conv_gemm_f32(-1, 64, 64, 1, 1, fp, 0, 0, 64, 1, 0, 64, 1, fp, 0, 64, nullptr, 0, nullptr, 0, 0,
                                 0, fp, 0, 0, 64, 0, st), "conv_gemm_f32 M<0");
    CHECK(hfa_conv_gemm_f32(64, 64, 60, 1, 1, fp, 0, 0, 64, 1, 0, 60, 64, fp, 0, 64, nullptr, 0, nullptr, 0, 0,
                                 0, fp, 0, 0, 64, 0, st), "conv_gemm_f32 K%16");
    CHECK(hfa_conv_gemm_f32(64, 64, 64, 1, 1, fp, 0, 0, 64, 1, 0, 64, 64, fmis, 0, 64, nullptr, 0, nullptr, 0,
                                 0, 0, fp, 0, 0, 64, 0, st), "conv_gemm_f32 W misaligned");
    CHECK(hfa_conv_gemm_f32(64, 64, 64, 1, 1, fp, 0, 0, 64, 1, 0, 64, 64, fp, 0, 64, nullptr, 0, nullptr, 0,
                                 0, 0, fp, 0, 0, 64, 7, st), "conv_gemm_f32 epilogue");
    CHECK(hfa_gemm_f32(64, 64, 64, nullptr, 64, fp, 64, nullptr, nullptr, 0, fp, 64, 0, st), "gemm_f32 NULL A");
    CHECK(hfa_conv_gemm_split(-1, 64, 64, 1, 1, hp, 0, 0, 0, 64, 1, 0, 64, 64, hp, 0, 0, 64, nullptr, 0, nullptr, 0, 0, 0, nullptr, 0, fp, nullptr, 0, 0, 0, 64, 0, op, st), "split M<0");
    CHECK(hfa_conv_gemm_split(64, 64, 48, 1, 1, hp, 0, 0, 0, 48, 1, 0, 48, 64, hp, 0, 0, 48, nullptr, 0, nullptr, 0, 0, 0, nullptr, 0, fp, nullptr, 0, 0, 0, 64, 0, op, st), "split K%32");
    CHECK(hfa_conv_gemm_split(64, 64, 64, 1, 1, hmis, 0, 0, 0, 64, 1, 0, 64, 64, hp, 0, 0, 64, nullptr, 0, nullptr, 0, 0, 0, nullptr, 0, fp, nullptr, 0, 0, 0, 64, 0, op, st), "split A misaligned");
    CHECK(hfa_conv_gemm_split(64, 64, 64, 1, 1, hp, 0, 0, 0, 64, 1, 0, 64, 64, hp, 0, 0, 64, nullptr, 0, nullptr, 0, 0, 0, nullptr, 0, nullptr, nullptr, 0, 0, 0, 64, 0, op, st), "split no output");
    CHECK(hfa_conv_gemm_split(64, 64, 64, 1, 1, hp, 0, 0, 0, 64, 1, 0, 64, 64, hp, 0, 0, 64, nullptr, 0, fp, 0, 0, 64, nullptr, 0, nullptr, hp, 0, 0, 0, 64, 0, op, st), "split planes-only + residual");
    CHECK(hfa_conv_gemm_split(64, 64, 64, 1, 1, hp, 0, 0, 0, 64, 1, 0, 64, 64, hp, 0, 0, 64, nullptr, 0, nullptr, 0, 0, 0, nullptr, 0, fmis, nullptr, 0, 0, 0, 64, 0, op, st), "split C misaligned");
    CHECK(hfa_conv_gemm_split(64, 64, 64, 1, 1, hp, 0, 0, 0, 64, 1, 0, 64, 64, hp, 0, 0, 64, nullptr, 0, fp, 0,
                              0, 64, hp, 4096, fp, nullptr, 0, 0, 0, 64, 0, op, st), "split R and Rs together");
    CHECK(hfa_split_f16(-1, 4, fp, 4, hp, 4, 16, op, st), "split_f16 rows<0");
    CHECK(hfa_split_f16(4, 4, nullptr, 4, hp, 4, 16, op, st), "split_f16 NULL x");
    // attention
    CHECK(hfa_attention_f32(-1, 12, 10, 64, 0.125f, fp, 0, 64, fp, 0, 64, fp, 0, 64, fp, 0, 64, nullptr, st),
               "attention_f32 B<0");
    CHECK(hfa_attention_f32(1, 12, 10, 80, 0.125f, fp, 0, 64, fp, 0, 64, fp, 0, 64, fp, 0, 64, nullptr, st),
               "attention_f32 head_dim");
    CHECK(hfa_attention_split(1, 12, 10, 96, 0.125f, hp, 0, 0, 64, hp, 0, 0, 64, hp, 0, 0, 64, hp, 0, 0, 64,
                                   nullptr, st), "attention_split head_dim");
    CHECK(hfa_attention_split_tuning(3), "attention tuning waves=3");
    CHECK(hfa_attention_split_form(8), "attention form 8");
    CHECK(hfa_set_grid_cap(-1), "grid cap -1");
    // norms
    CHECK(hfa_layernorm_f32(10, 6, fp, 8, nullptr, 0, fp, fp, 1e-5f, 0, fp, 8, 0, nullptr, st), "LN C%4");
    CHECK(hfa_layernorm_f32(10, 8, fmis, 8, nullptr, 0, fp, fp, 1e-5f, 0, fp, 8, 0, nullptr, st),
               "LN x misaligned");
    CHECK(hfa_layernorm_f32(10, 8, fp, 8, nullptr, 0, fp, fp, 1e-5f, 5, fp, 8, 0, nullptr, st), "LN act");
    CHECK(hfa_layernorm_split(10, 8, fp, 8, nullptr, 0, fp, fp, 1e-5f, 0, fp, 8, 0, nullptr, hmis, 8, 80, op,
                                   st), "LN planes misaligned");
    CHECK(hfa_layernorm_f32(10, 8, fp, 8, nullptr, 0, fp, fp, 1e-5f, 0, fp, 8, 3, ip, st), "LN rows%T");
    CHECK(hfa_groupnorm_f32(1, 10, 30, 16, fp, 300, 30, fp, fp, 1e-5f, 0, fp, 300, 30, nullptr, ws, st),
               "GN C%G");
    CHECK(hfa_groupnorm_f32(1, 10, 32, 16, nullptr, 320, 32, fp, fp, 1e-5f, 0, fp, 320, 32, nullptr, ws, st),
               "GN NULL x");
    CHECK(hfa_groupnorm_split(1, 10, 192, 16, fp, 1920, 192, fp, fp, 1e-5f, 2, nullptr, 0, 0, nullptr, nullptr,
                                   0, 0, 0, op, ws, st), "GN split no output");
    CHECK(hfa_groupnorm_split(1, 10, 200, 20, fp, 2000, 200, fp, fp, 1e-5f, 2, fp, 2000, 200, nullptr, hp, 2000,
                                   200, 4000, op, ws, st), "GN split Cg%4");
    CHECK(hfa_groupnorm_split(1, 10, 192, 16, fp, 1920, 192, fp, fp, 1e-5f, 2, fp, 1920, 192, nullptr, hp,
                                   1920, 192, 3840, op, nullptr, st), "GN split no workspace");
    if (hfa_groupnorm_workspace_bytes(4, 1000, 192, 16) <= 0) { std::printf("FAIL GN workspace\n"); ++g_fail; }
    // extractor / misc
    CHECK(hfa_conv0_f32(1, 5, fp, 5, fp, nullptr, 1, fp, fp, 1e-5f, ws, fp, 512, nullptr, st), "conv0 N<10");
    CHECK(hfa_conv0_f32(1, 1000, fp, 1000, fp, nullptr, 1, nullptr, fp, 1e-5f, ws, fp, 512, nullptr, st),
               "conv0 NULL gamma");
    CHECK(hfa_conv0_split(1, 1000, fp, 1000, fp, nullptr, 1, fp, fp, 1e-5f, ws, hmis, 512, 99 * 512, op,
                               nullptr, st), "conv0 split misaligned");
    if (hfa_conv0_workspace_bytes(2, 160000) <= 0) { std::printf("FAIL conv0 workspace\n"); ++g_fail; }
    CHECK(hfa_units_gather_f32(-1, 10, 768, fp, 0, 768, 20, 24, 1.7f, fp, 0, 768, nullptr, nullptr, st),
               "gather B<0");
    CHECK(hfa_wav_normalize_f32(2, 100, fp, 100, 1e-7f, fp, 100, nullptr, nullptr, st), "wav_norm no ws");
    CHECK(hfa_wav_normalize_f32(2, 0, fp, 100, 1e-7f, fp, 100, nullptr, ws, st), "wav_norm N=0");
    if (hfa_wav_normalize_workspace_bytes(3) <= 0) { std::printf("FAIL wav workspace\n"); ++g_fail; }
    CHECK(hfa_mask_rows_f32(-1, 10, 4, fp, 40, 4, ip, st), "mask B<0");
    CHECK(hfa_pad_rows_f32(1, 10, nullptr, 10, 2, 14, fp, 14, st), "pad NULL x");
    CHECK(hfa_add_f32(-4, fp, fp, fp, st), "add n<0");
    CHECK(hfa_flag_take(-1, op, op, st), "flag_take n<0");
    CHECK(hfa_flag_take(1, nullptr, op, st), "flag_take NULL flags");
    CHECK(hfa_selftest_erf(-1, fp, fp, fp, st), "erf n<0");
    CHECK(hfa_selftest_gelu(-1, fp, fp, st), "gelu n<0");
    CHECK(hfa_resample_f32(1, 100, fp, 100, 0, 441, fp, 16, 6, ws, fp, 300, st), "resample orig=0");
    CHECK(hfa_resample_chain_edges(1, 100, nullptr, fp, 100, 160, 441, fp, 174, 7, fp, 1155, 1155, ws, fp, 320, 320,
                                   st), "chain edges wd_width >= kwd");
    CHECK(hfa_resample_chain_edges(1, 100, nullptr, fp, 100, 160, 441, fp, 174, 7, fp, 20000, 357, ws, fp, 320, 320,
                                   st), "chain edges window past LDS");
    CHECK(hfa_resample_chain_edges(1, 100, nullptr, fp, 100, 160, 441, fp, 174, 7, fp, 1155, 357, ws, fp, 100, 320,
                                   st), "chain edges y_bs < y_cols");
    CHECK(hfa_resample_chain_edges(1, 100, nullptr, fp, 100, 160, 441, fp, 174, 7, fp, 1155, 357, nullptr, fp, 320,
                                   320, st), "chain edges NULL workspace");
    if (hfa_resample_chain_edges_workspace_bytes(2, 441, 1155, 357) <= 0) { std::printf("FAIL chain workspace\n"); ++g_fail; }
    // WAV front end (host memory): null arguments, a missing file, a non-RIFF file, a short buffer, a bad channel
    {
        int64_t nf = 0;
        int32_t ch = 0, sr = 0;
        float buf[64];
        CHECK(hfa_wav_info(nullptr, &nf, &ch, &sr), "wav_info NULL path");
        CHECK(hfa_wav_info("/nonexistent/x.wav", &nf, &ch, &sr), "wav_info missing file");
        CHECK(hfa_wav_read("/nonexistent/x.wav", 0, buf, 64, &nf, &sr), "wav_read missing file");
        CHECK(hfa_wav_read("/proc/self/cmdline", 0, buf, 64, &nf, &sr), "wav_read not RIFF");
        CHECK(hfa_wav_read(nullptr, 0, buf, 64, &nf, &sr), "wav_read NULL path");
        CHECK(hfa_wav_read("/proc/self/cmdline", 0, nullptr, 64, &nf, &sr), "wav_read NULL dst");
        CHECK(hfa_wav_read("/proc/self/cmdline", 0, buf, -1, &nf, &sr), "wav_read capacity<0");
        const char* tmp = "/tmp/hfa_abi_invalid.wav";   // 16-bit mono, 100 frames
        if (FILE* f = std::fopen(tmp, "wb")) {
            const unsigned char hdr[44] = {'R', 'I', 'F', 'F', 236, 0, 0, 0, 'W', 'A', 'V', 'E', 'f', 'm', 't', ' ',
                                           16, 0, 0, 0, 1, 0, 1, 0, 0x80, 0x3e, 0, 0, 0, 0x7d, 0, 0, 2, 0, 16, 0,
                                           'd', 'a', 't', 'a', 200, 0, 0, 0};
            std::fwrite(hdr, 1, 44, f);
            const short z[100] = {0};
            std::fwrite(z, 2, 100, f);
            std::fclose(f);
            CHECK(hfa_wav_read(tmp, 0, buf, 64, &nf, &sr), "wav_read short buffer");
            CHECK(hfa_wav_read(tmp, 1, buf, 64, &nf, &sr), "wav_read channel 1 of 1");
            CHECK(hfa_wav_read(tmp, -2, buf, 64, &nf, &sr), "wav_read channel -2");
            if (hfa_wav_info(tmp, &nf, &ch, &sr) != 0 || nf != 100 || ch != 1 || sr != 16000) {
                std::printf("FAIL wav_info on a valid file\n");
                ++g_fail;
            }
            std::remove(tmp);
        }
    }
    // host queries and tuning hooks (thread-local state; name strings stay valid, bounded)
    for (int cfg = -1; cfg < 28; ++cfg) {
        const bool built = cfg == 0 || (cfg >= 15 && cfg <= 20) || (cfg >= 23 && cfg <= 25);
        const int rc = hfa_gemm_split_tuning(cfg);   // retired / unknown tiles are refused, the override unchanged
        if ((rc == 0) != built) { std::printf("FAIL split tuning cfg %d rc %d\n", cfg, rc); ++g_fail; }
        const char* n = hfa_gemm_split_kernel_name(15968, 3072, 768, 1, 1, 1, 768);
        if (!n || std::strlen(n) == 0 || std::strlen(n) >= 128) { std::printf("FAIL split name cfg %d\n", cfg); ++g_fail; }
    }
    hfa_gemm_split_tuning(0);
    for (int pipe : {0, 16, 32, 102, 103})
        for (int cfg = 0; cfg < 10; ++cfg) {
            hfa_gemm_tuning(pipe, cfg);
            const char* n = hfa_gemm_kernel_name(1000, 768, 768, 1, 1, fp, 0, 0, 768, 1, 0, 768, 1000, fp, 0, 768,
                                                 nullptr, 0, nullptr, 0, 0, 0, fp, 0, 0, 768, 0);
            if (!n || std::strlen(n) == 0) { std::printf("FAIL gemm name %d %d\n", pipe, cfg); ++g_fail; }
        }
    hfa_gemm_tuning(0, 0);
    if (hfa_resample_workspace_bytes(2, 160000, 160, 256) <= 0) { std::printf("FAIL resample workspace\n"); ++g_fail; }
    std::printf("%d invalid-argument calls, %d failures\n", g_n, g_fail);
    return g_fail ? 1 : 0;
}
