// attn_params.h — the split attention's launch parameters, shared by attention.hip (the 32-queries-per-wave
// kernel and the C ABI) and attention64.hip (64 queries per wave, built without the VGPR MFMA form).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

struct AttnSP {
    int B, H, L;
    float scale;
    const _Float16* q; long long q_sp, q_bs; int q_ld;
    const _Float16* k; long long k_sp, k_bs; int k_ld;
    const _Float16* v; long long v_sp, v_bs; int v_ld;
    _Float16* o; long long o_sp, o_bs; int o_ld;
    const int32_t* key_len;
};

// attention64.hip: one workgroup of 4 waves = 256 queries of one (batch, head), 64 per wave
void launch_attn_split64(const AttnSP& p, hipStream_t stream);
