// Probe: does another kernel's work ever change this workgroup's LDS?  Each workgroup fills its LDS with a
// pattern, then re-reads it for `iters` rounds (s_sleep between) and counts words that changed.
// Built by scripts/probes/build_lds_guard.sh into scripts/probes/liblds_guard.so (debug only, not the product).
#include <hip/hip_runtime.h>
#include <cstdint>

template <int WORDS>
__global__ __launch_bounds__(256) void lds_guard_kernel(int iters, unsigned long long* bad, unsigned* first) {
    __shared__ uint32_t s[WORDS];
    const uint32_t tag = 0xA5000000u ^ (blockIdx.x << 12);
    for (int i = threadIdx.x; i < WORDS; i += 256) s[i] = tag ^ (uint32_t)i;
    __syncthreads();
    unsigned long long n = 0;
    for (int it = 0; it < iters; ++it) {
        for (int i = threadIdx.x; i < WORDS; i += 256) {
            const uint32_t v = s[i];
            if (v != (tag ^ (uint32_t)i)) {
                ++n;
                if (atomicCAS(first, 0u, 1u) == 0u) {
                    first[1] = (unsigned)i;
                    first[2] = v;
                    first[3] = blockIdx.x;
                }
                s[i] = tag ^ (uint32_t)i;
            }
        }
        __builtin_amdgcn_s_sleep(20);
    }
    if (n) atomicAdd(bad, n);
}

extern "C" int lds_guard_launch(int blocks, int words_kib, int iters, unsigned long long* bad, unsigned* first,
                                hipStream_t st) {
    if (words_kib == 16)
        hipLaunchKernelGGL((lds_guard_kernel<4096>), dim3(blocks), dim3(256), 0, st, iters, bad, first);
    else if (words_kib == 32)
        hipLaunchKernelGGL((lds_guard_kernel<8192>), dim3(blocks), dim3(256), 0, st, iters, bad, first);
    else
        hipLaunchKernelGGL((lds_guard_kernel<2048>), dim3(blocks), dim3(256), 0, st, iters, bad, first);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
