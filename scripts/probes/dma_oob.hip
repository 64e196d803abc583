// Probe: buffer_load_dwordx4 ... lds (LDS-DMA) lane layout and out-of-range behaviour on gfx950.
// Prints whether lane l lands at M0 + 16*l and whether an out-of-range voffset writes zeros or leaves LDS as is.
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ inline unsigned lds_addr(const void* p) {
    return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

__global__ void probe(const float* __restrict__ x, int nbytes, int* out) {
    __shared__ __attribute__((aligned(16))) float s[64 * 4];
    for (int i = threadIdx.x; i < 256; i += 64) s[i] = 7.0f;
    __syncthreads();
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, nbytes, 0x00020000);
    const int l = threadIdx.x;
    // lanes 0..47 read chunk (63-l) (reversed); lanes 48..63 read out of range
    unsigned voff = l < 48 ? (unsigned)(63 - l) * 16u : 0x80000000u;
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(r), "s"(lds_addr(s)) : "memory");
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    int ok_layout = 1, oob_zero = 1, oob_keep = 1;
    for (int i = 0; i < 64; ++i) {
        for (int e = 0; e < 4; ++e) {
            float v = s[i * 4 + e];
            if (i < 48) { if (v != x[(63 - i) * 4 + e]) ok_layout = 0; }
            else { if (v != 0.0f) oob_zero = 0; if (v != 7.0f) oob_keep = 0; }
        }
    }
    if (l == 0) { out[0] = ok_layout; out[1] = oob_zero; out[2] = oob_keep; }
}

int main() {
    float h[256];
    for (int i = 0; i < 256; ++i) h[i] = 1.0f + i;
    float* d; int* o; int ho[3];
    hipMalloc(&d, sizeof(h)); hipMalloc(&o, 12);
    hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, (int)sizeof(h), o);
    hipMemcpy(ho, o, 12, hipMemcpyDeviceToHost);
    printf("lane-linear layout ok=%d  oob writes zero=%d  oob leaves LDS=%d\n", ho[0], ho[1], ho[2]);
    return 0;
}
