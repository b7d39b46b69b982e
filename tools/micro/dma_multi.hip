// Semantics probe: LDS-DMA (global_load_lds_dwordx4) issued by several waves of one
// workgroup into disjoint LDS regions, then read back by every wave after a barrier.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void k(const float* __restrict__ src, float* __restrict__ dst, int nload) {
    __shared__ __attribute__((aligned(16))) f32x4 lds[16 * 64];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    // wave w < nload loads rows r = w, w + nload, ... (16 rows of 64 float4)
    if (wave < nload) {
        for (int r = wave; r < 16; r += nload) {
            const float* g = src + ((size_t)blockIdx.x * 16 * 64 + r * 64 + lane) * 4;
            __builtin_amdgcn_global_load_lds(g, lds + r * 64, 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    for (int i = threadIdx.x; i < 16 * 64; i += blockDim.x)
        reinterpret_cast<f32x4*>(dst)[(size_t)blockIdx.x * 16 * 64 + i] = lds[i];
}

int main() {
    const int nb = 64, n = nb * 16 * 64 * 4;
    float *s, *d;
    hipMalloc(&s, n * 4);
    hipMalloc(&d, n * 4);
    float* h = (float*)malloc(n * 4);
    for (int i = 0; i < n; ++i) h[i] = (float)i;
    hipMemcpy(s, h, n * 4, hipMemcpyHostToDevice);
    for (int nload = 1; nload <= 4; nload *= 2) {
        hipMemset(d, 0, n * 4);
        hipLaunchKernelGGL(k, dim3(nb), dim3(512), 0, 0, s, d, nload);
        hipMemcpy(h, d, n * 4, hipMemcpyDeviceToHost);
        int bad = 0, first = -1;
        for (int i = 0; i < n; ++i)
            if (h[i] != (float)i) { if (first < 0) first = i; ++bad; }
        printf("nload %d: %d mismatches (first %d: %f)\n", nload, bad, first, first >= 0 ? h[first] : 0.f);
    }
    return 0;
}
