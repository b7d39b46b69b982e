// Micro benchmark (GPU box): HBM write-only bandwidth for the cost volume's size
// (730 MB, config B), to price the cost build's store side.  Variants: 16-B and 4-B lane
// stores, contiguous grid-stride, plain and non-temporal.
//   hipcc --offload-arch=gfx950 -O3 -o build/micro/write_bw tools/micro/write_bw.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int MODE>  // 0: f4 plain, 1: f4 nt, 2: dword plain
__global__ __launch_bounds__(256) void k_write(float* p, size_t n4, float v) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        if (MODE == 0) reinterpret_cast<f4*>(p)[i] = f4{v, v, v, v};
        if (MODE == 1) __builtin_nontemporal_store(f4{v, v, v, v}, reinterpret_cast<f4*>(p) + i);
        if (MODE == 2) {
            // four dword stores, each a 256-B contiguous wave instruction
            const size_t w = i / blockDim.x * blockDim.x * 4 + threadIdx.x;
            p[w] = v; p[w + 256] = v; p[w + 512] = v; p[w + 768] = v;
        }
    }
}

template <int MODE>
static float run(float* p, size_t bytes, int blocks) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const size_t n4 = bytes / 16;
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k_write<MODE>, dim3(blocks), dim3(256), 0, 0, p, n4, 1.f);
    hipEventRecord(a);
    const int reps = 20;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_write<MODE>, dim3(blocks), dim3(256), 0, 0, p, n4, (float)r);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main() {
    const size_t bytes = (size_t)2 * 375 * 1242 * 196 * 4 / 4096 * 4096;  // one config-B volume
    float* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) return 2;
    const int grids[] = {1024, 4096, 16384};
    for (int g : grids) {
        const float t0 = run<0>(p, bytes, g), t1 = run<1>(p, bytes, g), t2 = run<2>(p, bytes, g);
        printf("grid %5d: f4 plain %.1f us (%.2f TB/s)  f4 nt %.1f us (%.2f TB/s)  dword %.1f us (%.2f TB/s)\n", g,
               t0 * 1e3, bytes / (t0 * 1e-3) / 1e12, t1 * 1e3, bytes / (t1 * 1e-3) / 1e12, t2 * 1e3,
               bytes / (t2 * 1e-3) / 1e12);
    }
    hipFree(p);
    return 0;
}
