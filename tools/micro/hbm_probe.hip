// hbm_probe.hip -- HBM calibration kernels for bench.py's hbm_calibration (measurement
// tooling, not the product): hand-written streaming copy / fill / read kernels over a
// buffer the size of one pair's two-view cost volume, so the roofline fractions sit under
// this GPU's own achievable rates rather than under torch's copy_.
//   make probe  ->  tools/lib/libtsm_hbm_probe.so
// C ABI: tsm_hbm_probe(bytes, reps, out[6]) -> 0, out = GB/s of
//   {copy, copy nt, fill, fill nt, read, read nt}  (copy counts read + write bytes)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int TPB = 256;
constexpr int UNR = 4;  // float4 per lane per iteration (4 loads in flight before the stores)

template <bool NT>
__global__ __launch_bounds__(TPB) void k_copy(const f4* __restrict__ src, f4* __restrict__ dst, size_t n4) {
    const size_t stride = (size_t)gridDim.x * TPB * UNR;
    for (size_t base = (size_t)blockIdx.x * TPB * UNR + threadIdx.x; base < n4; base += stride) {
        f4 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const size_t i = base + (size_t)u * TPB;
            v[u] = i < n4 ? (NT ? __builtin_nontemporal_load(src + i) : src[i]) : f4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const size_t i = base + (size_t)u * TPB;
            if (i < n4) {
                if (NT) __builtin_nontemporal_store(v[u], dst + i);
                else dst[i] = v[u];
            }
        }
    }
}

template <bool NT>
__global__ __launch_bounds__(TPB) void k_fill(f4* __restrict__ dst, size_t n4, float x) {
    const size_t stride = (size_t)gridDim.x * TPB * UNR;
    const f4 v = f4{x, x, x, x};
    for (size_t base = (size_t)blockIdx.x * TPB * UNR + threadIdx.x; base < n4; base += stride) {
#pragma unroll
        for (int u = 0; u < UNR; ++u) {  // UNR independent 16-B stores in flight per lane
            const size_t i = base + (size_t)u * TPB;
            if (i < n4) {
                if (NT) __builtin_nontemporal_store(v, dst + i);
                else dst[i] = v;
            }
        }
    }
}

template <bool NT>
__global__ __launch_bounds__(TPB) void k_read(const f4* __restrict__ src, size_t n4, float* __restrict__ sink) {
    const size_t stride = (size_t)gridDim.x * TPB * UNR;
    f4 acc = f4{0, 0, 0, 0};
    for (size_t base = (size_t)blockIdx.x * TPB * UNR + threadIdx.x; base < n4; base += stride) {
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const size_t i = base + (size_t)u * TPB;
            if (i < n4) acc += NT ? __builtin_nontemporal_load(src + i) : src[i];
        }
    }
    if (acc.x + acc.y + acc.z + acc.w == -1.f) sink[0] = 1.f;  // keeps the loads alive
}

template <class F>
static double time_ms(F launch, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) launch();
    hipEventRecord(a, 0);
    for (int i = 0; i < reps; ++i) launch();
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    hipEventDestroy(a);
    hipEventDestroy(b);
    return ms / reps;
}

extern "C" int tsm_hbm_probe(size_t bytes, int reps, double* out) {
    const size_t n4 = bytes / 16;
    f4 *x = nullptr, *y = nullptr;
    float* sink = nullptr;
    if (hipMalloc(&x, n4 * 16) != hipSuccess || hipMalloc(&y, n4 * 16) != hipSuccess ||
        hipMalloc(&sink, 256) != hipSuccess)
        return -1;
    hipMemset(x, 0, n4 * 16);
    int dev = 0, ncu = 256;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const int grid = ncu * 8;  // 8 workgroups (32 waves) per CU, grid-stride
    const double b = (double)n4 * 16;
    out[0] = 2 * b / (time_ms([&] { hipLaunchKernelGGL(k_copy<false>, dim3(grid), dim3(TPB), 0, 0, x, y, n4); }, reps) * 1e6);
    out[1] = 2 * b / (time_ms([&] { hipLaunchKernelGGL(k_copy<true>, dim3(grid), dim3(TPB), 0, 0, x, y, n4); }, reps) * 1e6);
    out[2] = b / (time_ms([&] { hipLaunchKernelGGL(k_fill<false>, dim3(grid), dim3(TPB), 0, 0, y, n4, 1.f); }, reps) * 1e6);
    out[3] = b / (time_ms([&] { hipLaunchKernelGGL(k_fill<true>, dim3(grid), dim3(TPB), 0, 0, y, n4, 1.f); }, reps) * 1e6);
    out[4] = b / (time_ms([&] { hipLaunchKernelGGL(k_read<false>, dim3(grid), dim3(TPB), 0, 0, x, n4, sink); }, reps) * 1e6);
    out[5] = b / (time_ms([&] { hipLaunchKernelGGL(k_read<true>, dim3(grid), dim3(TPB), 0, 0, x, n4, sink); }, reps) * 1e6);
    hipFree(x);
    hipFree(y);
    hipFree(sink);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -2;
}
