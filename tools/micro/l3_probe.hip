// l3_probe.hip -- measurement tooling (not the product): does a working set that fits the
// 256 MiB Infinity Cache (L3) stream faster than HBM when kernels re-read and re-write it
// back to back, as a label-sliced aggregation chain would?  For several working-set sizes:
//   rmw      : x = x * a + b in place, 10 launches back to back (plain loads / stores)
//   rmw_nt   : the same with non-temporal stores
//   fill+read: one fill launch, then a read launch of the same buffer
//   slice    : in place over a 196-B slice of every 784-B "pixel vector" (a quarter of a
//              config-B label vector), the slices' bytes = the working set
// Rates count the bytes the kernels move (read + write).
//   hipcc --offload-arch=gfx950 -O3 -o tools/micro/l3_probe tools/micro/l3_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int TPB = 256;

template <bool NT>
__global__ __launch_bounds__(TPB) void k_rmw(f4* __restrict__ p, size_t n4, float a) {
    const size_t stride = (size_t)gridDim.x * TPB;
    for (size_t i = (size_t)blockIdx.x * TPB + threadIdx.x; i < n4; i += stride) {
        f4 v = p[i];
        v = v * a + 1.0f;
        if (NT) __builtin_nontemporal_store(v, p + i);
        else p[i] = v;
    }
}

// slice of each 784-B vector: 196 B = 12.25 float4 -> 12 float4 + one float (kept simple:
// the first 12 float4 = 192 B of vector k at offset 784 k + 196 s)
__global__ __launch_bounds__(TPB) void k_rmw_slice(float* __restrict__ p, size_t nvec, int s, float a) {
    const size_t stride = (size_t)gridDim.x * TPB;
    const size_t n = nvec * 12;
    for (size_t i = (size_t)blockIdx.x * TPB + threadIdx.x; i < n; i += stride) {
        const size_t v = i / 12, q = i - v * 12;
        f4* e = reinterpret_cast<f4*>(p + v * 196 + (size_t)s * 49) + q;
        f4 x = *e;
        x = x * a + 1.0f;
        *e = x;
    }
}

__global__ __launch_bounds__(TPB) void k_fill(f4* __restrict__ p, size_t n4, float x) {
    const size_t stride = (size_t)gridDim.x * TPB;
    for (size_t i = (size_t)blockIdx.x * TPB + threadIdx.x; i < n4; i += stride) p[i] = f4{x, x, x, x};
}

__global__ __launch_bounds__(TPB) void k_read(const f4* __restrict__ p, size_t n4, float* sink) {
    const size_t stride = (size_t)gridDim.x * TPB;
    f4 acc = f4{0, 0, 0, 0};
    for (size_t i = (size_t)blockIdx.x * TPB + threadIdx.x; i < n4; i += stride) acc += p[i];
    if (acc.x == 12345.f) *sink = acc.y;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
    const size_t MiB = 1 << 20;
    const size_t sizes[] = {64 * MiB, 128 * MiB, 192 * MiB, 256 * MiB, 384 * MiB, 1024 * MiB};
    const size_t maxb = 4096 * MiB;
    float* buf = nullptr;
    float* sink = nullptr;
    CK(hipMalloc(&buf, maxb));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(buf, 0, maxb));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int grid = 256 * 8;
    auto timed = [&](auto fn, int reps) -> double {
        fn();
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0, 0);
        for (int r = 0; r < reps; ++r) fn();
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        return ms / reps;
    };
    std::printf("%10s %12s %12s %12s %12s %12s\n", "MiB", "rmw GB/s", "rmw_nt GB/s", "fill GB/s", "read_after GB/s", "slice GB/s");
    for (size_t S : sizes) {
        const size_t n4 = S / 16;
        f4* p = reinterpret_cast<f4*>(buf);
        const double t_rmw = timed([&] { hipLaunchKernelGGL(k_rmw<false>, dim3(grid), dim3(TPB), 0, 0, p, n4, 0.5f); }, 10);
        const double t_nt = timed([&] { hipLaunchKernelGGL(k_rmw<true>, dim3(grid), dim3(TPB), 0, 0, p, n4, 0.5f); }, 10);
        // fill, then the read right after it (one pair per rep)
        double t_fill = 0, t_read = 0;
        for (int r = 0; r < 5; ++r) {
            // evict: stream a 2 GiB region past the buffer first
            hipLaunchKernelGGL(k_fill, dim3(grid), dim3(TPB), 0, 0, reinterpret_cast<f4*>(buf + maxb / 8), (2048 * MiB) / 16, 1.0f);
            (void)hipEventRecord(e0, 0);
            hipLaunchKernelGGL(k_fill, dim3(grid), dim3(TPB), 0, 0, p, n4, 2.0f);
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            t_fill += ms;
            (void)hipEventRecord(e0, 0);
            hipLaunchKernelGGL(k_read, dim3(grid), dim3(TPB), 0, 0, p, n4, sink);
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
            t_read += ms;
        }
        t_fill /= 5;
        t_read /= 5;
        // slice pattern: vectors whose 196-B slices add up to S
        const size_t nvec = S / 196;
        double t_slice = -1;
        if (nvec * 784 <= maxb)
            t_slice = timed([&] { hipLaunchKernelGGL(k_rmw_slice, dim3(grid), dim3(TPB), 0, 0, buf, nvec, 1, 0.5f); }, 10);
        const double slice_bytes = 2.0 * nvec * 192;
        std::printf("%10zu %12.0f %12.0f %12.0f %12.0f %12.0f\n", S / MiB, 2.0 * S / (t_rmw * 1e-3) / 1e9,
                    2.0 * S / (t_nt * 1e-3) / 1e9, S / (t_fill * 1e-3) / 1e9, S / (t_read * 1e-3) / 1e9,
                    t_slice > 0 ? slice_bytes / (t_slice * 1e-3) / 1e9 : 0.0);
    }
    CK(hipFree(buf));
    return 0;
}
