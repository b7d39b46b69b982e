// granule_probe.hip -- measurement tooling (not the product): what does a vector that is
// not a whole number of 64-B granules cost when neighbouring vectors are written (or read
// and written) by different waves at different times, as the volume passes do with 784-B
// pixel vectors?  Every wave moves one vector at a time (16 B a lane), vectors visited in
// a scattered order (neighbours far apart in time) or in order.
//   hipcc --offload-arch=gfx950 -O3 -o tools/micro/granule_probe tools/micro/granule_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

// vec_bytes / 16 lanes move one vector; vector v sits at v * stride_bytes
template <bool READ>
__global__ __launch_bounds__(256) void k_vec(char* __restrict__ buf, size_t nvec, int q, size_t stride, int scatter,
                                             char* __restrict__ dst) {
    const int lane = threadIdx.x & 63;
    const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
    for (size_t i = wave; i < nvec; i += nw) {
        const size_t v = scatter ? (i * 7919) % nvec : i;  // 7919 prime, coprime to nvec
        f4* p = reinterpret_cast<f4*>(buf + v * stride) + lane;
        f4* o = reinterpret_cast<f4*>(dst + v * stride) + lane;  // == p: in place
        if (lane < q) {
            if (READ) {
                f4 x = *p;
                x = x * 0.5f + 1.0f;
                __builtin_nontemporal_store(x, o);
            } else {
                __builtin_nontemporal_store(f4{1.f, 2.f, 3.f, 4.f}, p);
            }
        }
    }
}

int main() {
    const size_t total = (size_t)1 << 30;  // 1 GiB of vectors
    char* buf = nullptr;
    char* buf2 = nullptr;
    if (hipMalloc(&buf, total + 4096) != hipSuccess) return 1;
    if (hipMalloc(&buf2, total + 4096) != hipSuccess) return 1;
    (void)hipMemset(buf, 0, total + 4096);
    (void)hipMemset(buf2, 0, total + 4096);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    struct Case { const char* name; int q; size_t stride; };
    const Case cases[] = {{"768 B at 768", 48, 768}, {"784 B at 784", 49, 784}, {"784 B at 832", 49, 832},
                          {"832 B at 832", 52, 832}, {"1024 B at 1024", 64, 1024}};
    std::printf("%-16s %8s %12s %12s %12s %12s %12s %12s\n", "vector", "", "write seq", "write scat", "rmw seq",
                "rmw scat", "r->w2 seq", "r->w2 scat");
    for (const Case& c : cases) {
        const size_t nvec = total / c.stride;
        double r[6];
        int k = 0;
        for (int rd = 0; rd < 3; ++rd)
            for (int sc = 0; sc < 2; ++sc) {
                char* dst = rd == 2 ? buf2 : buf;  // 2: read buf, write buf2 (out of place)
                auto launch = [&]() {
                    if (rd) hipLaunchKernelGGL(k_vec<true>, dim3(4096), dim3(256), 0, 0, buf, nvec, c.q, c.stride, sc, dst);
                    else hipLaunchKernelGGL(k_vec<false>, dim3(4096), dim3(256), 0, 0, buf, nvec, c.q, c.stride, sc, dst);
                };
                launch();
                (void)hipDeviceSynchronize();
                (void)hipEventRecord(e0, 0);
                for (int i = 0; i < 5; ++i) launch();
                (void)hipEventRecord(e1, 0);
                (void)hipEventSynchronize(e1);
                float ms = 0;
                (void)hipEventElapsedTime(&ms, e0, e1);
                const double useful = (double)nvec * c.q * 16 * (rd ? 2 : 1);
                r[k++] = useful / (ms / 5 * 1e-3) / 1e9;
            }
        std::printf("%-16s %8s %12.0f %12.0f %12.0f %12.0f %12.0f %12.0f\n", c.name, "GB/s", r[0], r[1], r[2], r[3],
                    r[4], r[5]);
    }
    (void)hipFree(buf);
    (void)hipFree(buf2);
    return 0;
}
