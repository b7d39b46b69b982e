// walk_probe.hip -- what bounds the scanline passes' memory stream (measurement tooling,
// not the product).  A wave walks one line (or LINES neighbouring lines) of a two-view
// volume of 784/1024/1040-B pixel vectors, K steps prefetched, updating every vector in
// place like k_scan_line (k_scanline.hip), with either a trivial per-step update or one
// that carries a wave-min dependency from step to step (CHAIN).  Prints per-launch time
// and the read + write rate.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/micro/walk_probe.hip -o tools/micro/walk_probe_bin
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <utility>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));

template <int N>
struct IC { static constexpr int value = N; };

__device__ __forceinline__ uint32_t row_min(uint32_t v) {
    // min over each row of 16 lanes by DPP, then across rows with the gfx950 lane swaps
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x141, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x140, 0xF, 0xF, false));
    const auto a = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    v = min((uint32_t)a[0], (uint32_t)a[1]);
    const auto b = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return min((uint32_t)b[0], (uint32_t)b[1]);
}

__device__ __forceinline__ int xcd_remap(int b, int n) {
    const int per = n >> 3;
    return b < 8 * per ? (b & 7) * per + (b >> 3) : b;
}

// MODE 0: in place; 1: read vol, write the second volume out; 2: read only; 3: write only
// EXTRA: per step also the scanline's two side loads (a uniform dword and a per-lane 8-B window
// of a byte map, as k_scan_line's d1 / d2), folded into the chain
template <int K, int LINES, bool NT, bool CHAIN, bool VERT, int MODE = 0, bool EXTRA = false>
__global__ __launch_bounds__(256) void k_walk(float* vol, float* out, int H, int W, int Lp, int Q) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int nl = VERT ? W : H, len = VERT ? H : W;
    const int blk = VERT ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int g = blk * 4 + wv;
    if (g * LINES >= nl) return;
    float* vb = vol + (size_t)blockIdx.y * H * W * Lp;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(vb, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t ws = MODE == 1 ? __builtin_amdgcn_make_buffer_rsrc(out + (size_t)blockIdx.y * H * W * Lp, (short)0, 0x7fffffff, 0x00020000) : rs;
    const uint32_t es = (uint32_t)(VERT ? (size_t)W * Lp * 4 : (size_t)Lp * 4);  // step stride (B)
    uint32_t vo[LINES];
#pragma unroll
    for (int l = 0; l < LINES; ++l) {
        const int line = min(g * LINES + l, nl - 1);
        const uint32_t lo = (uint32_t)(VERT ? (size_t)line * Lp * 4 : (size_t)line * W * Lp * 4);
        vo[l] = lane < Q ? lo + 16u * lane : 0x80000000u;  // lanes past the vector: out of range
    }
    constexpr int aux = NT ? 2 : 0;
    // byte map: the second volume's first bytes, row stride W + 2048
    const __amdgpu_buffer_rsrc_t gs = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, 0x7fffffff, 0x00020000);
    const uint32_t gl = 4u * lane + 1024u, grow = (uint32_t)(g % (VERT ? H : H)) * (uint32_t)(W + 2048);
    uint32_t gd[K], gw[K][2];
    auto side = [&](int k, int r) {
        if constexpr (EXTRA) {
            const uint32_t o = VERT ? (uint32_t)r * (uint32_t)(W + 2048) + (uint32_t)g : grow + (uint32_t)r;
            gd[k] = __builtin_amdgcn_raw_buffer_load_b32(gs, 0u, o & ~3u, 0);
            const auto w = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(gs, gl, o & ~3u, 0));
            gw[k][0] = w.x;
            gw[k][1] = w.y;
        }
    };
    f4 ring[K][LINES];
#pragma unroll
    for (int k = 0; k < K; ++k) {
#pragma unroll
        for (int l = 0; l < LINES; ++l)
            ring[k][l] = MODE == 3 ? f4{1, 2, 3, (float)k} : __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo[l], k * es, 0));
        side(k, k);
        __builtin_amdgcn_sched_barrier(0);
    }
    f4 q[LINES];
    uint32_t mq[LINES];
#pragma unroll
    for (int l = 0; l < LINES; ++l) {
        q[l] = f4{0, 0, 0, 0};
        mq[l] = 0;
    }
    auto step = [&](auto Kc, int r) {
        constexpr int k = decltype(Kc)::value;
#pragma unroll
        for (int l = 0; l < LINES; ++l) {
            const f4 p = ring[k][l];
            f4 np;
            if (CHAIN) {
                float m = __uint_as_float(mq[l]);
                if constexpr (EXTRA) {
                    const uint32_t d1 = ((uint32_t)__builtin_amdgcn_readfirstlane(gd[k]) >> (8 * (r & 3))) & 0xff;
                    const uint32_t gg = __builtin_amdgcn_perm(gw[k][1], gw[k][0], 0x03020100u + (uint32_t)(r & 3) * 0x01010101u);
                    m += (d1 < 16 ? 0.5f : 0.25f) + ((gg & 0xff) < 16 ? 0.125f : 0.f);
                }
                const float lo = __int_as_float(__builtin_amdgcn_update_dpp(0x7f800000, __float_as_int(q[l][3]), 0x138, 0xF, 0xF, false));
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float nb = fminf(e == 0 ? lo : q[l][e - 1], q[l][e]) + 0.25f;
                    np[e] = (p[e] - m + fminf(nb, m + 1.0f)) * 0.5f;
                }
                const uint32_t mn = min(min(__float_as_uint(np[0]), __float_as_uint(np[1])),
                                        min(__float_as_uint(np[2]), __float_as_uint(np[3])));
                mq[l] = row_min(mn);
            } else {
                np = (p + q[l]) * 0.5f;
            }
            q[l] = np;
            if (MODE != 2) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, np), ws, vo[l], (uint32_t)r * es, aux);
            const int rr = min(r + K, len - 1);
            if (MODE != 3) ring[k][l] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo[l], (uint32_t)rr * es, 0));
            else ring[k][l] = np + 1.0f;
        }
        side(k, min(r + K, len - 1));
        __builtin_amdgcn_sched_barrier(0x7);
    };
    for (int b = 0; b < len; b += K) {  // len is a multiple of K
        [&]<int... Ks>(std::integer_sequence<int, Ks...>) {
            (step(IC<Ks>{}, b + Ks), ...);
        }(std::make_integer_sequence<int, K>{});
    }
    if (MODE == 2 && q[0][0] == -1.f) out[0] = q[0][1];  // keeps the read-only walk's loads
}

template <int K, int LINES, bool NT, bool CHAIN, bool VERT, int MODE = 0, bool EXTRA = false>
static void run(const char* name, float* vol, int H, int W, int Lp, int reps, float* out = nullptr) {
    const int Q = Lp / 4;
    const int nl = VERT ? W : H;
    const int waves = (nl + LINES - 1) / LINES;
    int blocks = (waves + 3) / 4;
    if (VERT) blocks = (blocks + 7) / 8 * 8;
    auto launch = [&] {
        hipLaunchKernelGGL((k_walk<K, LINES, NT, CHAIN, VERT, MODE, EXTRA>), dim3(blocks, 2), dim3(256), 0, 0, vol, out, H, W, Lp, Q);
    };
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 2; ++i) launch();
    hipEventRecord(a, 0);
    for (int i = 0; i < reps; ++i) launch();
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    const double bytes = (MODE >= 2 ? 1.0 : 2.0) * 2.0 * H * W * (double)Lp * 4;  // read + write, two views
    printf("%-44s Lp %3d  %8.1f us  %6.0f GB/s  (%d waves, %.0f ns a step)\n", name, Lp, ms * 1e3,
           bytes / (ms * 1e6), 2 * waves, ms * 1e6 / (VERT ? H : W));
    hipEventDestroy(a);
    hipEventDestroy(b);
}

// placement: time the same walk in a series of large allocations kept alive side by side
static int placement(int nbuf, size_t gb) {
    const int H = 720, W = 1280;
    const size_t vol = (size_t)2 * H * W * 196 * 4;
    float* bufs[16] = {};
    for (int i = 0; i < nbuf && i < 16; ++i) {
        if (hipMalloc(&bufs[i], gb << 30) != hipSuccess) { printf("alloc %d failed\n", i); return 1; }
        hipMemset(bufs[i], 0, gb << 30);
        char name[64];
        for (size_t off = 0; off + vol <= (gb << 30); off += (gb << 30) / 3) {
            snprintf(name, sizeof name, "buf %d (%zu GB) at +%zu MB: V walk", i, gb, off >> 20);
            run<8, 1, true, true, true>(name, bufs[i] + off / 4, H, W, 196, 5, bufs[i]);
        }
        fflush(stdout);
    }
    for (int i = 0; i < nbuf && i < 16; ++i) hipFree(bufs[i]);
    return 0;
}

int main(int argc, char** argv) {
    if (argc > 1 && argv[1][0] == 'p') return placement(argc > 2 ? atoi(argv[2]) : 5, argc > 3 ? atoi(argv[3]) : 20);
    const int H = argc > 2 ? atoi(argv[1]) : 720, W = argc > 2 ? atoi(argv[2]) : 1280;  // default: the 0600 pair
    float* vol = nullptr;
    float* out = nullptr;
    if (hipMalloc(&vol, (size_t)2 * H * W * 260 * 4) != hipSuccess) return 1;
    if (hipMalloc(&out, (size_t)2 * H * W * 260 * 4) != hipSuccess) return 1;
    hipMemset(vol, 0, (size_t)2 * H * W * 260 * 4);
    hipMemset(out, 0, (size_t)2 * H * W * 260 * 4);
    const int reps = 5;
    printf("H %d W %d\n", H, W);
    run<16, 1, true, true, false>("H K16 1 line nt chain (k_scan_line<H>)", vol, H, W, 196, reps, out);
    run<16, 1, true, true, false, 0, true>("H K16 1 line nt chain + side loads", vol, H, W, 196, reps, out);
    run<8, 1, true, true, true>("V K8 1 line  nt chain (k_scan_line<V>)", vol, H, W, 196, reps, out);
    run<8, 1, true, true, true, 0, true>("V K8 1 line  nt chain + side loads", vol, H, W, 196, reps, out);
    hipFree(vol);
    hipFree(out);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 2;
}
