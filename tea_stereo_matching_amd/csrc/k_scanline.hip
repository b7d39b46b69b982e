// k_scanline.hip -- step 3 of AD-Census on gfx950: scanline optimisation
// (scanlineOptimize, ADCensus.cpp:997-1011; scanline :983-995; partialOptimization
// :869-913; computeP1P2 :915-981) and the WTA (cost2disparity :1394-1413) fused into
// the last pass.
//
// The four passes per view are CHAINED and IN PLACE: every pixel reads its predecessor's
// already-updated L-vector.  The reference parallelises each pass over the recursion
// dimension (a data race); the kernels implement the serial semantics: one wave owns one
// line (a column for the vertical passes, a row for the horizontal ones) and walks it,
// keeping the predecessor vector in registers (lanes own 4 consecutive disparities), so
// the min over disparities is a wave reduction and the d+-1 neighbours are DPP lane
// shifts.  Optional emulation of the race's lock-step outcome for T threads: the first
// pixel of each of the T static chunks reads its predecessor's pre-pass vector.
#include "tsm_device.h"
#include "tsm_launch.h"

namespace tsm {

// OpenMP static schedule (libgomp / vcomp): first n%T threads take q+1 iterations.
__device__ __forceinline__ bool omp_chunk_start(int it, int n, int T) {
    if (T <= 1 || n <= 0 || it == 0) return false;
    const int q = n / T, r = n % T;
    // chunk t starts at t*q + min(t, r)
    if (q == 0) return it < r; // every thread owns one iteration
    int t;
    if (it < r * (q + 1)) {
        if (it % (q + 1) != 0) return false;
        t = it / (q + 1);
    } else {
        const int k = it - r * (q + 1);
        if (k % q != 0) return false;
        t = r + k / q;
    }
    return t > 0 && t < T;
}

template <int J>
__device__ __forceinline__ float vec_min(const float4 (&x)[J], int lane, int Q, int L) {
    float m = __int_as_float(0x7f800000);
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int q = lane + 64 * j;
        if (q < Q) {
            const int d = 4 * q;
            if (d + 0 < L) m = fminf(m, x[j].x);
            if (d + 1 < L) m = fminf(m, x[j].y);
            if (d + 2 < L) m = fminf(m, x[j].z);
            if (d + 3 < L) m = fminf(m, x[j].w);
        }
    }
    return wave_min_nonneg(m);
}

// WTA over indices [minD, L-1] with the first minimum winning (strict <, :1404).
template <int J>
__device__ __forceinline__ int vec_argmin(const float4 (&x)[J], int lane, int Q, int L, int minD) {
    uint64_t best = ~0ull;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int q = lane + 64 * j;
        if (q < Q) {
            const float e[4] = {x[j].x, x[j].y, x[j].z, x[j].w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int d = 4 * q + k;
                if (d >= minD && d < L) {
                    const uint64_t key = ((uint64_t)__float_as_uint(e[k]) << 32) | (uint32_t)d;
                    best = key < best ? key : best;
                }
            }
        }
    }
    best = wave_min_u64(best);
    const uint32_t bits = (uint32_t)(best >> 32);
    // nothing strictly below FLT_MAX: the reference leaves the pixel uninitialised; we
    // return minD (defined behaviour, same as the oracle).
    if (best == ~0ull || !(__uint_as_float(bits) < 3.402823466e+38f)) return minD;
    return (int)(uint32_t)best;
}

// One partialOptimization step for the wave's pixel p given predecessor q (registers).
//   gsel(d) returns d2 (colour difference on the other view at the shifted column).
template <int J, typename G>
__device__ __forceinline__ void partial_opt(float4 (&p)[J], const float4 (&q)[J], float mq, int d1,
                                            G gsel, int lane, int Q, const DevParams& P) {
    const int L = P.L;
    const int cd = P.color_diff;
    const int s1 = d1 < cd ? 1 : 0;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        // neighbours across the float4 boundary: d-1 of element 0, d+1 of element 3
        float lo = dpp_f<DPP_WAVE_SHR1>(q[j].w, 0.f);
        float hi = dpp_f<DPP_WAVE_SHL1>(q[j].x, 0.f);
        if (j > 0) {
            const float prev = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(q[j - 1].w), 63));
            if (lane == 0) lo = prev;
        }
        if (j + 1 < J) {
            const float nxt = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(q[j + 1].x), 0));
            if (lane == 63) hi = nxt;
        }
        const int qi = lane + 64 * j;
        if (qi >= Q) continue;
        const float qe[6] = {lo, q[j].x, q[j].y, q[j].z, q[j].w, hi};
        float pe[4] = {p[j].x, p[j].y, p[j].z, p[j].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int d = 4 * qi + k;
            if (d >= L) break;
            const int d2 = gsel(d);
            const int cnt = s1 + (d2 < cd ? 1 : 0);
            const float p1 = P.p1t[cnt], p2 = P.p2t[cnt];
            const float cost = pe[k] - mq;
            float mo = mq + p2;
            const float t0 = qe[k + 1];
            if (mo > t0) mo = t0;
            if (d != 0) {
                const float t = qe[k] + p1;
                if (mo > t) mo = t;
            }
            if (d != L - 1) {
                const float t = qe[k + 2] + p1;
                if (mo > t) mo = t;
            }
            pe[k] = (cost + mo) / 2;
        }
        p[j] = make_float4(pe[0], pe[1], pe[2], pe[3]);
    }
}

template <int J>
__device__ __forceinline__ void load_vec(float4 (&x)[J], const float* ptr, int lane, int Q) {
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int q = lane + 64 * j;
        if (q < Q) x[j] = *reinterpret_cast<const float4*>(ptr + 4 * q);
        else x[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
}
template <int J>
__device__ __forceinline__ void store_vec(const float4 (&x)[J], float* ptr, int lane, int Q) {
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int q = lane + 64 * j;
        if (q < Q) *reinterpret_cast<float4*>(ptr + 4 * q) = x[j];
    }
}

// ---------------------------------------------------------------------------
// vertical passes: one wave per (column, view); dir = +1 (down) or -1 (up)
// ---------------------------------------------------------------------------
template <int J>
__global__ __launch_bounds__(256) void k_scan_vertical(float* __restrict__ vol,
                                                       const uint8_t* __restrict__ gv,
                                                       const uint32_t* __restrict__ img,
                                                       int dir, DevParams P) {
    const int H = P.H, W = P.W, Lp = P.Lp, Q = Lp >> 2;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    const int v = blockIdx.y;
    if (w >= W) return;
    const size_t rs = (size_t)W * Lp; // floats per image row
    float* col = vol + (size_t)v * H * rs + (size_t)w * Lp;
    const uint8_t* gown = gv + (size_t)v * H * W;
    const uint8_t* goth = gv + (size_t)(1 - v) * H * W;
    const uint32_t* im = img + (size_t)v * H * W;
    const int sgn = v == 0 ? 1 : -1;
    const int n = H - 1;
    const int T = P.omp_threads;

    float4 q[J], p[J], pn[J];
    const int h0 = dir > 0 ? 0 : H - 1;
    load_vec<J>(q, col + (size_t)h0 * rs, lane, Q);
    float mq = vec_min<J>(q, lane, Q, P.L);
    float4 qorig[J];
    float mqorig = mq;
#pragma unroll
    for (int j = 0; j < J; ++j) qorig[j] = q[j];
    if (n > 0) load_vec<J>(pn, col + (size_t)(dir > 0 ? 1 : H - 2) * rs, lane, Q);
    for (int it = 0; it < n; ++it) {
        const int h1 = dir > 0 ? 1 + it : H - 2 - it;
        const int h2 = h1 - dir;
#pragma unroll
        for (int j = 0; j < J; ++j) p[j] = pn[j];
        if (it + 1 < n) load_vec<J>(pn, col + (size_t)(h1 + dir) * rs, lane, Q);
        if (T > 1 && omp_chunk_start(it, n, T)) { // stale predecessor (racy schedule)
#pragma unroll
            for (int j = 0; j < J; ++j) q[j] = qorig[j];
            mq = mqorig;
        }
        // keep this pixel's pre-pass vector for a possible chunk start at it+1
        const bool keep = T > 1 && omp_chunk_start(it + 1, n, T);
        if (keep) {
#pragma unroll
            for (int j = 0; j < J; ++j) qorig[j] = p[j];
            mqorig = vec_min<J>(p, lane, Q, P.L);
        }
        const bool masked = P.mask && im[(size_t)h2 * W + w] == 0; // :824
        if (masked || mq == 0.f) { // :880-881 -- p untouched
#pragma unroll
            for (int j = 0; j < J; ++j) q[j] = p[j];
            mq = keep ? mqorig : vec_min<J>(p, lane, Q, P.L);
            continue;
        }
        const int hm = h1 > h2 ? h1 : h2;
        const int d1 = gown[(size_t)hm * W + w];
        const uint8_t* grow = goth + (size_t)hm * W;
        const int minD = P.minD, cd1 = P.color_diff + 1;
        auto gsel = [&](int d) -> int {
            const int x = w + sgn * (d + minD);
            return (x >= 0 && x < W) ? (int)grow[x] : cd1;
        };
        partial_opt<J>(p, q, mq, d1, gsel, lane, Q, P);
        store_vec<J>(p, col + (size_t)h1 * rs, lane, Q);
#pragma unroll
        for (int j = 0; j < J; ++j) q[j] = p[j];
        mq = vec_min<J>(q, lane, Q, P.L);
    }
}

// ---------------------------------------------------------------------------
// horizontal passes: one wave per (row, view); dir = +1 (rightward) or -1 (leftward).
// The leftward pass is the last one: it emits the WTA disparity of every pixel and,
// for view 1 (only needed for the WTA), can skip storing the volume.
// ---------------------------------------------------------------------------
template <int J>
__global__ __launch_bounds__(256) void k_scan_horizontal(float* __restrict__ vol,
                                                         const uint8_t* __restrict__ gh,
                                                         const uint32_t* __restrict__ img,
                                                         int dir, int32_t* __restrict__ wta,
                                                         int store_view1, DevParams P) {
    const int H = P.H, W = P.W, Lp = P.Lp, Q = Lp >> 2;
    const int lane = threadIdx.x & 63;
    const int h = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    const int v = blockIdx.y;
    if (h >= H) return;
    float* row = vol + ((size_t)v * H + h) * W * Lp;
    const uint8_t* gown = gh + ((size_t)v * H + h) * W;
    const uint8_t* goth = gh + ((size_t)(1 - v) * H + h) * W;
    const uint32_t* im = img + ((size_t)v * H + h) * W;
    const int sgn = v == 0 ? 1 : -1;
    const int n = W - 1;
    const int T = P.omp_threads;
    const bool store = !(wta && v == 1 && !store_view1);
    int32_t* wrow = wta ? wta + ((size_t)v * H + h) * W : nullptr;

    float4 q[J], p[J], pn[J];
    const int w0 = dir > 0 ? 0 : W - 1;
    load_vec<J>(q, row + (size_t)w0 * Lp, lane, Q);
    float mq = vec_min<J>(q, lane, Q, P.L);
    if (wrow) {
        const int d = vec_argmin<J>(q, lane, Q, P.L, P.minD);
        if (lane == 0) wrow[w0] = d;
    }
    float4 qorig[J];
    float mqorig = mq;
#pragma unroll
    for (int j = 0; j < J; ++j) qorig[j] = q[j];
    if (n > 0) load_vec<J>(pn, row + (size_t)(dir > 0 ? 1 : W - 2) * Lp, lane, Q);
    for (int it = 0; it < n; ++it) {
        const int w1 = dir > 0 ? 1 + it : W - 2 - it;
        const int w2 = w1 - dir;
#pragma unroll
        for (int j = 0; j < J; ++j) p[j] = pn[j];
        if (it + 1 < n) load_vec<J>(pn, row + (size_t)(w1 + dir) * Lp, lane, Q);
        if (T > 1 && omp_chunk_start(it, n, T)) {
#pragma unroll
            for (int j = 0; j < J; ++j) q[j] = qorig[j];
            mq = mqorig;
        }
        const bool keep = T > 1 && omp_chunk_start(it + 1, n, T);
        if (keep) {
#pragma unroll
            for (int j = 0; j < J; ++j) qorig[j] = p[j];
            mqorig = vec_min<J>(p, lane, Q, P.L);
        }
        const bool masked = P.mask && im[w2] == 0; // :862
        if (!(masked || mq == 0.f)) {
            const int d1 = gown[w1 > w2 ? w1 : w2];
            const int minD = P.minD, cd1 = P.color_diff + 1;
            const int off = dir > 0 ? 0 : 1; // max(x1, x2) - x1
            auto gsel = [&](int d) -> int {
                const int x1 = w1 + sgn * (d + minD);
                const int x2 = w2 + sgn * (d + minD);
                const bool in = x1 >= 0 && x1 < W && x2 >= 0 && x2 < W;
                return in ? (int)goth[x1 + off] : cd1;
            };
            partial_opt<J>(p, q, mq, d1, gsel, lane, Q, P);
            if (store) store_vec<J>(p, row + (size_t)w1 * Lp, lane, Q);
        }
#pragma unroll
        for (int j = 0; j < J; ++j) q[j] = p[j];
        mq = vec_min<J>(q, lane, Q, P.L);
        if (wrow) {
            const int d = vec_argmin<J>(q, lane, Q, P.L, P.minD);
            if (lane == 0) wrow[w1] = d;
        }
    }
}

int launch_scan_vertical(float* vol, const uint8_t* gv, const uint32_t* img, int dir,
                         const DevParams& P, hipStream_t st) {
    const int J = (P.Lp / 4 + 63) / 64;
    dim3 g((P.W + 3) / 4, 2);
    switch (J) {
        case 1: hipLaunchKernelGGL((k_scan_vertical<1>), g, dim3(256), 0, st, vol, gv, img, dir, P); trace_point("k_scan_vertical<1>", st); return 0;
        case 2: hipLaunchKernelGGL((k_scan_vertical<2>), g, dim3(256), 0, st, vol, gv, img, dir, P); trace_point("k_scan_vertical<2>", st); return 0;
        case 3: hipLaunchKernelGGL((k_scan_vertical<3>), g, dim3(256), 0, st, vol, gv, img, dir, P); trace_point("k_scan_vertical<3>", st); return 0;
        case 4: hipLaunchKernelGGL((k_scan_vertical<4>), g, dim3(256), 0, st, vol, gv, img, dir, P); trace_point("k_scan_vertical<4>", st); return 0;
        default: return -1;
    }
}

int launch_scan_horizontal(float* vol, const uint8_t* gh, const uint32_t* img, int dir,
                           int32_t* wta, int store_view1, const DevParams& P, hipStream_t st) {
    const int J = (P.Lp / 4 + 63) / 64;
    dim3 g((P.H + 3) / 4, 2);
    switch (J) {
        case 1: hipLaunchKernelGGL((k_scan_horizontal<1>), g, dim3(256), 0, st, vol, gh, img, dir, wta, store_view1, P); trace_point("k_scan_horizontal<1>", st); return 0;
        case 2: hipLaunchKernelGGL((k_scan_horizontal<2>), g, dim3(256), 0, st, vol, gh, img, dir, wta, store_view1, P); trace_point("k_scan_horizontal<2>", st); return 0;
        case 3: hipLaunchKernelGGL((k_scan_horizontal<3>), g, dim3(256), 0, st, vol, gh, img, dir, wta, store_view1, P); trace_point("k_scan_horizontal<3>", st); return 0;
        case 4: hipLaunchKernelGGL((k_scan_horizontal<4>), g, dim3(256), 0, st, vol, gh, img, dir, wta, store_view1, P); trace_point("k_scan_horizontal<4>", st); return 0;
        default: return -1;
    }
}

}  // namespace tsm
