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
__device__ __forceinline__ float vec_min(const f32x4 (&x)[J], int lane, int Q, int L, int from = 0) {
    float m = __int_as_float(0x7f800000);
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int q = lane + 64 * j;
        if (q < Q) {
            const int d = 4 * q;
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (d + e < L && d + e >= from) m = fminf(m, x[j][e]);
        }
    }
    return wave_min_nonneg(m);
}

// WTA over indices [minD, L-1], first minimum (strict <, ADCensus.cpp:1404): the first d
// whose cost equals the wave minimum, found by a ballot (no 64-bit shuffle reduction).
// `m` is the wave min over [0, L); recomputed over [minD, L) when minD > 0.
template <int J>
__device__ __forceinline__ int vec_argmin(const f32x4 (&x)[J], int lane, int Q, int L, int minD, float m) {
    if (minD > 0) m = vec_min<J>(x, lane, Q, L, minD);
    if (!(m < 3.402823466e+38f)) return minD;  // nothing below FLT_MAX: reference leaves it unset
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int q = lane + 64 * j;
        int first = 4;
        if (q < Q) {
#pragma unroll
            for (int e = 3; e >= 0; --e) {
                const int d = 4 * q + e;
                if (d < L && d >= minD && x[j][e] == m) first = e;
            }
        }
        const uint64_t mask = __ballot(first < 4);
        if (mask) {
            const int ln = __builtin_ctzll(mask);
            const int e = __builtin_amdgcn_readlane(first, ln);
            return 4 * (ln + 64 * j) + e;
        }
    }
    return minD;
}

// One partialOptimization step (ADCensus.cpp:869-913) for the wave's pixel p given its
// predecessor q (registers).  g[j] packs the four d2 bytes (other-view colour difference,
// or colorDiff+1 when out of range) of this lane's disparities.
// Scalars the hot loop needs, pinned in SGPRs: an empty asm makes each value opaque,
// so the compiler cannot rematerialise it from kernarg memory (a scalar load + lgkmcnt(0)
// wait per use inside the serial loop).
struct ScanConst {
    int L, Q, cd, minD, W;
    float p1[3], p2[3];
};
__device__ __forceinline__ ScanConst scan_const(const DevParams& P) {
    ScanConst c{P.L, P.Lp >> 2, P.color_diff, P.minD, P.W,
                {P.p1t[0], P.p1t[1], P.p1t[2]}, {P.p2t[0], P.p2t[1], P.p2t[2]}};
    asm volatile("" : "+s"(c.L), "+s"(c.Q), "+s"(c.cd), "+s"(c.minD), "+s"(c.W));
    asm volatile("" : "+s"(c.p1[0]), "+s"(c.p1[1]), "+s"(c.p1[2]), "+s"(c.p2[0]), "+s"(c.p2[1]), "+s"(c.p2[2]));
    return c;
}

template <int J>
__device__ __forceinline__ void partial_opt(f32x4 (&p)[J], const f32x4 (&q)[J], float mq, int d1,
                                            const uint32_t (&g)[J], int lane, const ScanConst& C) {
    const int L = C.L, Q = C.Q;
    const int cd = C.cd;
    const int s1 = d1 < cd ? 1 : 0;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        // neighbours across the float4 boundary: d-1 of element 0, d+1 of element 3
        float lo = dpp_f<DPP_WAVE_SHR1>(q[j][3], 0.f);
        float hi = dpp_f<DPP_WAVE_SHL1>(q[j][0], 0.f);
        if (j > 0) {
            const float prev = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(q[j - 1][3]), 63));
            if (lane == 0) lo = prev;
        }
        if (j + 1 < J) {
            const float nxt = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(q[j + 1][0]), 0));
            if (lane == 63) hi = nxt;
        }
        const int qi = lane + 64 * j;
        if (qi >= Q) continue;
        const float qe[6] = {lo, q[j][0], q[j][1], q[j][2], q[j][3], hi};
        f32x4 pe = p[j];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int d = 4 * qi + k;
            if (d >= L) break;
            const int d2 = (g[j] >> (8 * k)) & 0xff;
            const int cnt = s1 + (d2 < cd ? 1 : 0);
            const float p1 = cnt == 2 ? C.p1[2] : (cnt == 1 ? C.p1[1] : C.p1[0]);
            const float p2 = cnt == 2 ? C.p2[2] : (cnt == 1 ? C.p2[1] : C.p2[0]);
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
        p[j] = pe;
    }
}

// ---------------------------------------------------------------------------
// One wave walks one line (a column for vertical passes, a row for horizontal ones) of
// one view.  Everything a step needs that does not depend on the chain -- the pixel's
// L-vector, the uniform d1 and the per-disparity d2 bytes -- is prefetched K steps ahead
// into a register ring, so the serial critical path is only the update + wave min.
// The leftward horizontal pass is the last one: it emits the WTA disparity of every
// pixel and, for view 1 (only needed for the WTA), can skip storing the volume.
// ---------------------------------------------------------------------------
constexpr int SC_K = 8;  // prefetch depth (steps)

template <int J, bool HORIZ>
struct LineStep {
    f32x4 p[J];
    uint32_t g[J];
    int d1;
};

template <int J, bool HORIZ>
__device__ __forceinline__ void scan_issue(LineStep<J, HORIZ>& st, int it, int n, int dir, int line,
                                           const float* base, size_t es, const uint8_t* gown,
                                           const uint8_t* goth, int sgn, int lane,
                                           const ScanConst& C) {
    const int Q = C.Q;
    const int len = n + 1;
    const int pos = dir > 0 ? 1 + it : len - 2 - it;  // w1 (HORIZ) or h1 (vertical)
    const int pm = dir > 0 ? pos : pos + 1;            // max(pos, predecessor)
    const float* ptr = base + (size_t)pos * es;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int q = lane + 64 * j;
        st.p[j] = q < Q ? *reinterpret_cast<const f32x4*>(ptr + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const int W = C.W;
    const int cd1 = C.cd + 1;
    // d1's address is wave-uniform; a scalar load would need lgkmcnt(0) at its use and
    // serialise the prefetch, so the index is moved to a VGPR to get an ordered vector load
    int d1_idx = HORIZ ? pm : pm * W + line;
    asm volatile("v_mov_b32 %0, %1" : "=v"(d1_idx) : "v"(d1_idx));
    st.d1 = gown[d1_idx];
    if (HORIZ) {
        const int off = dir > 0 ? 0 : 1;  // max(x1, x2) - x1
#pragma unroll
        for (int j = 0; j < J; ++j) {
            uint32_t g = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int d = 4 * (lane + 64 * j) + e;
                const int x1 = pos + sgn * (d + C.minD);
                const int x2 = x1 - dir;
                const bool in = x1 >= 0 && x1 < W && x2 >= 0 && x2 < W && d < C.L;
                const uint32_t b = in ? goth[x1 + off] : (uint32_t)cd1;
                g |= b << (8 * e);
            }
            st.g[j] = g;
        }
    } else {
        const uint8_t* grow = goth + (size_t)pm * W;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            uint32_t g = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int d = 4 * (lane + 64 * j) + e;
                const int x = line + sgn * (d + C.minD);
                const uint32_t b = (x >= 0 && x < W && d < C.L) ? grow[x] : (uint32_t)cd1;
                g |= b << (8 * e);
            }
            st.g[j] = g;
        }
    }
}

template <int J, bool HORIZ>
__global__ __launch_bounds__(256) void k_scan_line(float* __restrict__ vol,
                                                   const uint8_t* __restrict__ grad,
                                                   const uint32_t* __restrict__ img, int dir,
                                                   int32_t* __restrict__ wta, int store_view1,
                                                   DevParams Pk) {
    const DevParams P = Pk;  // kernel args -> registers once (no per-use kernarg reloads)
    const int H = P.H, W = P.W, Lp = P.Lp, Q = Lp >> 2;
    const int lane = threadIdx.x & 63;
    const int line = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    const int v = blockIdx.y;
    if (line >= (HORIZ ? H : W)) return;
    const int len = HORIZ ? W : H;
    const size_t es = HORIZ ? (size_t)Lp : (size_t)W * Lp;
    float* base = vol + (size_t)v * H * W * Lp + (HORIZ ? (size_t)line * W * Lp : (size_t)line * Lp);
    const uint8_t* gown = grad + (size_t)v * H * W + (HORIZ ? (size_t)line * W : 0);
    const uint8_t* goth = grad + (size_t)(1 - v) * H * W + (HORIZ ? (size_t)line * W : 0);
    const uint32_t* im = img + (size_t)v * H * W;
    const int sgn = v == 0 ? 1 : -1;
    const int n = len - 1;
    const int T = P.omp_threads;
    const bool store = !(wta && v == 1 && !store_view1);
    int32_t* wrow = wta ? wta + ((size_t)v * H + line) * W : nullptr;  // only HORIZ passes emit WTA
    const ScanConst C = scan_const(P);

    f32x4 q[J];
    const int p0 = dir > 0 ? 0 : len - 1;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int qq = lane + 64 * j;
        q[j] = qq < Q ? *reinterpret_cast<const f32x4*>(base + (size_t)p0 * es + 4 * qq) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    float mq = vec_min<J>(q, lane, Q, P.L);
    if (wrow) {
        const int d = vec_argmin<J>(q, lane, Q, P.L, P.minD, mq);
        if (lane == 0) wrow[p0] = d;
    }
    f32x4 qorig[J];
    float mqorig = mq;
#pragma unroll
    for (int j = 0; j < J; ++j) qorig[j] = q[j];

    LineStep<J, HORIZ> ring[SC_K];
#pragma unroll
    for (int k = 0; k < SC_K; ++k)
        if (k < n) scan_issue<J, HORIZ>(ring[k], k, n, dir, line, base, es, gown, goth, sgn, lane, C);

    for (int b = 0; b < n; b += SC_K) {
#pragma unroll
        for (int k = 0; k < SC_K; ++k) {
            const int it = b + k;
            if (it < n) {
                f32x4 p[J];
                uint32_t g[J];
#pragma unroll
                for (int j = 0; j < J; ++j) { p[j] = ring[k].p[j]; g[j] = ring[k].g[j]; }
                const int d1 = ring[k].d1;
                if (it + SC_K < n)
                    scan_issue<J, HORIZ>(ring[k], it + SC_K, n, dir, line, base, es, gown, goth, sgn, lane, C);
                const int pos = dir > 0 ? 1 + it : len - 2 - it;
                const int pred = pos - dir;
                if (T > 1 && omp_chunk_start(it, n, T)) {  // stale predecessor (racy schedule)
#pragma unroll
                    for (int j = 0; j < J; ++j) q[j] = qorig[j];
                    mq = mqorig;
                }
                const bool keep = T > 1 && omp_chunk_start(it + 1, n, T);
                if (keep) {
#pragma unroll
                    for (int j = 0; j < J; ++j) qorig[j] = p[j];
                    mqorig = vec_min<J>(p, lane, C.Q, C.L);
                }
                const bool masked = P.mask && (HORIZ ? im[(size_t)line * W + pred] : im[(size_t)pred * W + line]) == 0;
                if (!(masked || mq == 0.f)) {  // :880-881 -- else p stays untouched
                    partial_opt<J>(p, q, mq, d1, g, lane, C);
                    if (store) {
#pragma unroll
                        for (int j = 0; j < J; ++j) {
                            const int qq = lane + 64 * j;
                            if (qq < Q) *reinterpret_cast<f32x4*>(base + (size_t)pos * es + 4 * qq) = p[j];
                        }
                    }
                }
#pragma unroll
                for (int j = 0; j < J; ++j) q[j] = p[j];
                mq = vec_min<J>(q, lane, C.Q, C.L);
                if (wrow) {
                    const int d = vec_argmin<J>(q, lane, C.Q, C.L, C.minD, mq);
                    if (lane == 0) wrow[pos] = d;
                }
            }
        }
    }
}

template <bool HORIZ>
static int launch_scan(float* vol, const uint8_t* grad, const uint32_t* img, int dir, int32_t* wta,
                       int store_view1, const DevParams& P, hipStream_t st) {
    const int J = (P.Lp / 4 + 63) / 64;
    dim3 g(((HORIZ ? P.H : P.W) + 3) / 4, 2);
    switch (J) {
        case 1: hipLaunchKernelGGL((k_scan_line<1, HORIZ>), g, dim3(256), 0, st, vol, grad, img, dir, wta, store_view1, P); break;
        case 2: hipLaunchKernelGGL((k_scan_line<2, HORIZ>), g, dim3(256), 0, st, vol, grad, img, dir, wta, store_view1, P); break;
        default: return -1;
    }
    trace_point(HORIZ ? "k_scan_line<H>" : "k_scan_line<V>", st);
    return 0;
}

int launch_scan_vertical(float* vol, const uint8_t* gv, const uint32_t* img, int dir,
                         const DevParams& P, hipStream_t st) {
    return launch_scan<false>(vol, gv, img, dir, nullptr, 1, P, st);
}

int launch_scan_horizontal(float* vol, const uint8_t* gh, const uint32_t* img, int dir,
                           int32_t* wta, int store_view1, const DevParams& P, hipStream_t st) {
    return launch_scan<true>(vol, gh, img, dir, wta, store_view1, P, st);
}

}  // namespace tsm
