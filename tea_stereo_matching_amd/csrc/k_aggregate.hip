// k_aggregate.hip -- step 2 of AD-Census on gfx950: cross arms (computeLimit,
// ADCensus.cpp:604-659), cross-window sizes and the 1-D arm aggregation passes
// (aggregation1D :685-723 / aggregation2D :725-751 / costAggregate :753-793).
//
// The reference sums each arm window SEQUENTIALLY in fp32 from -arm to +arm; the kernel
// keeps that exact order (no prefix sums), so aggregated volumes are bit-identical.
// One workgroup owns a whole line (an image row for horizontal passes, a column for
// vertical ones) of one view and streams along it in segments of SEG pixels through an
// LDS ring holding the segment plus +-A halo (A = maxLength1-1, the longest arm): every
// input vector is read from HBM once per pass and the pass runs IN PLACE.  A wave owns
// one output pixel at a time: the arm lengths are wave-uniform, lanes own 4 consecutive
// disparities and every LDS read is one conflict-free ds_read_b128 per lane.
#include "tsm_device.h"
#include "tsm_launch.h"

namespace tsm {

// computeLimit, ADCensus.cpp:604-659 (returns the arm length; one shorter when the walk
// ends at the image border, :650-658).
__device__ int compute_limit(const DevParams& P, const uint32_t* __restrict__ im, int h, int w,
                             int dH, int dW) {
    const int H = P.H, W = P.W;
    const uint32_t p = im[(size_t)h * W + w];
    int d = 1;
    int h1 = h + dH, w1 = w + dW;
    uint32_t p2 = p;
    bool inside = 0 <= h1 && h1 < H && 0 <= w1 && w1 < W;
    if (inside) {
        bool colorCond = true, wLimitCond = true, fColorCond = true;
        while (colorCond && wLimitCond && fColorCond && inside) {
            const uint32_t p1 = im[(size_t)h1 * W + w1];
            if (P.mask && p1 == 0) { d++; break; } // :625-629
            if (P.color_model == 0) {
                colorCond = color_diff(P, p, p1) < P.color_thresh1 &&
                            color_diff(P, p1, p2) < P.color_thresh1;
                fColorCond = (d <= P.max_length2) ||
                             (d > P.max_length2 && color_diff(P, p, p1) < P.color_thresh2);
            } else {
                // :632-636, :641-645 -- the saturation conditions are overwritten by the
                // intensity ones in the reference; only intensity survives.
                colorCond = iabs_(ch(p, 2) - ch(p1, 2)) < P.int_thresh1 &&
                            iabs_(ch(p1, 2) - ch(p2, 2)) < P.int_thresh1;
                fColorCond = (d <= P.max_length2) ||
                             (d > P.max_length2 && iabs_(ch(p, 2) - ch(p1, 2)) < P.int_thresh2);
            }
            wLimitCond = d < P.max_length1;
            p2 = p1;
            h1 += dH;
            w1 += dW;
            inside = 0 <= h1 && h1 < H && 0 <= w1 && w1 < W;
            d++;
        }
        d--;
    }
    return d - 1;
}

// arms[v][y][x] = up | down<<8 | left<<16 | right<<24  (computeLimits, :661-683)
__global__ void k_arms(const uint32_t* __restrict__ img, uint32_t* __restrict__ arms, DevParams P) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int v = blockIdx.z;
    if (x >= P.W) return;
    const uint32_t* im = img + (size_t)v * P.H * P.W;
    uint32_t packed = 0;
    if (!(P.mask && im[(size_t)y * P.W + x] == 0)) {
        const uint32_t up = compute_limit(P, im, y, x, -1, 0);
        const uint32_t dn = compute_limit(P, im, y, x, 1, 0);
        const uint32_t lf = compute_limit(P, im, y, x, 0, -1);
        const uint32_t rt = compute_limit(P, im, y, x, 0, 1);
        packed = up | (dn << 8) | (lf << 16) | (rt << 24);
    }
    arms[((size_t)v * P.H + y) * P.W + x] = packed;
}

__device__ __forceinline__ int arm_up(uint32_t a) { return a & 0xff; }
__device__ __forceinline__ int arm_down(uint32_t a) { return (a >> 8) & 0xff; }
__device__ __forceinline__ int arm_left(uint32_t a) { return (a >> 16) & 0xff; }
__device__ __forceinline__ int arm_right(uint32_t a) { return (a >> 24) & 0xff; }

// Cross-window sizes: identical for every d (aggregation1D accumulates windowSizes the
// same way for each slice, :716), so they are computed once per view and orientation.
//   ws[v][0]: horizontalFirst (row counts then column sums), ws[v][1]: vertical first.
__global__ void k_window_sizes(const uint32_t* __restrict__ arms, int32_t* __restrict__ ws,
                               DevParams P) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int v = blockIdx.z;
    const int H = P.H, W = P.W;
    if (x >= W) return;
    const uint32_t* A = arms + (size_t)v * H * W;
    const uint32_t a = A[(size_t)y * W + x];
    int hf = 0, vf = 0;
    for (int k = -arm_up(a); k <= arm_down(a); ++k) {
        const uint32_t b = A[(size_t)(y + k) * W + x];
        hf += arm_left(b) + arm_right(b) + 1;
    }
    for (int k = -arm_left(a); k <= arm_right(a); ++k) {
        const uint32_t b = A[(size_t)y * W + (x + k)];
        vf += arm_up(b) + arm_down(b) + 1;
    }
    ws[((size_t)(v * 2 + 0) * H + y) * W + x] = hf;
    ws[((size_t)(v * 2 + 1) * H + y) * W + x] = vf;
}

// colour differences between vertical / horizontal neighbours of each view image,
// used by the scanline P1/P2 rule (computeP1P2, :915-981; colorDiff is symmetric):
//   gv[v][y][x] = colorDiff(img_v(y,x), img_v(y-1,x))  (y >= 1)
//   gh[v][y][x] = colorDiff(img_v(y,x), img_v(y,x-1))  (x >= 1)
__global__ void k_color_grad(const uint32_t* __restrict__ img, uint8_t* __restrict__ gv,
                             uint8_t* __restrict__ gh, DevParams P) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int v = blockIdx.z;
    const int H = P.H, W = P.W;
    if (x >= W) return;
    const uint32_t* im = img + (size_t)v * H * W;
    const uint32_t c = im[(size_t)y * W + x];
    const size_t o = ((size_t)v * H + y) * W + x;
    gv[o] = (uint8_t)(y >= 1 ? color_diff(P, c, im[(size_t)(y - 1) * W + x]) : 0);
    gh[o] = (uint8_t)(x >= 1 ? color_diff(P, c, im[(size_t)y * W + (x - 1)]) : 0);
}

// ---------------------------------------------------------------------------
// 1-D aggregation along lines, in place, LDS ring
// ---------------------------------------------------------------------------
constexpr int AG_SEG = 16;     // outputs per step (4 per wave)
constexpr int AG_THREADS = 256;

// copy pixels [x0, x1) of the line into their ring slots (flattened float4 index t = px*Q + q:
// consecutive threads read consecutive 16-B pieces of a pixel's L-vector)
__device__ __forceinline__ void agg_fill(float4* ring, int RING, const float* base, size_t es, int Q,
                                         int x0, int x1, int tid) {
    const int cnt = (x1 - x0) * Q;
    for (int t = tid; t < cnt; t += AG_THREADS) {
        const int px = t / Q, q = t - px * Q;
        ring[((x0 + px) % RING) * Q + q] =
            *reinterpret_cast<const float4*>(base + (size_t)(x0 + px) * es + 4 * q);
    }
}

template <int J>
__global__ __launch_bounds__(AG_THREADS) void k_agg_line(float* __restrict__ vol,
                                                         const uint32_t* __restrict__ arms,
                                                         const int32_t* __restrict__ ws,
                                                         int horizontal, int A, DevParams P) {
    extern __shared__ __attribute__((aligned(16))) float4 ring[];
    const int H = P.H, W = P.W, Lp = P.Lp;
    const int Q = Lp >> 2;                      // float4 per pixel vector
    const int RING = AG_SEG + 2 * A;
    const int v = blockIdx.y;
    const int line = blockIdx.x;
    const int n = horizontal ? W : H;
    const size_t es = horizontal ? (size_t)Lp : (size_t)W * Lp;  // floats between neighbours
    float* base = vol + (size_t)v * H * W * Lp + (horizontal ? (size_t)line * W * Lp : (size_t)line * Lp);
    const uint32_t* ab = arms + (size_t)v * H * W + (horizontal ? (size_t)line * W : (size_t)line);
    const size_t as = horizontal ? 1 : (size_t)W;
    const int32_t* wsl = ws ? ws + (size_t)v * 2 * H * W + (horizontal ? (size_t)line * W : (size_t)line) : nullptr;
    const int shA = horizontal ? 16 : 0, shB = horizontal ? 24 : 8;

    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const int nsteps = (n + AG_SEG - 1) / AG_SEG;

    // initial window [0, min(n, SEG + A))
    agg_fill(ring, RING, base, es, Q, 0, min(n, AG_SEG + A), tid);
    __syncthreads();

    for (int s = 0; s < nsteps; ++s) {
        // the pixels step s+1 adds: [(s+1)*SEG + A, (s+2)*SEG + A)
        const int nx0 = min(n, (s + 1) * AG_SEG + A);
        const int nx1 = min(n, (s + 2) * AG_SEG + A);

        for (int i = 0; i < AG_SEG / 4; ++i) {
            const int o = s * AG_SEG + wave * (AG_SEG / 4) + i;
            if (o >= n) break;
            const uint32_t a = ab[(size_t)o * as];
            const int lo = (a >> shA) & 0xff, hi = (a >> shB) & 0xff;
            float4 acc[J];
#pragma unroll
            for (int j = 0; j < J; ++j) acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            int slot = (o - lo) % RING;
            for (int k = -lo; k <= hi; ++k) {
#pragma unroll
                for (int j = 0; j < J; ++j) {
                    const int q = lane + 64 * j;
                    if (q < Q) {
                        const float4 x = ring[slot * Q + q];
                        acc[j].x += x.x;
                        acc[j].y += x.y;
                        acc[j].z += x.z;
                        acc[j].w += x.w;
                    }
                }
                slot = slot + 1 == RING ? 0 : slot + 1;
            }
            if (wsl) {
                const float wsz = (float)wsl[(size_t)o * as];
#pragma unroll
                for (int j = 0; j < J; ++j) {
                    acc[j].x /= wsz;
                    acc[j].y /= wsz;
                    acc[j].z /= wsz;
                    acc[j].w /= wsz;
                }
            }
#pragma unroll
            for (int j = 0; j < J; ++j) {
                const int q = lane + 64 * j;
                if (q < Q) *reinterpret_cast<float4*>(base + (size_t)o * es + 4 * q) = acc[j];
            }
        }
        __syncthreads(); // everyone done reading the slots about to be overwritten
        if (nx0 < nx1) agg_fill(ring, RING, base, es, Q, nx0, nx1, tid);
        __syncthreads();
    }
}

void launch_arms(const uint32_t* img, uint32_t* arms, const DevParams& P, hipStream_t st) {
    dim3 g((P.W + 127) / 128, P.H, 2);
    hipLaunchKernelGGL(k_arms, g, dim3(128), 0, st, img, arms, P); trace_point("k_arms", st);
}

void launch_window_sizes(const uint32_t* arms, int32_t* ws, const DevParams& P, hipStream_t st) {
    dim3 g((P.W + 127) / 128, P.H, 2);
    hipLaunchKernelGGL(k_window_sizes, g, dim3(128), 0, st, arms, ws, P); trace_point("k_window_sizes", st);
}

void launch_color_grad(const uint32_t* img, uint8_t* gv, uint8_t* gh, const DevParams& P,
                       hipStream_t st) {
    dim3 g((P.W + 255) / 256, P.H, 2);
    hipLaunchKernelGGL(k_color_grad, g, dim3(256), 0, st, img, gv, gh, P); trace_point("k_color_grad", st);
}

size_t agg_lds_bytes(const DevParams& P) {
    const int A = P.max_length1 - 1;
    return (size_t)(AG_SEG + 2 * A) * (P.Lp / 4) * sizeof(float4);
}

int launch_agg_line(float* vol, const uint32_t* arms, const int32_t* ws, int horizontal,
                    const DevParams& P, hipStream_t st) {
    const int A = P.max_length1 - 1;
    const int J = (P.Lp / 4 + 63) / 64;
    dim3 g(horizontal ? P.H : P.W, 2);
    const size_t lds = agg_lds_bytes(P);
    if (lds > 160 * 1024) return -1;
    static bool attr_set = false;
    if (!attr_set) {
        hipFuncSetAttribute((const void*)k_agg_line<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        hipFuncSetAttribute((const void*)k_agg_line<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        hipFuncSetAttribute((const void*)k_agg_line<3>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        hipFuncSetAttribute((const void*)k_agg_line<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    switch (J) {
        case 1: hipLaunchKernelGGL((k_agg_line<1>), g, dim3(AG_THREADS), lds, st, vol, arms, ws, horizontal, A, P); trace_point("k_agg_line<1>", st); return 0;
        case 2: hipLaunchKernelGGL((k_agg_line<2>), g, dim3(AG_THREADS), lds, st, vol, arms, ws, horizontal, A, P); trace_point("k_agg_line<2>", st); return 0;
        case 3: hipLaunchKernelGGL((k_agg_line<3>), g, dim3(AG_THREADS), lds, st, vol, arms, ws, horizontal, A, P); trace_point("k_agg_line<3>", st); return 0;
        case 4: hipLaunchKernelGGL((k_agg_line<4>), g, dim3(AG_THREADS), lds, st, vol, arms, ws, horizontal, A, P); trace_point("k_agg_line<4>", st); return 0;
        default: return -1;
    }
}

}  // namespace tsm
