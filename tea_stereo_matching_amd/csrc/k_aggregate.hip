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
#include <stdlib.h>

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
__global__ void k_arms(const uint32_t* __restrict__ img, uint32_t* __restrict__ arms, DevParams Pk) {
    const DevParams P = Pk;  // kernel args -> registers once (no per-use kernarg reloads)
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int v = blockIdx.z & 1;
    if (x >= P.W) return;
    pair_shift(blockIdx.z >> 1, P.pstride, img, arms);
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
                               DevParams Pk) {
    const DevParams P = Pk;  // kernel args -> registers once (no per-use kernarg reloads)
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int v = blockIdx.z & 1;
    const int H = P.H, W = P.W;
    if (x >= W) return;
    pair_shift(blockIdx.z >> 1, P.pstride, arms, ws);
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
    // For the split streamer, per pass direction d (0 vertical: divides by hf, 1 horizontal:
    // by vf), same [v][d][H][W] layout: ws + 4HW the correctly rounded reciprocals of the
    // window sizes, ws + 8HW the packed descriptor lo | hi << 8 | size << 16.
    float* rcp = reinterpret_cast<float*>(ws + (size_t)4 * H * W);
    uint32_t* pk = reinterpret_cast<uint32_t*>(ws + (size_t)8 * H * W);
    const size_t i0 = ((size_t)(v * 2 + 0) * H + y) * W + x, i1 = ((size_t)(v * 2 + 1) * H + y) * W + x;
    rcp[i0] = 1.0f / (float)hf;
    rcp[i1] = 1.0f / (float)vf;
    pk[i0] = (a & 0xffffu) | ((uint32_t)hf << 16);
    pk[i1] = (a >> 16) | ((uint32_t)vf << 16);
}

// colour differences between vertical / horizontal neighbours of each view image,
// used by the scanline P1/P2 rule (computeP1P2, :915-981; colorDiff is symmetric):
//   gv[v][y][gpad + x] = colorDiff(img_v(y,x), img_v(y-1,x))  (y >= 1)
//   gh[v][y][gpad + x] = colorDiff(img_v(y,x), img_v(y,x-1))  (x >= 1)
// Every byte outside those ranges (margins, x = 0 for gh, y = 0 for gv) holds the
// sentinel colorDiff+1, which is exactly the reference's out-of-image value of d2
// (:928), so the scanline reads the maps without range checks.
__global__ void k_color_grad(const uint32_t* __restrict__ img, uint8_t* __restrict__ gv,
                             uint8_t* __restrict__ gh, DevParams Pk) {
    const DevParams P = Pk;
    const int xs = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int v = blockIdx.z & 1;
    const int H = P.H, W = P.W;
    if (xs >= P.gstride) return;
    pair_shift(blockIdx.z >> 1, P.pstride, img, gv, gh);
    const int x = xs - P.gpad;
    const uint8_t sent = (uint8_t)(P.color_diff + 1);
    const uint32_t* im = img + (size_t)v * H * W;
    const size_t o = ((size_t)v * H + y) * P.gstride + xs;
    uint8_t a = sent, b = sent;
    if (x >= 0 && x < W) {
        const uint32_t c = im[(size_t)y * W + x];
        if (y >= 1) a = (uint8_t)color_diff(P, c, im[(size_t)(y - 1) * W + x]);
        if (x >= 1) b = (uint8_t)color_diff(P, c, im[(size_t)y * W + (x - 1)]);
    }
    gv[o] = a;
    gh[o] = b;
}

// ---------------------------------------------------------------------------
// 1-D aggregation along lines, in place, LDS ring with register-staged prefetch
// ---------------------------------------------------------------------------
// One 512-thread workgroup owns a whole line of one view.  Per step it produces SEG
// outputs (4 per wave) from the LDS ring, while the SEG pixel vectors of the NEXT step
// are already in flight into registers (issued before the compute, written to the ring
// after the barrier), so HBM latency hides behind the compute.  The line's packed arms
// and window sizes are staged in LDS once, so the per-output arm lookup is an LDS
// broadcast instead of a dependent global load.
constexpr int AG_SEG = 32;
constexpr int AG_THREADS = 512;
constexpr int AG_WAVES = AG_THREADS / 64;
constexpr int AG_PER_WAVE = AG_SEG / AG_WAVES;  // outputs per wave per step

template <int PF>
__device__ __forceinline__ void agg_issue(f32x4 (&pf)[PF], const float* __restrict__ base, size_t es,
                                          int Q, int x0, int x1, int tid) {
    const int cnt = (x1 - x0) * Q;
#pragma unroll
    for (int r = 0; r < PF; ++r) {
        const int t = tid + r * AG_THREADS;
        const int tt = t < cnt ? t : 0;  // clamp: keeps every slot's load unconditional
        const int px = tt / Q, q = tt - px * Q;
        pf[r] = *reinterpret_cast<const f32x4*>(base + (size_t)(x0 + px) * es + 4 * q);
    }
}

template <int PF>
__device__ __forceinline__ void agg_commit(const f32x4 (&pf)[PF], f32x4* ring, int RING, int Q,
                                           int x0, int x1, int tid) {
    const int cnt = (x1 - x0) * Q;
#pragma unroll
    for (int r = 0; r < PF; ++r) {
        const int t = tid + r * AG_THREADS;
        if (t < cnt) {
            const int px = t / Q, q = t - px * Q;
            ring[((x0 + px) % RING) * Q + q] = pf[r];
        }
    }
}

template <int J>
__global__ __launch_bounds__(AG_THREADS) void k_agg_line(float* __restrict__ vol,
                                                         const uint32_t* __restrict__ arms,
                                                         const int32_t* __restrict__ ws,
                                                         int horizontal, int A, DevParams Pk) {
    const DevParams P = Pk;  // kernel args -> registers once (no per-use kernarg reloads)
    constexpr int PF = (AG_SEG * 64 * J + AG_THREADS - 1) / AG_THREADS;  // float4 per thread per step
    extern __shared__ __attribute__((aligned(16))) f32x4 smem_f4[];
    const int H = P.H, W = P.W, Lp = P.Lp;
    const int Q = Lp >> 2;                      // float4 per pixel vector
    const int RING = AG_SEG + 2 * A;
    const int v = blockIdx.y;
    const int line = blockIdx.x;
    pair_shift(blockIdx.z, P.pstride, vol, arms, ws);
    const int n = horizontal ? W : H;
    const size_t es = horizontal ? (size_t)Lp : (size_t)W * Lp;  // floats between neighbours
    float* base = vol + (size_t)v * H * W * Lp + (horizontal ? (size_t)line * W * Lp : (size_t)line * Lp);
    const uint32_t* ab = arms + (size_t)v * H * W + (horizontal ? (size_t)line * W : (size_t)line);
    const size_t as = horizontal ? 1 : (size_t)W;
    const int32_t* wsl = ws ? ws + (size_t)v * 2 * H * W + (horizontal ? (size_t)line * W : (size_t)line) : nullptr;
    const int shA = horizontal ? 16 : 0, shB = horizontal ? 24 : 8;
    f32x4* ring = smem_f4;
    uint32_t* arm_s = reinterpret_cast<uint32_t*>(ring + (size_t)RING * Q);
    float* ws_s = reinterpret_cast<float*>(arm_s + n);

    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const int nsteps = (n + AG_SEG - 1) / AG_SEG;

    f32x4 pf[PF];
    agg_issue<PF>(pf, base, es, Q, 0, min(n, AG_SEG), tid);
    for (int i = tid; i < n; i += AG_THREADS) {
        const uint32_t a = ab[(size_t)i * as];
        arm_s[i] = (((a >> shA) & 0xffu) << 16) | ((a >> shB) & 0xffu);  // lo<<16 | hi
        if (wsl) ws_s[i] = (float)wsl[(size_t)i * as];
    }
    agg_commit<PF>(pf, ring, RING, Q, 0, min(n, AG_SEG), tid);
    // rest of the initial window [SEG, SEG + A)
    for (int x0 = AG_SEG; x0 < min(n, AG_SEG + A); x0 += AG_SEG) {
        const int x1 = min(min(n, AG_SEG + A), x0 + AG_SEG);
        agg_issue<PF>(pf, base, es, Q, x0, x1, tid);
        agg_commit<PF>(pf, ring, RING, Q, x0, x1, tid);
    }
    __syncthreads();

    for (int s = 0; s < nsteps; ++s) {
        // the pixels step s+1 adds: [(s+1)*SEG + A, (s+2)*SEG + A), loads in flight now
        const int nx0 = min(n, (s + 1) * AG_SEG + A);
        const int nx1 = min(n, (s + 2) * AG_SEG + A);
        if (nx0 < nx1) agg_issue<PF>(pf, base, es, Q, nx0, nx1, tid);

#pragma unroll
        for (int i = 0; i < AG_PER_WAVE; ++i) {
            const int o = s * AG_SEG + wave * AG_PER_WAVE + i;
            if (o < n) {
                const uint32_t a = arm_s[o];
                const int lo = (int)(a >> 16), hi = (int)(a & 0xffffu);
                f32x4 acc[J];
#pragma unroll
                for (int j = 0; j < J; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
                int slot = o - lo;
                slot = slot >= RING ? slot % RING : slot;
                for (int k = -lo; k <= hi; ++k) {
#pragma unroll
                    for (int j = 0; j < J; ++j) {
                        const int q = lane + 64 * j;
                        if (q < Q) acc[j] += ring[slot * Q + q];  // 4 independent sequential fp32 sums
                    }
                    slot = slot + 1 == RING ? 0 : slot + 1;
                }
                if (wsl) {
                    const float wsz = ws_s[o];
#pragma unroll
                    for (int j = 0; j < J; ++j) acc[j] /= wsz;
                }
#pragma unroll
                for (int j = 0; j < J; ++j) {
                    const int q = lane + 64 * j;
                    if (q < Q) *reinterpret_cast<f32x4*>(base + (size_t)o * es + 4 * q) = acc[j];
                }
            }
        }
        __syncthreads(); // everyone done reading the slots about to be overwritten
        if (nx0 < nx1) agg_commit<PF>(pf, ring, RING, Q, nx0, nx1, tid);
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// 1-D aggregation v3: LDS-DMA line streamer (4 loader waves + 12 summing waves)
// ---------------------------------------------------------------------------
// The pass is bound by how many bytes each CU keeps in flight, not by arithmetic.
// A workgroup owns one line; the line's pixel vectors stream into an LDS ring in chunks
// of AGD_SEG pixels by LDS-DMA (global_load_lds_dwordx4, no registers), issued by a
// dedicated loader waves D chunks ahead of the chunk being summed, so ~D*AGD_SEG vectors
// (tens of KB per CU) are always in flight.  The ring holds the 2*AH+1 chunks a step's
// windows can touch (AH = ceil(A / AGD_SEG) halo chunks per side) plus the D in flight.
// Each loader waits only on its own DMAs (a counted vmcnt, younger DMAs stay in flight),
// then the step barrier publishes the chunk; summing waves never wait on memory.  Each
// summing wave produces AGD_OPW outputs per step with the sequential window sum of the
// reference (lanes own float4 of labels).  In place: an output overwrites pixel p only
// after the chunk holding p was staged, and later windows read p from the ring.
constexpr int AGD_SUM_WAVES = 12;
constexpr int AGD_LOAD_WAVES = 4;               // DMA issue is slow per wave: spread it
constexpr int AGD_OPW = 1;                      // outputs per summing wave per step
constexpr int AGD_SEG = AGD_SUM_WAVES * AGD_OPW;  // pixels per chunk = outputs per step
constexpr int AGD_THREADS = (AGD_SUM_WAVES + AGD_LOAD_WAVES) * 64;
constexpr int AGD_MAX_RING = 32;                // chunks

// s_waitcnt vmcnt(n) for a runtime n, rounded DOWN to a multiple of 8 (waiting for a few
// more operations than needed is safe) so the dispatch is a short branch tree
__device__ __forceinline__ void wait_vmcnt(int n) {
    n = n > 63 ? 63 : n;
    switch (n >> 3) {
        case 7: asm volatile("s_waitcnt vmcnt(56)" ::: "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(48)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(40)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(32)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
}

#ifdef TSM_EXP_STAMPS
__device__ unsigned long long g_agg_stamps[8192 * 16 * 4];  // [block][wave][total, vmwait, barrier, work]
#endif

template <int J>
__global__ __launch_bounds__(AGD_THREADS) void k_agg_dma(float* __restrict__ vol,
                                                         const uint32_t* __restrict__ arms,
                                                         const int32_t* __restrict__ ws,
                                                         int horizontal, int A, int RC, int D,
                                                         DevParams Pk) {
    const DevParams P = Pk;  // kernel args -> registers once (no per-use kernarg reloads)
    extern __shared__ __attribute__((aligned(16))) f32x4 smem_f4[];
    const int H = P.H, W = P.W, Lp = P.Lp;
    const int Q = Lp >> 2;                          // float4 per pixel vector
    const int CS = AGD_SEG * Q;                     // float4 per ring chunk (exact: pixel-linear ring)
    const int ndma = (CS + 63) >> 6;                // DMA instructions per chunk
    const int AH = (A + AGD_SEG - 1) / AGD_SEG;     // halo chunks per side
    const int v = blockIdx.y;
    const int line = blockIdx.x;
    pair_shift(blockIdx.z, P.pstride, vol, arms, ws);
    const int n = horizontal ? W : H;
    const size_t es = horizontal ? (size_t)Lp : (size_t)W * Lp;  // floats between neighbours
    float* base = vol + (size_t)v * H * W * Lp + (horizontal ? (size_t)line * W * Lp : (size_t)line * Lp);
    const uint32_t* ab = arms + (size_t)v * H * W + (horizontal ? (size_t)line * W : (size_t)line);
    const size_t as = horizontal ? 1 : (size_t)W;
    const int32_t* wsl = ws ? ws + (size_t)v * 2 * H * W + (horizontal ? (size_t)line * W : (size_t)line) : nullptr;
    const int shA = horizontal ? 16 : 0, shB = horizontal ? 24 : 8;
    f32x4* ring = smem_f4;
    uint32_t* arm_s = reinterpret_cast<uint32_t*>(ring + (size_t)RC * CS + 4 * Q + 64 * J);
    float* ws_s = reinterpret_cast<float*>(arm_s + n);

    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const int nchunks = (n + AGD_SEG - 1) / AGD_SEG;
    const bool loader = wave >= AGD_SUM_WAVES;
    const int li = wave - AGD_SUM_WAVES;            // loader index (valid when loader)

    // Loaders take whole chunks in turn (chunk c: loader c % NLOAD), so each has NLOAD
    // steps to issue a chunk's DMAs (their issue is slow per wave).  Chunk c goes to
    // ring slot c % RC; the ring is pixel-linear (pixel p at (p mod RC*SEG) * Q).
    // Instruction k moves chunk float4 f = 64 k + lane (pixel f / Q, group f % Q); the
    // last one runs with only the lanes that still hold chunk data, so no DMA writes
    // outside its chunk.  Pixels past the line end re-read a valid vector into slots
    // nobody reads.  Per-lane offsets are computed once (no per-step divisions).
    constexpr int KMAX = AGD_SEG * J;  // ndma <= SEG * ceil(Q / 64)
    int pxo[KMAX];
    uint32_t gofs[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
        const int f = k * 64 + lane;
        const bool data = f < AGD_SEG * Q;
        pxo[k] = data ? f / Q : 0;
        gofs[k] = data ? 4u * (uint32_t)(f - (f / Q) * Q) : 0u;
    }
    const bool last_lane_ok = (ndma - 1) * 64 + lane < CS;
    auto dma_chunk = [&](int c) {
        if (c % AGD_LOAD_WAVES != li) return;
        f32x4* slot = ring + (size_t)(c % RC) * CS;
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
            if (k < ndma && (k < ndma - 1 || last_lane_ok)) {
                int px = c * AGD_SEG + pxo[k];
                px = px < n ? px : n - 1;
                const float* src = base + (size_t)px * es + gofs[k];
                __builtin_amdgcn_global_load_lds(src, slot + k * 64, 16, 0, 0);
            }
        }
    };
    // D - 1 is a multiple of NLOAD (host side), so after chunk s+AH every loader has
    // issued exactly (D-1)/NLOAD younger chunks when step s begins
    const int younger = ndma * ((D - 1) / AGD_LOAD_WAVES);
    if (loader) {
        for (int c = 0; c < AH + D; ++c) dma_chunk(c);  // chunks past the end: dead slots
    }
    for (int i = tid; i < n; i += AGD_THREADS) {
        const uint32_t a = ab[(size_t)i * as];
        arm_s[i] = (((a >> shA) & 0xffu) << 16) | ((a >> shB) & 0xffu);  // lo<<16 | hi
        if (wsl) ws_s[i] = (float)wsl[(size_t)i * as];
    }
    __syncthreads();  // arms / window sizes staged (full fence: LDS writes visible)
#ifdef TSM_EXP_STAMPS
    unsigned long long t_start = __builtin_amdgcn_s_memtime(), t_vm = 0, t_bar = 0, t_work = 0;
#define AGS(x) unsigned long long x = __builtin_amdgcn_s_memtime()
#else
#define AGS(x)
#endif
    for (int s = 0; s < nchunks; ++s) {
        AGS(ta);
        if (loader) wait_vmcnt(younger);  // chunk s+AH landed (younger chunks stay in flight)
        AGS(tb);
        // bare s_barrier, NOT __syncthreads(): its fence would drain every wave's vmcnt,
        // i.e. wait for all DMAs in flight and serialise the stream.  Summing waves
        // write no LDS, and their ring reads of step s-1 have returned before they
        // arrive here, so chunk s-AH-1's slot is free for the next DMA.
        __builtin_amdgcn_s_barrier();
        AGS(tc);
#ifdef TSM_EXP_STAMPS
        t_vm += tb - ta;
        t_bar += tc - tb;
#endif
        if (loader) {
            dma_chunk(s + AH + D);               // into the slot of chunk s-AH-1
        } else {
#pragma unroll
            for (int u = 0; u < AGD_OPW; ++u) {
                const int o = s * AGD_SEG + u * AGD_SUM_WAVES + wave;
                if (o >= n) break;
                const uint32_t a = arm_s[o];
                const int lo = (int)(a >> 16), hi = (int)(a & 0xffffu);
                f32x4 acc[J];
#pragma unroll
                for (int j = 0; j < J; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
                // Window [o-lo, o+hi] in at most two runs of the pixel-linear ring (it wraps
                // once at most), summed strictly in window order in blocks of 4 reads;
                // a block's reads past the run end add +0.0 (exact: sums are >= +0).
                // Every lane reads (lanes >= Q read neighbouring ring data, never stored).
                const int RP = RC * AGD_SEG;
                int p = (o - lo) % RP;
                int len = lo + hi + 1;
                for (int run = 0; run < 2 && len > 0; ++run) {
                    const int rl = min(len, RP - p);
                    const f32x4* r = ring + (size_t)p * Q + lane;
                    for (int i = 0; i < rl; i += 4) {
                        f32x4 x[4][J];
#pragma unroll
                        for (int u = 0; u < 4; ++u)
#pragma unroll
                            for (int j = 0; j < J; ++j) x[u][j] = r[(i + u) * Q + 64 * j];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const bool in = i + u < rl;
#pragma unroll
                            for (int j = 0; j < J; ++j) {
                                acc[j].x += in ? x[u][j].x : 0.f;
                                acc[j].y += in ? x[u][j].y : 0.f;
                                acc[j].z += in ? x[u][j].z : 0.f;
                                acc[j].w += in ? x[u][j].w : 0.f;
                            }
                        }
                    }
                    len -= rl;
                    p = 0;
                }
                if (wsl) {
                    const float wsz = ws_s[o];
#pragma unroll
                    for (int j = 0; j < J; ++j) acc[j] /= wsz;
                }
#pragma unroll
                for (int j = 0; j < J; ++j) {
                    const int q = lane + 64 * j;
#ifdef TSM_EXP_AGG_NOSTORE
                    if (q < Q && acc[j].x == -1.f) *reinterpret_cast<f32x4*>(base + (size_t)o * es + 4 * q) = acc[j];
#else
                    if (q < Q) *reinterpret_cast<f32x4*>(base + (size_t)o * es + 4 * q) = acc[j];
#endif
                }
            }
        }
#ifdef TSM_EXP_STAMPS
        { AGS(td); t_work += td - tc; }
#endif
    }
    if (loader) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA outlives the WG
#ifdef TSM_EXP_STAMPS
    {
        const size_t bid = (size_t)blockIdx.y * gridDim.x + blockIdx.x;
        if (lane == 0 && bid < 8192) {
            unsigned long long* o = g_agg_stamps + (bid * 16 + wave) * 4;
            o[0] = __builtin_amdgcn_s_memtime() - t_start; o[1] = t_vm; o[2] = t_bar; o[3] = t_work;
        }
    }
#endif
}

// ---------------------------------------------------------------------------
// 1-D aggregation v4: label-grouped streamer, optionally two passes fused
// ---------------------------------------------------------------------------
// 1-D aggregation v5: persistent line streamer, same-direction pass pairs fused
// ---------------------------------------------------------------------------
// Each workgroup (one per CU) owns every G-th line of the pass (both views) and treats
// them as ONE continuous pixel stream: windows never cross a line (arms stop at the
// image border), so lines simply follow each other and there is no per-line warm-up.
// The stream moves in chunks of AS_SEG pixels, one chunk per step.  Eight loader waves
// stage chunk PAIRS in VGPRs (global_load_dwordx4; loader k % 8 owns pair k, one pair in
// flight per loader = 16 chunks = ~100 KB per CU for config B) and copy a landed pair
// into an LDS ring (ring1) AS_AHEAD steps before its first chunk is summed.  Each of the
// AS_SEG summing waves produces one output per step with the reference's strictly
// sequential window sum (lanes own float4 of labels).
//   FUSED: pass A (the 2nd pass of an iteration, divided by the window sizes) writes
//   its outputs to a second ring (ring2) and pass B (the 1st pass of the next
//   iteration, same direction) sums them AS_LAG steps later, so the volume makes one
//   HBM round trip for two passes.  Not fused: pass A's outputs go straight to HBM.
// In place: a pixel is overwritten AS_AHEAD (+AS_LAG) steps after it was staged.
// The per-pixel window sizes divide through an exact reciprocal-FMA quotient:
// q0 = a*y, r = fma(-q0, b, a), q = fma(r, y, q0) with y = RN(1/b) equals RN(a/b) for
// every integer b in [1, 4489] and every a in [2^-40, 2^16) (exhaustively checked,
// tools/micro/div_check.c); smaller a take the IEEE division.
#ifndef AS_GRP
#define AS_GRP 1                            // chunks per loader turn
#endif
constexpr int AS_SEG = 8;                   // pixels per chunk = summing waves
constexpr int AS_LOAD = 8;                  // loader waves (turn k: loader k % 8)
constexpr int AS_THREADS = (AS_SEG + AS_LOAD) * 64;
constexpr int AS_AH = 5;                    // windows reach at most 5 chunks either side
constexpr int AS_MAX_ARM = AS_AH * AS_SEG;
constexpr int AS_AHEAD = AS_AH + 1;         // chunk c is readable from step c - AHEAD + 1
constexpr int AS_RC1 = 2 * AS_AH + 1 + AS_GRP;  // ring1 chunks: 2*AH+1 read + a turn landing
constexpr int AS_RC2 = 2 * AS_AH + 2;       // ring2 chunks: 2*AH+1 read + one written
constexpr int AS_RP1 = AS_RC1 * AS_SEG;
constexpr int AS_RP2 = AS_RC2 * AS_SEG;
constexpr int AS_LAG = AS_AH + 1;           // pass B at step s outputs chunk s - LAG
constexpr int AS_MC = 16;                   // meta ring chunks (> AHEAD + GRP + LAG)
static_assert(AS_AHEAD % AS_GRP == 0, "turns land on steps NG*k - AHEAD");

// exact a / b for the aggregation's "C /= windowSize" (see above)
__device__ __forceinline__ f32x4 div_ws(f32x4 a, float b, float y) {
    const f32x4 q0 = a * y;
    const f32x4 r = __builtin_elementwise_fma(-q0, f32x4{b, b, b, b}, a);
    f32x4 q = __builtin_elementwise_fma(r, f32x4{y, y, y, y}, q0);
    // 0 < a < 2^-40 (never seen in practice) takes the IEEE path; a == 0 is exact above
    const u32x4 ab = __builtin_bit_cast(u32x4, a) - 1u;  // +0 wraps to 0xffffffff
    if (__builtin_expect(min(min(ab.x, ab.y), min(ab.z, ab.w)) < 0x2b800000u - 1u, 0)) {
        q.x = a.x / b; q.y = a.y / b; q.z = a.z / b; q.w = a.w / b;
    }
    return q;
}

// raw buffer resource over p (gfx9 dword3: 32-bit data format, no swizzle); offsets are
// unsigned 32-bit, the launcher checks that every line of a pass fits
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}

struct AggStream {
    float* vol;
    const uint32_t* arms;
    const int32_t* ws;     // window sizes of the dividing pass (nullptr: no divide)
    const uint32_t* pk;    // split streamer: packed descriptors of this direction, view 0
    const float* rcp;      // split streamer: reciprocals of this direction, view 0
    int qtot;              // split streamer: label vectors per pixel (Lp / 4)
    int qn0;               // split streamer: label vectors of slice 0 (blockIdx.y; = qtot if one slice)
    int horizontal;
    int n;                 // pixels per line
    int cpl;               // chunks per line
    int nlv;               // lines per view
    int nl;                // lines of both views
};

#ifdef TSM_EXP_STAMPS
__device__ unsigned long long g_as_stamps[1024 * 16 * 4];  // [block][wave][barrier, a/land, b/issue, total]
#define AST_T(x) const unsigned long long x = __builtin_amdgcn_s_memtime()
#define AST_ADD(i, v) ast[i] += (v)
#define AST_FLUSH() do { if (FUSED && lane == 0 && blockIdx.x < 1024) { unsigned long long* o_ = g_as_stamps + ((size_t)blockIdx.x * 16 + wave) * 4; \
    o_[0] = ast[0]; o_[1] = ast[1]; o_[2] = ast[2]; o_[3] = __builtin_amdgcn_s_memtime() - ast_t0; } } while (0)
#else
#define AST_T(x)
#define AST_ADD(i, v)
#define AST_FLUSH()
#endif

// Per-pixel window descriptor, precomputed by the loader when the pixel lands (so the
// summing waves spend no scalar work on ring arithmetic): 32 B per pixel.
//   [0] LDS byte offset of the pass-A window start in ring1   [1] window length
//   [2] y = RN(1/windowSize)                                   [3] windowSize as float
//   [4] LDS byte offset of the pass-B window start in ring2   [5] window length
constexpr int AS_MW = 8;  // meta words per pixel
constexpr int AX_MIR = 3;  // mirror slots after each ring (a 4-read block spans 3 slots past its start)

// QT > 0: the pixel vector has QT float4 (compile-time ring stride); 0: runtime Q.
template <bool FUSED, int QT>
__global__ __launch_bounds__(AS_THREADS) void k_agg_stream(AggStream S, DevParams Pk) {
    const DevParams P = Pk;
    pair_shift(blockIdx.z, P.pstride, S.vol, S.arms, S.ws, S.pk, S.rcp);
    extern __shared__ __attribute__((aligned(16))) f32x4 smem_f4[];
    const int H = P.H, W = P.W, Lp = P.Lp;
    const int Q = QT > 0 ? QT : Lp >> 2;
    const uint32_t Qs = (uint32_t)Q * 16;                                // bytes per ring pixel
    const size_t vstride = (size_t)H * W * Lp;
    const size_t es = S.horizontal ? (size_t)Lp : (size_t)W * Lp;         // floats per pixel step
    const size_t ls = S.horizontal ? (size_t)W * Lp : (size_t)Lp;          // floats per line step
    const size_t aes = S.horizontal ? 1 : (size_t)W;
    const size_t als = S.horizontal ? (size_t)W : 1;
    const int shA = S.horizontal ? 16 : 0, shB = S.horizontal ? 24 : 8;
    const int g = blockIdx.x, G = gridDim.x;
    const int my_lines = (S.nl - g + G - 1) / G;
    const int nch = my_lines * S.cpl;
    const uint32_t r1_off = 0;                                            // LDS byte offsets
    const uint32_t r2_off = (uint32_t)(AS_RP1 + AX_MIR) * Qs;  // each ring + AX_MIR mirror slots
    const uint32_t meta_off = r2_off + (FUSED ? (uint32_t)(AS_RP2 + AX_MIR) * Qs : 0u);
    char* lds = reinterpret_cast<char*>(smem_f4);

    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const bool loader = wave >= AS_SEG;
    const int li = wave - AS_SEG;
    const int nsteps = nch + (FUSED ? AS_LAG : 0);
    const uint32_t lane16 = (uint32_t)lane * 16;
    const bool vl = lane < Q;
#ifdef TSM_EXP_STAMPS
    unsigned long long ast[3] = {0, 0, 0};
    const unsigned long long ast_t0 = __builtin_amdgcn_s_memtime();
#endif
    // float offset of pixel 0 of local line lidx
    auto line_base = [&](int lidx) -> size_t {
        const int gl = g + lidx * G;
        const int v = gl / S.nlv, line = gl - v * S.nlv;
        return (size_t)v * vstride + (size_t)line * ls;
    };

    if (loader) {
        // ---- loader li: turns k = li, li + 8, ... (chunks NG*k .. NG*k+NG-1), one turn's
        // chunks in flight (one buffer per wave: the compiler's wait before the copy is a
        // plain vmcnt(0)).  Every load and LDS write is unconditional (lanes past the
        // vector repeat lane Q-1): with no exec branches the compiler's waits stay at the
        // copy (land) and never stall the next turn's issue.
        constexpr int NG = AS_GRP;
        f32x4 b[NG * AS_SEG];
        uint32_t ma[NG], mw[NG];                   // meta of chunk NG*k+h (pixel lane & 7)
        const int lanec = lane < Q ? lane : Q - 1;
        int lidx = 0, cc = NG * li;                // stream position of chunk NG*k
        while (cc >= S.cpl) { cc -= S.cpl; ++lidx; }
        // Byte offsets of the lines a turn can touch (vol, arms, window sizes), rebuilt
        // (one division) only when the turn moves to a new line.  Loads are buffer loads
        // off kernel-wide resources: a shared lane offset (VGPR) plus a per-pixel scalar
        // offset, so no 64-bit VGPR addresses compete with the staging buffer.
        const __amdgpu_buffer_rsrc_t rs_vol = make_rsrc(S.vol), rs_arm = make_rsrc(S.arms),
                                     rs_ws = make_rsrc(S.ws);
        struct LineRes { int l; uint32_t vol, arm, ws; };
        auto line_res = [&](int l) -> LineRes {
            const int gl = g + l * G;
            const int v = gl / S.nlv, line = gl - v * S.nlv;
            const uint32_t a = (uint32_t)(v * H * W + line * (int)als);
            return LineRes{l, (uint32_t)(((size_t)v * vstride + (size_t)line * ls) * 4), a * 4,
                           (a + (uint32_t)(v * H * W)) * 4};  // ws: per-view stride 2HW
        };
        LineRes lr[NG];
#pragma unroll
        for (int h = 0; h < NG; ++h) lr[h] = line_res(0);
        const int last_l = my_lines - 1, last_cc = S.cpl - 1;
        const uint32_t voff = (uint32_t)lanec * 16;
        const uint32_t es4 = (uint32_t)(es * 4), aes4 = (uint32_t)(aes * 4);
        const uint32_t mpx = (uint32_t)(lane & 7);
        auto issue = [&]() {  // the turn at (lidx, cc): chunk NG*k and its successors
            int l[NG], c[NG];
            l[0] = lidx; c[0] = cc;
#pragma unroll
            for (int h = 1; h < NG; ++h) {
                l[h] = c[h - 1] + 1 == S.cpl ? l[h - 1] + 1 : l[h - 1];
                c[h] = c[h - 1] + 1 == S.cpl ? 0 : c[h - 1] + 1;
            }
#pragma unroll
            for (int h = 0; h < NG; ++h) {
                if (l[h] > last_l) { l[h] = last_l; c[h] = last_cc; }  // past the end: re-read
                if (lr[h].l != l[h]) lr[h] = (h && lr[h - 1].l == l[h]) ? lr[h - 1] : line_res(l[h]);
            }
            // meta first: a wait the compiler places before a meta load then finds no
            // vector load of this turn in flight yet
#pragma unroll
            for (int h = 0; h < NG; ++h) {  // every lane loads (pixel lane & 7): no exec branches
                const uint32_t pos = min((uint32_t)c[h] * AS_SEG + mpx, (uint32_t)S.n - 1);
                ma[h] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs_arm, pos * aes4, lr[h].arm, 0);
                mw[h] = S.ws ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs_ws, pos * aes4, lr[h].ws, 0) : 1u;
            }
#pragma unroll
            for (int h = 0; h < NG; ++h) {
                const int p0 = c[h] * AS_SEG;
#pragma unroll
                for (int i = 0; i < AS_SEG; ++i) {
                    const uint32_t pos = (uint32_t)min(p0 + i, S.n - 1);
                    b[h * AS_SEG + i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs_vol, voff, lr[h].vol + pos * es4, 0));
                }
            }
        };
        auto land = [&](int k) {
#pragma unroll
            for (int h = 0; h < NG; ++h) {
                const int c = NG * k + h;
                char* slot = lds + r1_off + (uint32_t)(c % AS_RC1) * AS_SEG * Qs + (uint32_t)lanec * 16;
#pragma unroll
                for (int i = 0; i < AS_SEG; ++i) *reinterpret_cast<f32x4*>(slot + i * Qs) = b[h * AS_SEG + i];
                if (c % AS_RC1 == 0) {  // ring slots 0..AX_MIR-1 are mirrored past the ring's end
#pragma unroll
                    for (int i = 0; i < AX_MIR; ++i)
                        *reinterpret_cast<f32x4*>(slot + (AS_RP1 + i) * Qs) = b[h * AS_SEG + i];
                }
            }
            if (lane < NG * AS_SEG) {  // window descriptors of the turn's pixels
                const int hh = lane >> 3, c = NG * k + hh, px = lane & 7;
                uint32_t a = ma[0], wsz = mw[0];
#pragma unroll
                for (int h = 1; h < NG; ++h)
                    if (hh == h) { a = ma[h]; wsz = mw[h]; }
                const int lo = (a >> shA) & 0xff, hi = (a >> shB) & 0xff;
                const float bw = (float)(int)wsz;
                const int rp1 = (c % AS_RC1) * AS_SEG + px;
                const int rp2 = (c % AS_RC2) * AS_SEG + px;
                uint32_t* m = reinterpret_cast<uint32_t*>(lds + meta_off) + ((c % AS_MC) * AS_SEG + px) * AS_MW;
                m[0] = r1_off + (uint32_t)((rp1 - lo + AS_RP1) % AS_RP1) * Qs;
                m[1] = (uint32_t)(lo + hi + 1);
                m[2] = __float_as_uint(1.0f / bw);
                m[3] = __float_as_uint(bw);
                m[4] = r2_off + (uint32_t)((rp2 - lo + AS_RP2) % AS_RP2) * Qs;
                m[5] = (uint32_t)(lo + hi + 1);
            }
        };
        auto advance = [&]() {  // to the loader's next turn: NG * AS_LOAD chunks on
            cc += NG * AS_LOAD;
            while (cc >= S.cpl) { cc -= S.cpl; ++lidx; }
        };
        // prologue: turn li in flight; turns with chunks < AHEAD land before step 0
        issue();
        if (NG * li < AS_AHEAD) {
            land(li);
            advance();
            issue();
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        for (int t = 0; t < nsteps; ++t) {
            // turn k lands during step NG*k - AHEAD
            const int k = (t + AS_AHEAD) / NG;
            if ((t + AS_AHEAD) % NG == 0 && (k & (AS_LOAD - 1)) == li && NG * k < nch) {
                AST_T(t0);
                land(k);
                AST_T(t1);
                advance();
                issue();
                AST_T(t2);
                AST_ADD(1, t1 - t0);
                AST_ADD(2, t2 - t1);
            }
            AST_T(b0);
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            AST_T(b1);
            AST_ADD(0, b1 - b0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no load outlives the workgroup
        AST_FLUSH();
        return;
    }

    // ---- summing waves -------------------------------------------------------------
    // Sequential window sum of `len` ring pixels from LDS byte offset `off` in the ring
    // [rb, re): whole blocks of 4 at immediate offsets (AX_MIR mirror slots past each ring
    // make every block contiguous), then the 1-3 remaining pixels under uniform branches.
    auto window = [&](uint32_t off, int len, uint32_t rb, uint32_t re) -> f32x4 {
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        const char* lp = lds + lane16;
#ifdef TSM_EXP_AGG_W1
        return *reinterpret_cast<const f32x4*>(lp + off);  // timing experiment only
#endif
        const uint32_t span = re - rb;
#ifdef TSM_EXP_WIN8
        // two blocks of 4 in flight per LDS round trip (windows of up to 8: one round trip)
        for (; len > 4; len -= 8) {
            const char* p = lp + off;
            uint32_t off1 = off + 4 * Qs;
            off1 = off1 >= re ? off1 - span : off1;
            const char* q = lp + off1;
            const f32x4 x0 = *reinterpret_cast<const f32x4*>(p);
            const f32x4 x1 = *reinterpret_cast<const f32x4*>(p + Qs);
            const f32x4 x2 = *reinterpret_cast<const f32x4*>(p + 2 * Qs);
            const f32x4 x3 = *reinterpret_cast<const f32x4*>(p + 3 * Qs);
            const f32x4 x4 = *reinterpret_cast<const f32x4*>(q);
            const f32x4 x5 = *reinterpret_cast<const f32x4*>(q + Qs);
            const f32x4 x6 = *reinterpret_cast<const f32x4*>(q + 2 * Qs);
            const f32x4 x7 = *reinterpret_cast<const f32x4*>(q + 3 * Qs);
            acc += x0;
            acc += x1;
            acc += x2;
            acc += x3;
            acc += x4;
            if (len > 5) acc += x5;
            if (len > 6) acc += x6;
            if (len > 7) acc += x7;
            off = off1 + 4 * Qs;
            off = off >= re ? off - span : off;
        }
        if (len <= 0) return acc;
        if (len == 4) {
            const char* p = lp + off;
            const f32x4 x0 = *reinterpret_cast<const f32x4*>(p);
            const f32x4 x1 = *reinterpret_cast<const f32x4*>(p + Qs);
            const f32x4 x2 = *reinterpret_cast<const f32x4*>(p + 2 * Qs);
            const f32x4 x3 = *reinterpret_cast<const f32x4*>(p + 3 * Qs);
            acc += x0;
            acc += x1;
            acc += x2;
            acc += x3;
            return acc;
        }
#else
        for (int nb = len >> 2; nb > 0; --nb) {
            const char* p = lp + off;
            const f32x4 x0 = *reinterpret_cast<const f32x4*>(p);
            const f32x4 x1 = *reinterpret_cast<const f32x4*>(p + Qs);
            const f32x4 x2 = *reinterpret_cast<const f32x4*>(p + 2 * Qs);
            const f32x4 x3 = *reinterpret_cast<const f32x4*>(p + 3 * Qs);
            acc += x0;
            acc += x1;
            acc += x2;
            acc += x3;
            off += 4 * Qs;
            off = off >= re ? off - span : off;
        }
#endif
        const int r = len & 3;
        if (r) {
            const char* p = lp + off;
            const f32x4 x0 = *reinterpret_cast<const f32x4*>(p);
            const f32x4 x1 = *reinterpret_cast<const f32x4*>(p + Qs);
            const f32x4 x2 = *reinterpret_cast<const f32x4*>(p + 2 * Qs);
            acc += x0;
            if (r > 1) acc += x1;
            if (r > 2) acc += x2;
        }
        return acc;
    };
    // output position of chunk `c`'s pixel `wave`: running float offset, new line: one division
    struct Out {
        int lidx, cc;
        size_t off;
    };
#ifdef TSM_EXP_AGG_NOSTORE
    const bool st_ok = false;  // timing experiment only
#else
    const bool st_ok = true;
#endif
    auto out_init = [&](Out& o) { o.lidx = 0; o.cc = 0; o.off = line_base(0) + (size_t)wave * es; };
    auto out_step = [&](Out& o) {
        if (++o.cc == S.cpl) { o.cc = 0; ++o.lidx; if (o.lidx < my_lines) o.off = line_base(o.lidx) + (size_t)wave * es; }
        else o.off += (size_t)AS_SEG * es;
    };
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // prologue chunks landed
    Out oa, ob;
    out_init(oa);
    out_init(ob);
    const uint32_t mstep = AS_SEG * AS_MW * 4, mwrap = AS_MC * mstep;
    const uint32_t* mbase = reinterpret_cast<const uint32_t*>(lds + meta_off + (uint32_t)wave * AS_MW * 4);
    uint32_t ma_off = 0;                                            // meta of chunk s (pass A)
    uint32_t mb_off = (uint32_t)((AS_MC - AS_LAG) % AS_MC) * mstep; // meta of chunk s - LAG (pass B)
    uint32_t r2w = r2_off + (uint32_t)wave * Qs;                   // ring2 slot of chunk s
    // descriptors are read one step ahead (they landed AHEAD steps before use)
    u32x4 mA = *reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(mbase) + ma_off);
    uint2 mB = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(mbase) + mb_off + 16);
    for (int s = 0; s < nsteps; ++s) {
        const uint32_t a_off = __builtin_amdgcn_readfirstlane(mA.x);
        const int a_len = (int)__builtin_amdgcn_readfirstlane(mA.y);
        const float a_y = __uint_as_float(__builtin_amdgcn_readfirstlane(mA.z));
        const float a_b = __uint_as_float(__builtin_amdgcn_readfirstlane(mA.w));
        const uint32_t b_off = __builtin_amdgcn_readfirstlane(mB.x);
        const int b_len = (int)__builtin_amdgcn_readfirstlane(mB.y);
        ma_off += mstep;
        ma_off = ma_off >= mwrap ? ma_off - mwrap : ma_off;
        mb_off += mstep;
        mb_off = mb_off >= mwrap ? mb_off - mwrap : mb_off;
        mA = *reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(mbase) + ma_off);
        mB = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(mbase) + mb_off + 16);
        AST_T(ta0);
        const uint32_t r1_end = r1_off + (uint32_t)AS_RP1 * Qs, r2_end = r2_off + (uint32_t)AS_RP2 * Qs;
        // pass B first: it reads ring2 slots pass A does not write this step, so pass A's
        // ring1 reads can overlap it
        if (FUSED && s >= AS_LAG) {  // pass B on chunk s - LAG
            if (ob.cc * AS_SEG + wave < S.n) {
                const f32x4 acc = window(b_off, b_len, r2_off, r2_end);
                if (vl && (st_ok || acc.x == -1.f)) st_stream(S.vol + ob.off + 4 * lane, acc);
            }
            out_step(ob);
        }
        AST_T(ta1);
        AST_ADD(2, ta1 - ta0);
        if (s < nch) {  // pass A on chunk s
            if (oa.cc * AS_SEG + wave < S.n) {
                f32x4 acc = window(a_off, a_len, r1_off, r1_end);
                if (S.ws) acc = div_ws(acc, a_b, a_y);
                if (FUSED) {
                    if (vl) {
                        *reinterpret_cast<f32x4*>(lds + r2w + lane16) = acc;
                        if (r2w < r2_off + (uint32_t)AX_MIR * Qs)
                            *reinterpret_cast<f32x4*>(lds + r2w + (uint32_t)AS_RP2 * Qs + lane16) = acc;
                    }
                } else if (vl && (st_ok || acc.x == -1.f)) {
                    st_stream(S.vol + oa.off + 4 * lane, acc);
                }
            }
            out_step(oa);
            r2w += AS_SEG * Qs;
            r2w = r2w >= r2_end ? r2w - (uint32_t)AS_RP2 * Qs : r2w;
        }
        AST_T(ta2);
        AST_ADD(1, ta2 - ta1);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        AST_T(ta3);
        AST_ADD(0, ta3 - ta2);
    }
    AST_FLUSH();
}

// ---------------------------------------------------------------------------
// 1-D aggregation v6: role-split persistent streamer (the default)
// ---------------------------------------------------------------------------
// Same stream, rings and window descriptors as v5, but the 16 waves of a workgroup split
// by role so a step's two window sums run in parallel and no wave ever mixes loads with
// stores (the compiler drains vmcnt(0) whenever a wave with stores in flight consumes a
// load):
//   A waves (8): wave w owns pixel w of every chunk.  It stages its own pixel vectors
//     AX_D steps ahead in a VGPR ring (one 16-B-per-lane load and two meta words per step,
//     counted vmcnt waits, no stores), copies pixel w of chunk s + AHEAD into ring1,
//     writes its window descriptor, and sums pass A of chunk s into ring2.
//   B waves (8): pass B of chunk s - LAG over ring2 (FUSED), or the copy of pass A's
//     chunk s - 1 out of ring2 (single pass), and the stores to HBM.
// One barrier per step; every wave runs the same whole number of AX_D-step blocks.
#ifndef TSM_AGG_LDAUX
#define TSM_AGG_LDAUX 0  // cache-policy bits of the staging loads (experiments: 2 = nt)
#endif
constexpr int AX_THREADS = 16 * 64;
constexpr int AX_MW = 2;  // meta words per pixel: packed descriptor (lo, hi, size), RN(1/size)
constexpr int AX_D = 12;  // A-wave staging ring: steps in flight (AX_D * 8 px * Q * 16 B per CU)
constexpr int AX_MC = 12;  // meta ring chunks (B reads chunk s - LAG + 1 before A overwrites its slot)
static_assert(AX_D == AS_RC1 && AX_D == AS_RC2 && AX_D == AX_MC, "ring slots are compile-time per unrolled step");
static_assert(AS_AHEAD + AS_LAG <= AX_MC, "meta ring too short for the B lag");

// BIG: volumes of 2 GiB and more (configs C, E): vector loads through 64-bit addresses
// instead of 32-bit buffer offsets.  Label slices: past 64 label vectors a pixel, blockIdx.y
// picks one of two slices of the label axis (independent sums), each a narrower ring.
template <bool FUSED, int QT, bool BIG>
__global__ __launch_bounds__(AX_THREADS) void k_agg_split(AggStream S, DevParams Pk) {
    const DevParams P = Pk;
    pair_shift(blockIdx.z, P.pstride, S.vol, S.arms, S.ws, S.pk, S.rcp);
    extern __shared__ __attribute__((aligned(16))) f32x4 smem_f4[];
    const int H = P.H, W = P.W, Lp = P.Lp;
    const int slice = blockIdx.y;
    const int Q = QT > 0 ? QT : (slice == 0 ? S.qn0 : S.qtot - S.qn0);
    float* const volq = S.vol + 4 * (slice == 0 ? 0 : S.qn0);  // this slice's first label
    const uint32_t Qs = (uint32_t)Q * 16;                                // bytes per ring pixel
    const size_t vstride = (size_t)H * W * Lp;
    const size_t es = S.horizontal ? (size_t)Lp : (size_t)W * Lp;         // floats per pixel step
    const size_t ls = S.horizontal ? (size_t)W * Lp : (size_t)Lp;          // floats per line step
    const size_t aes = S.horizontal ? 1 : (size_t)W;
    const size_t als = S.horizontal ? (size_t)W : 1;
    const int g = blockIdx.x, G = gridDim.x;
    const int my_lines = (S.nl - g + G - 1) / G;
    const int nch = my_lines * S.cpl;
    const uint32_t r1_off = 0;                                            // LDS byte offsets
    // each ring is followed by AX_MIR mirror slots (copies of its first slots), so a block of
    // 4 window reads starting at any slot never wraps
    const uint32_t r2_off = (uint32_t)(AS_RP1 + AX_MIR) * Qs;
    const uint32_t meta_off = r2_off + (uint32_t)(AS_RP2 + AX_MIR) * Qs;
    const uint32_t r1_end = r1_off + (uint32_t)AS_RP1 * Qs, r2_end = r2_off + (uint32_t)AS_RP2 * Qs;
    char* lds = reinterpret_cast<char*>(smem_f4);

    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const bool roleA = wave < AS_SEG;
    const int w = roleA ? wave : wave - AS_SEG;  // pixel of the chunk this wave owns
    const int nsteps = nch + (FUSED ? AS_LAG : 1);
    const int nblk = (nsteps + AX_D - 1) / AX_D;  // every wave runs nblk * AX_D steps
    const uint32_t lane16 = (uint32_t)lane * 16;
    const bool vl = lane < Q;
    auto line_base = [&](int lidx) -> size_t {
        const int gl = g + lidx * G;
        const int v = gl / S.nlv, line = gl - v * S.nlv;
        return (size_t)v * vstride + (size_t)line * ls;
    };
#ifdef TSM_EXP_AGG_NOBAR
    auto barrier = [&]() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };  // timing experiment only
#else
    auto barrier = [&]() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
#endif
    // sequential window sum of `len` ring pixels from LDS byte offset `off` (a slot of the
    // ring [rb, re)): whole blocks of 4 at immediate offsets (the mirror slots make every
    // block contiguous), then the 1-3 remaining pixels under uniform branches -- the
    // reference's order, no padding reads, little scalar bookkeeping
    auto window = [&](uint32_t off, int len, uint32_t rb, uint32_t re) -> f32x4 {
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        const char* lp = lds + lane16;
#ifdef TSM_EXP_AGG_W1
        return *reinterpret_cast<const f32x4*>(lp + off);  // timing experiment only
#endif
        const uint32_t span = re - rb;
#ifdef TSM_EXP_WIN8
        // two blocks of 4 in flight per LDS round trip (windows of up to 8: one round trip)
        for (; len > 4; len -= 8) {
            const char* p = lp + off;
            uint32_t off1 = off + 4 * Qs;
            off1 = off1 >= re ? off1 - span : off1;
            const char* q = lp + off1;
            const f32x4 x0 = *reinterpret_cast<const f32x4*>(p);
            const f32x4 x1 = *reinterpret_cast<const f32x4*>(p + Qs);
            const f32x4 x2 = *reinterpret_cast<const f32x4*>(p + 2 * Qs);
            const f32x4 x3 = *reinterpret_cast<const f32x4*>(p + 3 * Qs);
            const f32x4 x4 = *reinterpret_cast<const f32x4*>(q);
            const f32x4 x5 = *reinterpret_cast<const f32x4*>(q + Qs);
            const f32x4 x6 = *reinterpret_cast<const f32x4*>(q + 2 * Qs);
            const f32x4 x7 = *reinterpret_cast<const f32x4*>(q + 3 * Qs);
            acc += x0;
            acc += x1;
            acc += x2;
            acc += x3;
            acc += x4;
            if (len > 5) acc += x5;
            if (len > 6) acc += x6;
            if (len > 7) acc += x7;
            off = off1 + 4 * Qs;
            off = off >= re ? off - span : off;
        }
        if (len <= 0) return acc;
        if (len == 4) {
            const char* p = lp + off;
            const f32x4 x0 = *reinterpret_cast<const f32x4*>(p);
            const f32x4 x1 = *reinterpret_cast<const f32x4*>(p + Qs);
            const f32x4 x2 = *reinterpret_cast<const f32x4*>(p + 2 * Qs);
            const f32x4 x3 = *reinterpret_cast<const f32x4*>(p + 3 * Qs);
            acc += x0;
            acc += x1;
            acc += x2;
            acc += x3;
            return acc;
        }
#else
        for (int nb = len >> 2; nb > 0; --nb) {
            const char* p = lp + off;
            const f32x4 x0 = *reinterpret_cast<const f32x4*>(p);
            const f32x4 x1 = *reinterpret_cast<const f32x4*>(p + Qs);
            const f32x4 x2 = *reinterpret_cast<const f32x4*>(p + 2 * Qs);
            const f32x4 x3 = *reinterpret_cast<const f32x4*>(p + 3 * Qs);
            acc += x0;
            acc += x1;
            acc += x2;
            acc += x3;
            off += 4 * Qs;
            off = off >= re ? off - span : off;
        }
#endif
        const int r = len & 3;
        if (r) {
            const char* p = lp + off;
            const f32x4 x0 = *reinterpret_cast<const f32x4*>(p);
            const f32x4 x1 = *reinterpret_cast<const f32x4*>(p + Qs);
            const f32x4 x2 = *reinterpret_cast<const f32x4*>(p + 2 * Qs);
            acc += x0;
            if (r > 1) acc += x1;
            if (r > 2) acc += x2;
        }
        return acc;
    };
    const uint32_t mstep = AS_SEG * AX_MW * 4;
    const char* mbase = lds + meta_off + (uint32_t)w * AX_MW * 4;  // this wave's pixel column
#ifdef TSM_EXP_STAMPS
    unsigned long long ast[3] = {0, 0, 0};
    const unsigned long long ast_t0 = __builtin_amdgcn_s_memtime();
#endif

    if (roleA) {
        // ---- A: staging ring, land, pass A ----------------------------------------------
        const int lanec = lane < Q ? lane : Q - 1;
        const __amdgpu_buffer_rsrc_t rs_vol = make_rsrc(volq), rs_pk = make_rsrc(S.pk),
                                     rs_rcp = make_rsrc(S.rcp);
        const uint32_t voff = (uint32_t)lanec * 16;
        const uint32_t es4 = (uint32_t)(es * 4), aes4 = (uint32_t)(aes * 4);
        // the meta words are uniform; an opaque zero lane offset keeps them in VGPRs
        // (uniform values would be moved to SGPRs right after the load: a wait per load)
        uint32_t vzero;
        asm volatile("v_mov_b32 %0, 0" : "=v"(vzero));
        // issue position (chunk ci = s + AHEAD + AX_D at step s), advanced one chunk a step
        int il = 0, icc = 0;
        uint32_t iv = 0, ia = 0;  // byte offsets of line il: vol, descriptors (= reciprocals)
        const float* ivp = volq;   // BIG: line il's first pixel
        auto set_line = [&]() {
            const int gl = g + il * G;
            const int v = gl / S.nlv, line = gl - v * S.nlv;
            if (BIG) ivp = volq + (size_t)v * vstride + (size_t)line * ls;
            else iv = (uint32_t)(((size_t)v * vstride + (size_t)line * ls) * 4);
            ia = (uint32_t)(2 * v * H * W + line * (int)als) * 4;  // per-view stride 2HW
        };
        set_line();
        f32x4 rv[AX_D];
        uint32_t rma[AX_D], rmy[AX_D];  // packed descriptor, RN(1/size) bits
        auto issue = [&](int k) {  // chunk at (il, icc) -> slot k; past the end: re-read the last pixel
            const bool past = il >= my_lines;
            const uint32_t pos = past ? (uint32_t)(S.n - 1) : (uint32_t)min(icc * AS_SEG + w, S.n - 1);
#ifdef TSM_EXP_AGG_NOLOAD
            rv[k] = f32x4{(float)pos, 0.f, 0.f, 0.f};  // timing experiment only
#else
            if (BIG)
                rv[k] = *reinterpret_cast<const f32x4*>(ivp + (size_t)pos * es + 4 * lanec);
            else
                rv[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs_vol, voff, iv + pos * es4, TSM_AGG_LDAUX));
#endif
            rma[k] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs_pk, vzero, ia + pos * aes4, 0);
            rmy[k] = S.ws ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs_rcp, vzero, ia + pos * aes4, 0) : vzero;
            if (!past && ++icc == S.cpl) {
                icc = 0;
                ++il;
                if (il < my_lines) set_line();
            }
        };
        // pixel w of chunk c -> ring1; its raw descriptor (arms, window size, reciprocal)
        // -> the meta ring (every lane writes the same 16 B: no exec branch)
        auto land = [&](const f32x4& val, uint32_t ma, uint32_t my, int c) {
            const int slot = (c % AS_RC1) * AS_SEG + w;
            *reinterpret_cast<f32x4*>(lds + r1_off + (uint32_t)slot * Qs + voff) = val;
            if (slot < AX_MIR) *reinterpret_cast<f32x4*>(lds + r1_off + (uint32_t)(AS_RP1 + slot) * Qs + voff) = val;
            *reinterpret_cast<u32x2*>(lds + meta_off + (uint32_t)((c % AX_MC) * AS_SEG + w) * AX_MW * 4) = u32x2{ma, my};
        };
        // prologue: chunks 0 .. AHEAD + AX_D - 1 in flight, chunks 0 .. AHEAD - 1 landed.
        // Slot of chunk c: (c - AHEAD) mod AX_D, so step s lands and refills slot s mod AX_D.
        f32x4 pre[AS_AHEAD];
        uint32_t pma[AS_AHEAD], pmy[AS_AHEAD];
#pragma unroll
        for (int c = 0; c < AS_AHEAD; ++c) {
            issue(0);
            pre[c] = rv[0];
            pma[c] = rma[0];
            pmy[c] = rmy[0];
        }
#pragma unroll
        for (int k = 0; k < AX_D; ++k) issue(k);
#pragma unroll
        for (int c = 0; c < AS_AHEAD; ++c) land(pre[c], pma[c], pmy[c], c);
        int ca = 0, cc_a = 0;  // pass-A chunk s: position in its line (validity of pixel w)
        // AX_D == ring chunks: every ring slot below is a compile-time function of u
        u32x2 mA;
        barrier();
        mA = *reinterpret_cast<const u32x2*>(mbase);
        for (int b = 0; b < nblk; ++b) {
#pragma unroll
            for (int u = 0; u < AX_D; ++u) {
                const int s = b * AX_D + u;
                // land chunk s + AHEAD from slot u, then refill the slot (chunk s + AHEAD + AX_D)
                AST_T(t0);
                land(rv[u], rma[u], rmy[u], s + AS_AHEAD);
                issue(u);
                AST_T(t1);
                AST_ADD(1, t1 - t0);
                const uint32_t arm = __builtin_amdgcn_readfirstlane(mA.x);
                const float a_y = __uint_as_float(__builtin_amdgcn_readfirstlane(mA.y));
                const float a_b = (float)(int)(arm >> 16);
                const int lo = (int)(arm & 0xffu), hi = (int)((arm >> 8) & 0xffu);
                int st = u * AS_SEG + w - lo;  // ring1 slot of chunk s pixel w, minus the arm
                st = st < 0 ? st + AS_RP1 : st;
                const uint32_t a_off = r1_off + (uint32_t)st * Qs;
                const int a_len = lo + hi + 1;
                mA = *reinterpret_cast<const u32x2*>(mbase + ((u + 1) % AX_MC) * mstep);  // chunk s + 1 (landed)
                const uint32_t r2w = r2_off + (uint32_t)(u * AS_SEG + w) * Qs;  // ring2 slot of chunk s
                if (s < nch && cc_a * AS_SEG + w < S.n) {
                    f32x4 acc = window(a_off, a_len, r1_off, r1_end);
                    if (S.ws) acc = div_ws(acc, a_b, a_y);
                    if (vl) {
                        *reinterpret_cast<f32x4*>(lds + r2w + lane16) = acc;
                        if (u == 0 && w < AX_MIR)
                            *reinterpret_cast<f32x4*>(lds + r2w + (uint32_t)AS_RP2 * Qs + lane16) = acc;
                    }
                }
                if (++cc_a == S.cpl) cc_a = 0;
                (void)ca;
                AST_T(t2);
                AST_ADD(2, t2 - t1);
                barrier();
                AST_T(t3);
                AST_ADD(0, t3 - t2);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no load outlives the workgroup
        AST_FLUSH();
        return;
    }

    // ---- B: pass B over ring2 (FUSED) or pass A's outputs out of ring2, stores ------------
    struct Out {
        int lidx, cc;
        size_t off;
    };
    auto out_init = [&](Out& o) { o.lidx = 0; o.cc = 0; o.off = line_base(0) + (size_t)w * es; };
    auto out_step = [&](Out& o) {
        if (++o.cc == S.cpl) { o.cc = 0; ++o.lidx; if (o.lidx < my_lines) o.off = line_base(o.lidx) + (size_t)w * es; }
        else o.off += (size_t)AS_SEG * es;
    };
    Out ob;
    out_init(ob);
    constexpr int lag = FUSED ? AS_LAG : 1;
    barrier();
    uint32_t mB = *reinterpret_cast<const uint32_t*>(mbase + ((AX_D - lag) % AX_MC) * mstep);  // arms of chunk -lag
    for (int b = 0; b < nblk; ++b) {
#pragma unroll
        for (int u = 0; u < AX_D; ++u) {
            const int s = b * AX_D + u;
            const int ub = (u - lag + 2 * AX_D) % AX_D;  // ring / meta chunk slot of chunk s - lag
            const uint32_t arm = __builtin_amdgcn_readfirstlane(mB);
            const int lo = (int)(arm & 0xffu), hi = (int)((arm >> 8) & 0xffu);
            int st = ub * AS_SEG + w - lo;
            st = st < 0 ? st + AS_RP2 : st;
            const uint32_t b_off = r2_off + (uint32_t)st * Qs;
            const int b_len = lo + hi + 1;
            mB = *reinterpret_cast<const uint32_t*>(mbase + ((ub + 1) % AX_MC) * mstep);
            const uint32_t r2r = r2_off + (uint32_t)(ub * AS_SEG + w) * Qs;  // single: chunk s - 1
            const int sb = s - lag;
            AST_T(t1);
            if (sb >= 0 && sb < nch) {
                if (ob.cc * AS_SEG + w < S.n) {
                    const f32x4 acc = FUSED ? window(b_off, b_len, r2_off, r2_end)
                                            : *reinterpret_cast<const f32x4*>(lds + r2r + lane16);
#ifdef TSM_EXP_AGG_NOSTORE
                    if (vl && acc.x == -1.f) *reinterpret_cast<f32x4*>(volq + ob.off + 4 * lane) = acc;  // timing only
#else
                    if (vl) st_stream(volq + ob.off + 4 * lane, acc);
#endif
                }
                out_step(ob);
            }
            AST_T(t2);
            AST_ADD(2, t2 - t1);
            barrier();
            AST_T(t3);
            AST_ADD(0, t3 - t2);
        }
    }
    AST_FLUSH();
}

// ---------------------------------------------------------------------------
// 1-D aggregation v7: the v6 role split with scalar-lean steps (the default)
// ---------------------------------------------------------------------------
// Same stream, rings, descriptors and roles as v6 (k_agg_split).  v6 is bound by the
// CU's single scalar unit: its 16 waves decode descriptors, loop over window blocks and
// track load positions in SGPRs (PMC: 1.7 scalar per vector instruction; with no HBM
// traffic at all the five launches still take 1.31 ms a pair).  Here every per-pixel
// quantity is a VGPR (descriptor decode, ring offsets, load offsets: uniform values
// kept per lane behind an opaque move), and a window of up to 8 ring pixels is summed
// without a loop: two blocks of 4 reads go out together and a read past the window is
// added as fma(x, 0, acc) == acc (fma(x, 1, acc) == acc + x: one rounding, the same
// value as the reference's add; every slot read holds a finite cost, or padding, whose
// NaN can only land in padding labels, which every consumer ignores).  The rings are
// zeroed once so no uninitialised LDS is ever read.  Lanes past the label vector work on
// the last lane's slot (identical values), so LDS writes need no exec mask.  What stays
// scalar: the window-length class branch, line changes, the B store's validity.
__device__ __forceinline__ uint32_t vopaque(uint32_t x) {
    asm volatile("" : "+v"(x));
    return x;
}
__device__ __forceinline__ f32x4 fmam(f32x4 acc, f32x4 x, float m) {
    return __builtin_elementwise_fma(x, f32x4{m, m, m, m}, acc);
}
// 1 if k < len else 0 (len, k small non-negative integers as floats)
__device__ __forceinline__ float wmask(float lenf, float k) { return __builtin_amdgcn_fmed3f(lenf - k, 0.f, 1.f); }

// WA / WB (roles A / B): 0 = the masked VGPR window above, 1 = v6's scalar window loop
// (uniform offsets and lengths in SGPRs).  Mixing the two moves a role's bookkeeping to
// the issue port the other role leaves idle (the CU issues one SALU and one VALU a cycle).
template <bool FUSED, bool DIV, int QT, int WA = 0, int WB = 0>
__global__ __launch_bounds__(AX_THREADS) void k_agg_v7(AggStream S, DevParams Pk) {
    const DevParams P = Pk;
    pair_shift(blockIdx.z, P.pstride, S.vol, S.arms, S.ws, S.pk, S.rcp);
    extern __shared__ __attribute__((aligned(16))) f32x4 smem_f4[];
    const int H = P.H, W = P.W, Lp = P.Lp;
    const int slice = blockIdx.y;
    const int Q = QT > 0 ? QT : (slice == 0 ? S.qn0 : S.qtot - S.qn0);
    float* const volq = S.vol + 4 * (slice == 0 ? 0 : S.qn0);
    const uint32_t Qs = (uint32_t)Q * 16;
    const size_t vstride = (size_t)H * W * Lp;
    const size_t es = S.horizontal ? (size_t)Lp : (size_t)W * Lp;
    const size_t ls = S.horizontal ? (size_t)W * Lp : (size_t)Lp;
    const size_t aes = S.horizontal ? 1 : (size_t)W;
    const size_t als = S.horizontal ? (size_t)W : 1;
    const int g = blockIdx.x, G = gridDim.x;
    const int my_lines = (S.nl - g + G - 1) / G;
    const int nch = my_lines * S.cpl;
    const uint32_t r2_off = (uint32_t)(AS_RP1 + AX_MIR) * Qs;
    const uint32_t meta_off = r2_off + (uint32_t)(AS_RP2 + AX_MIR) * Qs;
    const uint32_t span1 = (uint32_t)AS_RP1 * Qs, span2 = (uint32_t)AS_RP2 * Qs;
    char* lds = reinterpret_cast<char*>(smem_f4);
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const bool roleA = wave < AS_SEG;
    const int w = roleA ? wave : wave - AS_SEG;
    const int nsteps = nch + (FUSED ? AS_LAG : 1);
    const int nblk = (nsteps + AX_D - 1) / AX_D;
    const bool vl = lane < Q;
    const int lanec = vl ? lane : Q - 1;
    const uint32_t lc16 = (uint32_t)lanec * 16;
    const uint32_t mstep = AS_SEG * AX_MW * 4;
    auto barrier = [&]() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
    // zero both rings (and their mirror slots): masked window reads never see garbage
    for (uint32_t o = (uint32_t)tid * 16; o < meta_off; o += AX_THREADS * 16)
        *reinterpret_cast<f32x4*>(lds + o) = f32x4{0.f, 0.f, 0.f, 0.f};
    barrier();
    // sequential window sum of `len` ring pixels starting at ring-relative byte offset `rel`
    // (a VGPR) of the ring at `base` (lds + ring offset + this lane's 16 B) of `span` bytes
    auto window = [&](const char* base, uint32_t rel, uint32_t len_v, int len, uint32_t span) -> f32x4 {
        const float lenf = (float)len_v;
        const char* p = base + rel;
        const f32x4 x0 = *reinterpret_cast<const f32x4*>(p);
        const f32x4 x1 = *reinterpret_cast<const f32x4*>(p + Qs);
        const f32x4 x2 = *reinterpret_cast<const f32x4*>(p + 2 * Qs);
        const f32x4 x3 = *reinterpret_cast<const f32x4*>(p + 3 * Qs);
        if (len <= 4) {
            f32x4 acc = x0;
            acc = fmam(acc, x1, wmask(lenf, 1.f));
            acc = fmam(acc, x2, wmask(lenf, 2.f));
            acc = fmam(acc, x3, wmask(lenf, 3.f));
            return acc;
        }
        uint32_t r1 = rel + 4 * Qs;
        r1 = min(r1, r1 - span);  // wrap (ring-relative offsets: the subtraction underflows unless r1 >= span)
        const char* q = base + r1;
        const f32x4 x4 = *reinterpret_cast<const f32x4*>(q);
        const f32x4 x5 = *reinterpret_cast<const f32x4*>(q + Qs);
        const f32x4 x6 = *reinterpret_cast<const f32x4*>(q + 2 * Qs);
        const f32x4 x7 = *reinterpret_cast<const f32x4*>(q + 3 * Qs);
        f32x4 acc = x0;
        acc += x1;
        acc += x2;
        acc += x3;
        acc += x4;
        acc = fmam(acc, x5, wmask(lenf, 5.f));
        acc = fmam(acc, x6, wmask(lenf, 6.f));
        acc = fmam(acc, x7, wmask(lenf, 7.f));
        if (len > 8) {  // long windows (rare on natural images): blocks of 4, masked tail
            uint32_t r = r1 + 4 * Qs;
            r = min(r, r - span);
            for (int done = 8; done < len; done += 4) {
                const char* t = base + r;
                const f32x4 y0 = *reinterpret_cast<const f32x4*>(t);
                const f32x4 y1 = *reinterpret_cast<const f32x4*>(t + Qs);
                const f32x4 y2 = *reinterpret_cast<const f32x4*>(t + 2 * Qs);
                const f32x4 y3 = *reinterpret_cast<const f32x4*>(t + 3 * Qs);
                const float d = (float)done;
                acc += y0;
                acc = fmam(acc, y1, wmask(lenf, d + 1.f));
                acc = fmam(acc, y2, wmask(lenf, d + 2.f));
                acc = fmam(acc, y3, wmask(lenf, d + 3.f));
                r += 4 * Qs;
                r = min(r, r - span);
            }
        }
        return acc;
    };
    // ring-relative byte offset of the window start of pixel `slot` (ring pixel index)
    // with left arm lo, in a ring of `span` bytes: (slot - lo) * Qs, wrapped
    auto wstart = [&](uint32_t slotQs, uint32_t lo, uint32_t span) -> uint32_t {
        const uint32_t t = slotQs - lo * Qs;
        return min(t, t + span);
    };
    // v6's window: blocks of 4 at immediate offsets (the mirror slots keep a block
    // contiguous), the 1-3 remaining pixels under uniform branches; `off` ring-relative
    auto window_s = [&](const char* base, uint32_t off, int len, uint32_t span) -> f32x4 {
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int nb = len >> 2; nb > 0; --nb) {
            const char* p = base + off;
            const f32x4 x0 = *reinterpret_cast<const f32x4*>(p);
            const f32x4 x1 = *reinterpret_cast<const f32x4*>(p + Qs);
            const f32x4 x2 = *reinterpret_cast<const f32x4*>(p + 2 * Qs);
            const f32x4 x3 = *reinterpret_cast<const f32x4*>(p + 3 * Qs);
            acc += x0;
            acc += x1;
            acc += x2;
            acc += x3;
            off += 4 * Qs;
            off = off >= span ? off - span : off;
        }
        const int r = len & 3;
        if (r) {
            const char* p = base + off;
            const f32x4 x0 = *reinterpret_cast<const f32x4*>(p);
            const f32x4 x1 = *reinterpret_cast<const f32x4*>(p + Qs);
            const f32x4 x2 = *reinterpret_cast<const f32x4*>(p + 2 * Qs);
            acc += x0;
            if (r > 1) acc += x1;
            if (r > 2) acc += x2;
        }
        return acc;
    };
    const char* mbase = lds + meta_off + (uint32_t)w * AX_MW * 4;  // this wave's pixel column of the meta ring

    if (roleA) {
        // ---- A: staging ring, land, pass A ----------------------------------------------
        const __amdgpu_buffer_rsrc_t rs_vol = make_rsrc(volq), rs_pk = make_rsrc(S.pk),
                                     rs_rcp = make_rsrc(S.rcp);
        const uint32_t es4 = (uint32_t)(es * 4), aes4 = (uint32_t)(aes * 4);
        // issue position (chunk ci = s + AHEAD + AX_D at step s), advanced one chunk a step
        int il = 0, icc = 0;
        uint32_t iv = 0, ia = 0;  // byte offsets of line il: vol, descriptors (= reciprocals)
        auto set_line = [&]() {
            const int gl = g + il * G;
            const int v = gl / S.nlv, line = gl - v * S.nlv;
            iv = (uint32_t)(((size_t)v * vstride + (size_t)line * ls) * 4);
            ia = (uint32_t)(2 * v * H * W + line * (int)als) * 4;  // per-view stride 2HW
        };
        set_line();
        const uint32_t wv = vopaque((uint32_t)w), lastpx = vopaque((uint32_t)(S.n - 1));
        f32x4 rv[AX_D];
        uint32_t rma[AX_D], rmy[AX_D];  // packed descriptor, RN(1/size) bits
        auto issue = [&](int k) {  // chunk at (il, icc) -> slot k; past the end: re-read the last pixel
            const bool past = il >= my_lines;
            // position and offsets in VGPRs (the SGPRs only track the line)
            const uint32_t pos = past ? lastpx : min((uint32_t)(icc * AS_SEG) + wv, lastpx);
            const uint32_t vo = iv + pos * es4 + lc16, mo = ia + pos * aes4;
#ifdef TSM_EXP_AGG_NOLOAD
            rv[k] = f32x4{(float)vo, 0.f, 0.f, 0.f};  // timing experiment only
#else
            rv[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs_vol, vo, 0, 0));
#endif
            rma[k] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs_pk, mo, 0, 0);
            rmy[k] = DIV ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs_rcp, mo, 0, 0) : 0u;
            if (!past && ++icc == S.cpl) {
                icc = 0;
                ++il;
                if (il < my_lines) set_line();
            }
        };
        char* const r1w = lds + (uint32_t)w * Qs + lc16;            // ring1, this wave's pixel column
        const char* const r1b = lds + lc16;                         // ring1 window base
        char* const r2w = lds + r2_off + (uint32_t)w * Qs + lc16;   // ring2, this wave's pixel column
        // pixel w of chunk c -> ring1; its raw descriptor -> the meta ring
        auto land = [&](const f32x4& val, uint32_t ma, uint32_t my, int c) {
            const int cs = (c % AS_RC1) * AS_SEG;  // chunk slot (pixel index of its pixel 0)
            *reinterpret_cast<f32x4*>(r1w + (uint32_t)cs * Qs) = val;
            if (cs == 0 && w < AX_MIR) *reinterpret_cast<f32x4*>(r1w + (uint32_t)AS_RP1 * Qs) = val;
            *reinterpret_cast<u32x2*>(lds + meta_off + (uint32_t)((c % AX_MC) * AS_SEG + w) * AX_MW * 4) = u32x2{ma, my};
        };
        // prologue: chunks 0 .. AHEAD + AX_D - 1 in flight, chunks 0 .. AHEAD - 1 landed
        f32x4 pre[AS_AHEAD];
        uint32_t pma[AS_AHEAD], pmy[AS_AHEAD];
#pragma unroll
        for (int c = 0; c < AS_AHEAD; ++c) {
            issue(0);
            pre[c] = rv[0];
            pma[c] = rma[0];
            pmy[c] = rmy[0];
        }
#pragma unroll
        for (int k = 0; k < AX_D; ++k) issue(k);
#pragma unroll
        for (int c = 0; c < AS_AHEAD; ++c) land(pre[c], pma[c], pmy[c], c);
        barrier();
        u32x2 mA = *reinterpret_cast<const u32x2*>(mbase);
        for (int b = 0; b < nblk; ++b) {
#pragma unroll
            for (int u = 0; u < AX_D; ++u) {
                const int s = b * AX_D + u;
                // land chunk s + AHEAD from slot u, then refill the slot (chunk s + AHEAD + AX_D)
                land(rv[u], rma[u], rmy[u], s + AS_AHEAD);
                issue(u);
                // pass A on chunk s, pixel w (ring1 slot u*8 + w): descriptor in VGPRs
                f32x4 acc;
                if constexpr (WA == 0) {
                    const uint32_t pk = vopaque(mA.x);
                    const float a_y = __uint_as_float(vopaque(mA.y));
                    const uint32_t lo = pk & 0xffu, hi = (pk >> 8) & 0xffu;
                    const float a_b = (float)(pk >> 16);
                    const uint32_t len_v = lo + hi + 1;
                    const int len = (int)__builtin_amdgcn_readfirstlane(len_v);
                    const uint32_t rel = wstart((uint32_t)(u * AS_SEG) * Qs + wv * Qs, lo, span1);
                    mA = *reinterpret_cast<const u32x2*>(mbase + ((u + 1) % AX_MC) * mstep);  // chunk s + 1 (landed)
                    acc = window(r1b, rel, len_v, len, span1);
                    if (DIV) acc = div_ws(acc, a_b, a_y);
                } else {
                    const uint32_t arm = __builtin_amdgcn_readfirstlane(mA.x);
                    const float a_y = __uint_as_float(__builtin_amdgcn_readfirstlane(mA.y));
                    const float a_b = (float)(int)(arm >> 16);
                    const int lo = (int)(arm & 0xffu), hi = (int)((arm >> 8) & 0xffu);
                    int st = u * AS_SEG + w - lo;
                    st = st < 0 ? st + AS_RP1 : st;
                    mA = *reinterpret_cast<const u32x2*>(mbase + ((u + 1) % AX_MC) * mstep);  // chunk s + 1 (landed)
                    acc = window_s(r1b, (uint32_t)st * Qs, lo + hi + 1, span1);
                    if (DIV) acc = div_ws(acc, a_b, a_y);
                }
                // every step writes its ring2 slot (chunks past the stream are never read)
                *reinterpret_cast<f32x4*>(r2w + (uint32_t)(u * AS_SEG) * Qs) = acc;
                if (u == 0 && w < AX_MIR) *reinterpret_cast<f32x4*>(r2w + (uint32_t)AS_RP2 * Qs) = acc;
                barrier();
                (void)s;
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no load outlives the workgroup
        return;
    }

    // ---- B: pass B over ring2 (FUSED) or pass A's outputs out of ring2, stores ------------
    auto line_base = [&](int lidx) -> size_t {
        const int gl = g + lidx * G;
        const int v = gl / S.nlv, line = gl - v * S.nlv;
        return (size_t)v * vstride + (size_t)line * ls;
    };
    int o_l = 0, o_cc = 0;
    size_t o_off = line_base(0) + (size_t)w * es;
    constexpr int lag = FUSED ? AS_LAG : 1;
    const uint32_t wv = vopaque((uint32_t)w);
    const char* const r2b = lds + r2_off + lc16;
    barrier();
    uint32_t mB = *reinterpret_cast<const uint32_t*>(mbase + ((AX_D - lag) % AX_MC) * mstep);  // chunk -lag
    for (int b = 0; b < nblk; ++b) {
#pragma unroll
        for (int u = 0; u < AX_D; ++u) {
            const int s = b * AX_D + u;
            const int ub = (u - lag + 2 * AX_D) % AX_D;  // ring / meta chunk slot of chunk s - lag
            const uint32_t pk = WB == 0 ? vopaque(mB) : __builtin_amdgcn_readfirstlane(mB);
            const uint32_t lo = pk & 0xffu, hi = (pk >> 8) & 0xffu;
            const uint32_t len_v = lo + hi + 1;
            const uint32_t slotQs = (uint32_t)(ub * AS_SEG) * Qs + wv * Qs;
            mB = *reinterpret_cast<const uint32_t*>(mbase + ((ub + 1) % AX_MC) * mstep);
            const int sb = s - lag;
            if (sb >= 0 && sb < nch) {
                if (o_cc * AS_SEG + w < S.n) {
                    f32x4 acc;
                    if (FUSED && WB == 1) {
                        int st = ub * AS_SEG + w - (int)lo;
                        st = st < 0 ? st + AS_RP2 : st;
                        acc = window_s(r2b, (uint32_t)st * Qs, (int)len_v, span2);
                    } else if (FUSED) {
                        const int len = (int)__builtin_amdgcn_readfirstlane(len_v);
                        acc = window(r2b, wstart(slotQs, lo, span2), len_v, len, span2);
                    } else {
                        acc = *reinterpret_cast<const f32x4*>(r2b + slotQs);
                    }
#ifdef TSM_EXP_AGG_NOSTORE
                    if (vl && acc.x == -1.f) *reinterpret_cast<f32x4*>(volq + o_off + 4 * lane) = acc;  // timing only
#else
                    if (vl) st_stream(volq + o_off + 4 * lane, acc);
#endif
                }
                if (++o_cc == S.cpl) {
                    o_cc = 0;
                    ++o_l;
                    if (o_l < my_lines) o_off = line_base(o_l) + (size_t)w * es;
                } else {
                    o_off += (size_t)AS_SEG * es;
                }
            }
            barrier();
        }
    }
}

static size_t agg_split_lds(const DevParams& P) {
    const int Q = P.Lp / 4;
    return ((size_t)AS_RP1 + AS_RP2 + 2 * AX_MIR) * Q * 16 + (size_t)AX_MC * AS_SEG * AX_MW * 4;
}

static size_t agg_stream_lds(const DevParams& P, bool fused) {
    const int Q = P.Lp / 4;
    return ((size_t)AS_RP1 + AX_MIR + (fused ? AS_RP2 + AX_MIR : 0)) * Q * 16 + (size_t)AS_MC * AS_SEG * AS_MW * 4;
}

template <bool FUSED>
static void agg_stream_attrs() {
    (void)hipFuncSetAttribute((const void*)k_agg_stream<FUSED, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)k_agg_stream<FUSED, 49>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

template <bool FUSED, int QT, bool BIG>
static void launch_split_t(const AggStream& S, const DevParams& P, dim3 grid, size_t lds, hipStream_t st) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_agg_split<FUSED, QT, BIG>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
    }
    hipLaunchKernelGGL((k_agg_split<FUSED, QT, BIG>), grid, dim3(AX_THREADS), lds, st, S, P);
}

// Returns -1 if the streamer does not support the geometry (caller falls back).
int launch_agg_stream(float* vol, const uint32_t* arms, const int32_t* ws, const int32_t* ws_base,
                      int horizontal, bool fused, const DevParams& P, hipStream_t st) {
    const int Q = P.Lp / 4;
    if (Q > 128 || P.max_length1 - 1 > AS_MAX_ARM) return -1;
    const bool big = (size_t)2 * P.H * P.W * P.Lp * 4 >= ((size_t)1 << 31);  // past 32-bit offsets
    AggStream S;
    S.vol = vol;
    S.arms = arms;
    S.ws = ws;
    S.rcp = reinterpret_cast<const float*>(ws_base + (size_t)(4 + horizontal) * P.H * P.W);
    S.pk = reinterpret_cast<const uint32_t*>(ws_base + (size_t)(8 + horizontal) * P.H * P.W);
    S.qtot = Q;
    // past 64 label vectors: two slices (blockIdx.y); TSM_AGG_SLICES=2 forces two (A/B)
    static const int force_slices = [] { const char* e = getenv("TSM_AGG_SLICES"); return e ? atoi(e) : 0; }();
    const int nslice = (Q > 64 || force_slices == 2) ? 2 : 1;
    S.qn0 = nslice == 2 ? (Q + 1) / 2 : Q;
    S.horizontal = horizontal;
    S.n = horizontal ? P.W : P.H;
    S.cpl = (S.n + AS_SEG - 1) / AS_SEG;
    S.nlv = horizontal ? P.H : P.W;
    S.nl = 2 * S.nlv;
    static const int ncu = [] {
        int dev = 0, n = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        return n > 0 ? n : 256;
    }();
    const int G = S.nl < ncu ? S.nl : ncu;
    // fused pairs: the role-split v6; single passes: v5 (both sliced / big volumes: v6).
    // TSM_AGG_KERNEL=stream forces v5 where it fits, =split v6 for both.
    static const int pick = [] {
        const char* e = getenv("TSM_AGG_KERNEL");
        return !e ? 0 : (e[0] == 's' && e[1] == 't') ? 1 : (e[0] == 's' && e[1] == 'p') ? 2 : (e[0] == 'v' && e[1] == '7') ? 3 : 0;
    }();
    if (pick == 3 && !big) {  // v7: the scalar-lean role split (same LDS geometry as v6)
        const int qs = S.qn0;
        const size_t slds = ((size_t)AS_RP1 + AS_RP2 + 2 * AX_MIR) * qs * 16 + (size_t)AX_MC * AS_SEG * AX_MW * 4;
        if (slds <= 160 * 1024) {
            const dim3 sgrid(G, nslice, P.npairs);
            const bool div = ws != nullptr;
            auto go = [&](auto kern) {
                static bool attr = false;  // per instantiation
                (void)attr;
                (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
                hipLaunchKernelGGL(kern, sgrid, dim3(AX_THREADS), slds, st, S, P);
            };
            // TSM_AGG_MIX=<A><B>, each v (masked VGPR window) or s (scalar window loop)
            static const int mix = [] {
                const char* e = getenv("TSM_AGG_MIX");
                return !e || !e[0] || !e[1] ? 0 : (e[0] == 's' ? 2 : 0) + (e[1] == 's' ? 1 : 0);
            }();
            if (Q == 49 && nslice == 1 && mix == 2) {  // A scalar, B vector
                if (fused) div ? go(k_agg_v7<true, true, 49, 1, 0>) : go(k_agg_v7<true, false, 49, 1, 0>);
                else div ? go(k_agg_v7<false, true, 49, 1, 0>) : go(k_agg_v7<false, false, 49, 1, 0>);
            } else if (Q == 49 && nslice == 1 && mix == 1) {  // A vector, B scalar
                if (fused) div ? go(k_agg_v7<true, true, 49, 0, 1>) : go(k_agg_v7<true, false, 49, 0, 1>);
                else div ? go(k_agg_v7<false, true, 49, 0, 1>) : go(k_agg_v7<false, false, 49, 0, 1>);
            } else if (Q == 49 && nslice == 1 && mix == 3) {  // both scalar (v6 windows, v7 staging)
                if (fused) div ? go(k_agg_v7<true, true, 49, 1, 1>) : go(k_agg_v7<true, false, 49, 1, 1>);
                else div ? go(k_agg_v7<false, true, 49, 1, 1>) : go(k_agg_v7<false, false, 49, 1, 1>);
            } else if (Q == 49 && nslice == 1) {
                if (fused) div ? go(k_agg_v7<true, true, 49>) : go(k_agg_v7<true, false, 49>);
                else div ? go(k_agg_v7<false, true, 49>) : go(k_agg_v7<false, false, 49>);
            } else {
                if (fused) div ? go(k_agg_v7<true, true, 0>) : go(k_agg_v7<true, false, 0>);
                else div ? go(k_agg_v7<false, true, 0>) : go(k_agg_v7<false, false, 0>);
            }
            trace_point(fused ? "k_agg_v7<fused>" : "k_agg_v7", st);
            return 0;
        }
    }
    const bool v5_fits = Q <= 64 && !big && agg_stream_lds(P, fused) <= 160 * 1024;
    const bool split = pick == 2 || (pick == 0 && fused) || !v5_fits;
    if (split) {
        const int qs = S.qn0;  // the widest slice
        const size_t slds = ((size_t)AS_RP1 + AS_RP2 + 2 * AX_MIR) * qs * 16 + (size_t)AX_MC * AS_SEG * AX_MW * 4;
        if (slds > 160 * 1024) return -1;
        (void)agg_split_lds;
        const dim3 sgrid(G, nslice, P.npairs);
        if (fused) {
            if (big) launch_split_t<true, 0, true>(S, P, sgrid, slds, st);
            else if (Q == 49 && nslice == 1) launch_split_t<true, 49, false>(S, P, sgrid, slds, st);
            else launch_split_t<true, 0, false>(S, P, sgrid, slds, st);
        } else {
            if (big) launch_split_t<false, 0, true>(S, P, sgrid, slds, st);
            else if (Q == 49 && nslice == 1) launch_split_t<false, 49, false>(S, P, sgrid, slds, st);
            else launch_split_t<false, 0, false>(S, P, sgrid, slds, st);
        }
        trace_point(fused ? "k_agg_split<fused>" : "k_agg_split", st);
        return 0;
    }
    static bool attr_set = false;
    if (!attr_set) {
        agg_stream_attrs<false>();
        agg_stream_attrs<true>();
        attr_set = true;
    }
    const size_t lds = agg_stream_lds(P, fused);
    const dim3 grid(G, 1, P.npairs), block(AS_THREADS);
    if (fused) {
        if (Q == 49) hipLaunchKernelGGL((k_agg_stream<true, 49>), grid, block, lds, st, S, P);
        else hipLaunchKernelGGL((k_agg_stream<true, 0>), grid, block, lds, st, S, P);
    } else {
        if (Q == 49) hipLaunchKernelGGL((k_agg_stream<false, 49>), grid, block, lds, st, S, P);
        else hipLaunchKernelGGL((k_agg_stream<false, 0>), grid, block, lds, st, S, P);
    }
    trace_point(fused ? "k_agg_stream<fused>" : "k_agg_stream", st);
    return 0;
}


void launch_arms(const uint32_t* img, uint32_t* arms, const DevParams& P, hipStream_t st) {
    dim3 g((P.W + 127) / 128, P.H, 2 * P.npairs);
    hipLaunchKernelGGL(k_arms, g, dim3(128), 0, st, img, arms, P); trace_point("k_arms", st);
}

void launch_window_sizes(const uint32_t* arms, int32_t* ws, const DevParams& P, hipStream_t st) {
    dim3 g((P.W + 127) / 128, P.H, 2 * P.npairs);
    hipLaunchKernelGGL(k_window_sizes, g, dim3(128), 0, st, arms, ws, P); trace_point("k_window_sizes", st);
}

void launch_color_grad(const uint32_t* img, uint8_t* gv, uint8_t* gh, const DevParams& P,
                       hipStream_t st) {
    dim3 g((P.gstride + 255) / 256, P.H, 2 * P.npairs);
    hipLaunchKernelGGL(k_color_grad, g, dim3(256), 0, st, img, gv, gh, P); trace_point("k_color_grad", st);
}

size_t agg_lds_bytes(const DevParams& P) {
    const int A = P.max_length1 - 1;
    const int nmax = P.W > P.H ? P.W : P.H;
    return (size_t)(AG_SEG + 2 * A) * (P.Lp / 4) * 16 + (size_t)nmax * 8;
}

// Ring geometry of the DMA streamer: returns the LDS bytes and sets RC / D, or 0 when
// fewer than 2 chunks could be in flight (the register-staged kernel is used then).
static size_t agg_dma_geometry(const DevParams& P, int& RC, int& D) {
    const int A = P.max_length1 - 1;
    const int Q = P.Lp / 4;
    const int CS = AGD_SEG * Q;
    const int AH = (A + AGD_SEG - 1) / AGD_SEG;
    const int nmax = P.W > P.H ? P.W : P.H;
    // arms / window sizes, plus the tail pad a block of reads may touch past the ring
    // end (4 pixel vectors and 64 lanes per float4 group)
    const size_t fixed = (size_t)nmax * 8 + (size_t)(4 * Q + 64 * ((Q + 63) / 64)) * 16;
    const size_t chunk = (size_t)CS * 16;
    if (fixed >= 160 * 1024) return 0;
    int rc = (int)((160 * 1024 - fixed) / chunk);
    rc = rc > AGD_MAX_RING ? AGD_MAX_RING : rc;
    static const int dcap = [] {
        const char* e = getenv("TSM_AGG_D");  // tuning override: chunks in flight
        return e ? atoi(e) : 0;
    }();
    if (dcap >= 2 && rc > 2 * AH + 1 + dcap) rc = 2 * AH + 1 + dcap;
    D = rc - (2 * AH + 1);
    D -= (D - 1) % AGD_LOAD_WAVES;  // D - 1 a multiple of the loader count
    if (D < 2) return 0;
    rc = 2 * AH + 1 + D;
    RC = rc;
    return (size_t)rc * chunk + fixed;
}

int launch_agg_line(float* vol, const uint32_t* arms, const int32_t* ws, int horizontal,
                    const DevParams& P, hipStream_t st) {
    const int A = P.max_length1 - 1;
    const int J = (P.Lp / 4 + 63) / 64;
    dim3 g(horizontal ? P.H : P.W, 2, P.npairs);
    static bool attr_set = false;
    if (!attr_set) {
        hipFuncSetAttribute((const void*)k_agg_line<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        hipFuncSetAttribute((const void*)k_agg_line<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        hipFuncSetAttribute((const void*)k_agg_dma<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        hipFuncSetAttribute((const void*)k_agg_dma<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    static const bool use_dma = [] {
        const char* e = getenv("TSM_AGG_KERNEL");  // tuning override: "line" = register-staged
        return !(e && e[0] == 'l');
    }();
    int RC = 0, D = 0;
    const size_t lds_dma = use_dma ? agg_dma_geometry(P, RC, D) : 0;
    if (lds_dma) {
        switch (J) {
            case 1: hipLaunchKernelGGL((k_agg_dma<1>), g, dim3(AGD_THREADS), lds_dma, st, vol, arms, ws, horizontal, A, RC, D, P); break;
            case 2: hipLaunchKernelGGL((k_agg_dma<2>), g, dim3(AGD_THREADS), lds_dma, st, vol, arms, ws, horizontal, A, RC, D, P); break;
            default: return -1;
        }
        trace_point("k_agg_dma", st);
        return 0;
    }
    const size_t lds = agg_lds_bytes(P);
    if (lds > 160 * 1024) return -1;
    switch (J) {
        case 1: hipLaunchKernelGGL((k_agg_line<1>), g, dim3(AG_THREADS), lds, st, vol, arms, ws, horizontal, A, P); break;
        case 2: hipLaunchKernelGGL((k_agg_line<2>), g, dim3(AG_THREADS), lds, st, vol, arms, ws, horizontal, A, P); break;
        default: return -1;
    }
    trace_point("k_agg_line", st);
    return 0;
}

}  // namespace tsm

#ifdef TSM_EXP_STAMPS
extern "C" int tsm_exp_as_stamps(void* host, size_t bytes) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(tsm::g_as_stamps), bytes, 0, hipMemcpyDeviceToHost);
}
extern "C" int tsm_exp_agg_stamps(void* host, size_t bytes) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(tsm::g_agg_stamps), bytes, 0, hipMemcpyDeviceToHost);
}
#endif
