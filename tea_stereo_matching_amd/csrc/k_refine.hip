// k_refine.hip -- step 4 of AD-Census on gfx950: multi-step refinement
// (multiOptimize, ADCensus.cpp:1376-1392).  All maps are H x W int32/u8/fp32; these
// kernels move ~1-2 % of the bytes of the cost-volume stages.
//
//   outlierElimination  :1013-1044   per pixel
//   regionVoting x5     :1046-1159   per outlier; the reference's raster-order vote
//                                    histogram CARRY (cleared only by an outlier with
//                                    vote > votingThresh) is restated as a segmented
//                                    scan: a high-vote outlier's histogram = its own
//                                    samples + the samples of every low-vote outlier
//                                    since the previous high-vote outlier.
//   properInterpolation :1161-1239   per outlier
//   discontinuityAdj.   :1256-1342   equalizeHist + blur 3x3 + Canny(30,90,3,L1)
//                                    (OpenCV 4.x semantics) -> edge-pixel adjustment;
//                                    Canny hysteresis as lock-free union-find
//   subpixelEnhancement :1344-1374   parabola fit + medianBlur 3x3 (fp32, replicate)
#include <algorithm>
#include <utility>

#include "tsm_device.h"
#include "tsm_launch.h"

namespace tsm {

constexpr int kMaxSamples = 20; // = votingThresh: a low-vote outlier holds <= 20 samples
// RefineBufs.hist: the discontinuity stage's 256-bin histogram (+ 64 spare ints)
constexpr int kHistInts = 256 + 64;

// ---------------------------------------------------------------------------
// outlier elimination (LR check)
// ---------------------------------------------------------------------------

// Row form: the reference's occlusion search (does some k in [minD, maxD] have
// dR(x - k) == k?) asks whether any right-view pixel c maps onto x (c + dR(c) == x), so
// each row scatters that map into an LDS bitmap once and every pixel tests one byte.
__global__ __launch_bounds__(256) void k_outlier_row(const int32_t* __restrict__ dl, const int32_t* __restrict__ dr,
                                                     int32_t* __restrict__ out, int32_t* __restrict__ hist, DevParams Pk) {
    const DevParams P = Pk;
    pair_shift(blockIdx.z, P.pstride, dl, dr, out, hist);
    // the discontinuity stage's histogram, LUT and arrival counter start at zero
    if (blockIdx.x == 0)
        for (int k = threadIdx.x; k < kHistInts; k += blockDim.x) hist[k] = 0;
    extern __shared__ uint8_t hit[];
    const int y = blockIdx.x;
    const int W = P.W;
    const int32_t* r = dr + (size_t)y * W;
    for (int x = threadIdx.x; x < W; x += blockDim.x) hit[x] = 0;
    __syncthreads();
    for (int c = threadIdx.x; c < W; c += blockDim.x) {
        const int k = r[c];
        if (k >= P.minD && k <= P.maxD && c + k < W) hit[c + k] = 1;
    }
    __syncthreads();
    for (int x = threadIdx.x; x < W; x += blockDim.x) {
        int d = dl[(size_t)y * W + x];
        if (x - d < 0 || iabs_(d - r[x - d]) > P.disp_tolerance) d = hit[x] ? -2 : -1;  // (:415-416)
        out[(size_t)y * W + x] = d;
    }
}

// ---------------------------------------------------------------------------
// region voting
// ---------------------------------------------------------------------------
__device__ __forceinline__ void region_arms(uint32_t a, bool hf, int& oA, int& oB, int& iA, int& iB) {
    const int up = a & 0xff, dn = (a >> 8) & 0xff, lf = (a >> 16) & 0xff, rt = (a >> 24) & 0xff;
    if (hf) { oA = up; oB = dn; iA = lf; iB = rt; }
    else { oA = lf; oB = rt; iA = up; iB = dn; }
}

// Raster-order ranks of the outliers per block of SC_BLOCK pixels (k_vote_prep).
constexpr int SC_THREADS = 256, SC_ITEMS = 16, SC_BLOCK = SC_THREADS * SC_ITEMS;

// the SC_ITEMS disparities of a thread (16-B loads when the run is whole; the buffers are
// 256-B aligned); past n: INT_MAX, never an outlier
__device__ __forceinline__ void load_items(const int32_t* __restrict__ disp, int base, int n, int (&dv)[SC_ITEMS]) {
    if (base + SC_ITEMS <= n) {
#pragma unroll
        for (int k = 0; k < SC_ITEMS; k += 4) {
            const int4 v = *reinterpret_cast<const int4*>(disp + base + k);
            dv[k] = v.x; dv[k + 1] = v.y; dv[k + 2] = v.z; dv[k + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < SC_ITEMS; ++k) dv[k] = base + k < n ? disp[base + k] : 0x7fffffff;
    }
}

__device__ __forceinline__ void block_scan2(int& a, int& b, int* sa, int* sb) {
    // inclusive scan over the block of (a, b), returns exclusive prefix; totals in sa/sb[SC_THREADS]
    const int t = threadIdx.x;
    sa[t] = a;
    sb[t] = b;
    __syncthreads();
    for (int off = 1; off < SC_THREADS; off <<= 1) {
        int xa = 0, xb = 0;
        if (t >= off) { xa = sa[t - off]; xb = sb[t - off]; }
        __syncthreads();
        sa[t] += xa;
        sb[t] += xb;
        __syncthreads();
    }
    const int ia = sa[t], ib = sb[t];
    a = ia - a;
    b = ib - b;
}


constexpr int RI_B = 4;          // interpolation rays: steps loaded a round trip
constexpr int RW_B = 8;          // region walks: row-segment pixels loaded a round trip (minD >= 0,
                                 // so -1 marks a slot past the segment)


// ---------------------------------------------------------------------------
// region voting, outlier-list form
// ---------------------------------------------------------------------------
// The outliers (disp < minD) are ranked in raster order first (one block scan), so the
// vote count runs on them alone, 16 lanes an outlier, and writes its vote and (for a
// low-vote outlier) its samples straight in rank order; the decision walks, for each
// high-vote outlier, its region and then the low-vote outliers ranked just before it back
// to the previous high-vote one: exactly the histogram the reference carries in raster
// order (:1132-1151).  No per-pixel vote / sample / flag maps and no second scan.
//
// Single-pass scans: a block publishes its count (tagged with the launch's epoch, so a
// stale value from an earlier launch never matches), then sums its predecessors' counts,
// waiting for each to appear.  Workgroups are dispatched in index order, so every block
// waited on is resident or finished and itself waits only on earlier ones: no deadlock.
// One launch instead of a count launch and a scatter launch (round 6: 10 fewer launches a
// frame, the column prefixes 6 fewer).
__device__ __forceinline__ void flag_publish(uint64_t* f, uint32_t epoch, uint32_t v) {
    __hip_atomic_store(f, ((uint64_t)epoch << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t flag_wait(const uint64_t* f, uint32_t epoch) {
    uint64_t x;
    while (((x = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 32) != epoch)
        __builtin_amdgcn_s_sleep(1);
    return (uint32_t)x;
}
// the block's count is published by its last thread; returns the sum of blocks [0, b)
__device__ __forceinline__ int block_exclusive(uint64_t* flags, int b, uint32_t epoch, int total, int* s_base) {
    if (threadIdx.x == SC_THREADS - 1) flag_publish(flags + b, epoch, (uint32_t)total);
    int part = 0;
    for (int i = threadIdx.x; i < b; i += SC_THREADS) part += (int)flag_wait(flags + i, epoch);
    if (part) atomicAdd(s_base, part);
    __syncthreads();
    return *s_base;
}

// Valid-pixel counts of a voting pass's inner segments (valid: disp >= minD, the
// reference's sample test :1122) as differences of prefix counts, exact integer arithmetic in
// any order.  Rows (hf): the raster ranks.  Columns (!hf):
//   P(y, x) = cpre[(y >> 5) W + x] + pre[y W + x], the valid pixels of column x at rows < y
//   (y in [0, H]): pre holds the count inside 32-row chunks, cpre the counts of the chunks
//   before.
// vpre: rank[0 .. N], then pre[(H+1) W], then cpre[(H/32+2) W].
constexpr int VP_CH = 32;
size_t refine_vpre_ints(int H, int W) {
    return (size_t)H * W + 1 + (size_t)(H + 1) * W + (size_t)(H / VP_CH + 2) * W;
}
__host__ __device__ inline size_t vpre_cols_off(int H, int W) { return (size_t)H * W + 1; }
// 64-bit scan flags of a pair slot: the outlier ranking's blocks, the high-vote list's
// blocks, then one per (32-row chunk, column)
size_t refine_flag_words(int H, int W) {
    return 2 * refine_scan_blocks(H * W) + (size_t)(H / VP_CH + 1) * W;
}

// One launch per voting pass before the counts, two roles by block index:
//  * blocks [0, nb): the outliers' raster ranks.  out_list[rank] = pixel of each outlier;
//    dtmp = disp everywhere (the Jacobi output starts as the input; the decision overwrites
//    high-vote outliers); rank[p] = the outliers before pixel p in raster order (rank[n] =
//    all of them): the valid pixels of a raster range [p0, p1] are then
//    (p1 - p0 + 1) - (rank[p1 + 1] - rank[p0]).  The last block writes the totals.
//  * blocks [nb, nb + ncx * nch) (vertical passes only): thread (chunk c, column x) counts
//    the valid pixels of rows [32c, 32c + 32) into pre (local prefix), publishes the
//    chunk's total and sums the chunks above it into cpre[c W + x].
__global__ __launch_bounds__(SC_THREADS) void k_vote_prep(const int32_t* __restrict__ disp, int n, int nb,
                                                          uint64_t* __restrict__ flags, int32_t* __restrict__ out_list,
                                                          int32_t* __restrict__ dtmp, int32_t* __restrict__ counts,
                                                          int32_t* __restrict__ rank, uint32_t epoch, DevParams Pk) {
    const DevParams P = Pk;
    pair_shift(blockIdx.z, P.pstride, disp, flags, out_list, dtmp, counts, rank);
    const int minD = P.minD;
    if ((int)blockIdx.x >= nb) {  // column prefixes
        const int W = P.W, H = P.H;
        const int ncx = (W + SC_THREADS - 1) / SC_THREADS;
        const int j = (int)blockIdx.x - nb, c = j / ncx;
        const int x = (j - c * ncx) * SC_THREADS + threadIdx.x;
        if (x >= W) return;
        int32_t* pre = rank + vpre_cols_off(H, W);
        int32_t* cpre = pre + (size_t)(H + 1) * W;
        uint64_t* cflag = flags + 2 * (size_t)nb;
        const int y0 = c * VP_CH, y1 = min(H, y0 + VP_CH);
        int run = 0;
        int dv[VP_CH];
#pragma unroll
        for (int k = 0; k < VP_CH; ++k) dv[k] = y0 + k < y1 ? disp[(size_t)(y0 + k) * W + x] : -1;
#pragma unroll
        for (int k = 0; k < VP_CH; ++k) {
            // rows y0 .. y1 - 1, and y = H in the chunk holding it (P's local part at y = H)
            if (y0 + k < y1 || (y0 + k == H && H - y0 < VP_CH)) pre[(size_t)(y0 + k) * W + x] = run;
            run += dv[k] >= minD ? 1 : 0;
        }
        flag_publish(cflag + (size_t)c * W + x, epoch, (uint32_t)run);
        int above = 0;
        for (int cc = 0; cc < c; ++cc) above += (int)flag_wait(cflag + (size_t)cc * W + x, epoch);
        cpre[(size_t)c * W + x] = above;
        return;
    }
    __shared__ int sa[SC_THREADS], sb[SC_THREADS];
    __shared__ int s_base;
    if (threadIdx.x == 0) s_base = 0;
    const int base = blockIdx.x * SC_BLOCK + threadIdx.x * SC_ITEMS;
    int dv[SC_ITEMS];
    load_items(disp, base, n, dv);
    int a = 0, b = 0;
#pragma unroll
    for (int k = 0; k < SC_ITEMS; ++k) a += dv[k] < minD ? 1 : 0;
    block_scan2(a, b, sa, sb);  // its barriers also publish s_base = 0
    const int total = sa[SC_THREADS - 1];
    const int first = block_exclusive(flags, blockIdx.x, epoch, total, &s_base);
    a += first;
    if (threadIdx.x == SC_THREADS - 1 && (int)blockIdx.x == nb - 1) {
        counts[0] = first + total;
        counts[1] = 0;
        counts[2] = 0;  // the long-carry list (k_hv_list)
        rank[n] = first + total;
    }
    {
        int rk = a;
#pragma unroll
        for (int k = 0; k < SC_ITEMS; ++k) {
            if (base + k < n) rank[base + k] = rk;
            rk += dv[k] < minD ? 1 : 0;
        }
    }
    if (base + SC_ITEMS <= n) {
#pragma unroll
        for (int k = 0; k < SC_ITEMS; k += 4)
            *reinterpret_cast<int4*>(dtmp + base + k) = make_int4(dv[k], dv[k + 1], dv[k + 2], dv[k + 3]);
    } else {
        for (int k = 0; k < SC_ITEMS && base + k < n; ++k) dtmp[base + k] = dv[k];
    }
#pragma unroll
    for (int k = 0; k < SC_ITEMS; ++k)
        if (dv[k] < minD) out_list[a++] = base + k;
}

// valid pixels of the inner segment at (yy0, xx0), offsets [-a2, b2] along the inner direction
__device__ __forceinline__ int seg_votes(const int32_t* __restrict__ pre, bool hf, int H, int W, int yy0, int xx0,
                                         int a2, int b2) {
    if (hf) {  // raster ranks: the segment is the raster range [p0, p1]
        const size_t p0 = (size_t)yy0 * W + xx0 - a2, p1 = (size_t)yy0 * W + xx0 + b2;
        return (a2 + b2 + 1) - (pre[p1 + 1] - pre[p0]);
    }
    pre += vpre_cols_off(H, W);
    const int32_t* cpre = pre + (size_t)(H + 1) * W;
    const int ya = yy0 - a2, yb = yy0 + b2 + 1;
    return cpre[(size_t)(yb / VP_CH) * W + xx0] + pre[(size_t)yb * W + xx0] -
           cpre[(size_t)(ya / VP_CH) * W + xx0] - pre[(size_t)ya * W + xx0];
}

// Vote count of every ranked outlier, 16 lanes an outlier (4 a wave), grid-stride over
// ranks; lanes take every 16th outer-arm position and a low-vote outlier (every valid
// sample kept) walks its region again to place its samples at the lanes' prefix slots.
__global__ __launch_bounds__(256) void k_vote_count_rank(const int32_t* __restrict__ disp,
                                                         const uint32_t* __restrict__ arms,
                                                         const int32_t* __restrict__ out_list,
                                                         const int32_t* __restrict__ counts,
                                                         int32_t* __restrict__ cvote, uint16_t* __restrict__ csamp,
                                                         const int32_t* __restrict__ vpre, int hf, DevParams Pk) {
    const DevParams P = Pk;
    pair_shift(blockIdx.z, P.pstride, disp, arms, out_list, counts, cvote, csamp, vpre);
    const int lane = threadIdx.x & 63, sub = lane & 15, base = lane & ~15;
    const int W = P.W, minD = P.minD;
    const int nout = counts[0];
    const int ngroups = (gridDim.x * blockDim.x) >> 4;
    // every group of a wave runs the same number of iterations (shuffles stay in step)
    const int g0 = (blockIdx.x * blockDim.x + threadIdx.x) >> 4;
    const int wave_g0 = g0 & ~3;
    for (int it = wave_g0; it < nout; it += ngroups) {
        const int a = it + (g0 & 3);
        const bool valid = a < nout;
        const int p = valid ? out_list[a] : 0;
        const int y = p / W, x = p - y * W;
        int oA = 0, oB = -1, iA, iB;
        if (valid) region_arms(arms[p], hf, oA, oB, iA, iB);
        // the lane's votes: a prefix difference per inner segment (no pixel walk)
        auto votes = [&]() {
            int cnt = 0;
            for (int o = -oA + sub; o <= oB; o += 16) {
                const int yy0 = hf ? y + o : y, xx0 = hf ? x : x + o;
                int a1, b1, a2, b2;
                region_arms(arms[(size_t)yy0 * W + xx0], hf, a1, b1, a2, b2);
                cnt += seg_votes(vpre, hf, P.H, W, yy0, xx0, a2, b2);
            }
            return cnt;
        };
        // a low-vote outlier's samples in the reference's order (segments without a valid
        // pixel skipped)
        auto walk = [&](bool emit, int pos, uint16_t* smp) {
            int cnt = 0;
            for (int o = -oA + sub; o <= oB; o += 16) {
                const int yy0 = hf ? y + o : y, xx0 = hf ? x : x + o;
                int a1, b1, a2, b2;
                region_arms(arms[(size_t)yy0 * W + xx0], hf, a1, b1, a2, b2);
                if (seg_votes(vpre, hf, P.H, W, yy0, xx0, a2, b2) == 0) continue;
                const ptrdiff_t st = hf ? 1 : W;
                const int32_t* rp = disp + (size_t)yy0 * W + xx0;
                // the row segment RW_B pixels a round trip (loads issued back to back, then
                // used in order: the samples keep the reference's order)
                for (int i = -a2; i <= b2; i += RW_B) {
                    int dv[RW_B];
#pragma unroll
                    for (int k = 0; k < RW_B; ++k) dv[k] = i + k <= b2 ? rp[(ptrdiff_t)(i + k) * st] : -1;
#pragma unroll
                    for (int k = 0; k < RW_B; ++k)
                        if (dv[k] >= minD) {
                            if (emit) smp[pos + cnt] = (uint16_t)(dv[k] - minD);
                            cnt++;
                        }
                }
            }
            return cnt;
        };
        const int mine = votes();
        int incl = mine;
#pragma unroll
        for (int d = 1; d < 16; d <<= 1) {
            const int v = __shfl_up(incl, d, 16);
            if (sub >= d) incl += v;
        }
        const int total = __shfl(incl, base + 15);
        if (valid && total <= kMaxSamples && mine > 0) walk(true, incl - mine, csamp + (size_t)a * kMaxSamples);
        if (valid && sub == 0) cvote[a] = total;
    }
}


constexpr int VD_WAVES = 4;
constexpr int VD_CB = 8;      // carried votes loaded a lane per round trip (512 ranks a wave)
constexpr int VD_LONG = 512;  // carries longer than this are decided by a workgroup a rank
constexpr int VL_BLOCKS = 64; // the decision launch's long-carry workgroups

// The high-vote outliers (vote > votingThresh, :1132) listed in rank order: hv_list[k] = the
// rank of the k-th one, counts[1] = how many.  One single-pass launch over the ranks, as the
// outlier ranking (k_vote_prep): its own flags after the ranking's nb.  It also lists the
// high-vote ranks whose carry is longer than VD_LONG ranks (long_list[i] = k, counts[2] = how
// many, zeroed by k_vote_prep), which the decision launch's long-carry workgroups take while
// its waves take the rest: a rank is long when no high-vote rank lies in the VD_LONG + 1 ranks
// before it -- the previous one inside the block from a max-scan of the threads' last
// high-vote ranks, before the block from one search of the block's threads over that window,
// issued before the wait for the preceding blocks' counts (its latency hides behind it).
__global__ __launch_bounds__(SC_THREADS) void k_hv_list(const int32_t* __restrict__ cvote, int32_t* __restrict__ counts,
                                                        uint64_t* __restrict__ flags, int32_t* __restrict__ hv_list,
                                                        int32_t* __restrict__ long_list, int thresh, uint32_t epoch,
                                                        size_t ps) {
    pair_shift(blockIdx.z, ps, cvote, counts, flags, hv_list, long_list);
    constexpr int NW = SC_THREADS / 64;
    __shared__ int s_sum[NW], s_last[NW], s_first[NW];
    __shared__ int s_base, s_found;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    if (t == 0) { s_base = 0; s_found = -1; }
    const int nout = counts[0];
    const int base = blockIdx.x * SC_BLOCK + t * SC_ITEMS;
    int f[SC_ITEMS];
    int a = 0, mylast = -1, myfirst = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < SC_ITEMS; ++k) {
        f[k] = base + k < nout && cvote[base + k] > thresh ? 1 : 0;
        a += f[k];
        if (f[k]) {
            mylast = base + k;
            myfirst = min(myfirst, base + k);
        }
    }
    // per wave: inclusive sums of the counts, inclusive max of the last ranks, min of the first
    int isum = a, ilast = mylast, fmin = myfirst;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int vs = __shfl_up(isum, off), vl = __shfl_up(ilast, off);
        if (lane >= off) { isum += vs; ilast = max(ilast, vl); }
        fmin = min(fmin, __shfl_xor(fmin, off));
    }
    if (lane == 63) { s_sum[wv] = isum; s_last[wv] = ilast; s_first[wv] = fmin; }
    __syncthreads();
    int excl = isum - a, prev = __shfl_up(ilast, 1), total = 0, r0 = 0x7fffffff;
    if (lane == 0) prev = -1;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        if (w < wv) { excl += s_sum[w]; prev = max(prev, s_last[w]); }
        total += s_sum[w];
        r0 = min(r0, s_first[w]);
    }
    // before the block: the nearest high-vote rank among the VD_LONG + 1 ranks before r0, the
    // block's first one (loads issued now, used after the wait below)
    const int bbase = blockIdx.x * SC_BLOCK;
    const bool search = total > 0 && bbase > 0 && r0 - bbase <= VD_LONG;  // block-uniform
    const int lo = max(0, r0 - VD_LONG - 1);
    // (the window is at most VD_LONG + 1 = 513 ranks: two loads a thread and one more)
    static_assert(VD_LONG + 1 <= 2 * SC_THREADS + 1, "the search window's loads");
    int c0 = 0, c1 = 0, c2 = 0;
    const int q0 = bbase - 1 - t, q1 = q0 - SC_THREADS, q2 = bbase - 1 - 2 * SC_THREADS;
    if (search) {
        c0 = q0 >= lo ? cvote[q0] : 0;
        c1 = q1 >= lo ? cvote[q1] : 0;
        c2 = t == 0 && q2 >= lo ? cvote[q2] : 0;
    }
    const int first = block_exclusive(flags + gridDim.x, blockIdx.x, epoch, total, &s_base);
    if (t == SC_THREADS - 1 && blockIdx.x == gridDim.x - 1) counts[1] = first + total;
    int pos = first + excl;  // this thread's first list position
    if (total == 0) return;  // block-uniform
    if (search) {
        const int found = c0 > thresh ? q0 : (c1 > thresh ? q1 : (c2 > thresh ? q2 : -1));
        if (found >= 0) atomicMax(&s_found, found);
        __syncthreads();
    }
    if (prev < 0) prev = s_found;
#pragma unroll
    for (int k = 0; k < SC_ITEMS; ++k)
        if (f[k]) {
            const int r = base + k;
            hv_list[pos] = r;
            // a rank's carry: the ranks strictly between the previous high-vote rank and it
            if (r - prev - 1 > VD_LONG) long_list[atomicAdd(&counts[2], 1)] = pos;
            prev = r;
            ++pos;
        }
}

// The decision, one wave per high-vote outlier r_k (grid-stride over k): its own region into a
// wave-private LDS histogram, then the samples of the low-vote outliers ranked between the
// previous high-vote one r_{k-1} and r_k -- exactly the histogram the reference carries in
// raster order (:1132-1151: hist is cleared only by a high-vote decision) -- then the first
// argmax and the ratio test (:1137-1153).  No workgroup barrier: every wave is independent.
// One launch: workgroups [0, VL_BLOCKS) take the long carries listed by k_hv_list (a
// workgroup a rank, below), the others the rest (a wave a rank), side by side.
template <int NT>
__device__ void vote_decide_long(const int32_t* __restrict__ disp, int32_t* __restrict__ dtmp,
                                 const uint32_t* __restrict__ arms, const int32_t* __restrict__ out_list,
                                 const int32_t* __restrict__ cvote, const uint16_t* __restrict__ csamp,
                                 const int32_t* __restrict__ counts, const int32_t* __restrict__ hv_list,
                                 const int32_t* __restrict__ long_list, int hf, const DevParams& P, int* hist);

__global__ __launch_bounds__(VD_WAVES * 64) void k_vote_decide(
    const int32_t* __restrict__ disp, int32_t* __restrict__ dtmp, const uint32_t* __restrict__ arms,
    const int32_t* __restrict__ out_list, const int32_t* __restrict__ cvote, const uint16_t* __restrict__ csamp,
    const int32_t* __restrict__ counts, const int32_t* __restrict__ hv_list, const int32_t* __restrict__ long_list,
    int hf, DevParams Pk) {
    const DevParams P = Pk;
    pair_shift(blockIdx.z, P.pstride, disp, dtmp, arms, out_list, cvote, csamp, counts, hv_list, long_list);
    extern __shared__ int hist[];
    if ((int)blockIdx.x < VL_BLOCKS) {
        vote_decide_long<VD_WAVES * 64>(disp, dtmp, arms, out_list, cvote, csamp, counts, hv_list, long_list, hf, P,
                                        hist);
        return;
    }
    const int L = P.L, W = P.W, minD = P.minD;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int* h = hist + wv * L;
    const int nhv = counts[1];
    const int bx = (int)blockIdx.x - VL_BLOCKS, gx = (int)gridDim.x - VL_BLOCKS;
    for (int k = bx * VD_WAVES + wv; k < nhv; k += gx * VD_WAVES) {
        const int r = hv_list[k];
        const int prev = k > 0 ? hv_list[k - 1] : -1;
        if (r - prev - 1 > VD_LONG) continue;  // a long carry: one of the long-carry workgroups
        for (int d = lane; d < L; d += 64) h[d] = 0;
        wave_lds_sync();  // the zeroed bins before any lane's atomics (lanes share the histogram)
        const int p = out_list[r];
        const int v = cvote[r];
        const int y = p / W, x = p - y * W;
        int oA, oB, iA, iB;
        region_arms(arms[p], hf, oA, oB, iA, iB);
        // a region is mostly one or two disparities: each lane counts into a private two-entry
        // cache and adds an entry to the histogram only when it is evicted (64 lanes' atomics on
        // one bin serialise); the counts are exact either way
        int cd0 = -1, cn0 = 0, cd1 = -1, cn1 = 0;
        for (int o = -oA + lane; o <= oB; o += 64) {
            const int yy0 = hf ? y + o : y, xx0 = hf ? x : x + o;
            int a1, b1, a2, b2;
            region_arms(arms[(size_t)yy0 * W + xx0], hf, a1, b1, a2, b2);
            const ptrdiff_t st = hf ? 1 : W;
            const int32_t* rp = disp + (size_t)yy0 * W + xx0;
            for (int i = -a2; i <= b2; i += RW_B) {  // RW_B loads a round trip
                int dv[RW_B];
#pragma unroll
                for (int kk = 0; kk < RW_B; ++kk) dv[kk] = i + kk <= b2 ? rp[(ptrdiff_t)(i + kk) * st] : -1;
#pragma unroll
                for (int kk = 0; kk < RW_B; ++kk) {
                    const int d = dv[kk];
                    if (d >= minD) {
                        if (d == cd0) ++cn0;
                        else if (d == cd1) ++cn1;
                        else {
                            if (cn1) atomicAdd(&h[cd1 - minD], cn1);
                            cd1 = cd0; cn1 = cn0; cd0 = d; cn0 = 1;
                        }
                    }
                }
            }
        }
        if (cn0) atomicAdd(&h[cd0 - minD], cn0);
        if (cn1) atomicAdd(&h[cd1 - minD], cn1);
        // the carried samples: low-vote outliers ranked in (prev, r), VD_CB * 64 votes a round
        // trip (synthetic scenes carry thousands of ranks, most without a sample)
        for (int kb = prev + 1; kb < r; kb += VD_CB * 64) {
            int c[VD_CB];
#pragma unroll
            for (int j = 0; j < VD_CB; ++j) {
                const int kk = kb + j * 64 + lane;
                c[j] = kk < r ? cvote[kk] : 0;
            }
#pragma unroll
            for (int j = 0; j < VD_CB; ++j) {
                if (c[j] > 0 && c[j] <= P.voting_thresh) {
                    const int kk = kb + j * 64 + lane;
                    const uint32_t* sp = reinterpret_cast<const uint32_t*>(csamp + (size_t)kk * kMaxSamples);
                    uint32_t w2[kMaxSamples / 2];
#pragma unroll
                    for (int i = 0; i < kMaxSamples / 2; ++i) w2[i] = sp[i];
#pragma unroll
                    for (int m = 0; m < kMaxSamples; ++m)
                        if (m < c[j]) atomicAdd(&h[(w2[m >> 1] >> (16 * (m & 1))) & 0xffffu], 1);
                }
            }
        }
        wave_lds_sync();  // every lane's atomics before the argmax reads
        uint64_t best = ~0ull;
        for (int d = lane; d < L; d += 64) {
            const uint64_t key = ((uint64_t)(0xffffffffu - (uint32_t)h[d]) << 32) | (uint32_t)d;
            best = key < best ? key : best;
        }
        best = wave_min_u64(best);
        const int cmax = (int)(0xffffffffu - (uint32_t)(best >> 32));
        const int dbest = (int)(uint32_t)best;
        const float ratio = cmax / (float)v;
        if (lane == 0) dtmp[p] = ratio > P.voting_ratio && cmax > 0 ? dbest + minD : disp[p];
    }
}

// The high-vote outliers whose carry is longer than VD_LONG ranks (synthetic scenes: a few
// per pass, carrying thousands of low-vote outliers), a workgroup of NT threads each: the region split over
// its threads by outer position, the carry over all its threads, then the same decision.
template <int NT>
__device__ void vote_decide_long(const int32_t* __restrict__ disp, int32_t* __restrict__ dtmp,
                                 const uint32_t* __restrict__ arms, const int32_t* __restrict__ out_list,
                                 const int32_t* __restrict__ cvote, const uint16_t* __restrict__ csamp,
                                 const int32_t* __restrict__ counts, const int32_t* __restrict__ hv_list,
                                 const int32_t* __restrict__ long_list, int hf, const DevParams& P, int* hist) {
    constexpr int VL_THREADS = NT;
    const int L = P.L, W = P.W, minD = P.minD;
    const int tid = threadIdx.x, lane = tid & 63;
    const int nlong = counts[2];
    for (int i = blockIdx.x; i < nlong; i += VL_BLOCKS) {
        const int k = long_list[i];
        const int r = hv_list[k];
        const int prev = k > 0 ? hv_list[k - 1] : -1;
        for (int d = tid; d < L; d += VL_THREADS) hist[d] = 0;
        __syncthreads();
        const int p = out_list[r];
        const int v = cvote[r];
        const int y = p / W, x = p - y * W;
        int oA, oB, iA, iB;
        region_arms(arms[p], hf, oA, oB, iA, iB);
        for (int o = -oA + tid; o <= oB; o += VL_THREADS) {
            const int yy0 = hf ? y + o : y, xx0 = hf ? x : x + o;
            int a1, b1, a2, b2;
            region_arms(arms[(size_t)yy0 * W + xx0], hf, a1, b1, a2, b2);
            const ptrdiff_t st = hf ? 1 : W;
            const int32_t* rp = disp + (size_t)yy0 * W + xx0;
            for (int ii = -a2; ii <= b2; ii += RW_B) {  // RW_B loads a round trip
                int dv[RW_B];
#pragma unroll
                for (int kk = 0; kk < RW_B; ++kk) dv[kk] = ii + kk <= b2 ? rp[(ptrdiff_t)(ii + kk) * st] : -1;
#pragma unroll
                for (int kk = 0; kk < RW_B; ++kk)
                    if (dv[kk] >= minD) atomicAdd(&hist[dv[kk] - minD], 1);
            }
        }
        for (int kb = prev + 1; kb < r; kb += VD_CB * VL_THREADS) {
            int c[VD_CB];
#pragma unroll
            for (int j = 0; j < VD_CB; ++j) {
                const int kk = kb + j * VL_THREADS + tid;
                c[j] = kk < r ? cvote[kk] : 0;
            }
#pragma unroll
            for (int j = 0; j < VD_CB; ++j) {
                if (c[j] > 0 && c[j] <= P.voting_thresh) {
                    const int kk = kb + j * VL_THREADS + tid;
                    const uint32_t* sp = reinterpret_cast<const uint32_t*>(csamp + (size_t)kk * kMaxSamples);
                    uint32_t w2[kMaxSamples / 2];
#pragma unroll
                    for (int ii = 0; ii < kMaxSamples / 2; ++ii) w2[ii] = sp[ii];
#pragma unroll
                    for (int m = 0; m < kMaxSamples; ++m)
                        if (m < c[j]) atomicAdd(&hist[(w2[m >> 1] >> (16 * (m & 1))) & 0xffffu], 1);
                }
            }
        }
        __syncthreads();
        if (tid < 64) {
            uint64_t best = ~0ull;
            for (int d = lane; d < L; d += 64) {
                const uint64_t key = ((uint64_t)(0xffffffffu - (uint32_t)hist[d]) << 32) | (uint32_t)d;
                best = key < best ? key : best;
            }
            best = wave_min_u64(best);
            const int cmax = (int)(0xffffffffu - (uint32_t)(best >> 32));
            const int dbest = (int)(uint32_t)best;
            const float ratio = cmax / (float)v;
            if (lane == 0) dtmp[p] = ratio > P.voting_ratio && cmax > 0 ? dbest + minD : disp[p];
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// proper interpolation
// ---------------------------------------------------------------------------
// 16 rays of (:1166-1167); the reference steps d/2 then d - d/2 (C++ truncating /2).
__constant__ int c_ray_h[16] = {2, 2, 0, -2, -2, -2, 0, 2, 2, 1, -1, -2, -2, -1, 1, 2};
__constant__ int c_ray_w[16] = {0, 2, 2, 2, 0, -2, -2, -2, 1, 2, 2, 1, -1, -2, -2, -1};

// The per-ray results are folded as each ray finishes, in ray order, which is exactly
// the reference's two post-loops (:1211-1216 min for occlusions, :1222-1231 colour-diff
// selection for mismatches): no per-thread arrays, no dynamic register indexing.

// Ray-parallel form: 16 lanes per pixel, lane = ray, 4 pixels a wave.  The rays' dependent
// load chains (<= max_search_depth steps each) run side by side instead of one after
// another; the per-ray results are then folded in ray order exactly as above (a min for
// occlusions, the colour-difference rule for mismatches).
// Over the last voting pass's ranked outliers only (round 6; grid-stride over the ranks): the
// Jacobi output dtmp already equals the map everywhere else -- k_vote_prep copied the pass's
// input into it and the decision changed only ranked outliers -- so a ranked pixel that the
// decision made valid is copied, an outlier is interpolated, and nothing else is touched
// (one pixel group a rank instead of a 16-lane group for every pixel of the image).
__global__ __launch_bounds__(256) void k_interp_rays(const int32_t* __restrict__ disp, int32_t* __restrict__ out,
                                                     const uint32_t* __restrict__ img0,
                                                     const int32_t* __restrict__ out_list,
                                                     const int32_t* __restrict__ counts, DevParams Pk) {
    const DevParams P = Pk;
    pair_shift(blockIdx.z, P.pstride, disp, out, img0, out_list, counts);
    const int lane = threadIdx.x & 63;
    const int dir = lane & 15;
    const int H = P.H, W = P.W, minD = P.minD;
    const int nout = counts[0];
    const int ngroups = (gridDim.x * blockDim.x) >> 4;
    // every group of a wave runs the same number of iterations (shuffles stay in step)
    const int g0 = (blockIdx.x * blockDim.x + threadIdx.x) >> 4;
    for (int it = g0 & ~3; it < nout; it += ngroups) {
        const int a = it + (g0 & 3);
        const bool inside = a < nout;
        const int p = inside ? out_list[a] : out_list[nout - 1];
        const int y = p / W, x = p - y * W;
        const size_t idx = (size_t)p;
        const int cur = disp[idx];
        const bool outlier = inside && cur < minD;
        int nd = cur, ndiff = -1;
        if (outlier) {
            const uint32_t c0 = img0[idx];
            const int rh = c_ray_h[dir], rw = c_ray_w[dir];
            const int sh0 = rh / 2, sh1 = rh - rh / 2, sw0 = rw / 2, sw1 = rw - rw / 2;
            // RI_B steps a round trip: their positions, then their loads back to back, then the
            // first in-image valid one in step order (a ray moves monotonically, so it never
            // re-enters the image once it has left it)
            int hD = y, wD = x;
            bool done = false;
            for (int s0 = 0; s0 < P.max_search_depth && !done; s0 += RI_B) {
                size_t at[RI_B];
                bool ok[RI_B];
                int dv[RI_B];
#pragma unroll
                for (int k = 0; k < RI_B; ++k) {
                    const int s = s0 + k;
                    hD += (s & 1) ? sh1 : sh0;
                    wD += (s & 1) ? sw1 : sw0;
                    ok[k] = s < P.max_search_depth && hD >= 0 && hD < H && wD >= 0 && wD < W;
                    at[k] = ok[k] ? (size_t)hD * W + wD : idx;
                }
#pragma unroll
                for (int k = 0; k < RI_B; ++k) dv[k] = ok[k] ? disp[at[k]] : 0;
#pragma unroll
                for (int k = 0; k < RI_B; ++k) {
                    if (done) break;
                    if (!ok[k]) { done = true; break; }
                    if (dv[k] >= minD) {
                        nd = dv[k];
                        ndiff = color_diff(P, c0, img0[at[k]]);
                        done = true;
                    }
                }
            }
        }
        // fold the 16 rays of this lane's pixel in ray order (every lane of the group
        // computes the same result; lane dir == 0 writes it)
        const int base = lane & ~15;
        const bool occlusion = cur == minD - 1;  // :1209
        int res = 0, mdiff = -1;
#pragma unroll
        for (int d = 0; d < 16; ++d) {
            const int n_d = __shfl(nd, base + d);
            const int f_d = __shfl(ndiff, base + d);
            if (occlusion) {
                res = d == 0 ? n_d : min(res, n_d);
            } else if (d == 0) {
                res = n_d;
                mdiff = f_d;
            } else if (mdiff < 0 || (mdiff > f_d && f_d > 0)) {
                res = n_d;
                mdiff = f_d;
            }
        }
        if (inside && dir == 0) out[idx] = outlier ? res : cur;
    }
}

// ---------------------------------------------------------------------------
// discontinuity adjustment: gray -> equalizeHist -> blur -> Canny -> adjust, then subpixel +
// median.  Round 6: 14 launches -> 6 (the hist zeroing rides on k_outlier_row, the LUT is
// built by each block of the Canny launch, equalisation + blur + Sobel + NMS share one tiled launch, and the edge
// test, the adjustment, the subpixel step and the median another): every stage keeps its
// own arithmetic, so the outputs are the same bytes.
// ---------------------------------------------------------------------------
// gray = (uchar)max(d, 0) (:1249, wraps > 255) and its histogram (the LUT is built by every
// block of k_canny_front from it: a last-block LUT here needed a device-scope fence in every
// block, which wrote the gray bytes back out of L2 -- 67 against 15 us, round 6).  A thread
// takes 16 consecutive pixels (16-B loads and one 16-B store) and adds each run of equal
// values to the block's histogram once: a disparity map is piecewise constant, and one LDS
// atomic per pixel serialised on the few busy bins.
__global__ __launch_bounds__(256) void k_gray_hist(const int32_t* __restrict__ disp, uint8_t* __restrict__ gray,
                                                   int32_t* __restrict__ hist, int n, size_t ps) {
    pair_shift(blockIdx.z, ps, disp, gray, hist);
    __shared__ int h[256];
    const int k = threadIdx.x;
    h[k] = 0;
    __syncthreads();
    const int base = (blockIdx.x * 256 + k) * SC_ITEMS;
    if (base < n) {
        int dv[SC_ITEMS];
        load_items(disp, base, n, dv);  // past n: INT_MAX
        uint8_t g[SC_ITEMS];
#pragma unroll
        for (int i = 0; i < SC_ITEMS; ++i) g[i] = dv[i] < 0 ? 0 : (uint8_t)dv[i];  // (uchar) wraps > 255 (:1249)
        int run = 0;
        for (int i = 0; i < SC_ITEMS && base + i < n; ++i) {
            ++run;
            if (i + 1 == SC_ITEMS || base + i + 1 >= n || g[i + 1] != g[i]) {
                atomicAdd(&h[g[i]], run);
                run = 0;
            }
        }
        if (base + SC_ITEMS <= n) {
            uint32_t w[4];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                w[q] = g[4 * q] | (g[4 * q + 1] << 8) | (g[4 * q + 2] << 16) | ((uint32_t)g[4 * q + 3] << 24);
            *reinterpret_cast<uint4*>(gray + base) = make_uint4(w[0], w[1], w[2], w[3]);
        } else {
            for (int i = 0; i < SC_ITEMS && base + i < n; ++i) gray[base + i] = g[i];
        }
    }
    __syncthreads();
    if (h[k]) atomicAdd(&hist[k], h[k]);
}

// equalizeHist LUT (imgproc histogram.cpp) entry k of a 256-thread block: lut[i] =
// saturate_cast<uchar>(sum * scale), scale = 255.f / (total - hist[first nonzero]), from an
// exact integer prefix scan in LDS
__device__ __forceinline__ uint8_t eq_lut_entry(const int32_t* __restrict__ hist, int total, int* pre, int* first) {
    const int k = threadIdx.x;
    const int hk = hist[k];
    pre[k] = hk;
    if (k == 0) *first = 256;
    __syncthreads();
    if (hk != 0) atomicMin(first, k);
    for (int off = 1; off < 256; off <<= 1) {  // inclusive prefix sums
        const int add = k >= off ? pre[k - off] : 0;
        __syncthreads();
        pre[k] += add;
        __syncthreads();
    }
    const int i = *first;
    uint8_t out = 0;
    if (i < 256) {
        const int hi = pre[i] - (i > 0 ? pre[i - 1] : 0);
        if (hi == total) {
            out = k == i ? (uint8_t)i : 0;
        } else if (k > i) {
            const float scale = (256 - 1.f) / (float)(total - hi);
            const int sum = pre[k] - pre[i];  // hist[i + 1] + ... + hist[k], in the serial order's value
            const int v = (int)rintf((float)sum * scale);
            out = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
        }
    }
    return out;
}

__device__ __forceinline__ int reflect101(int i, int n) {
    if (n == 1) return 0;
    if (i < 0) i = -i;
    if (i >= n) i = 2 * n - 2 - i;
    return i;
}

// Canny front end on a TX x TY tile: the equalisation LUT (each block builds it from the
// histogram) -> the equalised map -> blur 3x3 BORDER_REFLECT_101
// with the ColumnSum<ushort,uchar> fixed-point divide ((s+4)*932068)>>23 == round(s/9) -> Sobel
// 3x3 (BORDER_REPLICATE), L1 magnitude -> non-maximum suppression (canny.cpp TG22 fixed point,
// zero magnitude outside the image).  Each stage runs on the tile plus the halo the next
// needs (3, 2, 1 pixels), in LDS.  map: 1 = not an edge, 0 = weak candidate, 2 = strong
// (m > high).  Also writes the equalised map (debug dumps) and zeroes the hysteresis's
// strong-root bytes.
constexpr int CF_TX = 32, CF_TY = 8;
__global__ __launch_bounds__(256) void k_canny_front(const uint8_t* __restrict__ gray, const int32_t* __restrict__ hist,
                                                     uint8_t* __restrict__ eq_out, uint8_t* __restrict__ map,
                                                     uint8_t* __restrict__ strong, int H, int W, int low, int high,
                                                     size_t ps) {
    pair_shift(blockIdx.z, ps, gray, hist, eq_out, map, strong);
    constexpr int EW = CF_TX + 6, EH = CF_TY + 6;  // equalised: halo 3
    constexpr int BW = CF_TX + 4, BH = CF_TY + 4;  // blurred: halo 2
    constexpr int SW = CF_TX + 2, SH = CF_TY + 2;  // Sobel: halo 1
    __shared__ uint8_t lut[256];
    __shared__ int pre[256];
    __shared__ int first;
    __shared__ uint8_t se[EH][EW];
    __shared__ uint8_t sbl[BH][BW];
    __shared__ int smag[SH][SW];
    __shared__ int16_t sdx[SH][SW], sdy[SH][SW];
    const int x0 = blockIdx.x * CF_TX, y0 = blockIdx.y * CF_TY;
    const int t = threadIdx.x;
    lut[t] = eq_lut_entry(hist, H * W, pre, &first);
    __syncthreads();
    // region coordinates: e(r, c) is image (y0 - 3 + r, x0 - 3 + c); only in-image cells are
    // ever read (reflect101 / clamps land inside the image, and inside these regions)
    for (int k = t; k < EH * EW; k += 256) {
        const int r = k / EW, c = k - r * EW;
        const int yy = y0 - 3 + r, xx = x0 - 3 + c;
        se[r][c] = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? lut[gray[(size_t)yy * W + xx]] : 0;
    }
    __syncthreads();
    for (int k = t; k < BH * BW; k += 256) {
        const int r = k / BW, c = k - r * BW;
        const int y = y0 - 2 + r, x = x0 - 2 + c;
        if (y < 0 || y >= H || x < 0 || x >= W) continue;
        int s = 0;
        for (int dy = -1; dy <= 1; ++dy) {
            const int yy = reflect101(y + dy, H) - (y0 - 3);
            for (int dx = -1; dx <= 1; ++dx) s += se[yy][reflect101(x + dx, W) - (x0 - 3)];
        }
        sbl[r][c] = (uint8_t)(((s + 4) * 932068) >> 23);
    }
    __syncthreads();
    for (int k = t; k < SH * SW; k += 256) {
        const int r = k / SW, c = k - r * SW;
        const int y = y0 - 1 + r, x = x0 - 1 + c;
        if (y < 0 || y >= H || x < 0 || x >= W) continue;
        auto S = [&](int yy, int xx) -> int {
            yy = yy < 0 ? 0 : (yy >= H ? H - 1 : yy);
            xx = xx < 0 ? 0 : (xx >= W ? W - 1 : xx);
            return sbl[yy - (y0 - 2)][xx - (x0 - 2)];
        };
        const int gx = (S(y - 1, x + 1) + 2 * S(y, x + 1) + S(y + 1, x + 1)) -
                       (S(y - 1, x - 1) + 2 * S(y, x - 1) + S(y + 1, x - 1));
        const int gy = (S(y + 1, x - 1) + 2 * S(y + 1, x) + S(y + 1, x + 1)) -
                       (S(y - 1, x - 1) + 2 * S(y - 1, x) + S(y - 1, x + 1));
        sdx[r][c] = (int16_t)gx;
        sdy[r][c] = (int16_t)gy;
        smag[r][c] = abs(gx) + abs(gy);
    }
    __syncthreads();
    const int x = x0 + (t % CF_TX), y = y0 + t / CF_TX;
    if (x >= W || y >= H) return;
    auto M = [&](int yy, int xx) -> int {
        if (yy < 0 || yy >= H || xx < 0 || xx >= W) return 0;
        return smag[yy - (y0 - 1)][xx - (x0 - 1)];
    };
    const int r = y - (y0 - 1), c = x - (x0 - 1);
    const int m = smag[r][c];
    bool keep = false;
    if (m > low) {
        const int xs = sdx[r][c], ys = sdy[r][c];
        const int ax = abs(xs);
        const int ay = abs(ys) << 15;
        const int tg22x = ax * 13573;  // (int)(0.4142135623730950488 * (1 << 15) + 0.5)
        if (ay < tg22x) {
            keep = m > M(y, x - 1) && m >= M(y, x + 1);
        } else {
            const int tg67x = tg22x + (ax << 16);
            if (ay > tg67x) {
                keep = m > M(y - 1, x) && m >= M(y + 1, x);
            } else {
                const int s = (xs ^ ys) < 0 ? -1 : 1;
                keep = m > M(y - 1, x - s) && m > M(y + 1, x + s);
            }
        }
    }
    const size_t i = (size_t)y * W + x;
    map[i] = !keep ? 1 : (m > high ? 2 : 0);
    eq_out[i] = se[y - (y0 - 3)][x - (x0 - 3)];
    strong[i] = 0;
}

// Hysteresis = 8-connected components of {map != 1} containing a strong pixel.
// Lock-free union-find: links always point to the smaller index (no cycles); a root is
// re-linked only by CAS, so stale reads just cost a retry.
__device__ __forceinline__ int uf_find(int* parent, int x) {
    int p = __hip_atomic_load(&parent[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (p != x) {
        x = p;
        p = __hip_atomic_load(&parent[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return x;
}
__device__ __forceinline__ void uf_union(int* parent, int a, int b) {
    while (true) {
        a = uf_find(parent, a);
        b = uf_find(parent, b);
        if (a == b) return;
        if (a < b) { const int t = a; a = b; b = t; }
        const int old = atomicCAS(&parent[a], a, b);
        if (old == a) return;
        a = old;
    }
}



// Tiled form: union-find inside a 32x32 tile in LDS (LDS atomics), global labels are
// the tile roots' pixel indices; then only the pairs crossing a tile edge merge in global
// memory.
constexpr int UT = 32;

__device__ __forceinline__ int lds_find(int* lab, int x) {
    int p = __hip_atomic_load(&lab[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (p != x) {
        x = p;
        p = __hip_atomic_load(&lab[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    return x;
}
__device__ __forceinline__ void lds_union(int* lab, int a, int b) {
    while (true) {
        a = lds_find(lab, a);
        b = lds_find(lab, b);
        if (a == b) return;
        if (a < b) { const int t = a; a = b; b = t; }
        const int old = atomicCAS(&lab[a], a, b);
        if (old == a) return;
        a = old;
    }
}

__global__ __launch_bounds__(256) void k_uf_tile(const uint8_t* __restrict__ map, int32_t* __restrict__ label,
                                                 int H, int W, size_t ps) {
    pair_shift(blockIdx.z, ps, map, label);
    __shared__ int lab[UT * UT];
    const int tx0 = blockIdx.x * UT, ty0 = blockIdx.y * UT;
    for (int k = threadIdx.x; k < UT * UT; k += 256) {
        const int x = tx0 + (k % UT), y = ty0 + k / UT;
        lab[k] = (x < W && y < H && map[(size_t)y * W + x] != 1) ? k : -1;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < UT * UT; k += 256) {
        if (lab[k] < 0) continue;
        const int lx = k % UT, ly = k / UT;
        if (lx > 0 && lab[k - 1] >= 0) lds_union(lab, k, k - 1);
        if (ly > 0) {
            if (lx > 0 && lab[k - UT - 1] >= 0) lds_union(lab, k, k - UT - 1);
            if (lab[k - UT] >= 0) lds_union(lab, k, k - UT);
            if (lx + 1 < UT && lab[k - UT + 1] >= 0) lds_union(lab, k, k - UT + 1);
        }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < UT * UT; k += 256) {
        const int x = tx0 + (k % UT), y = ty0 + k / UT;
        if (x >= W || y >= H) continue;
        int g = -1;
        if (lab[k] >= 0) {
            const int r = lds_find(lab, k);
            g = (ty0 + r / UT) * W + tx0 + r % UT;
        }
        label[(size_t)y * W + x] = g;
    }
}

__global__ void k_uf_edges(const uint8_t* __restrict__ map, int32_t* __restrict__ label, int H, int W, size_t ps) {
    pair_shift(blockIdx.z, ps, map, label);
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    if (x >= W) return;
    const int lx = x % UT, ly = y % UT;
    if (ly != 0 && lx != 0 && lx != UT - 1) return;  // no neighbour pair leaves the tile
    const int i = y * W + x;
    if (map[i] == 1) return;
    if (lx == 0 && x > 0 && map[i - 1] != 1) uf_union(label, i, i - 1);
    if (y > 0) {
        if ((lx == 0 || ly == 0) && x > 0 && map[i - W - 1] != 1) uf_union(label, i, i - W - 1);
        if (ly == 0 && map[i - W] != 1) uf_union(label, i, i - W);
        if ((ly == 0 || lx == UT - 1) && x + 1 < W && map[i - W + 1] != 1) uf_union(label, i, i - W + 1);
    }
}

__global__ void k_uf_flatten_mark(const uint8_t* __restrict__ map, int32_t* __restrict__ label,
                                  uint8_t* __restrict__ strong, int n, size_t ps) {
    pair_shift(blockIdx.z, ps, map, label, strong);
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || map[i] == 1) return;
    int r = i;
    while (label[r] != r) r = label[r];
    label[i] = r;
    if (map[i] == 2) strong[r] = 1;
}

// discontinuityAdjustment body (:1266-1339) for pixel (x, y) of the pre-adjust map; E(yy, xx):
// the Canny edge test of a neighbour
template <class EF>
__device__ __forceinline__ int adjust_px(const int32_t* __restrict__ disp, const float* __restrict__ vol0, int x, int y,
                                         const DevParams& P, EF E) {
    const int H = P.H, W = P.W, minD = P.minD, Lp = P.Lp;
    const size_t i = (size_t)y * W + x;
    int res = disp[i];
    if (y >= 1 && y < H - 1 && x >= 1 && x < W - 1 && E(y, x)) {
        int direction = -1;
        if (E(y - 1, x - 1) && E(y + 1, x + 1)) direction = 0;
        else if (E(y - 1, x + 1) && E(y + 1, x - 1)) direction = 4;
        else if (E(y - 1, x) || E(y + 1, x)) {
            if (E(y - 1, x - 1) || E(y - 1, x) || E(y - 1, x + 1))
                if (E(y + 1, x - 1) || E(y + 1, x) || E(y + 1, x + 1)) direction = 2;
        } else {
            if (E(y - 1, x - 1) || E(y, x - 1) || E(y + 1, x - 1))
                if (E(y - 1, x + 1) || E(y, x + 1) || E(y + 1, x + 1)) direction = 6;
        }
        if (direction != -1) {
            const int dHt[8] = {-1, 1, -1, 1, -1, 1, 0, 0};
            const int dWt[8] = {-1, 1, 0, 0, 1, -1, -1, 1};
            int dsel = res;
            direction = (direction + 4) % 8;
            if (dsel >= minD) {
                float cost = vol0[i * Lp + (dsel - minD)];
                const int y1 = y + dHt[direction], x1 = x + dWt[direction];
                const int y2 = y + dHt[direction + 1], x2 = x + dWt[direction + 1];
                const size_t i1 = (size_t)y1 * W + x1, i2 = (size_t)y2 * W + x2;
                const int d1 = disp[i1], d2 = disp[i2];
                const float cost1 = d1 >= minD ? vol0[i1 * Lp + (d1 - minD)] : -1.f;
                const float cost2 = d2 >= minD ? vol0[i2 * Lp + (d2 - minD)] : -1.f;
                if (cost1 != -1.f && cost1 < cost) { dsel = d1; cost = cost1; }
                if (cost2 != -1.f && cost2 < cost) { dsel = d2; }
            }
            res = dsel;
        }
    }
    return res;
}

// subpixelEnhancement (:1344-1374) of pixel i at disparity d
__device__ __forceinline__ float subpix_px(const float* __restrict__ vol0, size_t i, int d, const DevParams& P) {
    float inter = (float)d;
    if (d > P.minD && d < P.maxD) {
        const float* c = vol0 + i * P.Lp;
        const int minD = P.minD;
        const float c0 = c[d - minD], cp = c[d + 1 - minD], cm = c[d - 1 - minD];
        const float diff = (cp - cm) / (2 * (cp + cm - 2 * c0));
        if (diff > -1 && diff < 1) inter -= diff;
    }
    return inter;
}

__device__ __forceinline__ void sort2(float& a, float& b) {
    const float lo = fminf(a, b), hi = fmaxf(a, b);
    a = lo;
    b = hi;
}

// The refinement's last steps on a TX x TY tile: the edge map (hysteresis: a non-suppressed
// pixel whose component holds a strong one) on the tile + 2, the discontinuity adjustment and
// the subpixel step on the tile + 1, then medianBlur 3x3 CV_32F (BORDER_REPLICATE) + the ROI /
// mask post-processing (:388-403) and the store.  Also writes the edge map, the adjusted map
// (dtmp) and the subpixel map (debug dumps).
constexpr int RT_TX = 32, RT_TY = 8;
__global__ __launch_bounds__(256) void k_refine_tail(const uint8_t* __restrict__ map, const int32_t* __restrict__ label,
                                                     const uint8_t* __restrict__ strong, uint8_t* __restrict__ edges,
                                                     const int32_t* __restrict__ disp, int32_t* __restrict__ adj,
                                                     const float* __restrict__ vol0, float* __restrict__ sub,
                                                     PairOut outs, size_t out_step, const uint32_t* __restrict__ orig_left,
                                                     int roi_or_mask, int offset, DevParams Pk) {
    const DevParams P = Pk;
    float* out = outs.out[blockIdx.z];
    pair_shift(blockIdx.z, P.pstride, map, label, strong, edges, disp, adj, vol0, sub, orig_left);
    constexpr int EW = RT_TX + 4, EH = RT_TY + 4;  // edges: halo 2
    constexpr int AW = RT_TX + 2, AH = RT_TY + 2;  // adjusted + subpixel: halo 1
    __shared__ uint8_t se[EH][EW];
    __shared__ float ss[AH][AW];
    const int H = P.H, W = P.W;
    const int x0 = blockIdx.x * RT_TX, y0 = blockIdx.y * RT_TY;
    const int t = threadIdx.x;
    for (int k = t; k < EH * EW; k += 256) {
        const int r = k / EW, c = k - r * EW;
        const int yy = y0 - 2 + r, xx = x0 - 2 + c;
        uint8_t e = 0;
        if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
            const size_t i = (size_t)yy * W + xx;
            e = (map[i] != 1 && strong[label[i]]) ? 255 : 0;
        }
        se[r][c] = e;
    }
    __syncthreads();
    auto E = [&](int yy, int xx) -> bool { return se[yy - (y0 - 2)][xx - (x0 - 2)] != 0; };
    for (int k = t; k < AH * AW; k += 256) {
        const int r = k / AW, c = k - r * AW;
        const int y = y0 - 1 + r, x = x0 - 1 + c;
        if (y < 0 || y >= H || x < 0 || x >= W) continue;
        const int a = adjust_px(disp, vol0, x, y, P, E);
        const size_t i = (size_t)y * W + x;
        const float s = subpix_px(vol0, i, a, P);
        ss[r][c] = s;
        if (r >= 1 && r <= RT_TY && c >= 1 && c <= RT_TX) {  // the tile's own pixels
            adj[i] = a;
            sub[i] = s;
            edges[i] = se[r + 1][c + 1];
        }
    }
    __syncthreads();
    const int x = x0 + (t % RT_TX), y = y0 + t / RT_TX;
    if (x >= W || y >= H) return;
    float v[9];
    int k = 0;
    for (int dy = -1; dy <= 1; ++dy) {
        const int yy = min(max(y + dy, 0), H - 1) - (y0 - 1);
        for (int dx = -1; dx <= 1; ++dx) v[k++] = ss[yy][min(max(x + dx, 0), W - 1) - (x0 - 1)];
    }
    // odd-even transposition network: exact selection of the median (no arithmetic)
#pragma unroll
    for (int r = 0; r < 9; ++r) {
#pragma unroll
        for (int i = (r & 1); i + 1 < 9; i += 2) sort2(v[i], v[i + 1]);
    }
    float d = v[4];
    if (roi_or_mask) {
        if (d > 0) d = d + offset;                              // disparityOffset :1415-1427
        if ((orig_left[(size_t)y * W + x] == 0 && d > 0) || d == 0) d = -1.f;
    }
    *reinterpret_cast<float*>(reinterpret_cast<char*>(out) + (size_t)y * out_step + (size_t)x * 4) = d;
}

// ---------------------------------------------------------------------------
// debug layout conversions
// ---------------------------------------------------------------------------
__global__ void k_vol_to_ref(const float* __restrict__ vol, float* __restrict__ ref, DevParams Pk) {
    const DevParams P = Pk;  // kernel args -> registers once (no per-use kernarg reloads)
    const size_t N = (size_t)P.H * P.W;
    const int v = blockIdx.z;
    const int d = blockIdx.y;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < N; i += (size_t)gridDim.x * blockDim.x)
        ref[((size_t)v * P.L + d) * N + i] = vol[((size_t)v * N + i) * P.Lp + d];
}

__global__ void k_arms_to_ref(const uint32_t* __restrict__ arms, int32_t* __restrict__ ref, DevParams Pk) {
    const DevParams P = Pk;  // kernel args -> registers once (no per-use kernarg reloads)
    const size_t N = (size_t)P.H * P.W;
    const int v = blockIdx.y;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < N; i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t a = arms[(size_t)v * N + i];
        for (int k = 0; k < 4; ++k) ref[((size_t)v * 4 + k) * N + i] = (a >> (8 * k)) & 0xff;
    }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
size_t refine_scan_blocks(int n) { return (size_t)(n + SC_BLOCK - 1) / SC_BLOCK; }


// every refinement launch covers the group's P.npairs pairs (blockIdx.z = pair)
static dim3 grid2d(int W, int H, int bx, const DevParams& P) { return dim3((W + bx - 1) / bx, H, P.npairs); }
static dim3 grid1d(size_t n, const DevParams& P) { return dim3((unsigned)n, 1, P.npairs); }

void launch_outlier(RefineBufs& B, const DevParams& P, hipStream_t st) {
    hipLaunchKernelGGL(k_outlier_row, grid1d(P.H, P), dim3(256), (size_t)P.W, st, B.disp0, B.disp1, B.dm, B.hist, P);
    trace_point("k_outlier", st);
}

// Each Jacobi stage reads B.dm, writes B.dtmp, then the two maps swap roles (no copies).
void launch_region_voting(RefineBufs& B, const uint32_t* arms0, int hf, const DevParams& P,
                          hipStream_t st) {
    const int n = P.H * P.W;
    const int nb = (int)refine_scan_blocks(n);
    const size_t ps = P.pstride;
    // one launch: the outlier ranking (nb blocks) and, for vertical inner segments, the column
    // prefix counts (rows use the raster ranks)
    const int ncol = hf ? 0 : ((P.W + SC_THREADS - 1) / SC_THREADS) * (P.H / VP_CH + 1);
    const uint32_t ep = ++B.epoch;
    hipLaunchKernelGGL(k_vote_prep, grid1d(nb + ncol, P), dim3(SC_THREADS), 0, st, B.dm, n, nb, B.flags, B.out_list,
                       B.dtmp, B.counts, B.vpre, ep, P);
    trace_point("k_vote_prep", st);
    // grid-stride over the ranked outliers (their count stays on the device)
    // latency-bound walks: single pairs take enough waves to keep every SIMD several deep
    const int vc_blocks = std::max(64, 4096 / std::max(1, P.npairs));
    hipLaunchKernelGGL(k_vote_count_rank, grid1d(vc_blocks, P), dim3(256), 0, st, B.dm, arms0, B.out_list,
                       B.counts, B.cvote, B.csamp, B.vpre, hf, P);
    trace_point("k_vote_count_rank", st);
    hipLaunchKernelGGL(k_hv_list, grid1d(nb, P), dim3(SC_THREADS), 0, st, B.cvote, B.counts, B.flags, B.hv_list,
                       B.long_list, P.voting_thresh, ep, ps);
    trace_point("k_hv_list", st);
    // one wave per high-vote outlier, grid-stride; a histogram of L ints per wave; the first
    // VL_BLOCKS workgroups take the long carries (one histogram of L ints)
    const size_t lds = (size_t)VD_WAVES * P.L * sizeof(int);
    static_assert((size_t)VD_WAVES * 2048 * sizeof(int) <= 64 * 1024, "vote-decision LDS past the default limit");
    // a wave a high-vote rank where the list is long (real pairs: tens of thousands): 16384
    // blocks measured 110 against 121 us a launch on the 0600 pair (4096), config B unchanged
    const int vd_blocks = std::max(64, 16384 / std::max(1, P.npairs));
    hipLaunchKernelGGL(k_vote_decide, grid1d(VL_BLOCKS + vd_blocks, P), dim3(VD_WAVES * 64), lds, st, B.dm, B.dtmp,
                       arms0, B.out_list, B.cvote, B.csamp, B.counts, B.hv_list, B.long_list, hf, P);
    trace_point("k_vote_decide", st);
    std::swap(B.dm, B.dtmp);
}

void launch_interpolation(RefineBufs& B, const uint32_t* img0, const DevParams& P,
                          hipStream_t st) {
    // the ranked outliers of the last voting pass (out_list, counts[0]): dtmp equals dm elsewhere
    const int ib = std::max(64, 2048 / std::max(1, P.npairs));
    hipLaunchKernelGGL(k_interp_rays, grid1d(ib, P), dim3(256), 0, st, B.dm, B.dtmp, img0, B.out_list, B.counts, P);
    trace_point("k_interp", st);
    std::swap(B.dm, B.dtmp);
}

void launch_discontinuity(RefineBufs& B, const float* vol0, const DevParams& P,
                          hipStream_t st) {
    (void)vol0;
    const int n = P.H * P.W;
    const size_t ps = P.pstride;
    // the histogram was zeroed by k_outlier_row
    hipLaunchKernelGGL(k_gray_hist, grid1d((n + 256 * SC_ITEMS - 1) / (256 * SC_ITEMS), P), dim3(256), 0, st, B.dm,
                       B.gray, B.hist, n, ps); trace_point("k_gray_hist", st);
    hipLaunchKernelGGL(k_canny_front, dim3((P.W + CF_TX - 1) / CF_TX, (P.H + CF_TY - 1) / CF_TY, P.npairs), dim3(256), 0,
                       st, B.gray, B.hist, B.gray_eq, B.map, B.strong, P.H, P.W, P.canny_low, P.canny_high, ps);
    trace_point("k_canny_front", st);
    hipLaunchKernelGGL(k_uf_tile, dim3((P.W + UT - 1) / UT, (P.H + UT - 1) / UT, P.npairs), dim3(256), 0, st, B.map,
                       B.label, P.H, P.W, ps); trace_point("k_uf_tile", st);
    hipLaunchKernelGGL(k_uf_edges, grid2d(P.W, P.H, 256, P), dim3(256), 0, st, B.map, B.label, P.H, P.W, ps); trace_point("k_uf_edges", st);
    hipLaunchKernelGGL(k_uf_flatten_mark, grid1d((n + 255) / 256, P), dim3(256), 0, st, B.map, B.label, B.strong, n, ps); trace_point("k_uf_flatten_mark", st);
}

void launch_refine_tail(RefineBufs& B, const float* vol0, const uint32_t* orig_left, const PairOut& outs,
                        size_t out_step, int roi_or_mask, int offset, const DevParams& P, hipStream_t st) {
    hipLaunchKernelGGL(k_refine_tail, dim3((P.W + RT_TX - 1) / RT_TX, (P.H + RT_TY - 1) / RT_TY, P.npairs), dim3(256), 0,
                       st, B.map, B.label, B.strong, B.edges, B.dm, B.dtmp, vol0, B.subpix, outs, out_step, orig_left,
                       roi_or_mask, offset, P);
    trace_point("k_refine_tail", st);
    std::swap(B.dm, B.dtmp);  // dm = the adjusted map
}

void launch_vol_to_ref(const float* vol, float* ref, int views, const DevParams& P, hipStream_t st) {
    hipLaunchKernelGGL(k_vol_to_ref, dim3(256, P.L, views), dim3(256), 0, st, vol, ref, P); trace_point("k_vol_to_ref", st);
}

void launch_arms_to_ref(const uint32_t* arms, int32_t* ref, const DevParams& P, hipStream_t st) {
    hipLaunchKernelGGL(k_arms_to_ref, dim3(256, 2), dim3(256), 0, st, arms, ref, P); trace_point("k_arms_to_ref", st);
}

}  // namespace tsm
