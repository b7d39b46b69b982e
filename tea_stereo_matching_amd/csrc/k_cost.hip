// k_cost.hip -- step 1 of AD-Census on gfx950: image packing, ternary census
// descriptors and the cost-volume build (costInitialize, ADCensus.cpp:522-581).
//
// Census (ADCensus.cpp:454-498) is a ternary sign-disagreement count, not a Hamming
// distance of bit strings: a neighbour counts when (nL-cL)*(nR-cR) < 0, ties never
// count (:469).  Each pixel therefore carries two bit planes per channel, gt and lt
// (62 neighbours of the 9x7 window, centre excluded since it never counts), and
//     census = sum_w popc((gtL[w] & ltR[w]) | (ltL[w] & gtR[w]))
// over 6 words -- bit-exact with the reference's 186 sign products.
// HSI hue uses a NAND of "positive class" bits instead (:489-492).
//
// The AD-Census cost 2 - exp(-ad/lambdaAD) - exp(-census/lambdaCensus) (:518) is
// evaluated through two host-built tables (glibc expf on the exact arguments the
// reference feeds to std::exp), so the device result is bit-identical.
#include <utility>
#include <algorithm>
#include <stdlib.h>

#include "tsm_device.h"
#include "tsm_launch.h"

namespace tsm {

// ---------------------------------------------------------------------------
// image packing: BGR u8 (cv::Mat CV_8UC3, row step) -> u32 B | G<<8 | R<<16
// ---------------------------------------------------------------------------
__global__ void k_pack_bgr(PairIn in, size_t step, int H, int W, uint32_t* __restrict__ img, size_t ps) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int v = blockIdx.z & 1, pair = blockIdx.z >> 1;
    if (x >= W) return;
    pair_shift(pair, ps, img);
    const uint8_t* s = (v == 0 ? in.left[pair] : in.right[pair]) + (size_t)y * step + (size_t)x * 3;
    img[((size_t)v * H + y) * W + x] = (uint32_t)s[0] | ((uint32_t)s[1] << 8) | ((uint32_t)s[2] << 16);
}

// bgr2hsi, ADCensus.cpp:1429-1473 (filter: :1463-1470).  Float math as the reference;
// acosf comes from the device math library, so hue bytes are not guaranteed bit-equal
// to a given host libm (see DESIGN.md "HSI").
__global__ void k_bgr2hsi(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, int n,
                          int filter, size_t ps) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    pair_shift(blockIdx.z, ps, src, dst);
    const uint32_t p = src[i];
    const float b = ch(p, 0) / 255.f, g = ch(p, 1) / 255.f, r = ch(p, 2) / 255.f;
    const float sum = b + g + r;
    const float iv = sum / 3.0f;
    const uint32_t I = (uint32_t)(uint8_t)(iv * 255);
    float sv;
    if (sum == 0) sv = 0;
    else {
        float mn = fminf(fminf(b, g), r);
        sv = 1 - 3 * mn / sum;
    }
    const uint32_t S = (uint32_t)(uint8_t)(sv * 255);
    const float den = sqrtf((r - g) * (r - g) + (r - b) * (g - b));
    const float num = (2 * r - g - b) / 2.f;
    float hv;
    if (den == 0.f || den <= num || sv < 0.05f) hv = 0;
    else {
        const float theta = acosf(num / den);
        const double tp = 2 * 3.1415926535897932384626433832795;
        hv = b <= g ? (float)(theta / tp) : (float)(1 - theta / tp);
    }
    uint32_t Hh = (uint32_t)(uint8_t)(hv * 255);
    uint32_t out = Hh | (S << 8) | (I << 16);
    if (filter && (Hh >= 60 || Hh <= 10)) out = 0;
    dst[i] = out;
}

// computeGaussMedian, ADCensus.cpp:1475-1499: filter2D with the 3x3 Gaussian
// {1,2,1}x{1,2,1}/16 (exact in fp32), BORDER_CONSTANT, saturate_cast (half-to-even).
__global__ void k_gauss_median(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                               int H, int W, size_t ps) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int v = blockIdx.z & 1;
    if (x >= W) return;
    pair_shift(blockIdx.z >> 1, ps, src, dst);
    const uint32_t* s = src + (size_t)v * H * W;
    int acc[3] = {0, 0, 0};
    for (int dy = -1; dy <= 1; ++dy) {
        const int yy = y + dy;
        if (yy < 0 || yy >= H) continue;
        for (int dx = -1; dx <= 1; ++dx) {
            const int xx = x + dx;
            if (xx < 0 || xx >= W) continue;
            const int k = (dy == 0 ? 2 : 1) * (dx == 0 ? 2 : 1);
            const uint32_t q = s[(size_t)yy * W + xx];
            for (int c = 0; c < 3; ++c) acc[c] += k * ch(q, c);
        }
    }
    const uint32_t p = s[(size_t)y * W + x];
    uint32_t m[3];
    for (int c = 0; c < 3; ++c) {
        int q = acc[c] >> 4, r = acc[c] & 15;
        if (r > 8 || (r == 8 && (q & 1))) q++;
        m[c] = (uint32_t)min(q, 255);
    }
    uint32_t o[3] = {(uint32_t)ch(p, 0), (uint32_t)ch(p, 1), (uint32_t)ch(p, 2)};
    int hd = iabs_((int)o[0] - (int)m[0]);
    hd = min(hd, 255 - hd);
    if (hd >= 2) o[0] = m[0];
    for (int c = 1; c < 3; ++c)
        if (!(iabs_((int)o[c] - (int)m[c]) < 3)) o[c] = m[c];
    dst[((size_t)v * H + y) * W + x] = o[0] | (o[1] << 8) | (o[2] << 16);
}

// ---------------------------------------------------------------------------
// census descriptors: desc[v][y][x][16]
//   RGB: words 0..5 = gt planes (ch0 lo,hi, ch1 lo,hi, ch2 lo,hi), 6..11 = lt planes
//   HSI: words 0..1 = hue "positive" plane, 2..5 = sat/int gt, 6..9 = sat/int lt
//   word 12 = the pixel's packed colour (AD term, mask tests), words 13..15 = 0.
// One 64-B record per pixel, so the cost walk fetches a whole record with one scalar
// load.  Border pixels (window leaving the image) never reach the cost (:562-566):
// their planes are zero.
// ---------------------------------------------------------------------------
template <int CW, int CHh, bool HSI>
__global__ void k_census_desc(const uint32_t* __restrict__ img, uint32_t* __restrict__ desc,
                              DevParams Pk) {
    const DevParams P = Pk;  // kernel args -> registers once (no per-use kernarg reloads)
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int v = blockIdx.z & 1;
    const int H = P.H, W = P.W;
    if (x >= W) return;
    pair_shift(blockIdx.z >> 1, P.pstride, img, desc);
    constexpr int hw = CW / 2, hh = CHh / 2;
    uint32_t w[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) w[k] = 0;
    const uint32_t* im = img + (size_t)v * H * W;
    const uint32_t c = im[(size_t)y * W + x];
    if (x - hw >= 0 && x + hw < W && y - hh >= 0 && y + hh < H) {
        const int c0 = ch(c, 0), c1 = ch(c, 1), c2 = ch(c, 2);
        // fully unrolled: bit position and word index are compile-time constants
#pragma unroll
        for (int i = -hh; i <= hh; ++i) {
            const uint32_t* row = im + (size_t)(y + i) * W + x;
#pragma unroll
            for (int j = -hw; j <= hw; ++j) {
                if (i == 0 && j == 0) continue;
                const int bit = (i + hh) * CW + (j + hw) - (((i + hh) * CW + (j + hw)) > (hh * CW + hw) ? 1 : 0);
                const int wi = bit >> 5;
                const uint32_t m = 1u << (bit & 31);
                const uint32_t n = row[j];
                if (!HSI) {
                    const int d0 = ch(n, 0) - c0, d1 = ch(n, 1) - c1, d2 = ch(n, 2) - c2;
                    w[0 + wi] |= d0 > 0 ? m : 0u;
                    w[2 + wi] |= d1 > 0 ? m : 0u;
                    w[4 + wi] |= d2 > 0 ? m : 0u;
                    w[6 + wi] |= d0 < 0 ? m : 0u;
                    w[8 + wi] |= d1 < 0 ? m : 0u;
                    w[10 + wi] |= d2 < 0 ? m : 0u;
                } else {
                    const int dh = ch(n, 0) - c0, d1 = ch(n, 1) - c1, d2 = ch(n, 2) - c2;
                    w[0 + wi] |= ((dh <= -127) || (dh >= 0 && dh <= 127)) ? m : 0u;
                    w[2 + wi] |= d1 > 0 ? m : 0u;
                    w[4 + wi] |= d2 > 0 ? m : 0u;
                    w[6 + wi] |= d1 < 0 ? m : 0u;
                    w[8 + wi] |= d2 < 0 ? m : 0u;
                }
            }
        }
    }
    u32x4* o = reinterpret_cast<u32x4*>(desc + (((size_t)v * H + y) * W + x) * 16);
    o[0] = u32x4{w[0], w[1], w[2], w[3]};
    o[1] = u32x4{w[4], w[5], w[6], w[7]};
    o[2] = u32x4{w[8], w[9], w[10], w[11]};
    o[3] = u32x4{c, 0u, 0u, 0u};
}

// ---------------------------------------------------------------------------
// cost-volume build: one wave walks a row segment, the matched-against records held
// in a lane-shift register
// ---------------------------------------------------------------------------
// Lanes own E consecutive labels k = E*lane + e (E = 4 up to 256 labels, 8 up to 512), so
// a pixel's L-vector leaves as E/4 16-B stores per lane (784 contiguous bytes at L = 193).  View 0 pairs the fixed pixel
// left(j - minD) with right(j - k) at label k; view 1 pairs right(j + minD) with
// left(j + k) (costInitialize :542-579).  View 0 walks j upward and view 1 walks it
// downward, so in BOTH views the next pixel needs at label k the record that label k-1
// holds now: the label axis moves up one slot per step.  Inside a lane that is a
// rotation of the E slot registers (compile-time renaming, no data movement); one DPP
// wave_shr:1 per word carries the top slot into the next lane, and the one record that enters
// (label 0: varying column j) arrives by a wave-uniform scalar load and is written into
// lane 0.  The fixed pixel's record is wave-uniform as well (SGPR operands).  A cost
// cell is 6 x (and, and_or, bcnt) + one v_sad_u8 + two LDS table reads; no descriptor
// ever goes through LDS.  Census and AD are symmetric in (left, right), so both views
// run the same arithmetic.
struct F3 {  // 12-B store (global_store_dwordx3; an ext_vector of 3 would claim 16-B alignment)
    float a, b, c;
};
struct F5 {  // 20-B store of E = 5 lanes
    float a, b, c, d, e;
};
constexpr int CW_THREADS = 256;   // 4 independent waves per workgroup (tables shared)
constexpr int CW_LUTB = 192;      // lutB slot (188 used); padding entries follow it
constexpr int CW_CHUNK = 16;      // staging granule: 16 records x 64 B = one LDS-DMA per wave
constexpr int CW_SEG = 48;        // pixels per walk unit

template <int N>
struct IC { static constexpr int value = N; };

// staged records per stream: steps run in whole groups of E and read one record ahead
__host__ __device__ inline int cost_stage_slots(int seg_len, int E) {
    return (seg_len + E + 1 + CW_CHUNK - 1) / CW_CHUNK * CW_CHUNK;
}

// popcount accumulated in one instruction; opaque to the optimiser, which otherwise
// re-associates the census sum into add3 trees and distributes the table-address
// scaling over every term
__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc) {
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}

#ifdef TSM_EXP_STAMPS
// experiment build only: per-wave phase timestamps (s_memtime) for timeline analysis
__device__ unsigned long long g_stamps[65536 * 8];
#define CW_STAMP(i)                                                                   \
    do {                                                                              \
        if (lane == 0 && gw < 65536) g_stamps[(size_t)gw * 8 + (i)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define CW_STAMP(i) do { } while (0)
#endif

// MODE: CW_BOTH walks both views (unit -> view from the row index), CW_VIEW0 / CW_VIEW1
// one view per launch (one walk direction per kernel: fewer VGPRs, more waves per SIMD),
// CW_SHEAR the view-0 walk that also emits view 1.
enum { CW_BOTH = 0, CW_VIEW0 = 1, CW_VIEW1 = 2, CW_SHEAR = 3 };

template <int E, bool HSI, bool MASK, int MODE>
#ifndef TSM_CW_WPE3
#define TSM_CW_WPE3 4  // waves per SIMD asked of the E = 3 walk (measured: 3 -> 209 us, 4 -> 205, 5 / 6 spill: 341 / 384)
#endif
__global__ __launch_bounds__(CW_THREADS) __attribute__((amdgpu_waves_per_eu(E == 3 ? TSM_CW_WPE3 : (E == 4 ? 3 : 1)))) void k_cost_walk(
    const uint32_t* __restrict__ desc, const float* __restrict__ lutA, int lutA_n,
    const float* __restrict__ lutB, float* __restrict__ vol, DevParams Pk, int seg_len, int nseg,
    uint32_t* __restrict__ ctr, uint32_t ctr_base) {
    const DevParams P = Pk;  // kernel args -> registers once (no per-use kernarg reloads)
    // tables at fixed LDS addresses (table reads take the base as an immediate offset):
    //   sB[0..187] census term, sB[192..383] = -inf: padding labels (k >= L) start their
    //   census sum at 192, so 2 - A - (-inf) = +inf with no per-label select
    __shared__ __attribute__((aligned(16))) float s_lut[2 * CW_LUTB + (HSI ? 2816 : 768)];
    extern __shared__ __attribute__((aligned(16))) u32x4 smem_stage[];
    float* sB = s_lut;
    float* sA = s_lut + 2 * CW_LUTB;
    const int H = P.H, W = P.W, L = P.L, Lp = P.Lp;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    (void)ctr;
    (void)ctr_base;
    pair_shift(blockIdx.z, P.pstride, desc, vol);
    // one walk unit (view, row, segment) per wave; the unit's loads (ring prologue and
    // warm-up gather) are issued before the table fill's barrier so their latencies overlap
    // XCD-aware unit order: workgroups are dealt round-robin to the 8 XCDs, so block b runs
    // on XCD b % 8; remapping b -> (b % 8) * per + b / 8 gives each XCD a contiguous run of
    // units (neighbouring segments of the same rows), whose warm-up gathers and tails then
    // re-read records its own L2 already holds.  TSM_EXP_NO_XCD keeps the linear order.
    const int nb = gridDim.x, per = nb >> 3;
#ifdef TSM_EXP_NO_XCD
    const int blk = blockIdx.x;
#else
    const int blk = (int)blockIdx.x < 8 * per ? ((int)blockIdx.x & 7) * per + ((int)blockIdx.x >> 3) : (int)blockIdx.x;
#endif
    const int gw0 = blk * (CW_THREADS / 64) + wave;
    constexpr bool SHEAR = MODE == CW_SHEAR;
    const bool active = gw0 < (MODE == CW_BOTH ? 2 : 1) * H * nseg;
    const int gw = active ? gw0 : 0;
    CW_STAMP(0);
#ifdef TSM_EXP_STAMPS
    if (lane == 0 && gw < 65536) {
        unsigned hw_id, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_id));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        g_stamps[(size_t)gw * 8 + 5] = hw_id | ((unsigned long long)xcc << 32);
    }
#endif
    const int seg = gw % nseg;
    const int row = gw / nseg;
    // CW_BOTH interleaves the views row by row (unit row 2y + v): view 0 and view 1 of
    // image row y read the same two record rows (left y, right y), so both walks of a row
    // land on one XCD and its L2 fetches those records once
#ifdef TSM_EXP_VIEW_BLOCKS  // experiment build: view-major unit order (all of view 0 first)
    const int v = MODE == CW_BOTH ? row / H : (MODE == CW_VIEW1 ? 1 : 0);
    const int y = MODE == CW_BOTH ? row - v * H : row;
#else
    const int v = MODE == CW_BOTH ? (row & 1) : (MODE == CW_VIEW1 ? 1 : 0);
    const int y = MODE == CW_BOTH ? (row >> 1) : row;
#endif
    const int foff = v == 0 ? -P.minD : P.minD;
    const int x_lo = seg * seg_len;
    const int count0 = min(seg_len, W - x_lo);
    // SHEAR (minD = 0): view 1 is an exact shear of view 0, C1(x1, k) = C0(x1 + k, k), so
    // the view-0 walk also emits view 1.  Lane l completes the float4 of view-1 pixel
    // x1 = j - 4l - 3 (labels 4l..4l+3 come from steps j-3..j); a unit therefore starts
    // one group early (pre: those steps only fill the delay line) and the row's last unit
    // runs one group past the image (post: border cells, 2 / +inf, finish the float4s
    // that straddle the right edge).
    const int pre = (SHEAR && seg > 0) ? E : 0;
    const int post = (SHEAR && seg == nseg - 1) ? E : 0;
    const int count = pre + count0 + post;  // steps walked
    const int j0 = x_lo - pre;  // both views walk j upward: stores stream forward through HBM
    const int vtop = E * 64 - 1;  // view 1 feeds its shift register at the top label
    const int hw = P.censusW >> 1, hh = P.censusH >> 1;
    const bool rowOut = y - hh < 0 || y + hh >= H;
    constexpr int NW = HSI ? 11 : 13;  // shifted words: descriptor planes + colour
    constexpr int CWORD = 12;          // colour word of a record
    const uint32_t vmask_hi = (P.censusW * P.censusH - 1) >= 64
                                  ? 0xffffffffu
                                  : ((1u << ((P.censusW * P.censusH - 1) - 32)) - 1u);
    const uint32_t* dF = desc + ((size_t)v * H + y) * W * 16;        // fixed image
    const uint32_t* dV = desc + ((size_t)(1 - v) * H + y) * W * 16;  // varying image
    float* orow = vol + ((size_t)v * H + y) * W * Lp + E * lane;
    auto clampx = [&](int x) { return x < 0 ? 0 : (x >= W ? W - 1 : x); };

    // The unit's two wave-uniform record streams (fixed records x = j + foff, entering
    // records x = j (view 0) or j + vtop (view 1)) are staged in LDS up front by LDS-DMA
    // (global_load_lds_dwordx4: lane i's 16 bytes land at chunk base + 16 i, i.e. record
    // i/4, quarter i%4; no staging registers): per step they are broadcast LDS reads,
    // never an L2/HBM round trip.
    // steps run in groups of G (F/Fn double-buffering needs an even group)
    constexpr int G = (E & 1) ? 2 * E : E;
    const int slots = cost_stage_slots(seg_len + (SHEAR ? 2 * E : 0), G);
    u32x4* stF = smem_stage + (size_t)wave * 2 * slots * 4;
    u32x4* stE = stF + (size_t)slots * 4;
    const int rq = lane & 3, rr = lane >> 2;  // this lane's quarter / record of a chunk
    auto dma_chunk = [&](int t0) {  // records t0 .. t0+CW_CHUNK-1 (t0 a multiple of CW_CHUNK)
        const int t = t0 + rr;
        const int base = t0 * 4;
        __builtin_amdgcn_global_load_lds(
            reinterpret_cast<const u32x4*>(dF + (size_t)clampx(j0 + t + foff) * 16) + rq, stF + base, 16, 0, 0);
        __builtin_amdgcn_global_load_lds(
            reinterpret_cast<const u32x4*>(dV + (size_t)clampx(j0 + t + (v == 0 ? 0 : vtop)) * 16) + rq,
            stE + base, 16, 0, 0);
    };
    for (int c = 0; c < slots; c += CW_CHUNK) dma_chunk(c);

    // sA holds 2 - A[ad]: the reference's (2 - A) - B with its first subtraction done once
    for (int i = threadIdx.x; i < lutA_n; i += CW_THREADS) sA[i] = 2.f - lutA[i];
    for (int i = threadIdx.x; i < 2 * CW_LUTB; i += CW_THREADS)
        sB[i] = i < 188 ? lutB[i] : (i >= CW_LUTB ? -__int_as_float(0x7f800000) : 0.f);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // ring prologue landed (LDS-DMA)
    __syncthreads();  // tables ready: the kernel's only barrier
    if (!active) return;
    CW_STAMP(1);

    // warm-up: label k = E*lane + e holds the varying record at x = j0 - k (view 0) or
    // j0 + k (view 1), clamped: labels whose column leaves the image are border cells,
    // fixed up per step.  (Rotation 0: label offset e sits in slot e in both views.)
    uint32_t V[NW][E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        int x = v == 0 ? j0 - (E * lane + e) : j0 + (E * lane + e);
        x = x < 0 ? 0 : (x >= W ? W - 1 : x);
        const u32x4* r = reinterpret_cast<const u32x4*>(dV + (size_t)x * 16);
        const u32x4 a = r[0], b = r[1], c = r[2], d = r[3];
        const uint32_t rec[13] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w, d.x};
#pragma unroll
        for (int w = 0; w < NW; ++w) V[w][e] = rec[w < NW - 1 ? w : CWORD];
    }


    // record -> NW shifted words (descriptor planes, then the colour)
    auto pick = [&](const u32x4& a, const u32x4& b, const u32x4& c, const u32x4& d, uint32_t (&o)[NW]) {
        const uint32_t rec[13] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w, d.x};
#pragma unroll
        for (int w = 0; w < NW; ++w) o[w] = rec[w < NW - 1 ? w : CWORD];
    };
    auto load_staged = [&](const u32x4* st, int t, uint32_t (&o)[NW]) {
        const int i = t * 4;
        const uint32_t* r1 = reinterpret_cast<const uint32_t*>(st + i);
        pick(st[i + 0], st[i + 1], st[i + 2], u32x4{r1[CWORD], 0u, 0u, 0u}, o);
    };

    // View 0 pairs label k with right(j - k): the next pixel's label k is this pixel's
    // label k-1, so the label axis moves UP one slot per step (slot of offset e at
    // rotation R: (e - R) mod E; DPP wave_shr carries lanes up, lane 0 takes the entering
    // record x = j).  View 1 pairs label k with left(j + k): the label axis moves DOWN
    // (slot (e + R) mod E; wave_shl, lane 63 takes x = j + vtop).
    auto walk = [&](auto UPc) {
    constexpr bool UP = decltype(UPc)::value == 0;
    const float kInf = __int_as_float(0x7f800000);
    uint32_t padoff[E];  // census start: 0, or CW_LUTB for padding labels (+inf cost)
#pragma unroll
    for (int e = 0; e < E; ++e) padoff[e] = (!MASK && E * lane + e >= L) ? CW_LUTB : 0u;
    // fixed records double-buffered by step parity (compile-time), no register copies
    uint32_t FA[NW], FB[NW], En[NW];
    float dl0[4], dl1[4], dl2[4];  // SHEAR delay line (slots by step rotation)
#pragma unroll
    for (int i = 0; i < 4; ++i) dl0[i] = dl1[i] = dl2[i] = 0.f;
    float* o1row = vol + ((size_t)H + y) * W * Lp;  // view-1 row (SHEAR)
    load_staged(stF, 0, FA);

    // step S of a group: rotation R = S mod E, fixed-record buffer by the parity of S
    auto step = [&](auto Sc, bool fast, int t) {  // fast: interior group, no border tests
        constexpr int S = decltype(Sc)::value;
        constexpr int R = S % E;
        uint32_t(&F)[NW] = (S & 1) ? FB : FA;
        uint32_t(&Fn)[NW] = (S & 1) ? FA : FB;
        const int j = j0 + t;
        // the next step's records (steps past the segment end run on clamped records
        // and store nothing: no branches)
        load_staged(stF, t + 1, Fn);
        load_staged(stE, t + 1, En);
        // census of the E cells, interleaved word by word (E independent bcnt chains)
        uint32_t cen[E];
#pragma unroll
        for (int e = 0; e < E; ++e) cen[e] = padoff[e];
        if (!HSI) {
#pragma unroll
            for (int k = 0; k < 6; ++k)
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const int s = UP ? (e - R + E) % E : (e + R) % E;
                    cen[e] = bcnt_acc((F[k] & V[6 + k][s]) | (F[6 + k] & V[k][s]), cen[e]);
                }
        } else {
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const int s = UP ? (e - R + E) % E : (e + R) % E;
                cen[e] = padoff[e] + __builtin_popcount(~(F[0] & V[0][s])) +
                         __builtin_popcount(~(F[1] & V[1][s]) & vmask_hi);
#pragma unroll
                for (int k = 2; k < 6; ++k)
                    cen[e] += __builtin_popcount((F[k] & V[4 + k][s]) | (F[4 + k] & V[k][s]));
            }
        }
        float c[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int s = UP ? (e - R + E) % E : (e + R) % E;
            const uint32_t vc = V[NW - 1][s], fc = F[NW - 1];
            int ai;
            if (!HSI) {
                ai = (int)__builtin_amdgcn_sad_u8(fc, vc, 0u);
            } else {
                const int hd = (int)__builtin_amdgcn_sad_u8(fc & 0xffu, vc & 0xffu, 0u);
                ai = 2 * min(hd, 255 - hd) +
                     5 * (int)__builtin_amdgcn_sad_u8(fc & 0xffff00u, vc & 0xffff00u, 0u);
            }
            // mask mode: black centre on either side -> census = +inf (:459-460)
            if (MASK && (fc == 0 || vc == 0)) cen[e] = 187;
#ifdef TSM_EXP_NOLUT
            c[e] = (float)ai - (float)cen[e];
#else
            c[e] = sA[ai] - sB[cen[e]];
#endif
        }
        // border cells (either 9x7 window leaves the image, :562-566) and masked own
        // pixels (:551-555) cost 2; wave-uniform test first, per-label only near borders
        if (!fast) {
        const int xf = j + foff;
        bool fixed_ok = !rowOut && xf - hw >= 0 && xf + hw < W;
        if (MASK) fixed_ok = fixed_ok && dF[(size_t)__builtin_amdgcn_readfirstlane(j) * 16 + CWORD] != 0u;
        const int klo = v == 0 ? j - (W - 1 - hw) : hw - j;
        const int khi = v == 0 ? j - hw : W - 1 - hw - j;
        if (!(fixed_ok && klo <= 0 && khi >= L - 1)) {
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const int k = E * lane + e;
                c[e] = (fixed_ok && k >= klo && k <= khi) || k >= L ? c[e] : 2.f;
            }
        }
        }
        if (MASK) {  // mask mode overrides census indices: padding needs its own select
#pragma unroll
            for (int e = 1; e < E; ++e) c[e] = E * lane + e >= L ? kInf : c[e];
        }
        const bool own = SHEAR ? (t >= pre && t < pre + count0) : (fast || t < count);
#ifdef TSM_EXP_NOSTORE
        if (own && c[0] == -12345.f) {
#else
        if (own) {
#endif
            if constexpr (E == 3) {  // labels 3l .. 3l+2: one 12-B store per lane, 768 B a pixel
                F3 o3;
                o3.a = c[0];
                o3.b = c[1];
                o3.c = c[2];
                *reinterpret_cast<F3*>(orow + (size_t)j * Lp) = o3;  // (nt dwordx3: 206 -> 284 us)
            }
            if constexpr (E == 5) {  // labels 5l .. 5l+4: 20 B per lane, 1280 B a pixel
                F5 o5;
                o5.a = c[0];
                o5.b = c[1];
                o5.c = c[2];
                o5.d = c[3];
                o5.e = c[4];
                *reinterpret_cast<F5*>(orow + (size_t)j * Lp) = o5;
            }
#pragma unroll
            for (int q = 0; q < E / 4; ++q)
                if (E * lane + 4 * q < Lp)
                    st_stream(orow + (size_t)j * Lp + 4 * q, f32x4{c[4 * q], c[4 * q + 1], c[4 * q + 2], c[4 * q + 3]});
        }
        if constexpr (SHEAR) {
            // delay line by step rotation (compile-time slots): element e of the float4
            // completed now was computed 3 - e steps ago
            dl0[R & 3] = c[0];
            dl1[R & 3] = c[1];
            dl2[R & 3] = c[2];
            const int x1 = j - 4 * lane - 3;
#ifdef TSM_EXP_NOSTORE1
            if (t >= pre && x1 >= 0 && x1 < W && 4 * lane < Lp && c[3] == -12345.f)  // timing only
#else
            if (t >= pre && x1 >= 0 && x1 < W && 4 * lane < Lp)
#endif
                *reinterpret_cast<f32x4*>(o1row + (size_t)x1 * Lp + 4 * lane) =
                    f32x4{dl0[(R + 1) & 3], dl1[(R + 2) & 3], dl2[(R + 3) & 3], c[3]};
        }
        // advance: view 0: the slot of offset E-1 becomes offset 0 of the next rotation,
        // fed from lane-1 (lane 0 has no source and keeps `old`, the entering word);
        // view 1: the slot of offset 0 becomes offset E-1, fed from lane+1 (lane 63 keeps
        // the entering word)
        constexpr int s3 = UP ? (2 * E - 1 - R) % E : R % E;
#pragma unroll
        for (int w = 0; w < NW; ++w)
            V[w][s3] = (uint32_t)__builtin_amdgcn_update_dpp((int)En[w], (int)V[w][s3],
                                                             UP ? DPP_WAVE_SHR1 : DPP_WAVE_SHL1,
                                                             0xF, 0xF, false);
    };
    // interior steps (every label's windows inside the image) form one run of t: the
    // walk takes a branch-free body for whole groups of E steps inside it
    const int jlo = max(v == 0 ? hw + L - 1 : hw, hw - foff);
    const int jhi = min(v == 0 ? W - 1 - hw : W - hw - L, W - 1 - hw - foff);
    const int tf_lo = jlo - j0;
    const int tf_hi = min(jhi - j0, count - 1);
    const bool rows_ok = !MASK && !rowOut;
    CW_STAMP(2);
    for (int t = 0; t < count; t += G) {
        const bool fast = rows_ok && t >= tf_lo && t + G - 1 <= tf_hi;
        [&]<int... Ss>(std::integer_sequence<int, Ss...>) {
            (step(IC<Ss>{}, fast, t + Ss), ...);
        }(std::make_integer_sequence<int, G>{});
    }
    };
    if constexpr (MODE == CW_VIEW0 || MODE == CW_SHEAR) {
        walk(IC<0>{});
    } else if constexpr (MODE == CW_VIEW1) {
        walk(IC<1>{});
    } else {
        if (v == 0) walk(IC<0>{});
        else walk(IC<1>{});
    }
    // Lp = 64 E + 4 (E = 3: 193..196 labels, 4: 257..260, 5: 321..324): the lanes cover
    // labels 0 .. 64E-1, the pixel vector's last float4 (labels 64E .. Lp-1, the real ones
    // < L, the rest +inf padding) is the tail: lane l computes pixel x_lo + l of the unit
    // from global records (one gather per label, L2-resident)
    if constexpr (E == 3 || E == 4 || E == 5) {
        if (Lp > 64 * E && lane < count0) {
            const int j = x_lo + lane;
            const float inf = __int_as_float(0x7f800000);
            uint32_t Fr[NW];
            const u32x4* rf = reinterpret_cast<const u32x4*>(dF + (size_t)clampx(j + foff) * 16);
            pick(rf[0], rf[1], rf[2], rf[3], Fr);
            const int xf = j + foff;
            const bool fixed_ok = !rowOut && xf - hw >= 0 && xf + hw < W;
            const int klo = v == 0 ? j - (W - 1 - hw) : hw - j;
            const int khi = v == 0 ? j - hw : W - 1 - hw - j;
            float c4[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int k = 64 * E + t;
                c4[t] = inf;
                if (k < L) {
                    uint32_t Vr[NW];
                    const u32x4* rv = reinterpret_cast<const u32x4*>(dV + (size_t)clampx(v == 0 ? j - k : j + k) * 16);
                    pick(rv[0], rv[1], rv[2], rv[3], Vr);
                    uint32_t cen = 0;
                    if (!HSI) {
#pragma unroll
                        for (int w = 0; w < 6; ++w) cen = bcnt_acc((Fr[w] & Vr[6 + w]) | (Fr[6 + w] & Vr[w]), cen);
                    } else {
                        cen = __builtin_popcount(~(Fr[0] & Vr[0])) + __builtin_popcount(~(Fr[1] & Vr[1]) & vmask_hi);
#pragma unroll
                        for (int w = 2; w < 6; ++w) cen += __builtin_popcount((Fr[w] & Vr[4 + w]) | (Fr[4 + w] & Vr[w]));
                    }
                    const uint32_t vc = Vr[NW - 1], fc = Fr[NW - 1];
                    int ai;
                    if (!HSI) {
                        ai = (int)__builtin_amdgcn_sad_u8(fc, vc, 0u);
                    } else {
                        const int hd = (int)__builtin_amdgcn_sad_u8(fc & 0xffu, vc & 0xffu, 0u);
                        ai = 2 * min(hd, 255 - hd) + 5 * (int)__builtin_amdgcn_sad_u8(fc & 0xffff00u, vc & 0xffff00u, 0u);
                    }
                    const float c = sA[ai] - sB[cen];
                    c4[t] = (fixed_ok && k >= klo && k <= khi) ? c : 2.f;
                }
            }
            st_stream(vol + (((size_t)v * H + y) * W + j) * Lp + 64 * E, f32x4{c4[0], c4[1], c4[2], c4[3]});
        }
    }
    CW_STAMP(3);
}

// ---------------------------------------------------------------------------
// cost-volume build on the matrix cores (RGB, no mask): the census term as an fp4 MFMA
// ---------------------------------------------------------------------------
// The census count of a (fixed, varying) record pair is a dot product over the 384 bits
// of 12 words: census = sum_w popc(F[w] & V[(w + 6) % 12]) (gt planes against lt planes
// and back).  Expanding every bit to an fp4 (e2m1) element -- 2.0 where set, 0 where not --
// makes one 16x16x128 block-scaled MFMA (scales 1.0) sum 4 x the matches of 128 bits for a
// 16 x 16 tile of (fixed pixel j, varying pixel x) pairs, exactly (integers <= 1536 in
// f32), and three of them give 4 x census: the byte offset of the census table entry.
// Lane l of MFMA kk carries word 4 kk + (l >> 4) of row / column l & 15, expanded so that
// bit 4n + s of the word lands in nibble n of dword s: both operands place every bit at
// the same k, which is all a dot product needs (tools/micro/fp4_census_dot.hip checks it
// on the device).  The AD term and the two tables stay on the VALU / LDS: per cell one
// v_sad_u8, two table reads, one subtraction -- against 6 x (and, and_or, bcnt) + the
// shift-register DPP moves of the walk.
//
// A workgroup (8 waves) owns a unit (view, row, 128-pixel segment); wave w owns the 16
// pixels j0 = seg + 16 w.  Pixel j's labels k = 0..L-1 pair it with x = j - k (view 0)
// or j + k (view 1), so the wave's tiles are the x-blocks x0 = j0 -+ 16 m, m = 0..M with
// M = ceil((L - 1) / 16).  The unit's varying records (128 + 16 M pixels) are expanded
// once into LDS as B fragments, [word][pixel] 16 B each (a tile's 64 lanes read 16
// consecutive pixels per word: conflict-free ds_read_b128); the fixed records become
// the wave's A fragments in registers.  Output lane l of a tile holds x = x0 + (l & 15)
// and j = j0 + 4 (l >> 4) + r (C/D map col = lane & 15, row = 4 (lane >> 4) + reg), so one
// store per r writes 16 consecutive labels of 4 pixels (64-B runs, descending k).
// Cells: same formula and borders as k_cost_walk (costInitialize :542-579):
// c = (2 - A[ad]) - B[census] where the fixed pixel's and the varying pixel's windows
// are inside the image, 2 elsewhere, +inf on the padding labels L..Lp-1.
constexpr int CM_WAVES = 8;
constexpr int CM_THREADS = CM_WAVES * 64;
constexpr int CM_JB = 16;                   // pixels per wave (one tile row block)
constexpr int CM_SEG = CM_WAVES * CM_JB;    // pixels per unit
constexpr uint32_t CM_BIAS = 64;
#ifndef TSM_CM_STAUX
#define TSM_CM_STAUX 0  // cache-policy bits of the volume stores (experiments: 2 = nt)
#endif            // store buffer starts this many bytes before the row

typedef int v8i_ __attribute__((ext_vector_type(8)));
typedef float v4f_ __attribute__((ext_vector_type(4)));

// 32 census bits -> 32 fp4 elements (16 B): bit 4n + s -> nibble n of dword s, 0x4 = 2.0
__device__ __forceinline__ u32x4 fp4_expand(uint32_t w) {
    return u32x4{(w << 2) & 0x44444444u, (w << 1) & 0x44444444u, w & 0x44444444u, (w >> 1) & 0x44444444u};
}

__device__ __forceinline__ v4f_ mfma_fp4(u32x4 a, u32x4 b, v4f_ c) {
    const v8i_ av = {(int)a.x, (int)a.y, (int)a.z, (int)a.w, 0, 0, 0, 0};
    const v8i_ bv = {(int)b.x, (int)b.y, (int)b.z, (int)b.w, 0, 0, 0, 0};
    // cbsz = blgp = 4: both operands fp4 (e2m1); E8M0 scales 127 = 1.0
    return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, 4, 4, 0, 127, 0, 127);
}

__host__ __device__ inline int cost_mfma_tiles(int L) { return (L - 1 + CM_JB - 1) / CM_JB; }  // M
__host__ __device__ inline int cost_mfma_span(int L) { return CM_SEG + CM_JB * cost_mfma_tiles(L); }

// MT > 0: the tile count M at compile time (LDS offsets become immediates); 0: runtime
template <int MT>
__global__ __launch_bounds__(CM_THREADS) __attribute__((amdgpu_waves_per_eu(4))) void k_cost_mfma(const uint32_t* __restrict__ desc,
                                                          const float* __restrict__ lutA, int lutA_n,
                                                          const float* __restrict__ lutB,
                                                          float* __restrict__ vol, DevParams Pk, int nseg) {
    const DevParams P = Pk;
    __shared__ float sA2[768];  // 2 - A[ad]
    __shared__ float sB[192];   // B[census]
    extern __shared__ __attribute__((aligned(16))) u32x4 smem_frag[];
    const int H = P.H, W = P.W, L = P.L, Lp = P.Lp;
    const int M = MT > 0 ? MT : cost_mfma_tiles(L), XS = CM_SEG + CM_JB * M;
    u32x4* xfr = smem_frag;                                       // [12][XS]
    uint32_t* xcol = reinterpret_cast<uint32_t*>(smem_frag + 12 * XS);  // [XS]
    pair_shift(blockIdx.z, P.pstride, desc, vol);
    // XCD-aware unit order (as k_cost_walk): each XCD takes a contiguous run of units, so
    // the segments and both views of a row share one L2 for their records
    const int nb = gridDim.x, per = nb >> 3;
    const int blk = (int)blockIdx.x < 8 * per ? ((int)blockIdx.x & 7) * per + ((int)blockIdx.x >> 3) : (int)blockIdx.x;
    if (blk >= 2 * H * nseg) return;  // whole workgroup: no barrier is pending
    const int seg = blk % nseg, vy = blk / nseg;
    const int v = vy & 1, y = vy >> 1;
    const int seg_lo = seg * CM_SEG;
    const int xs0 = v == 0 ? seg_lo - CM_JB * M : seg_lo;  // first staged varying pixel
    const int hw = P.censusW >> 1, hh = P.censusH >> 1;
    const bool rowOut = y - hh < 0 || y + hh >= H;
    const int foff = v == 0 ? -P.minD : P.minD;
    const uint32_t* dF = desc + ((size_t)v * H + y) * W * 16;        // fixed image row
    const uint32_t* dV = desc + ((size_t)(1 - v) * H + y) * W * 16;  // varying image row

    for (int i = threadIdx.x; i < lutA_n && i < 768; i += CM_THREADS) sA2[i] = 2.f - lutA[i];
    for (int i = threadIdx.x; i < 192; i += CM_THREADS) sB[i] = i < 188 ? lutB[i] : 0.f;
    // stage the varying records as B fragments: word slot s holds V word (s + 6) % 12
    for (int p = threadIdx.x; p < XS; p += CM_THREADS) {
        const int x = xs0 + p;
        u32x4 r0 = {0u, 0u, 0u, 0u}, r1 = r0, r2 = r0, r3 = r0;
        if (x >= 0 && x < W) {
            const u32x4* r = reinterpret_cast<const u32x4*>(dV + (size_t)x * 16);
            r0 = r[0]; r1 = r[1]; r2 = r[2]; r3 = r[3];
        }
        const uint32_t w[12] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w, r2.x, r2.y, r2.z, r2.w};
#pragma unroll
        for (int s = 0; s < 12; ++s) xfr[s * XS + p] = fp4_expand(w[(s + 6) % 12]);
        xcol[p] = r3.x;
    }
    __syncthreads();
#ifdef TSM_EXP_CM_STAGEONLY  // timing only: the staging phase alone
    return;
#endif

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int j0 = seg_lo + CM_JB * wave;
    if (j0 >= W) return;
    const int col = lane & 15, grp = lane >> 4;
    auto clampx = [&](int x) { return x < 0 ? 0 : (x >= W ? W - 1 : x); };
    // A fragments: row j0 + col, words 4 kk + grp of its fixed record
    u32x4 af[3];
    {
        const uint32_t* rf = dF + (size_t)clampx(j0 + col + foff) * 16;
#pragma unroll
        for (int kk = 0; kk < 3; ++kk) af[kk] = fp4_expand(rf[4 * kk + grp]);
    }
    // this lane's four output rows j = j0 + 4 grp + r: fixed colour and window test
    uint32_t fc[4];
    bool fo[4];
    bool rows_in = j0 + CM_JB <= W;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int j = j0 + 4 * grp + r;
        const int xf = j + foff;
        fc[r] = dF[(size_t)clampx(xf) * 16 + 12];
        fo[r] = !rowOut && xf - hw >= 0 && xf + hw < W;
        rows_in = rows_in && fo[r];
    }
    rows_in = __all(rows_in);  // every row of the block inside the image with its window
    // cell (r, m): label k = kb + ks r + 16 m at byte ob[r] + 64 m of the row's volume
    const int kb = v == 0 ? 4 * grp - col : col - 4 * grp;
    const int ks = v == 0 ? 1 : -1;
    uint32_t ob[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) ob[r] = CM_BIAS + 4u * (uint32_t)((j0 + 4 * grp + r) * Lp + kb + ks * r);
    // fast tiles store quad-transposed float4s: pixel j0 + 4 grp + (col & 3), labels from
    // kq (m = 0) on, kq = 4 grp + i - 4 q - 3 (view 0) or 4 q - 4 grp - i (view 1)
    uint32_t oq;
    {
        const int i = col & 3, q4 = col & ~3;
        const int kq = v == 0 ? 4 * grp + i - q4 - 3 : q4 - 4 * grp - i;
        oq = CM_BIAS + 4u * (uint32_t)((j0 + 4 * grp + i) * Lp + kq);
    }
#ifdef TSM_EXP_CM_ALIGNED  // timing only: each tile's 16 labels as one 64-B aligned piece
#pragma unroll
    for (int r = 0; r < 4; ++r) ob[r] = CM_BIAS + (uint32_t)(j0 + 4 * grp + r) * 832u + 4u * (uint32_t)col;
    oq = CM_BIAS + (uint32_t)(j0 + 4 * grp + (col & 3)) * 832u + 4u * (uint32_t)(col & ~3);
#endif
    // the row's volume as a raw buffer: a store whose VGPR offset is past the buffer's
    // size is dropped, so cells outside the label band / image are masked without
    // branches.  The range check covers the VGPR offset only (the tile step 64 m rides in
    // soffset), so the buffer starts CM_BIAS bytes before the row: a valid cell's VGPR
    // part ob[r] >= 4 (k >= -15 at m = 0) stays non-negative.
    const uint32_t row_bytes = 4u * (uint32_t)(W * Lp);
    const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<char*>(vol + ((size_t)v * H + y) * W * Lp) - CM_BIAS, (short)0, (int)(row_bytes + CM_BIAS),
        0x00020000);
    // tile m's varying pixels start at staged pixel pb + ps m (uniform)
    const int pb = v == 0 ? CM_JB * (wave + M) : CM_JB * wave, ps = v == 0 ? -CM_JB : CM_JB;
    const u32x4* xl = xfr + grp * XS + col;
    const uint32_t* cl = xcol + col;
    // one tile: 3 MFMAs for the census, then per cell the AD term and the two tables.
    // FAST: every cell in the label band, both windows inside the image (no selects, no
    // masks); otherwise out-of-band / off-image cells get an offset past the buffer
    // (the store is dropped) and cells with a window off the image cost 2.
    auto mma = [&](int m) {
        const int p0 = pb + ps * m;
        v4f_ acc = {0.f, 0.f, 0.f, 0.f};
#ifdef TSM_EXP_CM_STOREONLY
        return acc;
#endif
#pragma unroll
        for (int kk = 0; kk < 3; ++kk) acc = mfma_fp4(af[kk], xl[4 * kk * XS + p0], acc);
        return acc;
    };
    // FASTc: 0 = general tile, 1 = fast tile of view 0, 2 = fast tile of view 1
    auto epilogue = [&](int m, v4f_ acc, auto FASTc) {
        constexpr bool FAST = decltype(FASTc)::value != 0;
        constexpr bool FV0 = decltype(FASTc)::value == 1;
        const int p0 = pb + ps * m;
        const uint32_t vc = cl[p0];
        const int mo = 64 * m;  // byte step of the tile's labels (soffset)
        bool xok = true;
        if (!FAST) {
            const int x = xs0 + p0 + col;
            xok = x - hw >= 0 && x + hw < W;
        }
        float c[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#ifdef TSM_EXP_CM_STOREONLY  // timing only: no MFMA results, no tables
            c[r] = (float)(m + r);
#else
            const uint32_t cen4 = (uint32_t)acc[r];  // 4 x census: byte offset into sB
            const uint32_t ad4 = __builtin_amdgcn_sad_u8(fc[r], vc, 0u) << 2;
            c[r] = *reinterpret_cast<const float*>(reinterpret_cast<const char*>(sA2) + ad4) -
                   *reinterpret_cast<const float*>(reinterpret_cast<const char*>(sB) + cen4);
#endif
        }
        if (FAST) {
            // 4x4 transpose inside each quad of lanes (two DPP butterflies): lane 4q + i
            // then holds pixel j0 + 4 grp + i at x = x0 + 4q + e in c[e], four consecutive
            // labels, and leaves them with one 16-B store instead of four 4-B ones
            const bool b1 = (col & 2) != 0, b0 = (col & 1) != 0;
            auto qp = [](float x, auto CTc) {  // quad_perm move (every lane has a source)
                return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), decltype(CTc)::value, 0xF, 0xF, true));
            };
            float r0 = qp(b1 ? c[0] : c[2], IC<DPP_QUAD_2301>{});
            float r1 = qp(b1 ? c[1] : c[3], IC<DPP_QUAD_2301>{});
            c[0] = b1 ? r0 : c[0]; c[1] = b1 ? r1 : c[1];
            c[2] = b1 ? c[2] : r0; c[3] = b1 ? c[3] : r1;
            r0 = qp(b0 ? c[0] : c[1], IC<DPP_QUAD_1032>{});
            r1 = qp(b0 ? c[2] : c[3], IC<DPP_QUAD_1032>{});
            c[0] = b0 ? r0 : c[0]; c[2] = b0 ? r1 : c[2];
            c[1] = b0 ? c[1] : r0; c[3] = b0 ? c[3] : r1;
            const u32x4 q = FV0 ? u32x4{__float_as_uint(c[3]), __float_as_uint(c[2]), __float_as_uint(c[1]), __float_as_uint(c[0])}
                                   : u32x4{__float_as_uint(c[0]), __float_as_uint(c[1]), __float_as_uint(c[2]), __float_as_uint(c[3])};
#ifdef TSM_EXP_CM_NOSTORE
            if (c[0] == -12345.f)
#endif
            __builtin_amdgcn_raw_buffer_store_b128(q, vrs, (int)oq, mo, 0);
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int k = kb + ks * r + CM_JB * m;
                const float cr = (fo[r] && xok) ? c[r] : 2.f;
                const int off = ((unsigned)k < (unsigned)L && j0 + 4 * grp + r < W) ? (int)ob[r] : -1;
#ifdef TSM_EXP_CM_NOSTORE
                if (cr == -12345.f)
#endif
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(cr), vrs, off, mo, TSM_CM_STAUX);
            }
        }
    };
    auto tile = [&](int m, auto FASTc) { epilogue(m, mma(m), FASTc); };
    // fast tiles: m in [1, (L - 16) / 16] (inside the label band) whose 16 varying pixels
    // and windows are inside the image, for a block whose rows all are
    int f_lo = 1, f_hi = (L - CM_JB) / CM_JB;
    {
        const int xb = xs0 + pb;  // x0(m) = xb + ps m
        const int lo_x = hw, hi_x = W - hw - CM_JB;  // x0 in [lo_x, hi_x]
        if (v == 0) {  // x0 = xb - 16 m
            f_lo = max(f_lo, (xb - hi_x + CM_JB - 1) >= 0 ? (xb - hi_x + CM_JB - 1) / CM_JB : 0);
            f_hi = min(f_hi, xb - lo_x >= 0 ? (xb - lo_x) / CM_JB : -1);
        } else {  // x0 = xb + 16 m
            f_lo = max(f_lo, lo_x - xb > 0 ? (lo_x - xb + CM_JB - 1) / CM_JB : 0);
            f_hi = min(f_hi, hi_x - xb >= 0 ? (hi_x - xb) / CM_JB : -1);
        }
        if (!rows_in || f_hi < f_lo) { f_lo = M + 1; f_hi = M; }
    }
#ifdef TSM_EXP_CM_BURST
    if constexpr (MT > 0) {
        // experiment: all tiles first, their cells held in registers, then the block's
        // stores in one burst (every pixel vector completed within a short window).
        // Measured slower than streaming the stores tile by tile: 208.8 vs 198.8 us.
        float cb[MT + 1][4];
#pragma unroll
        for (int m = 0; m <= MT; ++m) {
            const v4f_ acc = mma(m);
            const bool fast = m >= f_lo && m <= f_hi;
            const int p0 = pb + ps * m;
            const uint32_t vc = cl[p0];
            const int x = xs0 + p0 + col;
            const bool xok = fast || (x - hw >= 0 && x + hw < W);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t cen4 = (uint32_t)acc[r];
                const uint32_t ad4 = __builtin_amdgcn_sad_u8(fc[r], vc, 0u) << 2;
                const float c = *reinterpret_cast<const float*>(reinterpret_cast<const char*>(sA2) + ad4) -
                                *reinterpret_cast<const float*>(reinterpret_cast<const char*>(sB) + cen4);
                cb[m][r] = (fast || (fo[r] && xok)) ? c : 2.f;
            }
        }
#pragma unroll
        for (int m = 0; m <= MT; ++m) {
            const bool fast = m >= f_lo && m <= f_hi;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int k = kb + ks * r + CM_JB * m;
                const bool in = fast || ((unsigned)k < (unsigned)L && j0 + 4 * grp + r < W);
#ifdef TSM_EXP_CM_NOSTORE
                if (cb[m][r] == -12345.f)
#endif
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(cb[m][r]), vrs, in ? (int)ob[r] : -1, 64 * m, 0);
            }
        }
    } else
#endif
#ifdef TSM_EXP_CM_TILESTORE
    {  // experiment: every tile stores its own cells (4 x 64-B runs per store)
    for (int m = 0; m < min(f_lo, M + 1); ++m) tile(m, IC<0>{});
    auto fast_run = [&](auto Fc) {
        int m = f_lo;
        for (; m < f_hi; m += 2) {
            const v4f_ a0 = mma(m), a1 = mma(m + 1);
            epilogue(m, a0, Fc);
            epilogue(m + 1, a1, Fc);
        }
        if (m == f_hi) tile(m, Fc);
    };
    if (v == 0) fast_run(IC<1>{});
    else fast_run(IC<2>{});
    for (int m = max(f_hi + 1, min(f_lo, M + 1)); m <= M; ++m) tile(m, IC<0>{});
    }
#else
    {
    // Tiles 1.. in groups of four.  A tile's store would write 4 pixels x 64 B; instead the
    // group's four results per output row r are transposed between the lane rows and the
    // registers (v_permlane32_swap + v_permlane16_swap, 4 instructions per r), so lane row
    // t of register g holds tile m0 + t of pixel j0 + 4 g + r: one store then writes 64
    // consecutive labels (256 contiguous bytes) of one pixel.  Byte offset of (lane, g, r):
    // CM_BIAS + 4 (j Lp + k) = ab + st (4 g + r) + 64 m0, VGPR part ab, the rest uniform.
    const int kt = v == 0 ? CM_JB * grp - col : CM_JB * grp + col;  // k = kt + kg (4g + r) + 16 m0
    const int kg = v == 0 ? 1 : -1;
    const uint32_t ab = CM_BIAS + 4u * (uint32_t)(j0 * Lp + kt);
    const int st = 4 * (Lp + kg);
    auto group = [&](int m0, int cnt, auto FASTc) {
        constexpr bool FAST = decltype(FASTc)::value != 0;
        float X[4][4];  // [tile t][row r]
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            if (t < cnt) {
                const int m = m0 + t;
                const v4f_ acc = mma(m);
                const int p0 = pb + ps * m;
                const uint32_t vc = cl[p0];
                bool xok = true;
                if (!FAST) {
                    const int x = xs0 + p0 + col;
                    xok = x - hw >= 0 && x + hw < W;
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const uint32_t cen4 = (uint32_t)acc[r];  // 4 x census: byte offset into sB
                    const uint32_t ad4 = __builtin_amdgcn_sad_u8(fc[r], vc, 0u) << 2;
                    const float c = *reinterpret_cast<const float*>(reinterpret_cast<const char*>(sA2) + ad4) -
                                    *reinterpret_cast<const float*>(reinterpret_cast<const char*>(sB) + cen4);
                    X[t][r] = (FAST || (fo[r] && xok)) ? c : 2.f;
                }
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) X[t][r] = 0.f;  // past tile M: every store masked
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            uint32_t R0 = __float_as_uint(X[0][r]), R1 = __float_as_uint(X[1][r]);
            uint32_t R2 = __float_as_uint(X[2][r]), R3 = __float_as_uint(X[3][r]);
            auto a = __builtin_amdgcn_permlane32_swap(R0, R2, false, false);  // rows 2,3 <-> 0,1
            R0 = a[0]; R2 = a[1];
            a = __builtin_amdgcn_permlane32_swap(R1, R3, false, false);
            R1 = a[0]; R3 = a[1];
            a = __builtin_amdgcn_permlane16_swap(R0, R1, false, false);  // odd rows <-> even rows
            R0 = a[0]; R1 = a[1];
            a = __builtin_amdgcn_permlane16_swap(R2, R3, false, false);
            R2 = a[0]; R3 = a[1];
            const uint32_t Rg[4] = {R0, R1, R2, R3};
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int n = 4 * g + r;  // pixel j0 + n
                int voff = (int)ab;
                if (!FAST) {
                    const int k = kt + kg * n + CM_JB * m0;
                    voff = ((unsigned)k < (unsigned)L && grp < cnt && j0 + n < W) ? voff : -1;
                }
                __builtin_amdgcn_raw_buffer_store_b32(Rg[g], vrs, voff, 64 * m0 + st * n, TSM_CM_STAUX);
            }
        }
    };
    tile(0, IC<0>{});  // the band edge k = -15..15 (one tile, per-cell stores)
    for (int m0 = 1; m0 <= M; m0 += 4) {
        const int cnt = min(4, M + 1 - m0);
        if (cnt == 4 && m0 >= f_lo && m0 + 3 <= f_hi) group(m0, 4, IC<1>{});
        else group(m0, cnt, IC<0>{});
    }
    }
#endif
    // padding labels L..Lp-1: +inf (lane = pixel)
    if (Lp > L && lane < CM_JB && j0 + lane < W) {
        for (int k = L; k < Lp; ++k)
            __builtin_amdgcn_raw_buffer_store_b32(0x7f800000u, vrs, (int)(CM_BIAS + 4u * (uint32_t)((j0 + lane) * Lp + k)), 0, 0);
    }
}

size_t cost_mfma_lds_bytes(const DevParams& P) {
    const int XS = cost_mfma_span(P.L);
    return (size_t)XS * 12 * 16 + (size_t)XS * 4;
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
void launch_pack(const PairIn& in, size_t step, uint32_t* img, const DevParams& P, hipStream_t st) {
    dim3 g((P.W + 255) / 256, P.H, 2 * P.npairs);
    hipLaunchKernelGGL(k_pack_bgr, g, dim3(256), 0, st, in, step, P.H, P.W, img, P.pstride); trace_point("k_pack_bgr", st);
}

void launch_hsi(const uint32_t* src, uint32_t* tmp, uint32_t* dst, int filter, const DevParams& P,
                hipStream_t st) {
    const int H = P.H, W = P.W;
    const int n = 2 * H * W;
    const dim3 g1((n + 255) / 256, 1, P.npairs);
    if (filter) {
        hipLaunchKernelGGL(k_bgr2hsi, g1, dim3(256), 0, st, src, dst, n, 1, P.pstride); trace_point("k_bgr2hsi", st);
    } else {
        hipLaunchKernelGGL(k_bgr2hsi, g1, dim3(256), 0, st, src, tmp, n, 0, P.pstride); trace_point("k_bgr2hsi", st);
        dim3 g((W + 255) / 256, H, 2 * P.npairs);
        hipLaunchKernelGGL(k_gauss_median, g, dim3(256), 0, st, tmp, dst, H, W, P.pstride); trace_point("k_gauss_median", st);
    }
}

void launch_census(const uint32_t* img, uint32_t* desc, const DevParams& P, hipStream_t st) {
    dim3 g((P.W + 127) / 128, P.H, 2 * P.npairs);
    const bool hsi = P.color_model == 1;
    if (P.censusW == 7) {
        if (hsi) hipLaunchKernelGGL((k_census_desc<7, 5, true>), g, dim3(128), 0, st, img, desc, P);
        else hipLaunchKernelGGL((k_census_desc<7, 5, false>), g, dim3(128), 0, st, img, desc, P);
    } else {
        if (hsi) hipLaunchKernelGGL((k_census_desc<9, 7, true>), g, dim3(128), 0, st, img, desc, P);
        else hipLaunchKernelGGL((k_census_desc<9, 7, false>), g, dim3(128), 0, st, img, desc, P);
    }
    trace_point("k_census_desc", st);
}

// Walk unit length: each unit pays a 256-record warm-up gather, so units are long
// enough to amortise it and short enough that the pull queue balances the SIMDs.
static int cost_seg_len(const DevParams& P) {
    static const int env = [] {
        const char* e = getenv("TSM_COST_SEG");  // tuning override
        return e ? atoi(e) : 0;
    }();
    if (env >= 8) return (env + 7) / 8 * 8;
    (void)P;
    return CW_SEG;
}

size_t cost_volume_lds_bytes(const DevParams& P, int lutA_n) {
    // sized for E = 4 with the shear's margin: covers every E / group size the walk uses
    (void)P;
    (void)lutA_n;  // the tables are static LDS; this is the dynamic ring part
    const int E = P.Lp <= 256 ? 4 : 8;
    return (size_t)(CW_THREADS / 64) * 2 * cost_stage_slots(cost_seg_len(P) + 2 * E, E) * 64;
}

// View-1 float4s the shear walk never completes: lane l of pixel x1 with x1 + 4l > W
// (every label's left column x1 + k >= W: border cells, 2, or +inf padding).
__global__ void k_shear_tail(float* __restrict__ vol, DevParams Pk) {
    const DevParams P = Pk;
    const int Q = P.Lp >> 2;
    const int span = min(P.W, 4 * Q);  // x1 in [W - span, W)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    if (i >= span * Q) return;
    const int x1 = P.W - span + i / Q, l = i % Q;
    if (x1 + 4 * l <= P.W) return;
    pair_shift(blockIdx.z, P.pstride, vol);
    const float inf = __int_as_float(0x7f800000);
    f32x4 o;
    o.x = 4 * l + 0 < P.L ? 2.f : inf;
    o.y = 4 * l + 1 < P.L ? 2.f : inf;
    o.z = 4 * l + 2 < P.L ? 2.f : inf;
    o.w = 4 * l + 3 < P.L ? 2.f : inf;
    *reinterpret_cast<f32x4*>(vol + (((size_t)P.H + y) * P.W + x1) * P.Lp + 4 * l) = o;
}

template <int E, bool HSI, bool MASK, int MODE>
static void launch_cost_t(const uint32_t* desc, const float* lutA, int lutA_n, const float* lutB,
                          float* vol, const DevParams& P, uint32_t* ctr, uint32_t& ctr_base,
                          hipStream_t st) {
    const int seg_len = cost_seg_len(P);
    const int nseg = (P.W + seg_len - 1) / seg_len;
    const int units = (MODE == CW_BOTH ? 2 : 1) * P.H * nseg;
    const int waves = units;
    const int wpb = CW_THREADS / 64;
    // whole multiples of the 8 XCDs per pair, so every pair's blocks keep the same
    // block -> XCD dealing (the unit remap in the kernel relies on it)
    dim3 g(((waves + wpb - 1) / wpb + 7) / 8 * 8, 1, P.npairs);
    hipLaunchKernelGGL((k_cost_walk<E, HSI, MASK, MODE>), g, dim3(CW_THREADS), cost_volume_lds_bytes(P, lutA_n),
                       st, desc, lutA, lutA_n, lutB, vol, P, seg_len, nseg, ctr, ctr_base);
    trace_point("k_cost_walk", st);
    if (MODE == CW_SHEAR) {
        const int Q = P.Lp >> 2;
        const int n = (P.W < 4 * Q ? P.W : 4 * Q) * Q;
        hipLaunchKernelGGL(k_shear_tail, dim3((n + 255) / 256, P.H, P.npairs), dim3(256), 0, st, vol, P);
        trace_point("k_shear_tail", st);
    }
    ctr_base += (uint32_t)units + (uint32_t)(g.x * wpb);  // every wave overshoots once
}

// One launch walking both views (default), or -- TSM_COST_VIEWS=1 -- one launch per view,
// each kernel holding one walk direction (101-109 instead of 157 VGPRs, but the second
// launch's ramp costs more than the occupancy gains: 265 vs 255 us on config B).
template <int E, bool HSI, bool MASK>
static void launch_cost_views(const uint32_t* desc, const float* lutA, int lutA_n, const float* lutB,
                              float* vol, const DevParams& P, uint32_t* ctr, uint32_t& ctr_base,
                              hipStream_t st) {
    static const bool both = [] {
        const char* e = getenv("TSM_COST_VIEWS");
        return !(e && e[0] == '1');
    }();
    if (both) {
        launch_cost_t<E, HSI, MASK, CW_BOTH>(desc, lutA, lutA_n, lutB, vol, P, ctr, ctr_base, st);
        return;
    }
    launch_cost_t<E, HSI, MASK, CW_VIEW0>(desc, lutA, lutA_n, lutB, vol, P, ctr, ctr_base, st);
    launch_cost_t<E, HSI, MASK, CW_VIEW1>(desc, lutA, lutA_n, lutB, vol, P, ctr, ctr_base, st);
}

int launch_cost_volume(const uint32_t* img, const uint32_t* desc, const float* lutA, int lutA_n,
                       const float* lutB, float* vol, const DevParams& P, uint32_t* ctr,
                       uint32_t& ctr_base, hipStream_t st) {
    (void)img;
    const bool hsi = P.color_model == 1;
    // The product path is the walk (north_star: census by popcount, no MFMA).  The
    // matrix-core build is a measured experiment kept for the record: TSM_COST_MFMA=1
    // (RGB without mask mode) selects it.
    static const bool use_mfma = [] {
        const char* e = getenv("TSM_COST_MFMA");
        return e && e[0] == '1';
    }();
    const size_t mlds = cost_mfma_lds_bytes(P);
    if (use_mfma && !hsi && !P.mask && lutA_n <= 768 && mlds + 4 * (768 + 192) <= 160 * 1024) {
        static bool attr = false;
        if (!attr) {
            (void)hipFuncSetAttribute((const void*)k_cost_mfma<0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      160 * 1024 - 4 * (768 + 192));
            (void)hipFuncSetAttribute((const void*)k_cost_mfma<12>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      160 * 1024 - 4 * (768 + 192));
            attr = true;
        }
        const int nseg = (P.W + CM_SEG - 1) / CM_SEG;
        const int units = 2 * P.H * nseg;
        const dim3 g((units + 7) / 8 * 8, 1, P.npairs);  // whole multiples of the 8 XCDs
        if (cost_mfma_tiles(P.L) == 12)  // L = 178..193 (config B)
            hipLaunchKernelGGL(k_cost_mfma<12>, g, dim3(CM_THREADS), mlds, st, desc, lutA, lutA_n, lutB, vol, P, nseg);
        else
            hipLaunchKernelGGL(k_cost_mfma<0>, g, dim3(CM_THREADS), mlds, st, desc, lutA, lutA_n, lutB, vol, P, nseg);
        trace_point("k_cost_mfma", st);
        return 0;
    }
#define CASE(E)                                                                                  \
    if (hsi) {                                                                                     \
        if (P.mask) launch_cost_views<E, true, true>(desc, lutA, lutA_n, lutB, vol, P, ctr, ctr_base, st);  \
        else launch_cost_views<E, true, false>(desc, lutA, lutA_n, lutB, vol, P, ctr, ctr_base, st);        \
    } else {                                                                                       \
        if (P.mask) launch_cost_views<E, false, true>(desc, lutA, lutA_n, lutB, vol, P, ctr, ctr_base, st); \
        else launch_cost_views<E, false, false>(desc, lutA, lutA_n, lutB, vol, P, ctr, ctr_base, st);       \
    }
    // minD = 0 without mask mode: view 1 is an exact shear of view 0 and one walk can emit
    // both (parity-green).  Off by default: its view-1 stores are 16-B scatters (one per
    // lane, 64 different pixel vectors per instruction) and cost more than the second walk
    // saves (MI355X, config B: 390 us vs 254 us; 149 us with the view-1 stores removed).
    // TSM_COST_SHEAR=1 selects it.
    static const bool shear = [] {
        const char* e = getenv("TSM_COST_SHEAR");
        return e && e[0] == '1';
    }();
    if (P.minD == 0 && !P.mask && P.Lp <= 256 && shear) {
        if (hsi) launch_cost_t<4, true, false, CW_SHEAR>(desc, lutA, lutA_n, lutB, vol, P, ctr, ctr_base, st);
        else launch_cost_t<4, false, false, CW_SHEAR>(desc, lutA, lutA_n, lutB, vol, P, ctr, ctr_base, st);
        return 0;
    }
    // one wave holds the whole label axis: E labels per lane.  At Lp 192 / 196 three labels
    // a lane fill all 64 lanes (E = 4 would leave 15 of them idle) and a per-unit tail pass
    // writes labels 192..195.  TSM_COST_E4=1 keeps E = 4.
    static const bool e4 = [] {
        const char* e = getenv("TSM_COST_E4");
        return e && e[0] == '1';
    }();
    if (!e4 && !P.mask && (P.Lp == 192 || P.Lp == 196)) { CASE(3) }
    else if (!e4 && !P.mask && (P.Lp == 320 || P.Lp == 324)) { CASE(5) }
    else if (P.Lp <= 256 || (!P.mask && P.Lp == 260)) { CASE(4) }
    else if (P.Lp <= 512) { CASE(8) }
    else return -1;
#undef CASE
    return 0;
}

}  // namespace tsm

#ifdef TSM_EXP_STAMPS
extern "C" int tsm_exp_stamps(void* host, size_t bytes) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(tsm::g_stamps), bytes, 0, hipMemcpyDeviceToHost);
}
#endif
