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

// bgr2hsi, ADCensus.cpp:1429-1473 (filter: :1463-1470).  The conversion is a pure function
// of the pixel's (B, G, R), so it comes from a 2^24-entry table (H | S << 8 | I << 16) the
// host builds once with the reference's float expressions and its own libm acosf
// (engine.cpp hsi_table): the hue byte is then bit-identical to the host's, which a device
// acosf does not guarantee.
__global__ void k_bgr2hsi(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, int n,
                          int filter, const uint32_t* __restrict__ table, size_t ps) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    pair_shift(blockIdx.z, ps, src, dst);
    uint32_t out = table[src[i] & 0xffffffu];
    const uint32_t Hh = out & 0xffu;
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
//   HSI: words 0..1 = hue "positive" plane, 2..5 = sat/int gt, 6..9 = sat/int lt,
//        10 = the hue byte alone, 11 = the sat / int bytes alone (the AD term's two sums
//        without per-cell masks in the walk)
//   word 12 = the pixel's packed colour (AD term, mask tests), words 13..15 = 0.
// One 64-B record per pixel, so the cost walk fetches a whole record with one scalar
// load.  Border pixels (window leaving the image) never reach the cost (:562-566):
// their planes are zero.
// ---------------------------------------------------------------------------
constexpr int CD_TX = 128;  // pixels of a row per workgroup

template <int CW, int CHh, bool HSI>
__global__ __launch_bounds__(CD_TX) void k_census_desc(const uint32_t* __restrict__ img, uint32_t* __restrict__ desc,
                                                       DevParams Pk) {
    const DevParams P = Pk;  // kernel args -> registers once (no per-use kernarg reloads)
    constexpr int hw = CW / 2, hh = CHh / 2;
    constexpr int TW = CD_TX + 2 * hw;  // the window's rows for the block's pixels, staged in LDS
    __shared__ uint32_t s_win[CHh][TW];
    const int x0 = blockIdx.x * CD_TX;
    const int x = x0 + threadIdx.x;
    const int y = blockIdx.y;
    const int v = blockIdx.z & 1;
    const int H = P.H, W = P.W;
    pair_shift(blockIdx.z >> 1, P.pstride, img, desc);
    const uint32_t* im = img + (size_t)v * H * W;
    for (int i = threadIdx.x; i < CHh * TW; i += CD_TX) {
        const int r = i / TW, c = i - r * TW;
        const int yy = y - hh + r, xx = x0 - hw + c;
        s_win[r][c] = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? im[(size_t)yy * W + xx] : 0u;
    }
    __syncthreads();
    if (x >= W) return;
    uint32_t w[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) w[k] = 0;
    const int tx = threadIdx.x + hw;
    const uint32_t c = s_win[hh][tx];
    if (x - hw >= 0 && x + hw < W && y - hh >= 0 && y + hh < H) {
        const int c0 = ch(c, 0), c1 = ch(c, 1), c2 = ch(c, 2);
        // fully unrolled: bit position and word index are compile-time constants
#pragma unroll
        for (int i = -hh; i <= hh; ++i) {
#pragma unroll
            for (int j = -hw; j <= hw; ++j) {
                if (i == 0 && j == 0) continue;
                const int bit = (i + hh) * CW + (j + hw) - (((i + hh) * CW + (j + hw)) > (hh * CW + hw) ? 1 : 0);
                const int wi = bit >> 5;
                const uint32_t m = 1u << (bit & 31);
                const uint32_t n = s_win[i + hh][tx + j];
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
    if (HSI) {
        w[10] = c & 0xffu;
        w[11] = c & 0xffff00u;
    }
    o[0] = u32x4{w[0], w[1], w[2], w[3]};
    o[1] = u32x4{w[4], w[5], w[6], w[7]};
    o[2] = u32x4{w[8], w[9], w[10], w[11]};
    o[3] = u32x4{c, 0u, 0u, 0u};
}

// ---------------------------------------------------------------------------
// cost-volume build: one wave walks a row segment, the matched-against records held
// in a lane-shift register
// ---------------------------------------------------------------------------
// Lanes own E consecutive labels k = kb + E*lane + e (kb: the unit's label slice, 0 unless
// the range needs more than 64 E labels), so a pixel's L-vector leaves as E 4-B elements
// per lane in one run of contiguous bytes (768 B at L = 193, E = 3).  View 0 pairs the fixed
// pixel left(j - minD) with right(j - k) at label k; view 1 pairs right(j + minD) with
// left(j + k) (costInitialize :542-579).  View 0 walks j upward and view 1 walks it
// downward in label space, so in BOTH views the next pixel needs at label k the record
// that label k-1 holds now: the label axis moves up one slot per step.  Inside a lane that
// is a rotation of the E slot registers (compile-time renaming, no data movement); one DPP
// wave_shr:1 per word carries the top slot into the next lane, and the one record that
// enters (label kb: varying column j - kb) arrives as the DPP `old` operand of lane 0.  The
// fixed pixel's record is wave-uniform.  A cost cell is 6 x (and, and_or, bcnt) + one
// v_sad_u8 + two LDS table reads.  Census and AD are symmetric in (left, right), so both
// views run the same arithmetic.
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

// HSI AD table index (computeHSIADCost :439-451 with the lambdas 1, 2.5, 2.5 the engine
// requires, doubled: the table holds k / 2): 2 * circular hue distance + 5 * (|dS| + |dI|),
// the factor 5 as a 24-bit multiply (the compiler otherwise picks the quarter-rate
// v_mul_lo_u32)
// The records carry the hue byte and the sat / int bytes as separate words (10, 11), so
// neither sum needs a mask.
__device__ __forceinline__ int hsi_ad(uint32_t fh, uint32_t fsi, uint32_t vh, uint32_t vsi) {
    const uint32_t hd = __builtin_amdgcn_sad_u8(fh, vh, 0u);
    const uint32_t si = __builtin_amdgcn_sad_u8(fsi, vsi, 0u);
    return (int)(2u * min(hd, 255u - hd) + __umul24(si, 5u));
}

// labels one walk unit covers: 64 E, the tail float4 aside
__host__ __device__ constexpr int cw_slice(int E) { return 64 * E; }

// waves per SIMD asked of the walk: E = 3 is held to 128 VGPRs (measured: 3 -> 209 us,
// 4 -> 205, 5 / 6 spill: 341 / 384); the wider shift registers need more
template <int E, bool HSI, bool MASK>
__global__ __launch_bounds__(CW_THREADS) __attribute__((amdgpu_waves_per_eu(E == 3 ? 4 : (E == 4 ? 3 : 1)))) void k_cost_walk(
    const uint32_t* __restrict__ desc, const float* __restrict__ lutA, int lutA_n,
    const float* __restrict__ lutB, float* __restrict__ vol, DevParams Pk, int seg_len, int nseg, int nsl) {
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
    pair_shift(blockIdx.z, P.pstride, desc, vol);
    // one walk unit (view, row, segment, label slice) per wave.  XCD-aware unit order:
    // workgroups are dealt round-robin to the 8 XCDs, so block b runs on XCD b % 8;
    // remapping b -> (b % 8) * per + b / 8 gives each XCD a contiguous run of units
    // (neighbouring segments of the same rows), whose warm-up gathers and tails then
    // re-read records its own L2 already holds.
    const int nb = gridDim.x, per = nb >> 3;
    const int blk = (int)blockIdx.x < 8 * per ? ((int)blockIdx.x & 7) * per + ((int)blockIdx.x >> 3) : (int)blockIdx.x;
    const int gw0 = blk * (CW_THREADS / 64) + wave;
    const bool active = gw0 < 2 * H * nseg * nsl;
    const int gw = active ? gw0 : 0;
    const int sl = gw % nsl;
    const int seg = (gw / nsl) % nseg;
    const int row = gw / (nsl * nseg);
    // views interleaved row by row (unit row 2y + v): view 0 and view 1 of image row y read
    // the same two record rows (left y, right y), so both walks of a row land on one XCD
    // and its L2 fetches those records once
    const int v = row & 1;
    const int y = row >> 1;
    const int kb = sl * cw_slice(E);                    // first label of the slice
    const int kmax = min(L, kb + cw_slice(E)) - 1;      // last real label of the slice
    const int foff = v == 0 ? -P.minD : P.minD;
    const int x_lo = seg * seg_len;
    const int count = min(seg_len, W - x_lo);  // steps walked
    const int j0 = x_lo;  // both views walk j upward: stores stream forward through HBM
    const int vtop = E * 64 - 1;  // view 1 feeds its shift register at the top label
    const int hw = P.censusW >> 1, hh = P.censusH >> 1;
    const bool rowOut = y - hh < 0 || y + hh >= H;
    // shifted words: RGB the 12 descriptor planes + the colour (word 12); HSI the 10 planes +
    // the hue and sat / int words (10, 11).  Either way word w of a record.
    constexpr int NW = HSI ? 12 : 13;
    constexpr int CWORD = 12;          // colour word of a record
    const uint32_t vmask_hi = (P.censusW * P.censusH - 1) >= 64
                                  ? 0xffffffffu
                                  : ((1u << ((P.censusW * P.censusH - 1) - 32)) - 1u);
    const uint32_t* dF = desc + ((size_t)v * H + y) * W * 16;        // fixed image
    const uint32_t* dV = desc + ((size_t)(1 - v) * H + y) * W * 16;  // varying image
    float* orow = vol + ((size_t)v * H + y) * W * Lp + kb + E * lane;
    auto clampx = [&](int x) { return x < 0 ? 0 : (x >= W ? W - 1 : x); };

    // The unit's two wave-uniform record streams (fixed records x = j + foff, entering
    // records x = j - kb (view 0) or j + kb + vtop (view 1)) are staged in LDS up front by
    // LDS-DMA (global_load_lds_dwordx4: lane i's 16 bytes land at chunk base + 16 i, i.e.
    // record i/4, quarter i%4; no staging registers): per step they are broadcast LDS
    // reads, never an L2/HBM round trip.
    // steps run in groups of G (F/Fn double-buffering needs an even group)
    constexpr int G = (E & 1) ? 2 * E : E;
    const int slots = cost_stage_slots(seg_len, G);
    u32x4* stF = smem_stage + (size_t)wave * 2 * slots * 4;
    u32x4* stE = stF + (size_t)slots * 4;
    // the unit's tail float4s (Lp = 64 E + 4), one per pixel, computed before the walk
    f32x4* stT = reinterpret_cast<f32x4*>(smem_stage + (size_t)(CW_THREADS / 64) * 2 * slots * 4) + wave * CW_SEG;
    const bool tail = (E == 3 || E == 4 || E == 5) && Lp > 64 * E;
    const int rq = lane & 3, rr = lane >> 2;  // this lane's quarter / record of a chunk
    const int eoff = v == 0 ? -kb : kb + vtop;
    auto dma_chunk = [&](int t0) {  // records t0 .. t0+CW_CHUNK-1 (t0 a multiple of CW_CHUNK)
        const int t = t0 + rr;
        const int base = t0 * 4;
        __builtin_amdgcn_global_load_lds(
            reinterpret_cast<const u32x4*>(dF + (size_t)clampx(j0 + t + foff) * 16) + rq, stF + base, 16, 0, 0);
        __builtin_amdgcn_global_load_lds(
            reinterpret_cast<const u32x4*>(dV + (size_t)clampx(j0 + t + eoff) * 16) + rq, stE + base, 16, 0, 0);
    };
    for (int c = 0; c < slots; c += CW_CHUNK) dma_chunk(c);

    // sA holds 2 - A[ad]: the reference's (2 - A) - B with its first subtraction done once
    for (int i = threadIdx.x; i < lutA_n; i += CW_THREADS) sA[i] = 2.f - lutA[i];
    for (int i = threadIdx.x; i < 2 * CW_LUTB; i += CW_THREADS)
        sB[i] = i < 188 ? lutB[i] : (i >= CW_LUTB ? -__int_as_float(0x7f800000) : 0.f);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // ring prologue landed (LDS-DMA)
    __syncthreads();  // tables ready: the kernel's only barrier (waiting here costs nothing
                      // measurable: a probe without it ran 200.3 against 200.6 us, round 4)
    if (!active) return;

    // warm-up: label k = kb + E*lane + e holds the varying record at x = j0 - k (view 0)
    // or j0 + k (view 1), clamped: labels whose column leaves the image are border cells,
    // fixed up per step.  (Rotation 0: label offset e sits in slot e in both views.)
    uint32_t V[NW][E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int k = kb + E * lane + e;
        int x = v == 0 ? j0 - k : j0 + k;
        x = x < 0 ? 0 : (x >= W ? W - 1 : x);
        const u32x4* r = reinterpret_cast<const u32x4*>(dV + (size_t)x * 16);
        const u32x4 a = r[0], b = r[1], c = r[2], d = r[3];
        const uint32_t rec[13] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w, d.x};
#pragma unroll
        for (int w = 0; w < NW; ++w) V[w][e] = rec[w];
    }

    // record -> NW shifted words (descriptor planes, then the colour)
    auto pick = [&](const u32x4& a, const u32x4& b, const u32x4& c, const u32x4& d, uint32_t (&o)[NW]) {
        const uint32_t rec[13] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w, d.x};
#pragma unroll
        for (int w = 0; w < NW; ++w) o[w] = rec[w];
    };
    auto load_staged = [&](const u32x4* st, int t, uint32_t (&o)[NW]) {
        const int i = t * 4;
        const uint32_t* r1 = reinterpret_cast<const uint32_t*>(st + i);
        pick(st[i + 0], st[i + 1], st[i + 2], u32x4{r1[CWORD], 0u, 0u, 0u}, o);
    };

    // Lp = 64 E + 4 (E = 3: 193..196 labels, 4: 257..260, 5: 321..324): the lanes cover
    // labels 0 .. 64E-1, the pixel vector's last float4 (labels 64E .. Lp-1, the real ones
    // < L, the rest +inf padding) is the tail.  Lane l computes pixel x_lo + l's tail here,
    // before the walk -- its fixed record from the LDS stage, its varying records from L2,
    // where the warm-up has just brought that row segment -- into LDS; the walk's step for
    // the pixel stores it beside the pixel's main store, so the two land in one L2 line
    // while it is still there (a tail stored after the walk reached HBM as separate partial
    // lines: 46 MB of the launch's 776 MB written, and re-fetched its records: round 3 PMC).
    if (tail) {
        if (lane < count) {
            const int j = x_lo + lane;
            const float inf = __int_as_float(0x7f800000);
            uint32_t Fr[NW];
            load_staged(stF, lane, Fr);
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
                        cen = bcnt_acc(~(Fr[1] & Vr[1]) & vmask_hi, bcnt_acc(~(Fr[0] & Vr[0]), 0u));
#pragma unroll
                        for (int w = 2; w < 6; ++w) cen = bcnt_acc((Fr[w] & Vr[4 + w]) | (Fr[4 + w] & Vr[w]), cen);
                    }
                    int ai;
                    if (!HSI) {
                        ai = (int)__builtin_amdgcn_sad_u8(Fr[NW - 1], Vr[NW - 1], 0u);
                    } else {
                        ai = hsi_ad(Fr[10], Fr[11], Vr[10], Vr[11]);
                    }
                    const float c = sA[ai] - sB[cen];
                    c4[t] = (fixed_ok && k >= klo && k <= khi) ? c : 2.f;
                }
            }
            stT[lane] = f32x4{c4[0], c4[1], c4[2], c4[3]};
        }
        __builtin_amdgcn_wave_barrier();  // one wave: its LDS writes precede its reads in order
    }

    // View 0 pairs label k with right(j - k): the next pixel's label k is this pixel's
    // label k-1, so the label axis moves UP one slot per step (slot of offset e at
    // rotation R: (e - R) mod E; DPP wave_shr carries lanes up, lane 0 takes the entering
    // record x = j - kb).  View 1 pairs label k with left(j + k): the label axis moves DOWN
    // (slot (e + R) mod E; wave_shl, lane 63 takes x = j + kb + vtop).
    auto walk = [&](auto UPc, auto PADc) {
    constexpr bool UP = decltype(UPc)::value == 0;
    constexpr bool PAD = decltype(PADc)::value != 0;  // some lane label of the slice is >= L
    const float kInf = __int_as_float(0x7f800000);
    uint32_t padoff[E];  // census start: 0, or CW_LUTB for padding labels (+inf cost)
#pragma unroll
    for (int e = 0; e < E; ++e) padoff[e] = (PAD && !MASK && kb + E * lane + e >= L) ? CW_LUTB : 0u;
    // fixed records double-buffered by step parity (compile-time), no register copies
    uint32_t FA[NW], FB[NW], En[NW];
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
        } else {  // hue: NAND of the positive-class planes (:489-492), then 4 gt/lt words
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const int s = UP ? (e - R + E) % E : (e + R) % E;
                cen[e] = bcnt_acc(~(F[0] & V[0][s]), cen[e]);
            }
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const int s = UP ? (e - R + E) % E : (e + R) % E;
                cen[e] = bcnt_acc(~(F[1] & V[1][s]) & vmask_hi, cen[e]);
            }
#pragma unroll
            for (int k = 2; k < 6; ++k)
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const int s = UP ? (e - R + E) % E : (e + R) % E;
                    cen[e] = bcnt_acc((F[k] & V[4 + k][s]) | (F[4 + k] & V[k][s]), cen[e]);
                }
        }
        float c[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int s = UP ? (e - R + E) % E : (e + R) % E;
            int ai;
            uint32_t fc, vc;  // the packed colours (mask tests)
            if (!HSI) {
                fc = F[NW - 1];
                vc = V[NW - 1][s];
                ai = (int)__builtin_amdgcn_sad_u8(fc, vc, 0u);
            } else {
                fc = F[10] | F[11];
                vc = V[10][s] | V[11][s];
                ai = hsi_ad(F[10], F[11], V[10][s], V[11][s]);
            }
            // mask mode: black centre on either side -> census = +inf (:459-460)
            if (MASK && (fc == 0 || vc == 0)) cen[e] = 187;
            c[e] = sA[ai] - sB[cen[e]];
        }
        // border cells (either 9x7 window leaves the image, :562-566) and masked own
        // pixels (:551-555) cost 2; wave-uniform test first, per-label only near borders
        if (!fast) {
        const int xf = j + foff;
        bool fixed_ok = !rowOut && xf - hw >= 0 && xf + hw < W;
        if (MASK) fixed_ok = fixed_ok && dF[(size_t)__builtin_amdgcn_readfirstlane(j) * 16 + CWORD] != 0u;
        const int klo = v == 0 ? j - (W - 1 - hw) : hw - j;
        const int khi = v == 0 ? j - hw : W - 1 - hw - j;
        if (!(fixed_ok && klo <= kb && khi >= kmax)) {
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const int k = kb + E * lane + e;
                c[e] = (fixed_ok && k >= klo && k <= khi) || k >= L ? c[e] : 2.f;
            }
        }
        }
        if (MASK) {  // mask mode overrides census indices: padding needs its own select
#pragma unroll
            for (int e = 0; e < E; ++e) c[e] = kb + E * lane + e >= L ? kInf : c[e];
        }
        if (fast || t < count) {
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
            // E = 4 / 8: 16-B pieces, plain stores like E = 3 / 5.  A pixel vector of 260 labels is
            // 1040 B, not a whole number of 64-B granules: its neighbours' stores complete the
            // shared granules in L2 only if they stay there -- as non-temporal stores config C
            // wrote 3.46 GB for a 3.09 GB volume and the walk took 0.98 ms; plain: 3.12 GB,
            // 0.83 ms (round 6, profiles/r06_cost_walk_C.txt)
            if constexpr (E == 4 || E == 8) {  // (E = 5 is the F5 store above, whole)
#pragma unroll
                for (int q = 0; q < E / 4; ++q)
                    if (kb + E * lane + 4 * q < Lp)
                        *reinterpret_cast<f32x4*>(orow + (size_t)j * Lp + 4 * q) =
                            f32x4{c[4 * q], c[4 * q + 1], c[4 * q + 2], c[4 * q + 3]};
            }
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
    const int jlo = max(v == 0 ? hw + kmax : hw - kb, hw - foff);
    const int jhi = min(v == 0 ? W - 1 - hw + kb : W - 1 - hw - kmax, W - 1 - hw - foff);
    const int tf_lo = jlo - j0;
    const int tf_hi = min(jhi - j0, count - 1);
    const bool rows_ok = !MASK && !rowOut;
    for (int t = 0; t < count; t += G) {
        const bool fast = rows_ok && t >= tf_lo && t + G - 1 <= tf_hi;
        [&]<int... Ss>(std::integer_sequence<int, Ss...>) {
            (step(IC<Ss>{}, fast, t + Ss), ...);
        }(std::make_integer_sequence<int, G>{});
        // the group's tail float4s (labels 64E .. 64E+3), lane s for pixel j0 + t + s, a
        // few steps after those pixels' main stores: both still in L2.  The lane id is
        // recomputed here (2 VALU): held across the walk it was the register the allocator
        // spilled, and the reload's wait (vmcnt, in order with the volume stores) then
        // drained every group's stores before the walk went on.
        if (tail) {
            int ln;
            asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
            if (ln < G && t + ln < count)
                *reinterpret_cast<f32x4*>(vol + (((size_t)v * H + y) * W + j0 + t + ln) * Lp + 64 * E) = stT[t + ln];
        }
    }
    };
    // slices whose lane labels are all real (config B: 192 of 193) keep no padding offsets
    // live in registers
    if (kb + 64 * E <= L) {
        if (v == 0) walk(IC<0>{}, IC<0>{});
        else walk(IC<1>{}, IC<0>{});
    } else {
        if (v == 0) walk(IC<0>{}, IC<1>{});
        else walk(IC<1>{}, IC<1>{});
    }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
void launch_pack(const PairIn& in, size_t step, uint32_t* img, const DevParams& P, hipStream_t st) {
    dim3 g((P.W + 255) / 256, P.H, 2 * P.npairs);
    hipLaunchKernelGGL(k_pack_bgr, g, dim3(256), 0, st, in, step, P.H, P.W, img, P.pstride); trace_point("k_pack_bgr", st);
}

void launch_hsi(const uint32_t* src, uint32_t* tmp, uint32_t* dst, int filter, const uint32_t* table,
                const DevParams& P, hipStream_t st) {
    const int H = P.H, W = P.W;
    const int n = 2 * H * W;
    const dim3 g1((n + 255) / 256, 1, P.npairs);
    if (filter) {
        hipLaunchKernelGGL(k_bgr2hsi, g1, dim3(256), 0, st, src, dst, n, 1, table, P.pstride); trace_point("k_bgr2hsi", st);
    } else {
        hipLaunchKernelGGL(k_bgr2hsi, g1, dim3(256), 0, st, src, tmp, n, 0, table, P.pstride); trace_point("k_bgr2hsi", st);
        dim3 g((W + 255) / 256, H, 2 * P.npairs);
        hipLaunchKernelGGL(k_gauss_median, g, dim3(256), 0, st, tmp, dst, H, W, P.pstride); trace_point("k_gauss_median", st);
    }
}

void launch_hsi_convert(const uint32_t* src, uint32_t* dst, int n, int filter, const uint32_t* table, hipStream_t st) {
    hipLaunchKernelGGL(k_bgr2hsi, dim3((n + 255) / 256, 1, 1), dim3(256), 0, st, src, dst, n, filter, table, (size_t)0);
    trace_point("k_bgr2hsi", st);
}

void launch_census(const uint32_t* img, uint32_t* desc, const DevParams& P, hipStream_t st) {
    dim3 g((P.W + CD_TX - 1) / CD_TX, P.H, 2 * P.npairs);
    const bool hsi = P.color_model == 1;
    if (P.censusW == 7) {
        if (hsi) hipLaunchKernelGGL((k_census_desc<7, 5, true>), g, dim3(CD_TX), 0, st, img, desc, P);
        else hipLaunchKernelGGL((k_census_desc<7, 5, false>), g, dim3(CD_TX), 0, st, img, desc, P);
    } else {
        if (hsi) hipLaunchKernelGGL((k_census_desc<9, 7, true>), g, dim3(CD_TX), 0, st, img, desc, P);
        else hipLaunchKernelGGL((k_census_desc<9, 7, false>), g, dim3(CD_TX), 0, st, img, desc, P);
    }
    trace_point("k_census_desc", st);
}

// Labels a lane owns for the label range of P: three (Lp 192 / 196: all 64 lanes busy, the
// tail float4 writes labels 192..195; E = 4 would leave 15 lanes idle: 255 -> 220 us), five
// (Lp 320 / 324), four up to 256 (+ the tail at 260), else eight in slices of 512 labels.
static int cost_lanes(const DevParams& P) {
    if (!P.mask && (P.Lp == 192 || P.Lp == 196)) return 3;
    if (!P.mask && (P.Lp == 320 || P.Lp == 324)) return 5;
    if (P.Lp <= 256 || (!P.mask && P.Lp == 260)) return 4;
    return 8;
}

size_t cost_volume_lds_bytes(const DevParams& P) {
    const int E = cost_lanes(P);
    const int G = (E & 1) ? 2 * E : E;
    return (size_t)(CW_THREADS / 64) * (2 * cost_stage_slots(CW_SEG, G) * 64 + CW_SEG * 16);
}

template <int E, bool HSI, bool MASK>
static void launch_cost_t(const uint32_t* desc, const float* lutA, int lutA_n, const float* lutB,
                          float* vol, const DevParams& P, hipStream_t st) {
    const int nseg = (P.W + CW_SEG - 1) / CW_SEG;
    const int nsl = E == 8 ? (P.Lp + cw_slice(E) - 1) / cw_slice(E) : 1;  // label slices
    const int units = 2 * P.H * nseg * nsl;
    const int wpb = CW_THREADS / 64;
    // whole multiples of the 8 XCDs per pair, so every pair's blocks keep the same
    // block -> XCD dealing (the unit remap in the kernel relies on it)
    dim3 g(((units + wpb - 1) / wpb + 7) / 8 * 8, 1, P.npairs);
    ensure_lds_limit((const void*)k_cost_walk<E, HSI, MASK>, cost_volume_lds_bytes(P));
    hipLaunchKernelGGL((k_cost_walk<E, HSI, MASK>), g, dim3(CW_THREADS), cost_volume_lds_bytes(P), st, desc, lutA,
                       lutA_n, lutB, vol, P, CW_SEG, nseg, nsl);
    trace_point("k_cost_walk", st);
}

int launch_cost_volume(const uint32_t* desc, const float* lutA, int lutA_n, const float* lutB, float* vol,
                       const DevParams& P, hipStream_t st) {
    const bool hsi = P.color_model == 1;
#define CASE(E)                                                                                  \
    if (hsi) {                                                                                     \
        if (P.mask) launch_cost_t<E, true, true>(desc, lutA, lutA_n, lutB, vol, P, st);            \
        else launch_cost_t<E, true, false>(desc, lutA, lutA_n, lutB, vol, P, st);                  \
    } else {                                                                                       \
        if (P.mask) launch_cost_t<E, false, true>(desc, lutA, lutA_n, lutB, vol, P, st);           \
        else launch_cost_t<E, false, false>(desc, lutA, lutA_n, lutB, vol, P, st);                 \
    }
    switch (cost_lanes(P)) {  // E = 3 and 5 are never asked for in mask mode
        case 3: if (hsi) launch_cost_t<3, true, false>(desc, lutA, lutA_n, lutB, vol, P, st);
                else launch_cost_t<3, false, false>(desc, lutA, lutA_n, lutB, vol, P, st);
                break;
        case 4: CASE(4) break;
        case 5: if (hsi) launch_cost_t<5, true, false>(desc, lutA, lutA_n, lutB, vol, P, st);
                else launch_cost_t<5, false, false>(desc, lutA, lutA_n, lutB, vol, P, st);
                break;
        default: CASE(8) break;
    }
#undef CASE
    return 0;
}

}  // namespace tsm
