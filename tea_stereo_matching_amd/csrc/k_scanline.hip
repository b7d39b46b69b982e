// k_scanline.hip -- step 3 of AD-Census on gfx950: scanline optimisation
// (scanlineOptimize, ADCensus.cpp:997-1011; scanline :983-995; partialOptimization
// :869-913; computeP1P2 :915-981) and the WTA (cost2disparity :1394-1413) fused into
// the last pass.
//
// The four passes per view are CHAINED and IN PLACE: every pixel reads its predecessor's
// already-updated L-vector.  The reference parallelises each pass over the recursion
// dimension (a data race); the kernels implement the serial semantics: one wave owns one
// line (a column for the vertical passes, a row for the horizontal ones) and walks it,
// keeping the predecessor vector in registers (lanes own 4 consecutive disparities).
//
// The walk is serial, with under one wave per SIMD, so the cost of a step is its
// instruction count.  The step is kept branch-free and short:
//  * the padding disparities d >= L of every vector hold +inf (written by the cost
//    kernel, preserved by aggregation and by this update), so the d-1 / d+1 neighbours
//    of d = 0 and d = L-1 need no guards: +inf never wins a min;
//  * all values are non-negative floats, which order like their bit patterns, so every
//    min is an unsigned-integer v_min3_u32 (exact, no canonicalisation);
//  * d2 (the other view's colour difference, or colorDiff+1 out of range) comes from a
//    sentinel-padded byte map through one aligned 8-byte load + v_alignbyte per step;
//  * everything that does not depend on the chain (the pixel vector, d1, the d2 bytes)
//    is prefetched SC_K steps ahead into a register ring.
// Optional emulation of the reference's racy omp-static schedule for T threads: the
// first pixel of each of the T chunks reads its predecessor's pre-pass vector.
#include <utility>

#include "tsm_device.h"
#include "tsm_launch.h"

namespace tsm {

// OpenMP static schedule (libgomp / vcomp): first n%T threads take q+1 iterations.
__device__ __forceinline__ bool omp_chunk_start(int it, int n, int T) {
    if (T <= 1 || n <= 0 || it == 0) return false;
    const int q = n / T, r = n % T;
    if (q == 0) return it < r;  // every thread owns one iteration
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

constexpr uint32_t kInfBits = 0x7f800000u;

__device__ __forceinline__ uint32_t fbits(float x) { return __float_as_uint(x); }
__device__ __forceinline__ float bitsf(uint32_t x) { return __uint_as_float(x); }
__device__ __forceinline__ uint32_t umin3(uint32_t a, uint32_t b, uint32_t c) {
    return min(min(a, b), c);  // lowered to v_min3_u32
}

// wave min of non-negative floats held as bits (+inf padding is neutral).  VG: keep it in
// VGPRs via the gfx950 lane swaps (faster on the scanline's serial chain when every
// consumer is a vector op; the WTA's scalar uses prefer the readlane form).
template <int N>
struct IC { static constexpr int value = N; };

template <int J, bool VG = false>
__device__ __forceinline__ uint32_t vec_min_bits(const f32x4 (&x)[J]) {
    uint32_t m = min(min(fbits(x[0][0]), fbits(x[0][1])), min(fbits(x[0][2]), fbits(x[0][3])));
#pragma unroll
    for (int j = 1; j < J; ++j)
        m = min(m, min(min(fbits(x[j][0]), fbits(x[j][1])), min(fbits(x[j][2]), fbits(x[j][3]))));
    return VG ? wave_min_bits_v(m) : wave_min_bits(m);
}

// WTA over indices [minD, L-1], first minimum (strict <, ADCensus.cpp:1404): the first d
// whose cost equals the minimum, found by a ballot.
template <int J>
__device__ __forceinline__ int vec_argmin(const f32x4 (&x)[J], int lane, int L, int minD, uint32_t m) {
    if (minD > 0) {  // minimum over [minD, L) only
        uint32_t mm = ~0u;
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int d = 4 * (lane + 64 * j) + e;
                if (d >= minD) mm = min(mm, fbits(x[j][e]));
            }
        m = wave_min_bits(mm);
    }
    if (!(bitsf(m) < 3.402823466e+38f)) return minD;  // nothing below FLT_MAX (reference: unset)
#pragma unroll
    for (int j = 0; j < J; ++j) {
        int first = 4;
#pragma unroll
        for (int e = 3; e >= 0; --e) {
            const int d = 4 * (lane + 64 * j) + e;
            if (fbits(x[j][e]) == m && d >= minD && d < L) first = e;
        }
        const uint64_t mask = __ballot(first < 4);
        if (mask) {
            const int ln = __builtin_ctzll(mask);
            return 4 * (ln + 64 * j) + __builtin_amdgcn_readlane(first, ln);
        }
    }
    return minD;
}

// Same result, branch-free and with the minimum m held in VGPRs (every lane equal), for
// the fused WTA inside the scanline's serial loop: no basic-block boundary per step, so
// the compiler can interleave one step's argmin with the next step's dependent chain.
template <int J>
__device__ __forceinline__ int vec_argmin_nb(const f32x4 (&x)[J], int lane, int L, int minD, uint32_t m) {
    if (minD > 0) {
        uint32_t mm = ~0u;
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int d = 4 * (lane + 64 * j) + e;
                if (d >= minD) mm = min(mm, fbits(x[j][e]));
            }
        m = wave_min_bits_v(mm);
    }
    const bool valid = __ballot(bitsf(m) < 3.402823466e+38f) != 0;  // reference: unset otherwise
    int res = minD;
    bool found = false;
#pragma unroll
    for (int j = J - 1; j >= 0; --j) {  // descending: the lowest j that holds m wins
        int first = 4;
#pragma unroll
        for (int e = 3; e >= 0; --e) {
            const int d = 4 * (lane + 64 * j) + e;
            if (fbits(x[j][e]) == m && d >= minD && d < L) first = e;
        }
        const uint64_t mask = __ballot(first < 4);
        const int ln = mask ? (int)__builtin_ctzll(mask) : 0;
        const int cand = 4 * (ln + 64 * j) + __builtin_amdgcn_readlane(first, ln);
        res = mask ? cand : res;
        found = found || mask != 0;
    }
    return (valid && found) ? res : minD;
}

// Hot-loop scalars, pinned in SGPRs (an empty asm makes each value opaque, so the
// compiler cannot rematerialise it from kernarg memory inside the serial loop).
// The six P1 / P2 values live in VGPRs (loop-invariant copies): a step's per-label selects
// (v_cndmask with a lane-mask SGPR pair) may read only one scalar operand, so scalar copies
// would be moved to VGPRs again at every step.
struct ScanConst {
    int L, Q, cd, minD, W, gstride, gpad;
    float p1[3], p2[3];
};
__device__ __forceinline__ ScanConst scan_const(const DevParams& P) {
    ScanConst c{P.L, P.Lp >> 2, P.color_diff, P.minD, P.W, P.gstride, P.gpad,
                {P.p1t[0], P.p1t[1], P.p1t[2]}, {P.p2t[0], P.p2t[1], P.p2t[2]}};
    asm volatile("" : "+s"(c.L), "+s"(c.Q), "+s"(c.cd), "+s"(c.minD), "+s"(c.W), "+s"(c.gstride), "+s"(c.gpad));
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        asm volatile("v_mov_b32 %0, %1" : "=v"(c.p1[k]) : "s"(P.p1t[k]));
        asm volatile("v_mov_b32 %0, %1" : "=v"(c.p2[k]) : "s"(P.p2t[k]));
    }
    return c;
}

// Prefetched, chain-independent inputs of one step.
template <int J>
struct StepIn {
    f32x4 p[J];      // this pixel's L-vector (lanes >= Q: a constant +inf vector)
    uint32_t g0[J];  // aligned 8-byte window of the other view's colour differences
    uint32_t g1[J];
    int d1;          // own-view colour difference to the predecessor
    uint32_t mk;     // mask mode: predecessor's packed colour (0 = black)
};

// Per-lane addressing, fixed for the whole walk: the vector element of lane q lives at
// vbase + pos * ves (lanes >= Q: ves = 0 on a +inf vector, so no per-step select), its
// d2 bytes at dbase + pos * dstep (8-byte aligned window, sentinel-padded map).
template <int J>
struct LaneAddr {
    const float* vb[J];
    size_t ves[J];
};

// Buffer resources of the byte maps / image; offsets are 32-bit (checked by the launcher).
constexpr int SC_GBIAS = 2048;  // >= 4 * (max label vectors = 512): no negative buffer offset

struct ScanRes {
    __amdgpu_buffer_rsrc_t own;   // own-view colour differences (d1)
    __amdgpu_buffer_rsrc_t oth;   // other view's colour differences (d2), based SC_GBIAS B low
    __amdgpu_buffer_rsrc_t im;    // own-view image (mask mode)
};
__device__ __forceinline__ __amdgpu_buffer_rsrc_t scan_rsrc(const void* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}

// Chain-independent loads of one step.  The pixel vector comes through the lane's running
// pointer; d1, the mask colour and the d2 window are buffer loads whose offsets are
// scalar (uniform) plus, for d2, a per-lane constant: no per-step address arithmetic.
//   d2 window of lane q: aligned byte (x0 + gb) & ~3 = S + V with S = (x0 [- 3]) & ~3
//   (scalar) and V = +4q (view 0) or -4q (view 1); the rsrc sits SC_GBIAS B low so
//   V + SC_GBIAS >= 0 for every label vector q < 512 (J = 8).
template <int J, bool HORIZ, bool MASK>
__device__ __forceinline__ void scan_issue(StepIn<J>& s, int pos, int dir, int line,
                                           const float* const (&pv)[J], const uint32_t (&gv)[J],
                                           const ScanRes& R, uint32_t orow, int sgn,
                                           const ScanConst& C) {
    const int pm = dir > 0 ? pos : pos + 1;  // max(pos, predecessor)
#pragma unroll
    for (int j = 0; j < J; ++j) s.p[j] = *reinterpret_cast<const f32x4*>(pv[j]);  // (nt loads: -2 %)
    const uint32_t i1 = (uint32_t)(HORIZ ? C.gpad + pm : pm * C.gstride + C.gpad + line);
    // d1 as the aligned dword holding its byte (a byte load's value is narrowed by the
    // compiler, which then re-widens every ring slot at the loop back-edge, waiting for it)
    s.d1 = (int)__builtin_amdgcn_raw_buffer_load_b32(R.own, 0u, (orow + i1) & ~3u, 0);
    s.mk = 1u;
    if (MASK) {
        const uint32_t ii = (uint32_t)(HORIZ ? line * C.W + (pos - dir) : (pos - dir) * C.W + line);
        s.mk = __builtin_amdgcn_raw_buffer_load_b32(R.im, 0u, ii * 4u, 0);
    }
    // x of lane 0's first disparity; HORIZ reads byte max(x1, x2) = x1 + (dir < 0)
    const int x0 = (HORIZ ? pos + (dir < 0 ? 1 : 0) : line) + C.gpad + sgn * C.minD;
    const uint32_t so = (HORIZ ? orow : orow + (uint32_t)pm * C.gstride) +
                        (uint32_t)((sgn > 0 ? x0 : x0 - 3) & ~3);
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const uint2 w = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(R.oth, gv[j], so, 0));
        s.g0[j] = w.x;
        s.g1[j] = w.y;
    }
}

// One partialOptimization step (ADCensus.cpp:869-913), branch-free.  Everything that
// is uniform over the step (d1's P1/P2 class, m + P2, the d2 byte selector) is scalar
// work; per lane: one v_perm for the four d2 bytes, then per disparity two selects,
// the neighbour adds (packed), an integer min3/min and the packed (C - m + min) / 2.
//   psel: v_perm selector picking this step's 4 d2 bytes (in label order) out of the
//   aligned 8-byte window
template <int J>
__device__ __forceinline__ void partial_opt(f32x4 (&p)[J], const f32x4 (&q)[J], uint32_t mq,
                                            int d1, const StepIn<J>& s, uint32_t psel,
                                            int lane, const ScanConst& C) {
    const float mqf = bitsf(mq);
    // P1/P2 pairs by d1 class (:954-979): d2 similar -> a, dissimilar -> b (scalar)
    const bool sim1 = d1 < C.cd;
    const float p1a = sim1 ? C.p1[2] : C.p1[1], p1b = sim1 ? C.p1[1] : C.p1[0];
    const float p2a = sim1 ? C.p2[2] : C.p2[1], p2b = sim1 ? C.p2[1] : C.p2[0];
    const float m2a = mqf + p2a, m2b = mqf + p2b;  // m + P2 for both classes
    const float inf = bitsf(kInfBits);
#pragma unroll
    for (int j = 0; j < J; ++j) {
        // d-1 of element 0 / d+1 of element 3 from the neighbouring lanes (+inf past the
        // ends of the label axis: lanes >= Q hold the +inf vector, DPP feeds +inf at 0/63)
        float lo = dpp_f<DPP_WAVE_SHR1>(q[j][3], inf);
        float hi = dpp_f<DPP_WAVE_SHL1>(q[j][0], inf);
        if (j > 0) {
            const float prev = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(q[j - 1][3]), 63));
            lo = lane == 0 ? prev : lo;
        }
        if (j + 1 < J) {
            const float nxt = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(q[j + 1][0]), 0));
            hi = lane == 63 ? nxt : hi;
        }
        const uint32_t g = __builtin_amdgcn_perm(s.g1[j], s.g0[j], psel);
        const float qe[6] = {lo, q[j][0], q[j][1], q[j][2], q[j][3], hi};
        f32x4 pe = p[j];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const bool sim2 = (int)((g >> (8 * k)) & 0xffu) < C.cd;
            const float p1 = sim2 ? p1a : p1b;
            const float m2 = sim2 ? m2a : m2b;
            const float cost = pe[k] - mqf;
            // min{ m + P2, C(q,d), C(q,d-1) + P1, C(q,d+1) + P1 }: rounding is monotonic,
            // so min(a,b) + P1 == min(a + P1, b + P1) exactly (all >= 0: integer mins)
            const float nb = bitsf(min(fbits(qe[k]), fbits(qe[k + 2])));
            const uint32_t mo = umin3(fbits(m2), fbits(qe[k + 1]), fbits(nb + p1));
            pe[k] = (cost + bitsf(mo)) * 0.5f;  // == / 2 exactly
        }
        p[j] = pe;
    }
}

// ---------------------------------------------------------------------------
// One wave walks one line of one view.  The leftward horizontal pass is the last one:
// it emits the WTA disparity of every pixel (WTA) and, for view 1 (only needed for the
// WTA), can skip storing the volume.  MASK: mask-mode predecessor test.  The racy
// omp schedule emulation costs two scalar compares per step (chunk starts are tracked
// incrementally).
// ---------------------------------------------------------------------------
// Prefetch depth K (steps), a template parameter.  Alone, a pass of the horizontal kernel
// (under one wave per SIMD) is faster with 16 steps in flight, so single-pair launches take
// 16; in groups of pairs (tens of thousands of waves a launch) 8 steps win (+1 % pairs/s,
// same-box A/B): 79 instead of 135 VGPRs, 6 instead of 3 waves per SIMD.  The vertical
// passes are HBM-bound at 8.  Wider label vectors (J >= 3) shorten the ring to keep the
// registers in bounds.
// first iteration of omp-static chunk t (libgomp / vcomp: first n%T threads take q+1)
__device__ __forceinline__ int omp_start(int t, int n, int T) {
    const int q = n / T, r = n % T;
    return t * q + (t < r ? t : r);
}

// HELP (leftward pass of one or two pairs, J = 1): the argmin leaves the serial chain.
// A workgroup holds SH_LINES lines, each a chain wave plus a helper wave: the chain wave
// writes every step's final vector into an LDS ring of two blocks of SC_K steps, and after
// each block's barrier the helper takes the argmins of the block just finished (under one
// wave per SIMD the WTA's ballots and readlanes otherwise sit on every step of the chain:
// 0.57 against 0.30 ms a pass).
constexpr int SH_LINES = 4;

template <int J, int SC_K, bool HORIZ, bool MASK, bool WTA, bool OMP, bool HELP = false>
__global__ __launch_bounds__(HELP ? 2 * SH_LINES * 64 : 256) void k_scan_line(float* __restrict__ vol,
                                                   const uint8_t* __restrict__ grad,
                                                   const uint32_t* __restrict__ img, int dir,
                                                   int32_t* __restrict__ wta, int store_view1,
                                                   const float* __restrict__ infvec,
                                                   DevParams Pk) {
    const DevParams P = Pk;
    const int H = P.H, W = P.W, Lp = P.Lp;
    const int lane = threadIdx.x & 63;
    static_assert(!HELP || (J == 1 && HORIZ && WTA), "the helper form is the single-vector WTA pass");
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // vertical passes: neighbouring column groups on one XCD (xcd_remap; the launcher pads
    // gridDim.x to a multiple of 8, blocks past the image exit)
    int line = HELP ? (int)blockIdx.x * SH_LINES + wv % SH_LINES
                    : (HORIZ ? (int)blockIdx.x : xcd_remap(blockIdx.x, gridDim.x)) * 4 + wv;
    pair_shift(blockIdx.z, P.pstride, vol, grad, img, wta);  // infvec: shared, not per pair
    const int v = blockIdx.y;
    // HELP: every wave of the workgroup takes the same barriers, so a line past the image
    // re-walks the last line with its stores off instead of leaving
    const bool dummy = HELP && line >= H;
    if (dummy) line = H - 1;
    if (line >= (HORIZ ? H : W)) return;
    const ScanConst C = scan_const(P);
    const int len = HORIZ ? W : H;
    const size_t es = HORIZ ? (size_t)Lp : (size_t)W * Lp;
    float* base = vol + (size_t)v * H * W * Lp + (HORIZ ? (size_t)line * W * Lp : (size_t)line * Lp);
    const int sgn = v == 0 ? 1 : -1;
    ScanRes R;
    R.own = scan_rsrc(grad + (size_t)v * H * C.gstride);
    R.oth = scan_rsrc(grad + (size_t)(1 - v) * H * C.gstride - SC_GBIAS);
    R.im = scan_rsrc(img + (size_t)v * H * W);
    const uint32_t orow = HORIZ ? (uint32_t)line * (uint32_t)C.gstride : 0u;  // row offset in both maps
    const bool rev = sgn < 0;
    const int n = len - 1;
    const int T = OMP ? P.omp_threads : 1;
    const bool store = !(WTA && v == 1 && !store_view1) && !dummy;
    int32_t* wrow = WTA ? wta + ((size_t)v * H + line) * W : nullptr;
    extern __shared__ __attribute__((aligned(16))) f32x4 sh_ring[];
    // per line: the vectors of 2 * SC_K steps (1 KB each), then their minima (one dword a lane)
    char* const hline = reinterpret_cast<char*>(sh_ring) + (size_t)(wv % SH_LINES) * (2 * SC_K * 1280);
    char* const hring = hline + lane * 16;
    char* const mring = hline + 2 * SC_K * 1024 + lane * 4;
    auto barrier = [&]() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
    if constexpr (HELP) if (wv >= SH_LINES) {
        // helper: after the barrier closing block i, the argmins of block i's steps
        const int nfull = n / SC_K;
        const int posbase = dir > 0 ? 1 : len - 2;
        int dacc = 0;
        // the block's vectors first (one LDS latency a block), then its argmins: a full
        // block is branch-free straight-line code, so the 16 steps' chains interleave
        // the first d holding the step's minimum m (the chain's own): four ballots, the rest
        // scalar.  m not below FLT_MAX: the reference leaves the disparity unset (minD).
        // minD > 0 restricts the minimum to [minD, L): the general form.
        const bool fast = P.minD == 0;
        auto argmin_of = [&](const f32x4& xk, uint32_t mv) {
            const f32x4 (&xv)[1] = *reinterpret_cast<const f32x4(*)[1]>(&xk);
            if (!fast) return vec_argmin_nb<J>(xv, lane, P.L, P.minD, vec_min_bits<J, true>(xv));
            const uint32_t m = __builtin_amdgcn_readfirstlane(mv);
            int d = 1 << 20;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint64_t b = __ballot(fbits(xk[e]) == m);
                d = b ? min(d, 4 * (int)__builtin_ctzll(b) + e) : d;
            }
            return (bitsf(m) < 3.402823466e+38f && d < (1 << 20)) ? d : 0;
        };
        auto flush = [&](int it) {  // the group of 64 steps holding step it, up to it
            const int g0 = it & ~63;
            if (!dummy && lane <= it - g0) wrow[posbase + dir * (g0 + lane)] = dacc;
        };
        for (int i = 0; i <= nfull; ++i) {
            barrier();
            f32x4 x[SC_K];
            uint32_t mk[SC_K];
            const char* hb = hring + (i & 1) * (SC_K * 1024);
            const char* mb = mring + (i & 1) * (SC_K * 256);
#pragma unroll
            for (int k = 0; k < SC_K; ++k) {
                x[k] = *reinterpret_cast<const f32x4*>(hb + k * 1024);
                mk[k] = *reinterpret_cast<const uint32_t*>(mb + k * 256);
            }
            const int i0 = i * SC_K;
            if (i < nfull) {
#pragma unroll
                for (int k = 0; k < SC_K; ++k) {
                    const int d = argmin_of(x[k], mk[k]);
                    dacc = lane == ((i0 + k) & 63) ? d : dacc;
                }
                if (((i0 + SC_K) & 63) == 0) flush(i0 + SC_K - 1);
            } else {
#pragma unroll
                for (int k = 0; k < SC_K; ++k) {
                    if (i0 + k < n) {
                        const int d = argmin_of(x[k], mk[k]);
                        dacc = lane == ((i0 + k) & 63) ? d : dacc;
                    }
                }
                if ((n & 63) != 0) flush(n - 1);
            }
        }
        return;
    }
    // byte misalignment of every lane's d2 window (uniform: lanes differ by multiples of 4)
    const int x0a = (HORIZ ? (dir < 0 ? 1 : 0) : line) + C.gpad + sgn * C.minD - (sgn > 0 ? 0 : 3);
    const int posbase = dir > 0 ? 1 : len - 2;  // pos(it) = posbase + dir*it (HORIZ shifts x0)
    // v_perm selector of the 4 d2 bytes at byte offset 0 of the (lo, hi) window: view 0
    // reads x ascending, view 1 descending (byte-reversed); + sh * 0x01010101 per step
    const uint32_t psel0 = rev ? 0x00010203u : 0x03020100u;
    LaneAddr<J> la;
    uint32_t gv[J];  // d2 lane offsets (+SC_GBIAS: the rsrc sits that low)
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int q = lane + 64 * j;
        const bool in = q < C.Q;
        la.vb[j] = in ? base + 4 * q : infvec;
        la.ves[j] = in ? es : 0;
        gv[j] = (uint32_t)(SC_GBIAS + (in ? (sgn > 0 ? 4 * q : -4 * q) : 0));
    }

    f32x4 q[J];
    const int p0 = dir > 0 ? 0 : len - 1;
#pragma unroll
    for (int j = 0; j < J; ++j) q[j] = *reinterpret_cast<const f32x4*>(la.vb[j] + (size_t)p0 * la.ves[j]);
    uint32_t mq = vec_min_bits<J>(q);
    if (WTA) {
        const int d = vec_argmin<J>(q, lane, C.L, C.minD, mq);
        if (lane == 0 && !dummy) wrow[p0] = d;
    }
    f32x4 qorig[J];
    uint32_t mqorig = mq;
    if (OMP) {
#pragma unroll
        for (int j = 0; j < J; ++j) qorig[j] = q[j];
    }
    // omp emulation: next chunk start (INT_MAX when off)
    int ct = 1;
    int cs = (OMP && T > 1 && n > 0) ? omp_start(1, n, T) : 0x7fffffff;

    // running per-lane pointers: the prefetch position and the step being written
    // (lanes past the label axis stay on the +inf vector: step 0; storing +inf there is a no-op)
    const float* pf[J];
    float* cur[J];
    ptrdiff_t dstep[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        dstep[j] = (ptrdiff_t)dir * (ptrdiff_t)la.ves[j];
        cur[j] = const_cast<float*>(la.vb[j]) + (ptrdiff_t)posbase * (ptrdiff_t)la.ves[j];
        pf[j] = cur[j];
    }
    StepIn<J> ring[SC_K];
#pragma unroll
    for (int k = 0; k < SC_K; ++k) {
        const int kk = k < n ? k : n - 1;  // past the end: re-read the last pixel (unused)
        scan_issue<J, HORIZ, MASK>(ring[k], posbase + dir * kk, dir, line, pf, gv, R, orow, sgn, C);
        if (k + 1 < n) {
#pragma unroll
            for (int j = 0; j < J; ++j) pf[j] += dstep[j];
        }
        // slots issued in order (the loop's waits assume slot k is the k-th oldest load set)
        __builtin_amdgcn_sched_barrier(0);
    }
    int pfi = SC_K < n ? SC_K : n - 1;  // step index pf points at (clamped to the last)

    static_assert(64 % SC_K == 0, "WTA groups of 64 steps hold whole unrolled blocks");
    int dacc = 0;  // WTA: indices of the current group of 64 steps, one per lane
    // one step: ring slot k (compile-time), step index it
    auto step = [&](auto Kc, int it) {
        constexpr int k = decltype(Kc)::value;
        const StepIn<J>& s = ring[k];
        const int pos = posbase + dir * it;
        const uint32_t sh = (uint32_t)((HORIZ ? x0a + pos : x0a) & 3);
        if (OMP) {
            if (it == cs) {  // chunk start of the racy schedule: stale predecessor
#pragma unroll
                for (int j = 0; j < J; ++j) q[j] = qorig[j];
                mq = mqorig;
                ++ct;
                cs = ct < T ? omp_start(ct, n, T) : 0x7fffffff;
            }
            if (it + 1 == cs) {  // the next chunk's first pixel sees this pre-pass vector
#pragma unroll
                for (int j = 0; j < J; ++j) qorig[j] = s.p[j];
                mqorig = vec_min_bits<J>(s.p);
            }
        }
        const bool masked = MASK && __builtin_amdgcn_readfirstlane(s.mk) == 0;  // :824, :862
        // :880-881: m == 0 leaves p untouched (branch-free: compute, then select)
        f32x4 np[J];
#pragma unroll
        for (int j = 0; j < J; ++j) np[j] = s.p[j];
        const uint32_t i1 = (uint32_t)(HORIZ ? C.gpad + (dir > 0 ? pos : pos + 1)
                                             : (dir > 0 ? pos : pos + 1) * C.gstride + C.gpad + line);
        const int d1 = ((uint32_t)__builtin_amdgcn_readfirstlane(s.d1) >> (8 * ((orow + i1) & 3u))) & 0xff;
        partial_opt<J>(np, q, mq, d1, s, psel0 + sh * 0x01010101u, lane, C);
        const bool upd = !(masked || mq == 0u);
        // q gets registers of its own (early-clobber copy): coalesced with the ring slot, it
        // would keep the slot's registers live past the refill, and the compiler would then
        // rotate the whole ring by copies at the loop back-edge (each copy waiting for its
        // in-flight load: the prefetch gone)
        // the select itself writes q's registers (early clobber): no separate copy
        const uint64_t umask = __builtin_amdgcn_ballot_w64(upd);
#pragma unroll
        for (int j = 0; j < J; ++j) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float o;
                asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=&v"(o) : "v"(s.p[j][e]), "v"(np[j][e]), "s"(umask));
                q[j][e] = o;
            }
        }
        if (store && upd) {  // untouched vectors are not rewritten
#pragma unroll
            for (int j = 0; j < J; ++j) st_stream(cur[j], q[j]);
        }
#pragma unroll
        for (int j = 0; j < J; ++j) cur[j] += dstep[j];
        mq = vec_min_bits<J, true>(q);
        if constexpr (HELP) {  // the final vector to the helper's ring (slot it mod 2K)
            *reinterpret_cast<f32x4*>(hring + (size_t)((it % (2 * SC_K)) * 1024)) = q[0];
            *reinterpret_cast<uint32_t*>(mring + (size_t)((it % (2 * SC_K)) * 256)) = mq;
        } else if (WTA) {  // step it's index lands in lane it & 63, stored 64 steps at a time
            const int d = vec_argmin_nb<J>(q, lane, C.L, C.minD, mq);  // whole wave
            dacc = lane == (it & 63) ? d : dacc;
        }
        // refill this slot only now that its data is consumed (a load into a live slot would
        // make the compiler stage it in temporaries and copy it back, waiting for the load
        // right away); past the line end the last pixel is re-read (a select, no branch)
        scan_issue<J, HORIZ, MASK>(ring[k], posbase + dir * pfi, dir, line, pf, gv, R, orow, sgn, C);
        const bool adv = pfi + 1 < n;
        pfi = adv ? pfi + 1 : pfi;
#pragma unroll
        for (int j = 0; j < J; ++j) pf[j] += adv ? dstep[j] : 0;
        // keep the refill in its step: the scheduler otherwise sinks early slots' loads to the
        // block end, and the next block's first steps wait for them almost at once (ALU work
        // may still cross: mask 0x7 = ALU / VALU / SALU)
        __builtin_amdgcn_sched_barrier(0x7);
    };
    auto flush_wta = [&](int b) {  // the group of 64 steps holding step b
        const int g0 = b & ~63;
        if (lane < min(n, g0 + 64) - g0) wrow[posbase + dir * (g0 + lane)] = dacc;
    };
    // Whole blocks of SC_K steps as straight-line code (no per-step range branches): the
    // waitcnt pass then counts each slot's loads across the loop back-edge, so a step waits
    // only for its own prefetched data (with range branches it drained vmcnt(0) at every
    // block, one full memory latency per SC_K steps).
    int b = 0;
    for (; b + SC_K <= n; b += SC_K) {
        [&]<int... Ks>(std::integer_sequence<int, Ks...>) {
            (step(IC<Ks>{}, b + Ks), ...);
        }(std::make_integer_sequence<int, SC_K>{});
        if constexpr (HELP) barrier();
        else if (WTA && ((b + SC_K) & 63) == 0) flush_wta(b);
    }
    [&]<int... Ks>(std::integer_sequence<int, Ks...>) {
        ((b + Ks < n ? step(IC<Ks>{}, b + Ks) : (void)0), ...);
    }(std::make_integer_sequence<int, SC_K>{});
    if constexpr (HELP) barrier();
    else if (WTA && (n & 63) != 0) flush_wta(n - 1);
}

// the helper form of the leftward WTA pass (single-vector label axis, K = 16)
template <bool MASK, bool OMP>
static void launch_scan_help_t(float* vol, const uint8_t* grad, const uint32_t* img, int dir, int32_t* wta,
                               int store_view1, const float* infvec, const DevParams& P, hipStream_t st) {
    constexpr int K = 16;
    const size_t lds = (size_t)SH_LINES * 2 * K * 1280;
    ensure_lds_limit((const void*)k_scan_line<1, K, true, MASK, true, OMP, true>, lds);
    const dim3 g((P.H + SH_LINES - 1) / SH_LINES, 2, P.npairs);
    hipLaunchKernelGGL((k_scan_line<1, K, true, MASK, true, OMP, true>), g, dim3(2 * SH_LINES * 64), lds, st, vol,
                       grad, img, dir, wta, store_view1, infvec, P);
}

static void launch_scan_help(float* vol, const uint8_t* grad, const uint32_t* img, int dir, int32_t* wta,
                             int store_view1, const float* infvec, const DevParams& P, hipStream_t st) {
    const bool omp = P.omp_threads > 1;
    if (P.mask) {
        if (omp) launch_scan_help_t<true, true>(vol, grad, img, dir, wta, store_view1, infvec, P, st);
        else launch_scan_help_t<true, false>(vol, grad, img, dir, wta, store_view1, infvec, P, st);
    } else {
        if (omp) launch_scan_help_t<false, true>(vol, grad, img, dir, wta, store_view1, infvec, P, st);
        else launch_scan_help_t<false, false>(vol, grad, img, dir, wta, store_view1, infvec, P, st);
    }
}

template <int J, int K, bool HORIZ, bool MASK, bool WTA>
static void launch_scan_t(float* vol, const uint8_t* grad, const uint32_t* img, int dir, int32_t* wta,
                          int store_view1, const float* infvec, const DevParams& P, hipStream_t st) {
    dim3 g(HORIZ ? (P.H + 3) / 4 : ((P.W + 3) / 4 + 7) / 8 * 8, 2, P.npairs);
    if (P.omp_threads > 1)
        hipLaunchKernelGGL((k_scan_line<J, K, HORIZ, MASK, WTA, true>), g, dim3(256), 0, st, vol, grad, img, dir,
                           wta, store_view1, infvec, P);
    else
        hipLaunchKernelGGL((k_scan_line<J, K, HORIZ, MASK, WTA, false>), g, dim3(256), 0, st, vol, grad, img, dir,
                           wta, store_view1, infvec, P);
}

template <int J, int K, bool HORIZ, bool WTA>
static void launch_scan_m(float* vol, const uint8_t* grad, const uint32_t* img, int dir, int32_t* wta,
                          int store_view1, const float* infvec, const DevParams& P, hipStream_t st) {
    if (P.mask) launch_scan_t<J, K, HORIZ, true, WTA>(vol, grad, img, dir, wta, store_view1, infvec, P, st);
    else launch_scan_t<J, K, HORIZ, false, WTA>(vol, grad, img, dir, wta, store_view1, infvec, P, st);
}

// label vectors per lane J = ceil(Lp / 256) (J = 5..8 run as 8, lanes past the axis on +inf)
int scan_max_lp() { return 8 * 256; }

template <bool HORIZ, bool WTA>
static int launch_scan(float* vol, const uint8_t* grad, const uint32_t* img, int dir, int32_t* wta,
                       int store_view1, const float* infvec, const DevParams& P, hipStream_t st) {
    const int J = (P.Lp / 4 + 63) / 64;
    // a horizontal pass of one or two pairs runs under one wave per SIMD: the deeper ring
    const bool deep = HORIZ && P.npairs <= 2;
    if (J == 1) {
        if constexpr (HORIZ) {
            if (deep && WTA) launch_scan_help(vol, grad, img, dir, wta, store_view1, infvec, P, st);
            else if (deep) launch_scan_m<1, 16, HORIZ, WTA>(vol, grad, img, dir, wta, store_view1, infvec, P, st);
            else launch_scan_m<1, 8, HORIZ, WTA>(vol, grad, img, dir, wta, store_view1, infvec, P, st);
        } else {
            (void)deep;
            launch_scan_m<1, 8, HORIZ, WTA>(vol, grad, img, dir, wta, store_view1, infvec, P, st);
        }
    } else if (J == 2) {
        launch_scan_m<2, 8, HORIZ, WTA>(vol, grad, img, dir, wta, store_view1, infvec, P, st);
    } else if (J == 3) {
        launch_scan_m<3, 4, HORIZ, WTA>(vol, grad, img, dir, wta, store_view1, infvec, P, st);
    } else if (J == 4) {
        launch_scan_m<4, 4, HORIZ, WTA>(vol, grad, img, dir, wta, store_view1, infvec, P, st);
    } else if (J <= 8) {
        launch_scan_m<8, 2, HORIZ, WTA>(vol, grad, img, dir, wta, store_view1, infvec, P, st);
    } else {
        return -1;
    }
    trace_point(HORIZ ? "k_scan_line<H>" : "k_scan_line<V>", st);
    return 0;
}

int launch_scan_vertical(float* vol, const uint8_t* gv, const uint32_t* img, int dir,
                         const float* infvec, const DevParams& P, hipStream_t st) {
    return launch_scan<false, false>(vol, gv, img, dir, nullptr, 1, infvec, P, st);
}

int launch_scan_horizontal(float* vol, const uint8_t* gh, const uint32_t* img, int dir,
                           int32_t* wta, int store_view1, const float* infvec, const DevParams& P,
                           hipStream_t st) {
    if (wta) return launch_scan<true, true>(vol, gh, img, dir, wta, store_view1, infvec, P, st);
    return launch_scan<true, false>(vol, gh, img, dir, nullptr, store_view1, infvec, P, st);
}

}  // namespace tsm
