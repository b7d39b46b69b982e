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
// ends at the image border, :650-658).  p: the pixel; fetch(k): the pixel k steps along the
// arm's direction; avail: how many such steps stay inside the image.
template <class F>
__device__ __forceinline__ int compute_limit(const DevParams& P, uint32_t p, int avail, F fetch) {
    int d = 1;
    uint32_t p2 = p;
    bool inside = 1 <= avail;
    if (inside) {
        bool colorCond = true, wLimitCond = true, fColorCond = true;
        while (colorCond && wLimitCond && fColorCond && inside) {
            const uint32_t p1 = fetch(d);
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
            inside = d + 1 <= avail;
            d++;
        }
        d--;
    }
    return d - 1;
}

// arms[v][y][x] = up | down<<8 | left<<16 | right<<24  (computeLimits, :661-683): the
// four walks of a pixel on four lanes, reading the image through L1/L2.  Arms are short on real
// scenes (mean 2.1 px), so the walks are a few dependent cached loads; staging row and
// column tiles with a maxLength1 halo in LDS measured slower (round 3: 0.089 -> 0.161 ms a
// pair for the stage, the column tile serialising 16 pixels a thread).
__global__ void k_arms(const uint32_t* __restrict__ img, uint32_t* __restrict__ arms, DevParams Pk) {
    const DevParams P = Pk;  // kernel args -> registers once (no per-use kernarg reloads)
    // four lanes a pixel, one direction each (0 up, 1 down, 2 left, 3 right): the four
    // dependent load chains run side by side; the pixel's lane 0 packs and stores
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int x = t >> 2, dir = t & 3;
    const int y = blockIdx.y;
    const int v = blockIdx.z & 1;
    pair_shift(blockIdx.z >> 1, P.pstride, img, arms);
    const int W = P.W;
    const bool inside = x < W;
    const int xc = inside ? x : W - 1;
    const uint32_t* row = img + ((size_t)v * P.H + y) * W;
    const uint32_t p = row[xc];
    const ptrdiff_t step = dir == 0 ? -(ptrdiff_t)W : dir == 1 ? (ptrdiff_t)W : dir == 2 ? -1 : 1;
    const int avail = dir == 0 ? y : dir == 1 ? P.H - 1 - y : dir == 2 ? xc : W - 1 - xc;
    uint32_t arm = 0;
    if (!(P.mask && p == 0)) arm = compute_limit(P, p, avail, [&](int k) { return row[xc + (ptrdiff_t)k * step]; });
    // gather the quad's four arms into lane dir == 0 (up | down << 8 | left << 16 | right << 24)
    uint32_t packed = arm << (8 * dir);
    packed |= (uint32_t)__shfl_xor((int)packed, 1);
    packed |= (uint32_t)__shfl_xor((int)packed, 2);
    if (inside && dir == 0) arms[((size_t)v * P.H + y) * W + x] = packed;
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
// every integer b in [1, 6561] (arms up to 40) and every a in [2^-40, 2^16) (exhaustively checked,
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

// Cache policy of the single-pass streamer's volume loads (the first and the last pass):
// streaming (slc).  Each vector is read once; the following scanline pass then ran 4 %
// faster for a single pair (1.106 against 1.152 ms, same box, round 3) with the
// aggregation unchanged.  The fused streamer keeps default loads (slc there: 1.55 against
// 1.47 ms).
constexpr int kNtLoad = 2;
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
    int qn0;               // split streamer: label vectors per slice (blockIdx.y; the last may be narrower)
    int horizontal;
    int n;                 // pixels per line
    int cpl;               // chunks per line
    int nlv;               // lines per view
    int nl;                // lines of both views
};


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
    const int g = xcd_remap(blockIdx.x, gridDim.x), G = gridDim.x;
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
                    b[h * AS_SEG + i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs_vol, voff, lr[h].vol + pos * es4, kNtLoad));
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
                land(k);
                advance();
                issue();
            }
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no load outlives the workgroup
        return;
    }

    // ---- summing waves -------------------------------------------------------------
    // Sequential window sum of `len` ring pixels from LDS byte offset `off` in the ring
    // [rb, re): whole blocks of 4 at immediate offsets (AX_MIR mirror slots past each ring
    // make every block contiguous), then the 1-3 remaining pixels under uniform branches.
    auto window = [&](uint32_t off, int len, uint32_t rb, uint32_t re) -> f32x4 {
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        const char* lp = lds + lane16;
        const uint32_t span = re - rb;
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
        const uint32_t r1_end = r1_off + (uint32_t)AS_RP1 * Qs, r2_end = r2_off + (uint32_t)AS_RP2 * Qs;
        // pass B first: it reads ring2 slots pass A does not write this step, so pass A's
        // ring1 reads can overlap it
        if (FUSED && s >= AS_LAG) {  // pass B on chunk s - LAG
            if (ob.cc * AS_SEG + wave < S.n) {
                const f32x4 acc = window(b_off, b_len, r2_off, r2_end);
                if (vl) st_stream(S.vol + ob.off + 4 * lane, acc);
            }
            out_step(ob);
        }
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
                } else if (vl) {
                    st_stream(S.vol + oa.off + 4 * lane, acc);
                }
            }
            out_step(oa);
            r2w += AS_SEG * Qs;
            r2w = r2w >= r2_end ? r2w - (uint32_t)AS_RP2 * Qs : r2w;
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
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
constexpr int AX_THREADS = 16 * 64;
constexpr int AX_MW = 2;  // meta words per pixel: packed descriptor (lo, hi, size), RN(1/size)
constexpr int AX_D = 12;  // A-wave staging ring: steps in flight (AX_D * 8 px * Q * 16 B per CU)
constexpr int AX_MC = 12;  // meta ring chunks (B reads chunk s - LAG + 1 before A overwrites its slot)
static_assert(AX_D == AS_RC1 && AX_D == AS_RC2 && AX_D == AX_MC, "ring slots are compile-time per unrolled step");
static_assert(AS_AHEAD + AS_LAG <= AX_MC, "meta ring too short for the B lag");

// BIG: volumes of 2 GiB and more (configs C, E): vector loads through 64-bit addresses
// instead of 32-bit buffer offsets.  Label slices: when a pixel vector's rings would not fit
// the CU's LDS, blockIdx.y picks one slice of the label axis (the sums of different labels
// are independent), each a narrower ring.
template <bool FUSED, int QT, bool BIG>
__global__ __launch_bounds__(AX_THREADS) void k_agg_split(AggStream S, DevParams Pk) {
    const DevParams P = Pk;
    pair_shift(blockIdx.z, P.pstride, S.vol, S.arms, S.ws, S.pk, S.rcp);
    extern __shared__ __attribute__((aligned(16))) f32x4 smem_f4[];
    const int H = P.H, W = P.W, Lp = P.Lp;
    const int slice = blockIdx.y;
    const int Q = QT > 0 ? QT : min(S.qn0, S.qtot - slice * S.qn0);
    float* const volq = S.vol + 4 * slice * S.qn0;  // this slice's first label
    const uint32_t Qs = (uint32_t)Q * 16;                                // bytes per ring pixel
    const size_t vstride = (size_t)H * W * Lp;
    const size_t es = S.horizontal ? (size_t)Lp : (size_t)W * Lp;         // floats per pixel step
    const size_t ls = S.horizontal ? (size_t)W * Lp : (size_t)Lp;          // floats per line step
    const size_t aes = S.horizontal ? 1 : (size_t)W;
    const size_t als = S.horizontal ? (size_t)W : 1;
    const int g = xcd_remap(blockIdx.x, gridDim.x), G = gridDim.x;
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
    auto barrier = [&]() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
    // sequential window sum of `len` ring pixels from LDS byte offset `off` (a slot of the
    // ring [rb, re)): whole blocks of 4 at immediate offsets (the mirror slots make every
    // block contiguous), then the 1-3 remaining pixels under uniform branches -- the
    // reference's order, no padding reads, little scalar bookkeeping
    auto window = [&](uint32_t off, int len, uint32_t rb, uint32_t re) -> f32x4 {
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        const char* lp = lds + lane16;
        const uint32_t span = re - rb;
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
            if (BIG)
                rv[k] = *reinterpret_cast<const f32x4*>(ivp + (size_t)pos * es + 4 * lanec);
            else
                rv[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs_vol, voff, iv + pos * es4, 0));
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
                land(rv[u], rma[u], rmy[u], s + AS_AHEAD);
                issue(u);
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
                barrier();
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no load outlives the workgroup
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
            if (sb >= 0 && sb < nch) {
                if (ob.cc * AS_SEG + w < S.n) {
                    const f32x4 acc = FUSED ? window(b_off, b_len, r2_off, r2_end)
                                            : *reinterpret_cast<const f32x4*>(lds + r2r + lane16);
                    if (vl) st_stream(volq + ob.off + 4 * lane, acc);
                }
                out_step(ob);
            }
            barrier();
        }
    }
}

// ---------------------------------------------------------------------------
// 1-D aggregation for long arms (maxLength1 > AS_MAX_ARM + 1): one workgroup per (line,
// label slice) holds the whole line's slice of the volume in LDS, so every window sum
// reads LDS and the pass can overwrite the line in place.  Plain IEEE division (the
// library builds with correctly rounded fp32 division).  Not a throughput path: it serves
// the arm lengths the streamers' rings cannot reach.
// ---------------------------------------------------------------------------
constexpr int AL_THREADS = 512;

__global__ __launch_bounds__(AL_THREADS) void k_agg_wholeline(float* __restrict__ vol, const uint32_t* __restrict__ arms,
                                                              const int32_t* __restrict__ ws, int horizontal, int qs,
                                                              DevParams Pk) {
    const DevParams P = Pk;
    pair_shift(blockIdx.z, P.pstride, vol, arms, ws);
    extern __shared__ __attribute__((aligned(16))) f32x4 smem_f4[];
    const int H = P.H, W = P.W, Lp = P.Lp, Q = Lp >> 2;
    const int nlv = horizontal ? H : W;
    const int v = blockIdx.x / nlv, line = blockIdx.x - v * nlv;
    const int q0 = blockIdx.y * qs, nq = min(qs, Q - q0);
    const int n = horizontal ? W : H;
    const size_t es = horizontal ? (size_t)Lp : (size_t)W * Lp;  // floats per pixel step
    float* base = vol + (size_t)v * H * W * Lp + (horizontal ? (size_t)line * W * Lp : (size_t)line * Lp) + 4 * q0;
    const size_t aes = horizontal ? 1 : (size_t)W;
    const uint32_t* A = arms + (size_t)v * H * W + (horizontal ? (size_t)line * W : (size_t)line);
    const int32_t* WS = ws ? ws + (size_t)v * 2 * H * W + (horizontal ? (size_t)line * W : (size_t)line) : nullptr;
    const int shA = horizontal ? 16 : 0, shB = horizontal ? 24 : 8;  // left/right or up/down arm
    for (int t = threadIdx.x; t < n * nq; t += AL_THREADS) {
        const int px = t / nq, q = t - px * nq;
        smem_f4[t] = *reinterpret_cast<const f32x4*>(base + (size_t)px * es + 4 * q);
    }
    __syncthreads();
    for (int t = threadIdx.x; t < n * nq; t += AL_THREADS) {
        const int px = t / nq, q = t - px * nq;
        const uint32_t a = A[(size_t)px * aes];
        const int lo = (a >> shA) & 0xff, hi = (a >> shB) & 0xff;
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};  // the reference's sequential order (:725-751)
        for (int k = px - lo; k <= px + hi; ++k) acc += smem_f4[k * nq + q];
        if (WS) {
            const float b = (float)WS[(size_t)px * aes];
            acc.x = acc.x / b; acc.y = acc.y / b; acc.z = acc.z / b; acc.w = acc.w / b;
        }
        *reinterpret_cast<f32x4*>(base + (size_t)px * es + 4 * q) = acc;
    }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
static size_t agg_stream_lds(const DevParams& P, bool fused) {
    const int Q = P.Lp / 4;
    return ((size_t)AS_RP1 + AX_MIR + (fused ? AS_RP2 + AX_MIR : 0)) * Q * 16 + (size_t)AS_MC * AS_SEG * AS_MW * 4;
}
// LDS of the split streamer for a slice of qs label vectors
static size_t agg_split_lds(int qs) {
    return ((size_t)AS_RP1 + AS_RP2 + 2 * AX_MIR) * qs * 16 + (size_t)AX_MC * AS_SEG * AX_MW * 4;
}
constexpr size_t kLdsBytes = 160 * 1024;

template <bool FUSED, int QT, bool BIG>
static void launch_split_t(const AggStream& S, const DevParams& P, dim3 grid, size_t lds, hipStream_t st) {
    ensure_lds_limit((const void*)k_agg_split<FUSED, QT, BIG>, kLdsBytes);
    hipLaunchKernelGGL((k_agg_split<FUSED, QT, BIG>), grid, dim3(AX_THREADS), lds, st, S, P);
}

static int launch_wholeline(float* vol, const uint32_t* arms, const int32_t* ws, int horizontal, const DevParams& P,
                            hipStream_t st) {
    const int n = horizontal ? P.W : P.H;
    const int Q = P.Lp / 4;
    int qs = (int)(kLdsBytes / ((size_t)n * 16));
    if (qs < 1) return -1;  // one label vector of the line does not fit the CU's LDS
    qs = qs > Q ? Q : qs;
    const int nsl = (Q + qs - 1) / qs;
    qs = (Q + nsl - 1) / nsl;  // balanced slices
    ensure_lds_limit((const void*)k_agg_wholeline, kLdsBytes);
    const dim3 g(2 * (horizontal ? P.H : P.W), nsl, P.npairs);
    hipLaunchKernelGGL(k_agg_wholeline, g, dim3(AL_THREADS), (size_t)n * qs * 16, st, vol, arms, ws, horizontal, qs, P);
    trace_point("k_agg_wholeline", st);
    return 0;
}

int agg_max_streamer_arm() { return AS_MAX_ARM; }

int launch_aggregation_pass(float* vol, const uint32_t* arms, const int32_t* ws, const int32_t* ws_base,
                            int horizontal, bool fused, const DevParams& P, hipStream_t st) {
    const int Q = P.Lp / 4;
    if (P.max_length1 - 1 > AS_MAX_ARM) {  // arms past the streamers' rings: one pass at a time
        if (fused) return -1;
        return launch_wholeline(vol, arms, ws, horizontal, P, st);
    }
    const bool big = (size_t)2 * P.H * P.W * P.Lp * 4 >= ((size_t)1 << 31);  // past 32-bit offsets
    AggStream S;
    S.vol = vol;
    S.arms = arms;
    S.ws = ws;
    S.rcp = reinterpret_cast<const float*>(ws_base + (size_t)(4 + horizontal) * P.H * P.W);
    S.pk = reinterpret_cast<const uint32_t*>(ws_base + (size_t)(8 + horizontal) * P.H * P.W);
    S.qtot = Q;
    // label slices: as few as keep each slice's two rings inside the CU's LDS (balanced)
    int nslice = 1;
    while (agg_split_lds((Q + nslice - 1) / nslice) > kLdsBytes || (Q + nslice - 1) / nslice > 64) ++nslice;
    S.qn0 = (Q + nslice - 1) / nslice;
    S.horizontal = horizontal;
    S.n = horizontal ? P.W : P.H;
    S.cpl = (S.n + AS_SEG - 1) / AS_SEG;
    S.nlv = horizontal ? P.H : P.W;
    S.nl = 2 * S.nlv;
    const int ncu = P.ncu;
    const int G = S.nl < ncu ? S.nl : ncu;
    // fused pass pairs: the role-split streamer (v6); single passes: v5 where its rings fit
    // (v6 for single passes too measured 1 % fewer pairs/s: round 3, same box)
    const bool v5_fits = !fused && Q <= 64 && !big && agg_stream_lds(P, false) <= kLdsBytes;
    if (!v5_fits) {
        const size_t slds = agg_split_lds(S.qn0);
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
    const size_t lds = agg_stream_lds(P, false);
    const dim3 grid(G, 1, P.npairs), block(AS_THREADS);
    if (Q == 49) {
        ensure_lds_limit((const void*)k_agg_stream<false, 49>, kLdsBytes);
        hipLaunchKernelGGL((k_agg_stream<false, 49>), grid, block, lds, st, S, P);
    } else {
        ensure_lds_limit((const void*)k_agg_stream<false, 0>, kLdsBytes);
        hipLaunchKernelGGL((k_agg_stream<false, 0>), grid, block, lds, st, S, P);
    }
    trace_point("k_agg_stream", st);
    return 0;
}

void launch_arms(const uint32_t* img, uint32_t* arms, const DevParams& P, hipStream_t st) {
    dim3 g((4 * P.W + 255) / 256, P.H, 2 * P.npairs);
    hipLaunchKernelGGL(k_arms, g, dim3(256), 0, st, img, arms, P); trace_point("k_arms", st);
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

}  // namespace tsm
