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
// arm's direction; avail: how many such steps stay inside the image.  The walk loads
// ARM_B pixels a round trip (those inside the image), then takes its steps over them in
// order with the reference's conditions; the loads past where the walk stops go unused.
constexpr int ARM_B = 4;
template <class F>
__device__ __forceinline__ int compute_limit(const DevParams& P, uint32_t p, int avail, F fetch) {
    int d = 1;
    uint32_t p2 = p;
    bool go = 1 <= avail;
    const bool any = go;
    while (go) {
        uint32_t q[ARM_B];
#pragma unroll
        for (int k = 0; k < ARM_B; ++k) q[k] = d + k <= avail ? fetch(d + k) : 0u;
#pragma unroll
        for (int k = 0; k < ARM_B; ++k) {
            if (!go) break;
            const uint32_t p1 = q[k];
            if (P.mask && p1 == 0) {  // :625-629
                d++;
                go = false;
                break;
            }
            bool colorCond, fColorCond;
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
            const bool wLimitCond = d < P.max_length1;
            p2 = p1;
            const bool inside = d + 1 <= avail;
            d++;
            go = colorCond && wLimitCond && fColorCond && inside;
        }
    }
    if (any) d--;
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
    // integer sums (any order): ARM_B arms loaded a round trip
    int hf = 0, vf = 0;
    for (int k0 = -arm_up(a); k0 <= arm_down(a); k0 += ARM_B) {
        uint32_t b[ARM_B];
#pragma unroll
        for (int j = 0; j < ARM_B; ++j) b[j] = k0 + j <= arm_down(a) ? A[(size_t)(y + k0 + j) * W + x] : 0xffffffffu;
#pragma unroll
        for (int j = 0; j < ARM_B; ++j)
            if (k0 + j <= arm_down(a)) hf += arm_left(b[j]) + arm_right(b[j]) + 1;
    }
    for (int k0 = -arm_left(a); k0 <= arm_right(a); k0 += ARM_B) {
        uint32_t b[ARM_B];
#pragma unroll
        for (int j = 0; j < ARM_B; ++j) b[j] = k0 + j <= arm_right(a) ? A[(size_t)y * W + (x + k0 + j)] : 0xffffffffu;
#pragma unroll
        for (int j = 0; j < ARM_B; ++j)
            if (k0 + j <= arm_right(a)) vf += arm_up(b[j]) + arm_down(b[j]) + 1;
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
// 1-D aggregation: persistent line streamer, same-direction pass pairs fused
// ---------------------------------------------------------------------------
// Each workgroup (one per CU) owns every G-th line of the pass (both views) and treats
// them as ONE continuous pixel stream: windows never cross a line (arms stop at the
// image border), so lines simply follow each other and there is no per-line warm-up.
// The stream moves in chunks of AS_SEG pixels, one chunk per step; a chunk's pixel
// vectors land in an LDS ring (ring1) AS_AHEAD steps before the chunk is summed, and each
// pixel's window is summed with the reference's strictly sequential order (lanes own
// float4 of labels).
//   FUSED: pass A (the 2nd pass of an iteration, divided by the window sizes) writes
//   its outputs to a second ring (ring2) and pass B (the 1st pass of the next
//   iteration, same direction) sums them AS_LAG steps later, so the volume makes one
//   HBM round trip for two passes.  Not fused (the first and the last pass): pass A's
//   outputs are copied out of ring2 to HBM.
// In place: a pixel is overwritten AS_AHEAD (+AS_LAG) steps after it was staged.
// The per-pixel window sizes divide through an exact reciprocal-FMA quotient:
// q0 = a*y, r = fma(-q0, b, a), q = fma(r, y, q0) with y = RN(1/b) equals RN(a/b) for
// every integer b in [1, 6561] (arms up to 40) and every a in [2^-40, 2^16) (exhaustively checked,
// tools/micro/div_check.c); smaller a take the IEEE division.
constexpr int AS_SEG = 8;                   // pixels per chunk = A waves = B waves
constexpr int AS_AH = 5;                    // windows reach at most 5 chunks either side
constexpr int AS_MAX_ARM = AS_AH * AS_SEG;
constexpr int AS_AHEAD = AS_AH + 1;         // chunk c is readable from step c - AHEAD + 1
constexpr int AS_RC1 = 2 * AS_AH + 2;       // ring1 chunks: 2*AH+1 read + one landing
constexpr int AS_RC2 = 2 * AS_AH + 2;       // ring2 chunks: 2*AH+1 read + one written
constexpr int AS_RP1 = AS_RC1 * AS_SEG;
constexpr int AS_RP2 = AS_RC2 * AS_SEG;
constexpr int AS_LAG = AS_AH + 1;           // pass B at step s outputs chunk s - LAG

// Cache policy of the single passes' volume loads (the first and the last pass):
// streaming (slc).  Each vector is read once; the scanline pass after the last one then ran
// 4 % faster for a single pair (1.106 against 1.152 ms, same box, round 3).  The fused
// pass pairs keep default loads (slc there: 1.55 against 1.47 ms).
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
    const uint32_t* pk;    // packed descriptors of this direction, view 0
    const float* rcp;      // reciprocals of this direction, view 0
    int qtot;              // label vectors per pixel (Lp / 4)
    int qn0;               // label vectors per slice (blockIdx.y; the last may be narrower)
    int horizontal;
    int n;                 // pixels per line
    int cpl;               // chunks per line
    int nlv;               // lines per view
    int nl;                // lines of both views
    uint32_t* err;         // CHK: the stream's trace flag (trace_flag(st))
    int slices_x;          // > 1: the label slices interleaved along blockIdx.x (see k_agg_split)
};

constexpr int AX_MIR = 3;  // mirror slots after each ring (a 4-read block spans 3 slots past its start)

// The label vector a lane owns.  A ds_read_b128 serves a wave in four 16-lane groups, one LDS
// cycle each: {0-3,12-15,20-27}, {4-11,16-19,28-31}, {32-35,44-47,52-59}, {36-43,48-51,60-63}
// (MI355X_MICROARCH.md, LDS).  Lanes take the vectors group by group, so a slice of q vectors
// occupies ceil(q / 16) groups: config E's slices of 41 / 40 vectors read in 3 + 3 cycles an
// element instead of 4 + 4 with lane = vector (configs B, C: unchanged, 4 and 3 + 2).
__device__ __forceinline__ int agg_lane_vec(int l) {
    const int m = l & 31;
    int b, pos;  // group (0: the first of the half-wave's two, 1: the second), position in it
    if (m < 4) { b = 0; pos = m; }
    else if (m < 12) { b = 1; pos = m - 4; }
    else if (m < 16) { b = 0; pos = m - 8; }
    else if (m < 20) { b = 1; pos = m - 8; }
    else if (m < 28) { b = 0; pos = m - 12; }
    else { b = 1; pos = m - 16; }
    return (l & 32) + 16 * b + pos;
}

// ---------------------------------------------------------------------------
// The streamer's 16 waves split by role, so a step's two window sums run in parallel and
// no wave ever mixes loads with
// stores (the compiler drains vmcnt(0) whenever a wave with stores in flight consumes a
// load):
//   A waves (8): wave w owns pixel w of every chunk.  It stages its own pixel vectors
//     AX_D steps ahead in a VGPR ring (one 16-B-per-lane load and two meta words per step,
//     counted vmcnt waits, no stores), copies pixel w of chunk s + AHEAD into ring1,
//     writes its window descriptor, and sums pass A of chunk s into ring2.
//   B waves (8): pass B of chunk s - LAG over ring2 (FUSED), or the copy of pass A's
//     chunk s - 1 out of ring2 (single pass), and the stores to HBM.
// One barrier per step; every wave runs the same whole number of AX_D-step blocks.
//
// Scalar work: one workgroup fills a CU (16 waves, 4 a SIMD) and a CU issues about one
// scalar instruction a cycle, so per-step scalar bookkeeping of 16 waves sets the step's
// floor (round 4: ~85 SALU a wave and step in the ISA of the previous form, SQ_INSTS_SALU
// 1.7x SQ_INSTS_VALU).  Per-pixel bookkeeping is therefore vector work done once a block
// of AX_D steps, lane k for the block's k-th chunk:
//   * issue positions (line, chunk, volume offset) and the pixels' packed arms / window
//     sizes / reciprocals (one per-lane load each, a block ahead of use);
//   * the window descriptors of the block's landing chunks (ring offsets of both passes,
//     length, divisor and reciprocal, the pixel's volume offset), written to a meta ring of
//     2 * AX_D chunks, so a step only reads its descriptor (v_readfirstlane);
//   * the window loops keep their ring offset in a VGPR (wrap by v_cndmask).
constexpr int AX_THREADS = 16 * 64;
constexpr int AX_MW = 8;   // meta words per pixel (32 B): see k_agg_split
constexpr int AX_D = 12;   // A-wave staging ring: steps in flight (AX_D * 8 px * Q * 16 B per CU)
constexpr int AX_MC = 2 * AX_D;  // meta ring chunks: a block's descriptors are written at its start
static_assert(AX_D == AS_RC1 && AX_D == AS_RC2, "ring slots are compile-time per unrolled step");
static_assert(AS_AHEAD + AS_LAG <= AX_D, "meta ring too short for the B lag");
static_assert(AS_RP1 == AS_RP2, "pass B's ring2 window starts at pass A's ring1 slot");

// BIG: volumes of 2 GiB and more (configs C, E): vector loads and stores through 64-bit
// addresses instead of 32-bit buffer offsets.  Label slices: when a pixel vector's rings
// would not fit the CU's LDS, blockIdx.y picks one slice of the label axis (the sums of
// different labels are independent), each a narrower ring.
//
// Meta of pixel w of chunk c (slot c % AX_MC), written by A wave w at the start of the block
// in which the pixel lands:
//   [0] LDS byte offset of the pass-A window start in ring1 (pass B: + ring2 - ring1)
//   [1] window length, 0 = no output (past the line or the workgroup's stream)
//   [2] RN(1/windowSize) bits   [3] windowSize as float
//   [4] the pixel's volume byte offset from the slice base, low word   [5] high word
//
// CHK (TSM_TRACE builds of a launch): every descriptor a wave consumes is range-checked
// (ring offset inside its ring and on a pixel slot, window length within the rings' reach,
// volume offset inside the slice); a bad one sets the trace flag and its step does nothing.
template <bool FUSED, int QT, bool BIG, bool CHK = false>
__global__ __launch_bounds__(AX_THREADS) void k_agg_split(AggStream S, DevParams Pk) {
    const DevParams P = Pk;
    pair_shift(blockIdx.z, P.pstride, S.vol, S.arms, S.ws, S.pk, S.rcp);
    extern __shared__ __attribute__((aligned(16))) f32x4 smem_f4[];
    const int H = P.H, W = P.W, Lp = P.Lp;
    // label slices: when the grid interleaves them (slices_x > 1), the slices of one line group
    // are blocks 8 apart (same XCD) and dispatched together, so the 64-B granules two slices'
    // pieces of a pixel vector share are fetched once into that XCD's L2
    const int nsx = S.slices_x;
    const int slice = nsx > 1 ? (int)((blockIdx.x >> 3) % nsx) : (int)blockIdx.y;
    const int Q = QT > 0 ? QT : min(S.qn0, S.qtot - slice * S.qn0);
    float* const volq = S.vol + 4 * slice * S.qn0;  // this slice's first label
    const uint32_t Qs = (uint32_t)Q * 16;                                // bytes per ring pixel
    const size_t vstride = (size_t)H * W * Lp;
    const size_t es = S.horizontal ? (size_t)Lp : (size_t)W * Lp;         // floats per pixel step
    const size_t ls = S.horizontal ? (size_t)W * Lp : (size_t)Lp;          // floats per line step
    const uint32_t aes = S.horizontal ? 1u : (uint32_t)W;
    const uint32_t als = S.horizontal ? (uint32_t)W : 1u;
    const int G = gridDim.x / nsx;
    const int g = nsx > 1 ? (int)(blockIdx.x & 7) * (G >> 3) + (int)((blockIdx.x >> 3) / nsx)
                          : xcd_remap(blockIdx.x, gridDim.x);
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
    const int vq = agg_lane_vec(lane);  // this lane's label vector within the slice
    const uint32_t lane16 = (uint32_t)vq * 16;
    const bool vl = vq < Q;
    // CHK: descriptor ranges (see above); kind 1 = pass-A window, 2 = pass-B window, 3 = store
    const size_t vol_bytes = 2 * vstride * 4 - (size_t)16 * slice * S.qn0;  // slice base to volume end
    // lw = len | n1 << 16: n1 <= len, and the first piece ends inside the ring (or at its end)
    auto bad_desc = [&](uint32_t kind, uint32_t off, uint32_t lw, uint32_t rb, uint32_t re) -> bool {
        const uint32_t len = lw & 0xffffu, n1 = lw >> 16;
        const bool bad = len > 2 * AS_MAX_ARM + 1 || n1 > len ||
                         (len > 0 && (off < rb || off >= re || (off - rb) % Qs != 0 ||
                                      off + n1 * Qs > re || (n1 < len && off + n1 * Qs != re)));
        if (bad && lane == 0) { S.err[1] = off; S.err[0] = kind; }
        return bad;
    };
    auto bad_store = [&](uint32_t lo, uint32_t hi) -> bool {
        const size_t o = BIG ? ((size_t)hi << 32 | lo) : (size_t)lo;
        const bool bad = (o & 15) != 0 || o + (size_t)Q * 16 > vol_bytes;
        if (bad && lane == 0) { S.err[1] = lo; S.err[0] = 3u; }
        return bad;
    };
    // the step's barrier is the descriptor protocol: a descriptor is read only after the
    // barrier that follows its write (a probe without it faulted, round 4)
    auto barrier = [&]() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
    // sequential window sum of `len` ring pixels from LDS byte offset `off` (a slot of the
    // ring [rb, re)): whole blocks of 4 at immediate offsets (the mirror slots make every
    // block contiguous), then the 1-3 remaining pixels under uniform branches -- the
    // reference's order, no padding reads.  The running offset is a VGPR (its wrap a
    // v_cndmask): only the block count is scalar.
    // The descriptor also holds n1, the elements before the ring's end (len | n1 << 16), so
    // the window runs as two straight pieces -- n1 elements from off, the rest from the
    // ring's start -- with no per-block wrap test: per block of 4 elements one address add.
    auto piece = [&](f32x4& acc, uint32_t off, int n) {
        const char* p = lds + off + lane16;
        // 8 reads a round trip, then a block of 4 (the long windows of real pairs: one LDS latency
        // per 8 elements; round 6: 0600 aggregate 4.65 -> 4.55 ms, Motorcycle 15.9 -> 15.4)
        for (int nb = n >> 3; nb > 0; --nb) {
            f32x4 x[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] = *reinterpret_cast<const f32x4*>(p + k * Qs);
#pragma unroll
            for (int k = 0; k < 8; ++k) acc += x[k];
            p += 8 * Qs;
        }
        if (n & 4) {
            const f32x4 x0 = *reinterpret_cast<const f32x4*>(p);
            const f32x4 x1 = *reinterpret_cast<const f32x4*>(p + Qs);
            const f32x4 x2 = *reinterpret_cast<const f32x4*>(p + 2 * Qs);
            const f32x4 x3 = *reinterpret_cast<const f32x4*>(p + 3 * Qs);
            acc += x0;
            acc += x1;
            acc += x2;
            acc += x3;
            p += 4 * Qs;
        }
        const int r = n & 3;
        if (r) {  // the mirror slots keep a block starting at the ring's last slot in range
            const f32x4 x0 = *reinterpret_cast<const f32x4*>(p);
            const f32x4 x1 = *reinterpret_cast<const f32x4*>(p + Qs);
            const f32x4 x2 = *reinterpret_cast<const f32x4*>(p + 2 * Qs);
            acc += x0;
            if (r > 1) acc += x1;
            if (r > 2) acc += x2;
        }
    };
    auto window = [&](uint32_t off, uint32_t lw, uint32_t rb, uint32_t re) -> f32x4 {
        (void)re;
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        const int len = (int)(lw & 0xffffu), n1 = (int)(lw >> 16);
        piece(acc, off, n1);
        if (len > n1) piece(acc, rb, len - n1);
        return acc;
    };
    const uint32_t mstep = AS_SEG * AX_MW * 4;
    const char* mbase = lds + meta_off + (uint32_t)w * AX_MW * 4;  // this wave's pixel column
    // meta slot of chunk 12 b + u + d (b: the block, odd -> par): compile-time d and u
    auto mslot = [&](bool par, int ud) -> uint32_t {
        const int e = (ud % AX_MC + AX_MC) % AX_MC, o = (ud + AX_D) % AX_MC;
        return (uint32_t)(par ? (o + AX_MC) % AX_MC : e) * mstep;
    };
    // the volume store of pass B / the single pass: byte offset from the slice base
    const __amdgpu_buffer_rsrc_t rs_vol = make_rsrc(volq);
    auto store = [&](uint32_t lo, uint32_t hi, const f32x4& acc) {
        if (!vl) return;
        if (BIG) {  // plain stores (configs C / E: non-temporal ones measured 2 % slower on C, round 6)
            const size_t o = ((size_t)hi << 32 | lo) >> 2;
            *reinterpret_cast<f32x4*>(volq + o + 4 * vq) = acc;
        } else {
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc), rs_vol, lane16, lo, 2);
        }
    };

    if (roleA) {
        // ---- A: staging ring, land, pass A ----------------------------------------------
        const int lanec = vq < Q ? vq : Q - 1;
        const __amdgpu_buffer_rsrc_t rs_pk = make_rsrc(S.pk), rs_rcp = make_rsrc(S.rcp);
        const uint32_t voff = (uint32_t)lanec * 16;
        // Chunks c0 .. c0 + AX_D - 1, lane k for chunk c0 + k: the volume byte offset of pixel
        // w (64-bit), whether the pixel is inside the workgroup's stream, and its packed
        // arms + window size and reciprocal (loaded here, used a block later).  (bl, bc):
        // line / chunk-in-line of c0, advanced AX_D chunks a block (scalar, once a block).
        struct Batch { uint32_t olo, ohi, valid, ma, my; };
        int bl = 0, bc = 0;
        auto batch = [&]() -> Batch {
            int c = bc + (lane < AX_D ? lane : 0), l = bl;
            while (c >= S.cpl) { c -= S.cpl; ++l; }
            const bool past = l >= my_lines;
            const int lc = past ? my_lines - 1 : l;  // past the end: re-read the last pixel
            const int pos = past ? S.n - 1 : min(c * AS_SEG + w, S.n - 1);
            const int gl = g + lc * G;
            const int v = gl >= S.nlv ? 1 : 0, line = gl - v * S.nlv;
            const size_t ob = ((size_t)v * vstride + (size_t)line * ls + (size_t)pos * es) * 4;
            const uint32_t mo = ((uint32_t)(2 * v * H * W) + (uint32_t)line * als + (uint32_t)pos * aes) * 4;  // per-view stride 2HW
            Batch B;
            B.olo = (uint32_t)ob;
            B.ohi = BIG ? (uint32_t)(ob >> 32) : 0u;
            B.valid = (!past && c * AS_SEG + w < S.n) ? 1u : 0u;
            B.ma = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs_pk, mo, 0, 0);
            B.my = S.ws ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs_rcp, mo, 0, 0) : 0u;
            return B;
        };
        auto advance = [&](int k) {
            bc += k;
            while (bc >= S.cpl) { bc -= S.cpl; ++bl; }
        };
        // descriptors of batch Bt's chunks (chunk c0 + k in lane k, lanes < n) -> the meta
        // ring; the chunks' ring slot index is (r0 + k) % AX_D, their meta slot (m0 + k) % AX_MC
        auto finish = [&](const Batch& Bt, int r0, int m0, int n) {
            if (lane < n) {
                const int slot = ((r0 + lane) % AX_D) * AS_SEG + w;
                const int lo = (int)(Bt.ma & 0xffu), hi = (int)((Bt.ma >> 8) & 0xffu);
                int st = slot - lo;
                st = st < 0 ? st + AS_RP1 : st;
                const uint32_t len = Bt.valid ? (uint32_t)(lo + hi + 1) : 0u;
                const uint32_t n1 = min(len, (uint32_t)(AS_RP1 - st));  // elements before the ring end
                char* m = lds + meta_off + (uint32_t)(((m0 + lane) % AX_MC) * AS_SEG + w) * AX_MW * 4;
                *reinterpret_cast<u32x4*>(m) = u32x4{r1_off + (uint32_t)st * Qs, len | n1 << 16, Bt.my,
                                                     __float_as_uint((float)(int)(Bt.ma >> 16))};
                *reinterpret_cast<u32x2*>(m + 16) = u32x2{Bt.olo, Bt.ohi};
            }
        };
        f32x4 rv[AX_D];
        auto issue = [&](int k, const Batch& Bt, int i) {  // chunk of lane i of batch Bt -> slot k
            const uint32_t lo = __builtin_amdgcn_readlane(Bt.olo, i);
            if (BIG) {
                const uint32_t hi = __builtin_amdgcn_readlane(Bt.ohi, i);
                const size_t o = ((size_t)hi << 32 | lo) >> 2;
                rv[k] = *reinterpret_cast<const f32x4*>(volq + o + 4 * lanec);
            } else {
                // single passes (the first and the last) load with the streaming policy (kNtLoad)
                rv[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs_vol, voff, lo, FUSED ? 0 : kNtLoad));
            }
        };
        auto land = [&](const f32x4& val, int ci) {  // pixel w of a chunk -> ring1 slot index ci
            const int slot = ci * AS_SEG + w;
            *reinterpret_cast<f32x4*>(lds + r1_off + (uint32_t)slot * Qs + voff) = val;
            if (slot < AX_MIR) *reinterpret_cast<f32x4*>(lds + r1_off + (uint32_t)(AS_RP1 + slot) * Qs + voff) = val;
        };
        // prologue: chunks 0 .. AHEAD + AX_D - 1 in flight, chunks 0 .. AHEAD - 1 landed.
        // Slot of chunk c: (c - AHEAD) mod AX_D, so step s lands and refills slot s mod AX_D.
        const Batch b0 = batch();  // chunks 0 .. AX_D - 1
        f32x4 pre[AS_AHEAD];
#pragma unroll
        for (int c = 0; c < AS_AHEAD; ++c) {
            issue(0, b0, c);
            pre[c] = rv[0];
        }
        advance(AS_AHEAD);
        Batch prev = batch();  // chunks AHEAD .. AHEAD + AX_D - 1: land in block 0
#pragma unroll
        for (int k = 0; k < AX_D; ++k) issue(k, prev, k);
        advance(AX_D);
        finish(b0, 0, 0, AS_AHEAD);
#pragma unroll
        for (int c = 0; c < AS_AHEAD; ++c) land(pre[c], c % AX_D);
        u32x4 mA;
        barrier();
        mA = *reinterpret_cast<const u32x4*>(mbase);
        for (int b = 0; b < nblk; ++b) {
            const bool par = b & 1;
            const Batch cur = batch();  // chunks issued in this block (land in the next)
            advance(AX_D);
            // the descriptors of this block's landing chunks 12 b + AHEAD + k
            finish(prev, AS_AHEAD, (par ? AX_D : 0) + AS_AHEAD, AX_D);
#pragma unroll
            for (int u = 0; u < AX_D; ++u) {
                // land chunk s + AHEAD from slot u, then refill the slot (chunk s + AHEAD + AX_D)
                land(rv[u], (u + AS_AHEAD) % AX_D);
                issue(u, cur, u);
                const uint32_t a_off = __builtin_amdgcn_readfirstlane(mA.x);
                uint32_t a_lw = __builtin_amdgcn_readfirstlane(mA.y);
                if constexpr (CHK) if (bad_desc(1u, a_off, a_lw, r1_off, r1_end)) a_lw = 0;
                const int a_len = (int)(a_lw & 0xffffu);
                const float a_y = __uint_as_float(__builtin_amdgcn_readfirstlane(mA.z));
                const float a_b = __uint_as_float(__builtin_amdgcn_readfirstlane(mA.w));
                mA = *reinterpret_cast<const u32x4*>(mbase + mslot(par, u + 1));  // chunk s + 1
                const uint32_t r2w = r2_off + (uint32_t)(u * AS_SEG + w) * Qs;  // ring2 slot of chunk s
                if (a_len) {
                    f32x4 acc = window(a_off, a_lw, r1_off, r1_end);
                    if (S.ws) acc = div_ws(acc, a_b, a_y);
                    if (vl) {
                        *reinterpret_cast<f32x4*>(lds + r2w + lane16) = acc;
                        if (u == 0 && w < AX_MIR)
                            *reinterpret_cast<f32x4*>(lds + r2w + (uint32_t)AS_RP2 * Qs + lane16) = acc;
                    }
                }
                barrier();
            }
            prev = cur;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no load outlives the workgroup
        return;
    }

    // ---- B: pass B over ring2 (FUSED) or pass A's outputs out of ring2, stores ------------
    constexpr int lag = FUSED ? AS_LAG : 1;
    const uint32_t d21 = r2_off - r1_off;  // pass B's window: pass A's ring1 start, in ring2
    barrier();
    u32x2 mB = u32x2{0u, 0u}, mO = u32x2{0u, 0u};  // chunk -lag: never used (s < lag)
    for (int b = 0; b < nblk; ++b) {
        const bool par = b & 1;
#pragma unroll
        for (int u = 0; u < AX_D; ++u) {
            const int s = b * AX_D + u;
            const int ub = (u - lag + 2 * AX_D) % AX_D;  // ring chunk slot of chunk s - lag
            const uint32_t b_off = __builtin_amdgcn_readfirstlane(mB.x) + d21;
            uint32_t b_lw = __builtin_amdgcn_readfirstlane(mB.y);
            const uint32_t olo = __builtin_amdgcn_readfirstlane(mO.x);
            const uint32_t ohi = BIG ? __builtin_amdgcn_readfirstlane(mO.y) : 0u;
            if constexpr (CHK) {
                if (s >= lag && b_lw && ((FUSED && bad_desc(2u, b_off, b_lw, r2_off, r2_end)) || bad_store(olo, ohi)))
                    b_lw = 0;
            }
            const int b_len = (int)(b_lw & 0xffffu);
            const char* mn = mbase + mslot(par, u - lag + 1);  // chunk s - lag + 1
            mB = *reinterpret_cast<const u32x2*>(mn);
            mO = *reinterpret_cast<const u32x2*>(mn + 16);
            const uint32_t r2r = r2_off + (uint32_t)(ub * AS_SEG + w) * Qs;  // single: chunk s - 1
            if (s >= lag && b_len) {
                const f32x4 acc = FUSED ? window(b_off, b_lw, r2_off, r2_end)
                                        : *reinterpret_cast<const f32x4*>(lds + r2r + lane16);
                store(olo, ohi, acc);
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
// LDS of the split streamer for a slice of qs label vectors
static size_t agg_split_lds(int qs) {
    return ((size_t)AS_RP1 + AS_RP2 + 2 * AX_MIR) * qs * 16 + (size_t)AX_MC * AS_SEG * AX_MW * 4;  // rings + meta
}
constexpr size_t kLdsBytes = 160 * 1024;

template <bool FUSED, int QT, bool BIG>
static void launch_split_t(const AggStream& S, const DevParams& P, dim3 grid, size_t lds, hipStream_t st) {
    if (S.err) {  // TSM_TRACE: the descriptor-checked variant of the instance production runs
        ensure_lds_limit((const void*)k_agg_split<FUSED, QT, BIG, true>, kLdsBytes);
        hipLaunchKernelGGL((k_agg_split<FUSED, QT, BIG, true>), grid, dim3(AX_THREADS), lds, st, S, P);
        return;
    }
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
    S.err = trace_flag(st);
    const int ncu = P.ncu;
    const int G = S.nl < ncu ? S.nl : ncu;
    // every pass through the role-split streamer (round 4, same box: 409 against 406.5
    // pairs/s with the single passes on the former loader/summer streamer)
    const size_t slds = agg_split_lds(S.qn0);
    // several slices: interleaved along x, G / nslice line groups (a multiple of 8: one per XCD
    // slot), each slice of a group on the same XCD at the same time
    int Gs = (ncu / nslice) & ~7;
    if (Gs > S.nl) Gs = S.nl & ~7;
    S.slices_x = (nslice > 1 && Gs >= 8) ? nslice : 1;
    const dim3 sgrid = S.slices_x > 1 ? dim3(Gs * nslice, 1, P.npairs) : dim3(G, nslice, P.npairs);
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
