// tsm_device.h -- shared device-side definitions for the gfx950 AD-Census kernels.
//
// HBM layout of one pair's workspace (see DESIGN.md "Data layout"):
//   img   [2][H][W]      u32  packed B|G<<8|R<<16 of the matched view images
//   desc  [2][H][W][16]  u32  ternary census records (gt/lt bit planes + colour)
//   vol   [2][H][W][Lp]  f32  pixel-major cost volume, Lp = round_up(L, 4)
//   arms  [2][H][W]      u32  packed u8 arms: up | down<<8 | left<<16 | right<<24
//   ws    [2][2][H][W]   i32  cross-window sizes (horizontal-first, vertical-first)
// Pixel-major volumes make every per-pixel L-vector one contiguous 16-B-aligned run:
// a wave owns a pixel, lanes own 4 consecutive disparities (float4), so arm lengths,
// scanline minima and WTA are wave-uniform / wave reductions with no divergence.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace tsm {

constexpr int kWave = 64;

// native 4-wide vectors: register arrays of these stay in VGPRs (HIP's float4 class
// type defeats SROA in arrays and spills them to scratch)
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// POD kernel parameters (ADCensusParams, stereo_utils.h:209-244, plus geometry).
struct DevParams {
    int H, W;          // image size
    int L, Lp;         // labels (max-min+1) and padded vector length (multiple of 4)
    int minD, maxD;    // disparity range (inclusive)
    int color_model;   // 0 RGB, 1 HSI
    int mask;          // mask matching
    int censusW, censusH;
    int color_thresh1, color_thresh2;
    int sat_thresh1, sat_thresh2;
    int int_thresh1, int_thresh2;
    int max_length1, max_length2;
    int color_diff;
    float pi1, pi2;
    float p1t[3], p2t[3]; // P1/P2 by #similar (d1<colorDiff)+(d2<colorDiff): /10, /4, x1 (ADCensus.cpp:954-979)
    int disp_tolerance;
    int voting_thresh;
    float voting_ratio;
    int max_search_depth;
    int canny_low, canny_high;
    int omp_threads;   // scanline race emulation (0/1 = serial semantics)
    int gpad, gstride; // colour-difference maps: row stride and left margin (sentinel bytes)
    // Pair groups: a launch runs `npairs` pairs; pair p's per-pair buffers sit p * pstride
    // bytes past pair 0's (one arena, one slot per pair), and every kernel takes its pair
    // from blockIdx.z (kernels with a view axis: blockIdx.z = 2 * pair + view).
    size_t pstride;
    int npairs;
    int ncu;           // compute units of the handle's device (persistent grids)
};

// Streaming store of a volume vector: non-temporal (nt), since nothing reads it back
// before it has left the caches anyway.  Measured on the aggregation streamer: -6.6 %
// per launch against plain stores (nt LOADS measured slower and are not used).
__device__ __forceinline__ void st_stream(float* p, f32x4 v) {
    __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p));
}

// Exact a / b for the aggregation's "C /= windowSize" (ADCensus.cpp:743-748): with
// y = RN(1/b), q0 = a*y, r = fma(-q0, b, a), q = fma(r, y, q0) equals RN(a/b) for every
// integer b in [1, 6561] and every a in [2^-40, 2^16) (exhaustively checked,
// tools/micro/div_check.c); 0 < a < 2^-40 (never seen in practice) takes the IEEE path,
// a == 0 is exact.
__device__ __forceinline__ f32x4 div_ws(f32x4 a, float b, float y) {
    const f32x4 q0 = a * y;
    const f32x4 r = __builtin_elementwise_fma(-q0, f32x4{b, b, b, b}, a);
    f32x4 q = __builtin_elementwise_fma(r, f32x4{y, y, y, y}, q0);
    const u32x4 ab = __builtin_bit_cast(u32x4, a) - 1u;  // +0 wraps to 0xffffffff
    if (__builtin_expect(min(min(ab.x, ab.y), min(ab.z, ab.w)) < 0x2b800000u - 1u, 0)) {
        q.x = a.x / b; q.y = a.y / b; q.z = a.z / b; q.w = a.w / b;
    }
    return q;
}

// XCD-aware block order.  Workgroups are dealt round-robin to the 8 XCDs (flat block b runs
// on XCD b % 8; with gridDim.x a multiple of 8, blockIdx.x % 8 is the XCD whatever y / z).
// Mapping b -> (b % 8) * per + b / 8 gives each XCD a contiguous run of the index space, so
// workgroups that run side by side on one XCD own neighbouring lines: the 64-B granules two
// neighbouring pixel vectors share (a 784-B vector is not a granule multiple) are then
// fetched once into that XCD's L2 instead of once by each of two XCDs.  A permutation of
// [0, n); blocks past the last multiple of 8 keep their index.
__device__ __forceinline__ int xcd_remap(int b, int n) {
    const int per = n >> 3;
    return b < 8 * per ? (b & 7) * per + (b >> 3) : b;
}

// Largest group a launch carries (pointer tables of per-pair user buffers are kernel
// arguments of this many entries).
constexpr int kMaxGroup = 64;

// Per-pair user buffers of a group (inputs, outputs), passed by value.
struct PairIn {
    const uint8_t* left[kMaxGroup];
    const uint8_t* right[kMaxGroup];
};
struct PairOut {
    float* out[kMaxGroup];
};

// Move arena pointers from pair 0's slot to pair `pair`'s (null pointers stay null).
// Byte-pointer arithmetic, not an integer round trip: the shifted pointer keeps the
// kernel argument's provenance, so the compiler still knows it addresses global memory
// and emits global_* instead of flat_* accesses (a flat access also counts against
// lgkmcnt, so every LDS wait after it would wait for the memory access too).
template <class Ptr>
__device__ __forceinline__ void pair_shift1(size_t off, Ptr& p) {
    using B = std::conditional_t<std::is_const_v<std::remove_pointer_t<Ptr>>, const char*, char*>;
    if (p) p = (Ptr)((B)p + off);
}
template <class... Ptr>
__device__ __forceinline__ void pair_shift(unsigned pair, size_t pstride, Ptr&... p) {
    const size_t off = (size_t)pair * pstride;
    (pair_shift1(off, p), ...);
}

// Left/right margin of the colour-difference maps gv/gh: a scanline step reads 4
// consecutive bytes at x = line +- (d + minD), d < L, through an aligned 8-byte load.
__host__ __device__ inline int grad_pad(int maxD) { return ((maxD + 12 + 15) / 16) * 16; }

__device__ __forceinline__ int iabs_(int x) { return x < 0 ? -x : x; }
__device__ __forceinline__ int ch(uint32_t p, int c) { return (p >> (8 * c)) & 0xff; }

// colorDiff, ADCensus.cpp:583-602.
__device__ __forceinline__ int color_diff(const DevParams& P, uint32_t a, uint32_t b) {
    if (P.color_model == 0) {
        int d0 = iabs_(ch(a, 0) - ch(b, 0));
        int d1 = iabs_(ch(a, 1) - ch(b, 1));
        int d2 = iabs_(ch(a, 2) - ch(b, 2));
        return max(d0, max(d1, d2));
    }
    int hd = iabs_(ch(a, 0) - ch(b, 0));
    return min(hd, 255 - hd);
}

// DPP move with an `old` fallback for lanes whose source is out of range.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v, float old) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), CTRL,
                                                      0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u(uint32_t v, uint32_t old) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, 0xF, 0xF, false);
}

constexpr int DPP_QUAD_1032 = 0xB1;     // quad_perm [1,0,3,2]
constexpr int DPP_QUAD_2301 = 0x4E;     // quad_perm [2,3,0,1]
constexpr int DPP_ROW_MIRROR = 0x140;
constexpr int DPP_ROW_HALF_MIRROR = 0x141;
constexpr int DPP_WAVE_SHL1 = 0x130;    // lane l <- lane l+1
constexpr int DPP_WAVE_SHR1 = 0x138;    // lane l <- lane l-1

// Wave-wide min of NON-NEGATIVE floats (cost values), result uniform in every lane.
// Non-negative IEEE floats order like their bit patterns, so the whole reduction runs
// as unsigned integer min (DPP within rows, scalar across the four rows): exact, and
// without the canonicalising v_max the compiler puts in front of every fminf.  The row
// steps read every lane (quad_perm / mirrors), so bound_ctrl DPP moves fold into
// v_min_u32_dpp (one instruction per level).
__device__ __forceinline__ uint32_t dpp_row_min(uint32_t v) {
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, DPP_QUAD_1032, 0xF, 0xF, true));
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, DPP_QUAD_2301, 0xF, 0xF, true));
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, DPP_ROW_HALF_MIRROR, 0xF, 0xF, true));
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, DPP_ROW_MIRROR, 0xF, 0xF, true));
    return v;
}
__device__ __forceinline__ uint32_t wave_min_bits(uint32_t v) {
    v = dpp_row_min(v);
    const uint32_t r0 = __builtin_amdgcn_readlane(v, 0);
    const uint32_t r1 = __builtin_amdgcn_readlane(v, 16);
    const uint32_t r2 = __builtin_amdgcn_readlane(v, 32);
    const uint32_t r3 = __builtin_amdgcn_readlane(v, 48);
    return min(min(r0, r1), min(r2, r3));
}
// Same, kept in VGPRs (every lane ends with the wave min): the row minima are combined
// by the gfx950 lane swaps v_permlane32_swap (rows 0,1 <-> 2,3) and v_permlane16_swap
// (rows 0 <-> 1, 2 <-> 3) instead of readlanes, so a VALU consumer needs no
// VALU -> SGPR -> VALU round trip.
__device__ __forceinline__ uint32_t wave_min_bits_v(uint32_t v) {
    v = dpp_row_min(v);
    const auto a = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    v = min((uint32_t)a[0], (uint32_t)a[1]);
    const auto b = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return min((uint32_t)b[0], (uint32_t)b[1]);
}
__device__ __forceinline__ float wave_min_nonneg(float x) {
    return __uint_as_float(wave_min_bits(__float_as_uint(x)));
}

// Wave-wide min of u64 keys (e.g. (float_bits << 32) | d for WTA first-min).
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
    for (int off = 32; off >= 1; off >>= 1) {
        uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
        uint32_t olo = (uint32_t)__shfl_xor((int)lo, off);
        uint32_t ohi = (uint32_t)__shfl_xor((int)hi, off);
        uint64_t o = ((uint64_t)ohi << 32) | olo;
        v = o < v ? o : v;
    }
    return v;
}

__device__ __forceinline__ int wave_max_i32(int v) {
    for (int off = 32; off >= 1; off >>= 1) v = max(v, __shfl_xor(v, off));
    return v;
}

__device__ __forceinline__ int wave_sum_i(int v) {
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Orders one wave's LDS accesses across its lanes (lanes sharing LDS words without a workgroup
// barrier): every access before it completes before any after it, and the compiler moves none
// across it.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace tsm
