// k_stereo_ops.hip -- the gfx950 operators either side of the AD-Census path (SURVEY
// §8f f2-f4) and their C ABI (include/tsm_stereo_ops.h):
//   f2  applyColorMap (source/stereo.cpp:94-134): a min/max pass + a LUT pass
//   f3  reprojectToDepth / reprojectTo3D x2 (stereo.cpp:136-202): elementwise
//   f4  cv::remap INTER_LINEAR of EpipolarRectify::rectify (EpipolarRectify.cpp:87-101)
// All are HBM-bound streams: 4 pixels a lane along a row, so the byte-wide BGR outputs
// leave as whole dwords (12 B a lane), and no divergent per-pixel branches beyond the
// reference's own validity tests.  Every kernel takes tables of up to kOpsBatch maps
// (blockIdx.z = map): the _batch_device forms run a whole group of the matcher's outputs
// in one launch (one map per call is launch-latency bound at config-B sizes); the single
// forms are a table of one.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <map>
#include <mutex>
#include <type_traits>
#include <utility>

#include "tsm_adcensus.h"
#include "tsm_stereo_ops.h"

namespace tsm {
namespace {

constexpr int OPS_THREADS = 256;
constexpr int OPS_PX = 4;  // pixels per lane along a row
constexpr int kOpsBatch = 64;  // maps per launch (pointer tables ride in the kernel arguments)

template <class T>
struct Tab {
    T* p[kOpsBatch];
};

// (unsigned char)t with x86 cvttss2si semantics: NaN / out of int range -> 0x80000000
__device__ __forceinline__ uint32_t cast_u8_x86(float t) {
    return (t > -2147483648.0f && t < 2147483648.0f) ? ((uint32_t)(int32_t)t & 0xffu) : 0u;
}

// Pixel groups: 4 consecutive pixels of a row per lane, the (row, group) pairs of a map
// flattened over blockIdx.x (no idle lanes at the row ends).  Dense maps (rows packed
// back to back, every map of the call) run as one row of rows*cols pixels, so groups never
// straddle a misaligned row start and the loads / stores are whole vectors.
struct Grp {
    int y, x0, n;  // row, first pixel, pixels in the group (0: past the map)
};
__device__ __forceinline__ Grp pixel_group(int rows, int cols) {
    const uint32_t gpr = (uint32_t)(cols + OPS_PX - 1) / OPS_PX;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;  // grids stay below 2^32 threads
    if ((long)t >= (long)rows * gpr) return Grp{0, 0, 0};
    const uint32_t y = rows == 1 ? 0u : t / gpr;  // dense maps run as one row: no division
    const int x0 = (int)(t - y * gpr) * OPS_PX;
    return Grp{(int)y, x0, min(OPS_PX, cols - x0)};
}

typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));

// the group's n <= 4 floats at s: two 8-B loads when whole and 8-B aligned
__device__ __forceinline__ void load4(const float* __restrict__ s, int n, float (&v)[OPS_PX]) {
    if (n == OPS_PX && ((uintptr_t)s & 7) == 0) {
        const f2v a = reinterpret_cast<const f2v*>(s)[0], b = reinterpret_cast<const f2v*>(s)[1];
        v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
        return;
    }
#pragma unroll
    for (int k = 0; k < OPS_PX; ++k) v[k] = k < n ? s[k] : 0.f;
}

// n <= 4 groups of 3 floats (12 n bytes) at d: 16-B / 8-B vectors when whole and aligned
__device__ __forceinline__ void store4x3(float* __restrict__ d, int n, const float (&o)[3 * OPS_PX]) {
    if (n == OPS_PX && ((uintptr_t)d & 15) == 0) {
#pragma unroll
        for (int i = 0; i < 3; ++i)
            reinterpret_cast<f4v*>(d)[i] = f4v{o[4 * i], o[4 * i + 1], o[4 * i + 2], o[4 * i + 3]};
        return;
    }
    if (n == OPS_PX && ((uintptr_t)d & 7) == 0) {
#pragma unroll
        for (int i = 0; i < 6; ++i) reinterpret_cast<f2v*>(d)[i] = f2v{o[2 * i], o[2 * i + 1]};
        return;
    }
    for (int i = 0; i < 3 * n; ++i) d[i] = o[i];
}

// ---- f2 ---------------------------------------------------------------------------

struct Lut {
    uint32_t bgr[256];  // b | g << 8 | r << 16
};

// min / max over pixels >= 0 and not inf (stereo.cpp:96-104).  Every such value is a
// non-negative float (NaN is skipped as std::min/max skip it; -0.0 folds to +0.0, which
// changes no index downstream), so the bit patterns order like the values and the
// reduction is on integers.  Two launches: per-block partials, then one block folds them
// into mm[0..1] (plain stores read by the next launch: no cross-XCD atomics on a word
// other XCDs' caches may hold).
constexpr int MM_BLOCKS = 512;

__device__ __forceinline__ void block_minmax(uint32_t& lo, int& hi, uint32_t* s_lo, int* s_hi) {
    for (int o = 32; o > 0; o >>= 1) {
        lo = min(lo, (uint32_t)__shfl_xor((int)lo, o));
        hi = max(hi, __shfl_xor(hi, o));
    }
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s_lo[w] = lo;
        s_hi[w] = hi;
    }
    __syncthreads();
    lo = 0x7f800000u;
    hi = (int)0xff800000u;
    for (int i = 0; i < nw; ++i) {
        lo = min(lo, s_lo[i]);
        hi = max(hi, s_hi[i]);
    }
}

// part: MM_BLOCKS partial pairs per map (map z at part + 2 * MM_BLOCKS * z); a grid-stride
// walk over the map's pixel groups, two groups in flight per lane
__global__ void k_minmax(Tab<const float> srcs, int rows, int cols, size_t step_f, uint32_t* __restrict__ part) {
    __shared__ uint32_t s_lo[16];
    __shared__ int s_hi[16];
    const float* __restrict__ src = srcs.p[blockIdx.z];
    part += (size_t)2 * MM_BLOCKS * blockIdx.z;
    const int gpr = (cols + OPS_PX - 1) / OPS_PX;
    const long ng = (long)rows * gpr, stride = (long)gridDim.x * blockDim.x;
    uint32_t lo = 0x7f800000u;
    int hi = (int)0xff800000u;  // -inf: no valid pixel
    auto fold = [&](const float (&v)[OPS_PX], int n) {
#pragma unroll
        for (int k = 0; k < OPS_PX; ++k)
            if (k < n && v[k] >= 0.f && v[k] != __int_as_float(0x7f800000)) {
                const uint32_t b = __float_as_uint(v[k] + 0.f);
                lo = min(lo, b);
                hi = max(hi, (int)b);
            }
    };
    auto at = [&](long t, int& n) {
        const int y = (int)(t / gpr), x0 = (int)(t - (long)y * gpr) * OPS_PX;
        n = min(OPS_PX, cols - x0);
        return src + (size_t)y * step_f + x0;
    };
    long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    for (; t + stride < ng; t += 2 * stride) {
        int n0, n1;
        const float* s0 = at(t, n0);
        const float* s1 = at(t + stride, n1);
        float v0[OPS_PX], v1[OPS_PX];
        load4(s0, n0, v0);
        load4(s1, n1, v1);
        fold(v0, n0);
        fold(v1, n1);
    }
    if (t < ng) {
        int n0;
        const float* s0 = at(t, n0);
        float v0[OPS_PX];
        load4(s0, n0, v0);
        fold(v0, n0);
    }
    block_minmax(lo, hi, s_lo, s_hi);
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = lo;
        part[2 * blockIdx.x + 1] = (uint32_t)hi;
    }
}

// mm: the folded (min, max) of map z at mm + 2 z
__global__ void k_minmax_final(uint32_t* __restrict__ part, int nparts, uint32_t* __restrict__ mm) {
    __shared__ uint32_t s_lo[16];
    __shared__ int s_hi[16];
    part += (size_t)2 * MM_BLOCKS * blockIdx.z;
    mm += 2 * blockIdx.z;
    uint32_t lo = 0x7f800000u;
    int hi = (int)0xff800000u;
    for (int i = threadIdx.x; i < nparts; i += blockDim.x) {
        lo = min(lo, part[2 * i]);
        hi = max(hi, (int)part[2 * i + 1]);
    }
    block_minmax(lo, hi, s_lo, s_hi);
    if (threadIdx.x == 0) {
        mm[0] = lo;
        mm[1] = (uint32_t)hi;
    }
}

__global__ void k_colormap(Tab<const float> srcs, int rows, int cols, size_t step_f,
                           const uint32_t* __restrict__ mm, int use_range, float rmin, float rmax,
                           Lut lut, Tab<uint8_t> dsts, size_t dstep) {
    const Grp p = pixel_group(rows, cols);
    if (p.n == 0) return;
    const float* __restrict__ src = srcs.p[blockIdx.z];
    uint8_t* __restrict__ dst = dsts.p[blockIdx.z];
    if (!use_range) mm += 2 * blockIdx.z;
    const float mn = use_range ? rmin : __uint_as_float(mm[0]);
    const float mx = use_range ? rmax : __int_as_float((int)mm[1]);
    uint8_t* d = dst + (size_t)p.y * dstep + 3 * (size_t)p.x0;
    const int n = p.n;
    float v[OPS_PX];
    load4(src + (size_t)p.y * step_f + p.x0, n, v);
    uint32_t c[OPS_PX];
#pragma unroll
    for (int k = 0; k < OPS_PX; ++k) {
        const bool black = use_range ? (v[k] < mn || v[k] > mx) : (v[k] < 0.f);
        c[k] = black ? 0u : lut.bgr[cast_u8_x86(((v[k] - mn) / (mx - mn)) * 255)];
    }
    if (n == OPS_PX && ((uintptr_t)d & 3) == 0) {  // 12 B: three dword stores
        uint32_t* d4 = reinterpret_cast<uint32_t*>(d);
        d4[0] = c[0] | (c[1] << 24);
        d4[1] = (c[1] >> 8) | (c[2] << 16);
        d4[2] = (c[2] >> 16) | (c[3] << 8);
    } else if (n == OPS_PX && ((uintptr_t)d & 1) == 0) {  // 2-B aligned: six halfword stores
        uint16_t* d2 = reinterpret_cast<uint16_t*>(d);
        d2[0] = (uint16_t)c[0];
        d2[1] = (uint16_t)((c[0] >> 16) | (c[1] << 8));
        d2[2] = (uint16_t)(c[1] >> 8);
        d2[3] = (uint16_t)c[2];
        d2[4] = (uint16_t)((c[2] >> 16) | (c[3] << 8));
        d2[5] = (uint16_t)(c[3] >> 8);
    } else {
        for (int k = 0; k < n; ++k) {
            d[3 * k + 0] = (uint8_t)c[k];
            d[3 * k + 1] = (uint8_t)(c[k] >> 8);
            d[3 * k + 2] = (uint8_t)(c[k] >> 16);
        }
    }
}

// ---- f3 ---------------------------------------------------------------------------

__global__ void k_depth(Tab<const float> srcs, int rows, int cols, size_t step_f, float fb,
                        Tab<float> dsts, size_t dstep_f) {
    const Grp p = pixel_group(rows, cols);
    if (p.n == 0) return;
    const float* __restrict__ src = srcs.p[blockIdx.z];
    float* __restrict__ d = dsts.p[blockIdx.z] + (size_t)p.y * dstep_f + p.x0;
    float v[OPS_PX];
    load4(src + (size_t)p.y * step_f + p.x0, p.n, v);
#pragma unroll
    for (int k = 0; k < OPS_PX; ++k) v[k] = (v[k] < 0.f || isinf(v[k])) ? 0.f : fb / v[k];
    if (p.n == OPS_PX && ((uintptr_t)d & 7) == 0) {
        reinterpret_cast<f2v*>(d)[0] = f2v{v[0], v[1]};
        reinterpret_cast<f2v*>(d)[1] = f2v{v[2], v[3]};
    } else {
        for (int k = 0; k < p.n; ++k) d[k] = v[k];
    }
}

// image coordinates of the group's first pixel: a dense map runs as one row of rows*cols
// pixels, wcols is the image width (= cols for a strided map, which has y = the row)
__device__ __forceinline__ void group_uv(const Grp& p, int wcols, int& u, int& v) {
    const int i = p.x0;  // dense: flat pixel index (y = 0)
    v = p.y + i / wcols;
    u = i - (i / wcols) * wcols;
}

__global__ void k_xyz(Tab<const float> srcs, int rows, int cols, size_t step_f, int wcols, float f,
                      float fb, float cx, float cy, Tab<float> dsts, size_t dstep_f) {
    const Grp p = pixel_group(rows, cols);
    if (p.n == 0) return;
    const float* __restrict__ src = srcs.p[blockIdx.z];
    float* __restrict__ d = dsts.p[blockIdx.z] + (size_t)p.y * dstep_f + 3 * (size_t)p.x0;
    float dv[OPS_PX];
    load4(src + (size_t)p.y * step_f + p.x0, p.n, dv);
    int u, v;
    group_uv(p, wcols, u, v);
    float o[3 * OPS_PX];
#pragma unroll
    for (int k = 0; k < OPS_PX; ++k) {
        o[3 * k] = o[3 * k + 1] = o[3 * k + 2] = 0.f;
        if (!(dv[k] < 0.f || isinf(dv[k]))) {
            const float Z = fb / dv[k];
            const float Zf = Z / f;
            o[3 * k] = ((float)u - cx) * Zf;
            o[3 * k + 1] = ((float)v - cy) * Zf;
            o[3 * k + 2] = Z;
        }
        if (++u == wcols) {  // next pixel: the row wraps (dense maps)
            u = 0;
            ++v;
        }
    }
    store4x3(d, p.n, o);
}

struct Q16 {
    float q[16];
};

__global__ void k_xyz_q(Tab<const float> srcs, int rows, int cols, size_t step_f, int wcols, Q16 Q,
                        Tab<float> dsts, size_t dstep_f) {
    const Grp p = pixel_group(rows, cols);
    if (p.n == 0) return;
    const float* __restrict__ src = srcs.p[blockIdx.z];
    float* __restrict__ d = dsts.p[blockIdx.z] + (size_t)p.y * dstep_f + 3 * (size_t)p.x0;
    float dv[OPS_PX];
    load4(src + (size_t)p.y * step_f + p.x0, p.n, dv);
    int u, v;
    group_uv(p, wcols, u, v);
    float o[3 * OPS_PX];
#pragma unroll
    for (int k = 0; k < OPS_PX; ++k) {
        const float pv[4] = {(float)u, (float)v, dv[k], 1.f};
        float r[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float sacc = 0.f;
#pragma unroll
            for (int j = 0; j < 4; ++j) sacc += Q.q[4 * i + j] * pv[j];
            r[i] = sacc;
        }
        o[3 * k] = r[0] / r[3];
        o[3 * k + 1] = r[1] / r[3];
        o[3 * k + 2] = r[2] / r[3];
        if (++u == wcols) {
            u = 0;
            ++v;
        }
    }
    store4x3(d, p.n, o);
}

// ---- f4 ---------------------------------------------------------------------------

// One source row's two taps (2*C bytes from byte x*C): a 12-B dword window at the
// aligned base, bytes picked by v_alignbyte; rows outside, or taps past either edge,
// read the border value 0 byte by byte.
template <int C>
__device__ __forceinline__ void row_taps(const uint8_t* __restrict__ src, int sh, int sw,
                                         size_t sstep, int sx, int sy, uint32_t (&b)[2 * C]) {
    if (sy < 0 || sy >= sh) {
#pragma unroll
        for (int i = 0; i < 2 * C; ++i) b[i] = 0;
        return;
    }
    const uint8_t* row = src + (size_t)sy * sstep;
    const long off = (long)sx * C;
    // the dword-aligned 12 B holding the taps (any row alignment), while they stay inside
    // the image's bytes (the last row's end is the buffer's)
    const uintptr_t pa = (uintptr_t)(row + off);
    const uintptr_t a = pa & ~(uintptr_t)3;
    if (sx >= 0 && sx + 1 < sw && a + 12 - (uintptr_t)src <= (size_t)(sh - 1) * sstep + (size_t)sw * C) {
        const uint32_t* w = reinterpret_cast<const uint32_t*>(a);
        const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
        const uint32_t sh8 = (uint32_t)(pa & 3) * 8;
        const uint32_t lo = __builtin_amdgcn_alignbit(w1, w0, sh8);
        const uint32_t hi = __builtin_amdgcn_alignbit(w2, w1, sh8);
#pragma unroll
        for (int i = 0; i < 2 * C; ++i) b[i] = ((i < 4 ? lo : hi) >> (8 * (i & 3))) & 0xffu;
        return;
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const int x = sx + t;
        const bool in = x >= 0 && x < sw;
#pragma unroll
        for (int c = 0; c < C; ++c) b[t * C + c] = in ? row[(size_t)x * C + c] : 0u;
    }
}

template <int C>
__device__ __forceinline__ void remap_px(const uint8_t* __restrict__ src, int sh, int sw, size_t sstep,
                                         int sx, int sy, int fx, int fy, uint32_t (&o)[C]) {
    const uint32_t w00 = (uint32_t)((32 - fx) * (32 - fy) * 32), w01 = (uint32_t)(fx * (32 - fy) * 32);
    const uint32_t w10 = (uint32_t)((32 - fx) * fy * 32), w11 = (uint32_t)(fx * fy * 32);
    uint32_t t0[2 * C], t1[2 * C];
    row_taps<C>(src, sh, sw, sstep, sx, sy, t0);
    row_taps<C>(src, sh, sw, sstep, sx, sy + 1, t1);
#pragma unroll
    for (int c = 0; c < C; ++c)
        o[c] = (__umul24(t0[c], w00) + __umul24(t0[C + c], w01) + __umul24(t1[c], w10) + __umul24(t1[C + c], w11) +
                (1u << 14)) >> 15;
}

template <int C>
__device__ __forceinline__ void store_px(uint8_t* d, int n, const uint32_t (&o)[OPS_PX][C]) {
    uint8_t bytes[OPS_PX * C];
#pragma unroll
    for (int k = 0; k < OPS_PX; ++k)
#pragma unroll
        for (int c = 0; c < C; ++c) bytes[k * C + c] = (uint8_t)o[k][c];
    if (n == OPS_PX && ((uintptr_t)d & 3) == 0) {  // 4*C bytes as C dwords
        uint32_t* d4 = reinterpret_cast<uint32_t*>(d);
#pragma unroll
        for (int i = 0; i < C; ++i)
            d4[i] = (uint32_t)bytes[4 * i] | ((uint32_t)bytes[4 * i + 1] << 8) |
                    ((uint32_t)bytes[4 * i + 2] << 16) | ((uint32_t)bytes[4 * i + 3] << 24);
    } else {
        for (int i = 0; i < n * C; ++i) d[i] = bytes[i];
    }
}

template <int C>
__global__ void k_remap_fixed(Tab<const uint8_t> srcs, int sh, int sw, size_t sstep,
                              const int16_t* __restrict__ xy, size_t xy_step_e,
                              const uint16_t* __restrict__ fxy, size_t fxy_step_e, int rows, int cols,
                              Tab<uint8_t> dsts, size_t dstep) {
    const Grp p = pixel_group(rows, cols);
    if (p.n == 0) return;
    const uint8_t* __restrict__ src = srcs.p[blockIdx.z];
    uint8_t* __restrict__ dst = dsts.p[blockIdx.z];
    const int n = p.n;
    // the group's map entries: 16 B of (x, y) pairs and 8 B of fractions, as two vector
    // loads when whole and aligned
    const int16_t* xr = xy + (size_t)p.y * xy_step_e + 2 * (size_t)p.x0;
    const uint16_t* fr = fxy + (size_t)p.y * fxy_step_e + p.x0;
    uint32_t mxy[OPS_PX], mf[OPS_PX];
    if (n == OPS_PX && ((uintptr_t)xr & 15) == 0 && ((uintptr_t)fr & 7) == 0) {
        const uint4 a = *reinterpret_cast<const uint4*>(xr);
        const uint2 b = *reinterpret_cast<const uint2*>(fr);
        mxy[0] = a.x; mxy[1] = a.y; mxy[2] = a.z; mxy[3] = a.w;
        mf[0] = b.x; mf[1] = b.x >> 16; mf[2] = b.y; mf[3] = b.y >> 16;
    } else {
#pragma unroll
        for (int k = 0; k < OPS_PX; ++k) {
            const int kk = k < n ? k : n - 1;
            mxy[k] = (uint32_t)(uint16_t)xr[2 * kk] | ((uint32_t)(uint16_t)xr[2 * kk + 1] << 16);
            mf[k] = fr[kk];
        }
    }
    uint32_t o[OPS_PX][C];
#pragma unroll
    for (int k = 0; k < OPS_PX; ++k) {
        const int sx = (int)(int16_t)(mxy[k] & 0xffffu);
        const int sy = (int)(int16_t)(mxy[k] >> 16);
        const int f = (int)(mf[k] & 1023u);
        remap_px<C>(src, sh, sw, sstep, sx, sy, f & 31, f >> 5, o[k]);
    }
    store_px<C>(dst + (size_t)p.y * dstep + (size_t)p.x0 * C, n, o);
}

// saturate_cast<int>(v * 32) = cvRound, x86: nearest-even, NaN / out of range -> INT_MIN
__device__ __forceinline__ int round32(float v) {
    const float a = v * 32.f;
    return (a >= -2147483648.0f && a < 2147483648.0f) ? (int)rintf(a) : (int)0x80000000u;
}

template <int C>
__global__ void k_remap_float(Tab<const uint8_t> srcs, int sh, int sw, size_t sstep,
                              const float* __restrict__ mapx, const float* __restrict__ mapy,
                              size_t map_step_f, int rows, int cols, Tab<uint8_t> dsts,
                              size_t dstep) {
    const Grp p = pixel_group(rows, cols);
    if (p.n == 0) return;
    const uint8_t* __restrict__ src = srcs.p[blockIdx.z];
    uint8_t* __restrict__ dst = dsts.p[blockIdx.z];
    const int n = p.n;
    uint32_t o[OPS_PX][C];
#pragma unroll
    for (int k = 0; k < OPS_PX; ++k) {
        const int x = min(p.x0 + k, cols - 1);
        const int ix = round32(mapx[(size_t)p.y * map_step_f + x]);
        const int iy = round32(mapy[(size_t)p.y * map_step_f + x]);
        const int sx = min(max(ix >> 5, -32768), 32767), sy = min(max(iy >> 5, -32768), 32767);
        remap_px<C>(src, sh, sw, sstep, sx, sy, ix & 31, iy & 31, o[k]);
    }
    store_px<C>(dst + (size_t)p.y * dstep + (size_t)p.x0 * C, n, o);
}

// Buffer form of the remap (sources whose bytes fit 31-bit offsets and row steps < 2^23, the
// usual case): one code path for every pixel, border taps included, no per-pixel branches.
//  * the taps of a row come from one 12-B window at the clamped column xw = clamp(sx, 0,
//    sw-2) of the clamped row, read through a buffer resource whose range check returns 0
//    for dwords past the image (no read leaves the buffer);
//  * a tap outside the image (BORDER_CONSTANT 0) gets weight 0 instead of a branch: the
//    vertical weights (32-fy, fy) of rows outside are 0, and the horizontal weights go to
//    the window slot that holds the tap's column (sx = -1: tap 1 in slot 0; sx = sw-1:
//    tap 0 in slot 1) or nowhere;
//  * per channel the two slots as 16-bit pairs (v_perm of the aligned window), the column
//    sums v = t0 * wy0 + t1 * wy1 <= 255 * 32 by packed 16-bit multiply-adds, then one
//    2-term dot product with the horizontal weights.  Exact: sum_ij t_ij w_ij * 32 + 2^14
//    >> 15 with w = (32-fx | fx) x (32-fy | fy) equals ((32-fx) v0 + fx v1 + 512) >> 10,
//    and with the horizontal weights scaled by 64 the result is byte 2 of the dot product.
//  * the last row's last windows read 12 B of which the tail dwords lie past num_records: the
//    form relies on the raw buffer range check being per dword (in-range dwords return their
//    data, the others 0), which gfx950 does (tests/test_gpu_stereo_ops.py
//    test_remap_last_row_end pins it on the box).  The library is built for gfx950 only; the
//    guard below stops a device compile for any target where that was not measured.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "k_remap_*_buf: per-dword buffer range checks are verified on gfx950 only"
#endif
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x3v __attribute__((ext_vector_type(3)));

struct RemapSrc {
    __amdgpu_buffer_rsrc_t r;  // the image's bytes, from the dword holding its first byte
    uint32_t mis;              // offset of the first byte in that dword
};
__device__ __forceinline__ RemapSrc remap_src(const uint8_t* p, uint32_t nbytes) {
    const uintptr_t u = (uintptr_t)p;
    const uint32_t mis = (uint32_t)u & 3u;
    // the dword-rounded range stays in the allocation's last page
    return RemapSrc{__builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p - mis), (short)0,
                                                     (int)((nbytes + mis + 3u) & ~3u), 0x00020000),
                    mis};
}

// One pixel's taps, independent of the image (a group of images shares the maps): the two
// rows' window offsets (without the image's misalignment) and the packed weights.
struct RemapTap {
    uint32_t oa, ob;
    u16x2 vya, vyb, wx;
};
// IN: the caller knows every tap of the pixel is inside the image and not in the last row
// (a wave-uniform test over its lanes' pixels): no clamps, no weight selection.
template <int C, bool IN>
__device__ __forceinline__ RemapTap remap_tap(uint32_t sstep, int sh, int sw, int sx, int sy, int fx, int fy) {
    const int xw = IN ? sx : max(0, min(sx, sw - 2));
    const int ya = IN ? sy : min(max(sy, 0), sh - 1), yb = IN ? sy + 1 : min(max(sy + 1, 0), sh - 1);
    const uint32_t cb = __umul24((uint32_t)xw, (uint32_t)C);
    RemapTap T;
    T.oa = __umul24((uint32_t)ya, sstep) + cb;
    T.ob = IN ? T.oa + sstep : __umul24((uint32_t)yb, sstep) + cb;
    // weights of the two window slots and the two rows (0 for taps outside the image)
    uint32_t ws0, ws1, wa, wb;
    if constexpr (IN) {
        ws0 = (uint32_t)(32 - fx), ws1 = (uint32_t)fx, wa = (uint32_t)(32 - fy), wb = (uint32_t)fy;
    } else {
        const int d = sx - xw;  // window slot of tap 0 (tap 1 is in slot d + 1)
        const bool in0 = (sx >= 0) & (sx < sw), in1 = (sx >= -1) & (sx + 1 < sw);
        const uint32_t w0 = (uint32_t)(32 - fx), w1 = (uint32_t)fx;
        ws0 = ((in0 & (d == 0)) ? w0 : 0u) + ((in1 & (d == -1)) ? w1 : 0u);
        ws1 = ((in0 & (d == 1)) ? w0 : 0u) + ((in1 & (d == 0)) ? w1 : 0u);
        wa = ((sy >= 0) & (sy < sh)) ? (uint32_t)(32 - fy) : 0u;
        wb = ((sy >= -1) & (sy + 1 < sh)) ? (uint32_t)fy : 0u;
    }
    T.vya = __builtin_bit_cast(u16x2, wa | (wa << 16));
    T.vyb = __builtin_bit_cast(u16x2, wb | (wb << 16));
    T.wx = __builtin_bit_cast(u16x2, (ws0 << 6) | (ws1 << 22));
    return T;
}

// the pixel of one image: its two windows, the channels' column sums and dot products
template <int C>
__device__ __forceinline__ uint32_t remap_apply(const RemapSrc& S, const RemapTap& T) {
    const uint32_t oa = T.oa + S.mis, ob = T.ob + S.mis;
    const u32x3v ra = __builtin_amdgcn_raw_buffer_load_b96(S.r, oa & ~3u, 0, 0);
    const u32x3v rb = __builtin_amdgcn_raw_buffer_load_b96(S.r, ob & ~3u, 0, 0);
    const uint32_t sa = (oa & 3u) * 8u, sb = (ob & 3u) * 8u;
    const uint32_t loa = __builtin_amdgcn_alignbit(ra.y, ra.x, sa), hia = __builtin_amdgcn_alignbit(ra.z, ra.y, sa);
    const uint32_t lob = __builtin_amdgcn_alignbit(rb.y, rb.x, sb), hib = __builtin_amdgcn_alignbit(rb.z, rb.y, sb);
    uint32_t dc[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
        // [slot 0 byte c, 0, slot 1 byte C + c, 0]: pool bytes 0-3 = lo, 4-7 = hi
        constexpr uint32_t z = 0x0c;
        const uint32_t sel = (uint32_t)c | (z << 8) | ((uint32_t)(C + c) << 16) | (z << 24);
        const u16x2 ta = __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(hia, loa, sel));
        const u16x2 tb = __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(hib, lob, sel));
        const u16x2 v = ta * T.vya + tb * T.vyb;
        dc[c] = __builtin_amdgcn_udot2(v, T.wx, 512u << 6, false);
    }
    // the channels' byte 2s as one packed pixel
    if constexpr (C == 1) return dc[0] >> 16;
    const uint32_t p01 = __builtin_amdgcn_perm(dc[1], dc[0], 0x0c0c0602u);
    if constexpr (C == 3) return (dc[2] & 0xff0000u) | p01;
    return p01 | __builtin_amdgcn_perm(dc[3], dc[2], 0x06020c0cu);
}

// 4 packed pixels of C bytes at d: C dwords when whole and aligned
template <int C>
__device__ __forceinline__ void store_packed(uint8_t* d, int n, const uint32_t (&px)[OPS_PX]) {
    uint32_t w[C];
    if constexpr (C == 1) {
        w[0] = px[0] | (px[1] << 8) | (px[2] << 16) | (px[3] << 24);
    } else if constexpr (C == 3) {
        w[0] = px[0] | (px[1] << 24);
        w[1] = (px[1] >> 8) | (px[2] << 16);
        w[2] = (px[2] >> 16) | (px[3] << 8);
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) w[k] = px[k];
    }
    if (n == OPS_PX && ((uintptr_t)d & 3) == 0) {
        uint32_t* d4 = reinterpret_cast<uint32_t*>(d);
#pragma unroll
        for (int i = 0; i < C; ++i) d4[i] = w[i];
    } else {
        for (int i = 0; i < n * C; ++i) d[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
    }
}

// blockIdx.z: a run of MI images of the call (nimg in all); a lane's taps serve all of them
template <int C, int MI>
__global__ __launch_bounds__(OPS_THREADS) void k_remap_fixed_buf(Tab<const uint8_t> srcs, int nimg, int sh, int sw,
                                                                 uint32_t sstep, uint32_t nbytes,
                                                                 const int16_t* __restrict__ xy, size_t xy_step_e,
                                                                 const uint16_t* __restrict__ fxy, size_t fxy_step_e,
                                                                 int rows, int cols, Tab<uint8_t> dsts, size_t dstep) {
    const Grp p = pixel_group(rows, cols);
    if (p.n == 0) return;
    const int n = p.n;
    const int16_t* xr = xy + (size_t)p.y * xy_step_e + 2 * (size_t)p.x0;
    const uint16_t* fr = fxy + (size_t)p.y * fxy_step_e + p.x0;
    uint32_t mxy[OPS_PX], mf[OPS_PX];
    if (n == OPS_PX && ((uintptr_t)xr & 15) == 0 && ((uintptr_t)fr & 7) == 0) {
        const uint4 a = *reinterpret_cast<const uint4*>(xr);
        const uint2 b = *reinterpret_cast<const uint2*>(fr);
        mxy[0] = a.x; mxy[1] = a.y; mxy[2] = a.z; mxy[3] = a.w;
        mf[0] = b.x; mf[1] = b.x >> 16; mf[2] = b.y; mf[3] = b.y >> 16;
    } else {
#pragma unroll
        for (int k = 0; k < OPS_PX; ++k) {
            const int kk = k < n ? k : n - 1;
            mxy[k] = (uint32_t)(uint16_t)xr[2 * kk] | ((uint32_t)(uint16_t)xr[2 * kk + 1] << 16);
            mf[k] = fr[kk];
        }
    }
    RemapTap T[OPS_PX];
    auto taps = [&](auto INc) {
#pragma unroll
        for (int k = 0; k < OPS_PX; ++k) {
            const int f = (int)(mf[k] & 1023u);
            T[k] = remap_tap<C, decltype(INc)::value>(sstep, sh, sw, (int)(int16_t)(mxy[k] & 0xffffu),
                                                     (int)(int16_t)(mxy[k] >> 16), f & 31, f >> 5);
        }
    };
    bool in = true;
#pragma unroll
    for (int k = 0; k < OPS_PX; ++k) {
        const int sx = (int)(int16_t)(mxy[k] & 0xffffu), sy = (int)(int16_t)(mxy[k] >> 16);
        in = in & (sx >= 0) & (sx <= sw - 2) & (sy >= 0) & (sy <= sh - 3);
    }
    if (__builtin_amdgcn_ballot_w64(!in) == 0) taps(std::true_type{});
    else taps(std::false_type{});
    const int i0 = (int)blockIdx.z * MI;
    auto image = [&](int i) {
        const RemapSrc S = remap_src(srcs.p[i], nbytes);
        uint32_t px[OPS_PX];
#pragma unroll
        for (int k = 0; k < OPS_PX; ++k) px[k] = remap_apply<C>(S, T[k]);
        store_packed<C>(dsts.p[i] + (size_t)p.y * dstep + (size_t)p.x0 * C, n, px);
    };
    if (i0 + MI <= nimg) {  // a whole run: no per-image guards between the images' loads
#pragma unroll
        for (int m = 0; m < MI; ++m) image(i0 + m);
    } else {
        for (int i = i0; i < nimg; ++i) image(i);
    }
}

template <int C>
__global__ __launch_bounds__(OPS_THREADS) void k_remap_float_buf(Tab<const uint8_t> srcs, int sh, int sw, uint32_t sstep,
                                                                 uint32_t nbytes, const float* __restrict__ mapx,
                                                                 const float* __restrict__ mapy, size_t map_step_f,
                                                                 int rows, int cols, Tab<uint8_t> dsts, size_t dstep) {
    const Grp p = pixel_group(rows, cols);
    if (p.n == 0) return;
    const RemapSrc S = remap_src(srcs.p[blockIdx.z], nbytes);
    int sx[OPS_PX], sy[OPS_PX], fx[OPS_PX], fy[OPS_PX];
    bool in = true;
#pragma unroll
    for (int k = 0; k < OPS_PX; ++k) {
        const int x = min(p.x0 + k, cols - 1);
        const int ix = round32(mapx[(size_t)p.y * map_step_f + x]);
        const int iy = round32(mapy[(size_t)p.y * map_step_f + x]);
        sx[k] = min(max(ix >> 5, -32768), 32767), sy[k] = min(max(iy >> 5, -32768), 32767);
        fx[k] = ix & 31, fy[k] = iy & 31;
        in = in & (sx[k] >= 0) & (sx[k] <= sw - 2) & (sy[k] >= 0) & (sy[k] <= sh - 3);
    }
    RemapTap T[OPS_PX];
    auto taps = [&](auto INc) {
#pragma unroll
        for (int k = 0; k < OPS_PX; ++k)
            T[k] = remap_tap<C, decltype(INc)::value>(sstep, sh, sw, sx[k], sy[k], fx[k], fy[k]);
    };
    if (__builtin_amdgcn_ballot_w64(!in) == 0) taps(std::true_type{});
    else taps(std::false_type{});
    uint32_t px[OPS_PX];
#pragma unroll
    for (int k = 0; k < OPS_PX; ++k) px[k] = remap_apply<C>(S, T[k]);
    store_packed<C>(dsts.p[blockIdx.z] + (size_t)p.y * dstep + (size_t)p.x0 * C, p.n, px);
}

// the buffer form's limits: every source byte at a 31-bit offset, 24-bit row products
static bool remap_buf_ok(int src_rows, int src_cols, size_t src_step, int C) {
    const size_t bytes = (size_t)(src_rows - 1) * src_step + (size_t)src_cols * C;
    return src_step < (1u << 23) && src_rows < (1 << 23) && bytes + 16 < 0x7fffffffu;
}

// ---- host side --------------------------------------------------------------------

// the flattened (row, pixel group) grid of pixel_group(), n maps
dim3 row_blocks(int rows, int cols, int n = 1) {
    const long groups = (long)rows * ((cols + OPS_PX - 1) / OPS_PX);
    return dim3((unsigned)((groups + OPS_THREADS - 1) / OPS_THREADS), 1, n);
}

// A map whose rows are packed (step = row bytes, input and output) runs as one row of
// rows * cols pixels: rows -> 1, cols -> rows * cols (the f3 kernels keep the true width
// for the pixel coordinates).
struct Shape {
    int rows, cols;
};
Shape dense_shape(int rows, int cols, size_t step, size_t in_bpp, size_t out_step, size_t out_bpp) {
    if (step == in_bpp * cols && out_step == out_bpp * cols && (long)rows * cols <= 0x7fffffffL)
        return Shape{1, rows * cols};
    return Shape{rows, cols};
}

template <class T, class U>
Tab<T> tab_of(const U* const* ptrs, int n) {
    Tab<T> t{};
    for (int i = 0; i < n; ++i) t.p[i] = const_cast<T*>(reinterpret_cast<const T*>(ptrs[i]));
    return t;
}
template <class T, class U>
Tab<T> tab_one(U* p) {
    Tab<T> t{};
    t.p[0] = const_cast<T*>(reinterpret_cast<const T*>(p));
    return t;
}
bool null_in(const void* const* ptrs, int n) {
    if (!ptrs) return true;
    for (int i = 0; i < n; ++i)
        if (!ptrs[i]) return true;
    return false;
}

bool bad_dims(int rows, int cols) { return rows <= 0 || cols <= 0; }

Lut make_lut(const uint8_t* lut768) {
    uint8_t jet[768];
    if (!lut768) {
        tsm_jet_colormap(jet);
        lut768 = jet;
    }
    Lut L;
    for (int i = 0; i < 256; ++i)
        L.bgr[i] = lut768[3 * i] | ((uint32_t)lut768[3 * i + 1] << 8) | ((uint32_t)lut768[3 * i + 2] << 16);
    return L;
}

// RAII device buffer for the host forms
struct DevBuf {
    void* p = nullptr;
    hipError_t e = hipSuccess;
    explicit DevBuf(size_t n) { e = hipMalloc(&p, n ? n : 1); }
    ~DevBuf() { if (p) (void)hipFree(p); }
};

int status(hipError_t e) {
    if (e == hipSuccess) return TSM_OK;
    return e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation ? TSM_ERR_OUT_OF_MEMORY : TSM_ERR_DEVICE;
}

int device_ok() {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess && n > 0;
}

// host form helper: upload `in` (rows of in_row bytes at in_step), run `op` on the dense
// device copies, download `out` rows of out_row bytes to out_step
template <class Op>
int host_form(const void* in, size_t in_row, size_t in_step, int rows, void* out, size_t out_row,
              size_t out_step, Op op) {
    if (!device_ok()) return TSM_ERR_DEVICE;
    DevBuf di(in_row * rows), dout(out_row * rows);
    if (di.e != hipSuccess) return status(di.e);
    if (dout.e != hipSuccess) return status(dout.e);
    hipError_t e = hipMemcpy2D(di.p, in_row, in, in_step, in_row, rows, hipMemcpyHostToDevice);
    if (e != hipSuccess) return status(e);
    int rc = op(di.p, in_row, dout.p, out_row);
    if (rc != TSM_OK) return rc;
    e = hipMemcpy2D(out, out_step, dout.p, out_row, out_row, rows, hipMemcpyDeviceToHost);
    return status(e);
}


// [0, 2 kOpsBatch): folded (min, max) per map; then MM_BLOCKS partial pairs per map
constexpr size_t MM_SCRATCH_BYTES = (size_t)(2 * kOpsBatch + 2 * MM_BLOCKS * kOpsBatch) * 4;

// the min/max scratch of the _device form: one buffer per (device, stream), kept for the
// process lifetime (launches on one stream are ordered, so reuse is safe)
uint32_t* stream_scratch(void* stream) {
    static std::mutex mu;
    static std::map<std::pair<int, void*>, void*> bufs;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    void*& p = bufs[{dev, stream}];
    if (!p && hipMalloc(&p, MM_SCRATCH_BYTES) != hipSuccess) p = nullptr;
    return (uint32_t*)p;
}

// nm maps (<= kOpsBatch) of one size; the min/max scratch holds every map's folds
int colormap_launch(const Tab<const float>& src, int nm, int rows, int cols, size_t step, const uint8_t* lut768,
                    int use_range, float min_val, float max_val, const Tab<uint8_t>& dst, size_t out_step,
                    uint32_t* scratch, hipStream_t st) {
    const Lut L = make_lut(lut768);
    uint32_t* mm = scratch;
    const Shape sh = dense_shape(rows, cols, step, 4, out_step, 3);
    if (!use_range) {
        const long groups = (long)rows * ((cols + OPS_PX - 1) / OPS_PX);
        // about 2048 partial blocks a launch (8 a CU), at most MM_BLOCKS per map
        const int per_map = min(MM_BLOCKS, max(8, 2048 / nm));
        const int blocks = (int)min((groups + OPS_THREADS - 1) / OPS_THREADS, (long)per_map);
        hipLaunchKernelGGL(k_minmax, dim3(blocks, 1, nm), dim3(OPS_THREADS), 0, st, src, sh.rows, sh.cols,
                           step / 4, mm + 2 * kOpsBatch);
        hipLaunchKernelGGL(k_minmax_final, dim3(1, 1, nm), dim3(1024), 0, st, mm + 2 * kOpsBatch, blocks, mm);
    }
    hipLaunchKernelGGL(k_colormap, row_blocks(sh.rows, sh.cols, nm), dim3(OPS_THREADS), 0, st, src, sh.rows,
                       sh.cols, step / 4, mm, use_range, min_val, max_val, L, dst, out_step);
    return status(hipGetLastError());
}

}  // namespace
}  // namespace tsm

using namespace tsm;

extern "C" {

int tsm_stream_synchronize(void* hip_stream) {
    return status(hipStreamSynchronize((hipStream_t)hip_stream));
}

int tsm_jet_colormap(uint8_t* lut) {
    if (!lut) return TSM_ERR_ARGUMENT;
    auto set = [&](int i, int b, int g, int r) {
        lut[3 * i] = (uint8_t)b;
        lut[3 * i + 1] = (uint8_t)g;
        lut[3 * i + 2] = (uint8_t)r;
    };
    for (int i = 0; i < 32; ++i) set(i, 128 + 4 * i, 0, 0);
    set(32, 255, 0, 0);
    for (int i = 0; i < 63; ++i) set(33 + i, 255, 4 + 4 * i, 0);
    set(96, 254, 255, 2);
    for (int i = 0; i < 62; ++i) set(97 + i, 250 - 4 * i, 255, 6 + 4 * i);
    set(159, 1, 255, 254);
    for (int i = 0; i < 64; ++i) set(160 + i, 0, 252 - 4 * i, 255);
    for (int i = 0; i < 32; ++i) set(224 + i, 0, 0, 252 - 4 * i);
    return TSM_OK;
}

int tsm_apply_colormap_device(const float* d_disp, int rows, int cols, size_t step, const uint8_t* lut768,
                              int use_range, float min_val, float max_val, uint8_t* d_bgr,
                              size_t out_step, void* hip_stream) {
    if (!d_disp || !d_bgr || bad_dims(rows, cols) || step % 4 || step < 4 * (size_t)cols ||
        out_step < 3 * (size_t)cols)
        return TSM_ERR_ARGUMENT;
    uint32_t* scratch = nullptr;
    if (!use_range) {
        scratch = stream_scratch(hip_stream);
        if (!scratch) return TSM_ERR_OUT_OF_MEMORY;
    }
    return colormap_launch(tab_one<const float>(d_disp), 1, rows, cols, step, lut768, use_range, min_val, max_val,
                           tab_one<uint8_t>(d_bgr), out_step, scratch, (hipStream_t)hip_stream);
}

int tsm_apply_colormap_batch_device(int n, const float* const* d_disps, int rows, int cols, size_t step,
                                    const uint8_t* lut768, int use_range, float min_val, float max_val,
                                    uint8_t* const* d_bgrs, size_t out_step, void* hip_stream) {
    if (n < 0 || (n > 0 && (null_in((const void* const*)d_disps, n) || null_in((const void* const*)d_bgrs, n))) ||
        bad_dims(rows, cols) || step % 4 || step < 4 * (size_t)cols || out_step < 3 * (size_t)cols)
        return TSM_ERR_ARGUMENT;
    uint32_t* scratch = nullptr;
    if (!use_range && n > 0) {
        scratch = stream_scratch(hip_stream);
        if (!scratch) return TSM_ERR_OUT_OF_MEMORY;
    }
    for (int i = 0; i < n; i += kOpsBatch) {  // the scratch is reused chunk after chunk (stream order)
        const int k = min(kOpsBatch, n - i);
        const int rc = colormap_launch(tab_of<const float>(d_disps + i, k), k, rows, cols, step, lut768, use_range,
                                       min_val, max_val, tab_of<uint8_t>(d_bgrs + i, k), out_step, scratch,
                                       (hipStream_t)hip_stream);
        if (rc != TSM_OK) return rc;
    }
    return TSM_OK;
}

int tsm_apply_colormap(const float* disp, int rows, int cols, size_t step, const uint8_t* lut768,
                       int use_range, float min_val, float max_val, uint8_t* bgr, size_t out_step) {
    if (!disp || !bgr || bad_dims(rows, cols) || step < 4 * (size_t)cols || out_step < 3 * (size_t)cols)
        return TSM_ERR_ARGUMENT;
    if (!device_ok()) return TSM_ERR_DEVICE;
    DevBuf scratch(MM_SCRATCH_BYTES);
    if (scratch.e != hipSuccess) return status(scratch.e);
    return host_form(disp, 4 * (size_t)cols, step, rows, bgr, 3 * (size_t)cols, out_step,
                     [&](void* di, size_t is, void* dout, size_t os) {
                         int rc = colormap_launch(tab_one<const float>(di), 1, rows, cols, is, lut768, use_range,
                                                  min_val, max_val, tab_one<uint8_t>(dout), os,
                                                  (uint32_t*)scratch.p, nullptr);
                         return rc != TSM_OK ? rc : status(hipDeviceSynchronize());
                     });
}

int tsm_reproject_to_depth_device(const float* d_disp, int rows, int cols, size_t step, float focal,
                                  float baseline, float* d_depth, size_t out_step, void* hip_stream) {
    if (!d_disp || !d_depth || bad_dims(rows, cols) || step % 4 || out_step % 4 ||
        step < 4 * (size_t)cols || out_step < 4 * (size_t)cols)
        return TSM_ERR_ARGUMENT;
    return tsm_reproject_to_depth_batch_device(1, &d_disp, rows, cols, step, focal, baseline, &d_depth, out_step,
                                               hip_stream);
}

int tsm_reproject_to_depth_batch_device(int n, const float* const* d_disps, int rows, int cols, size_t step,
                                        float focal, float baseline, float* const* d_depths, size_t out_step,
                                        void* hip_stream) {
    if (n < 0 || (n > 0 && (null_in((const void* const*)d_disps, n) || null_in((const void* const*)d_depths, n))) ||
        bad_dims(rows, cols) || step % 4 || out_step % 4 || step < 4 * (size_t)cols || out_step < 4 * (size_t)cols)
        return TSM_ERR_ARGUMENT;
    const Shape sh = dense_shape(rows, cols, step, 4, out_step, 4);
    for (int i = 0; i < n; i += kOpsBatch) {
        const int k = min(kOpsBatch, n - i);
        hipLaunchKernelGGL(k_depth, row_blocks(sh.rows, sh.cols, k), dim3(OPS_THREADS), 0, (hipStream_t)hip_stream,
                           tab_of<const float>(d_disps + i, k), sh.rows, sh.cols, step / 4, focal * baseline,
                           tab_of<float>(d_depths + i, k), out_step / 4);
    }
    return status(hipGetLastError());
}

int tsm_reproject_to_depth(const float* disp, int rows, int cols, size_t step, float focal,
                           float baseline, float* depth, size_t out_step) {
    if (!disp || !depth || bad_dims(rows, cols) || step < 4 * (size_t)cols || out_step < 4 * (size_t)cols)
        return TSM_ERR_ARGUMENT;
    return host_form(disp, 4 * (size_t)cols, step, rows, depth, 4 * (size_t)cols, out_step,
                     [&](void* di, size_t is, void* dout, size_t os) {
                         int rc = tsm_reproject_to_depth_device((const float*)di, rows, cols, is, focal,
                                                                baseline, (float*)dout, os, nullptr);
                         return rc != TSM_OK ? rc : status(hipDeviceSynchronize());
                     });
}

int tsm_reproject_to_3d_device(const float* d_disp, int rows, int cols, size_t step, float focal,
                               float baseline, float cx, float cy, float* d_xyz, size_t out_step,
                               void* hip_stream) {
    if (!d_disp || !d_xyz || bad_dims(rows, cols) || step % 4 || out_step % 4 ||
        step < 4 * (size_t)cols || out_step < 12 * (size_t)cols)
        return TSM_ERR_ARGUMENT;
    return tsm_reproject_to_3d_batch_device(1, &d_disp, rows, cols, step, focal, baseline, cx, cy, &d_xyz,
                                            out_step, hip_stream);
}

int tsm_reproject_to_3d_batch_device(int n, const float* const* d_disps, int rows, int cols, size_t step,
                                     float focal, float baseline, float cx, float cy, float* const* d_xyzs,
                                     size_t out_step, void* hip_stream) {
    if (n < 0 || (n > 0 && (null_in((const void* const*)d_disps, n) || null_in((const void* const*)d_xyzs, n))) ||
        bad_dims(rows, cols) || step % 4 || out_step % 4 || step < 4 * (size_t)cols || out_step < 12 * (size_t)cols)
        return TSM_ERR_ARGUMENT;
    const Shape sh = dense_shape(rows, cols, step, 4, out_step, 12);
    for (int i = 0; i < n; i += kOpsBatch) {
        const int k = min(kOpsBatch, n - i);
        hipLaunchKernelGGL(k_xyz, row_blocks(sh.rows, sh.cols, k), dim3(OPS_THREADS), 0, (hipStream_t)hip_stream,
                           tab_of<const float>(d_disps + i, k), sh.rows, sh.cols, step / 4, cols, focal,
                           focal * baseline, cx, cy, tab_of<float>(d_xyzs + i, k), out_step / 4);
    }
    return status(hipGetLastError());
}

int tsm_reproject_to_3d(const float* disp, int rows, int cols, size_t step, float focal,
                        float baseline, float cx, float cy, float* xyz, size_t out_step) {
    if (!disp || !xyz || bad_dims(rows, cols) || step < 4 * (size_t)cols || out_step < 12 * (size_t)cols)
        return TSM_ERR_ARGUMENT;
    return host_form(disp, 4 * (size_t)cols, step, rows, xyz, 12 * (size_t)cols, out_step,
                     [&](void* di, size_t is, void* dout, size_t os) {
                         int rc = tsm_reproject_to_3d_device((const float*)di, rows, cols, is, focal, baseline,
                                                             cx, cy, (float*)dout, os, nullptr);
                         return rc != TSM_OK ? rc : status(hipDeviceSynchronize());
                     });
}

int tsm_reproject_to_3d_q_device(const float* d_disp, int rows, int cols, size_t step,
                                 const double* q16, float* d_xyz, size_t out_step, void* hip_stream) {
    if (!d_disp || !d_xyz || !q16 || bad_dims(rows, cols) || step % 4 || out_step % 4 ||
        step < 4 * (size_t)cols || out_step < 12 * (size_t)cols)
        return TSM_ERR_ARGUMENT;
    Q16 Q;
    for (int i = 0; i < 16; ++i) Q.q[i] = (float)q16[i];  // Q.convertTo(CV_32F), stereo.cpp:190
    const Shape sh = dense_shape(rows, cols, step, 4, out_step, 12);
    hipLaunchKernelGGL(k_xyz_q, row_blocks(sh.rows, sh.cols), dim3(OPS_THREADS), 0, (hipStream_t)hip_stream,
                       tab_one<const float>(d_disp), sh.rows, sh.cols, step / 4, cols, Q, tab_one<float>(d_xyz),
                       out_step / 4);
    return status(hipGetLastError());
}

int tsm_reproject_to_3d_q(const float* disp, int rows, int cols, size_t step, const double* q16,
                          float* xyz, size_t out_step) {
    if (!disp || !xyz || !q16 || bad_dims(rows, cols) || step < 4 * (size_t)cols || out_step < 12 * (size_t)cols)
        return TSM_ERR_ARGUMENT;
    return host_form(disp, 4 * (size_t)cols, step, rows, xyz, 12 * (size_t)cols, out_step,
                     [&](void* di, size_t is, void* dout, size_t os) {
                         int rc = tsm_reproject_to_3d_q_device((const float*)di, rows, cols, is, q16,
                                                               (float*)dout, os, nullptr);
                         return rc != TSM_OK ? rc : status(hipDeviceSynchronize());
                     });
}

int tsm_remap_linear_fixed_device(const uint8_t* d_src, int src_rows, int src_cols, size_t src_step,
                                  int channels, const int16_t* d_xy, size_t xy_step,
                                  const uint16_t* d_fxy, size_t fxy_step, int rows, int cols,
                                  uint8_t* d_dst, size_t dst_step, void* hip_stream) {
    const int C = channels;
    if (!d_src || !d_xy || !d_fxy || !d_dst || bad_dims(rows, cols) || bad_dims(src_rows, src_cols) ||
        (C != 1 && C != 3 && C != 4) || src_step < (size_t)C * src_cols || xy_step % 2 || fxy_step % 2 ||
        xy_step < 4 * (size_t)cols || fxy_step < 2 * (size_t)cols || dst_step < (size_t)C * cols)
        return TSM_ERR_ARGUMENT;
    return tsm_remap_linear_fixed_batch_device(1, &d_src, src_rows, src_cols, src_step, C, d_xy, xy_step, d_fxy,
                                               fxy_step, rows, cols, &d_dst, dst_step, hip_stream);
}

int tsm_remap_linear_fixed_batch_device(int n, const uint8_t* const* d_srcs, int src_rows, int src_cols,
                                        size_t src_step, int channels, const int16_t* d_xy, size_t xy_step,
                                        const uint16_t* d_fxy, size_t fxy_step, int rows, int cols,
                                        uint8_t* const* d_dsts, size_t dst_step, void* hip_stream) {
    const int C = channels;
    if (n < 0 || (n > 0 && (null_in((const void* const*)d_srcs, n) || null_in((const void* const*)d_dsts, n))) ||
        !d_xy || !d_fxy || bad_dims(rows, cols) || bad_dims(src_rows, src_cols) ||
        (C != 1 && C != 3 && C != 4) || src_step < (size_t)C * src_cols || xy_step % 2 || fxy_step % 2 ||
        xy_step < 4 * (size_t)cols || fxy_step < 2 * (size_t)cols || dst_step < (size_t)C * cols)
        return TSM_ERR_ARGUMENT;
    hipStream_t st = (hipStream_t)hip_stream;
    // packed maps and output run as one row (the source is addressed through the maps)
    const bool dense = xy_step == 4 * (size_t)cols && fxy_step == 2 * (size_t)cols && dst_step == (size_t)C * cols &&
                       (long)rows * cols <= 0x7fffffffL;
    const int rr = dense ? 1 : rows, cc = dense ? rows * cols : cols;
    const bool buf = remap_buf_ok(src_rows, src_cols, src_step, C);
    // images a lane: their taps (offsets, weights, border handling) are computed once for the
    // run (measured, 64 maps of 1242x375: 1 -> 72 us a call, 2 -> 58, 4 -> 53, 8 -> 53)
    const int mi = n >= 4 ? 4 : (n >= 2 ? 2 : 1);
    for (int i = 0; i < n; i += kOpsBatch) {
        const int k = min(kOpsBatch, n - i);
        const dim3 g = row_blocks(rr, cc, k);
        const Tab<const uint8_t> s = tab_of<const uint8_t>(d_srcs + i, k);
        const Tab<uint8_t> d = tab_of<uint8_t>(d_dsts + i, k);
        const uint32_t nb = (uint32_t)((size_t)(src_rows - 1) * src_step + (size_t)src_cols * C);
#define TSM_REMAP_BUF(CC, M)                                                                                      \
        hipLaunchKernelGGL((k_remap_fixed_buf<CC, M>), row_blocks(rr, cc, (k + M - 1) / M), dim3(OPS_THREADS), 0, st, \
                           s, k, src_rows, src_cols, (uint32_t)src_step, nb, d_xy, xy_step / 2, d_fxy, fxy_step / 2,  \
                           rr, cc, d, dst_step)
#define TSM_REMAP_FIXED(CC)                                                                                       \
        if (buf && mi == 4) TSM_REMAP_BUF(CC, 4);                                                                 \
        else if (buf && mi == 2) TSM_REMAP_BUF(CC, 2);                                                            \
        else if (buf) TSM_REMAP_BUF(CC, 1);                                                                       \
        else                                                                                                      \
            hipLaunchKernelGGL(k_remap_fixed<CC>, g, dim3(OPS_THREADS), 0, st, s, src_rows, src_cols, src_step,   \
                               d_xy, xy_step / 2, d_fxy, fxy_step / 2, rr, cc, d, dst_step)
        if (C == 1) TSM_REMAP_FIXED(1);
        else if (C == 3) TSM_REMAP_FIXED(3);
        else TSM_REMAP_FIXED(4);
#undef TSM_REMAP_FIXED
#undef TSM_REMAP_BUF
    }
    return status(hipGetLastError());
}

int tsm_remap_linear_float_device(const uint8_t* d_src, int src_rows, int src_cols, size_t src_step,
                                  int channels, const float* d_mapx, const float* d_mapy,
                                  size_t map_step, int rows, int cols, uint8_t* d_dst,
                                  size_t dst_step, void* hip_stream) {
    const int C = channels;
    if (!d_src || !d_mapx || !d_mapy || !d_dst || bad_dims(rows, cols) || bad_dims(src_rows, src_cols) ||
        (C != 1 && C != 3 && C != 4) || src_step < (size_t)C * src_cols || map_step % 4 ||
        map_step < 4 * (size_t)cols || dst_step < (size_t)C * cols)
        return TSM_ERR_ARGUMENT;
    hipStream_t st = (hipStream_t)hip_stream;
    const dim3 g = row_blocks(rows, cols);
    const Tab<const uint8_t> s = tab_one<const uint8_t>(d_src);
    const Tab<uint8_t> d = tab_one<uint8_t>(d_dst);
    const bool buf = remap_buf_ok(src_rows, src_cols, src_step, C);
    const uint32_t nb = (uint32_t)((size_t)(src_rows - 1) * src_step + (size_t)src_cols * C);
#define TSM_REMAP_FLOAT(CC)                                                                                     \
    if (buf)                                                                                                    \
        hipLaunchKernelGGL(k_remap_float_buf<CC>, g, dim3(OPS_THREADS), 0, st, s, src_rows, src_cols,           \
                           (uint32_t)src_step, nb, d_mapx, d_mapy, map_step / 4, rows, cols, d, dst_step);      \
    else                                                                                                        \
        hipLaunchKernelGGL(k_remap_float<CC>, g, dim3(OPS_THREADS), 0, st, s, src_rows, src_cols, src_step,     \
                           d_mapx, d_mapy, map_step / 4, rows, cols, d, dst_step)
    if (C == 1) TSM_REMAP_FLOAT(1);
    else if (C == 3) TSM_REMAP_FLOAT(3);
    else TSM_REMAP_FLOAT(4);
#undef TSM_REMAP_FLOAT
    return status(hipGetLastError());
}

// host forms of the remap: three inputs (image, two maps), one output
static int remap_host(const uint8_t* src, int src_rows, int src_cols, size_t src_step, int C,
                      const void* m1, size_t m1_row, size_t m1_step, const void* m2, size_t m2_row,
                      size_t m2_step, int rows, int cols, uint8_t* dst, size_t dst_step, bool fixed) {
    if (!device_ok()) return TSM_ERR_DEVICE;
    const size_t srow = (size_t)C * src_cols, drow = (size_t)C * cols;
    DevBuf ds(srow * src_rows), d1(m1_row * rows), d2(m2_row * rows), dd(drow * rows);
    for (DevBuf* b : {&ds, &d1, &d2, &dd})
        if (b->e != hipSuccess) return status(b->e);
    hipError_t e = hipMemcpy2D(ds.p, srow, src, src_step, srow, src_rows, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy2D(d1.p, m1_row, m1, m1_step, m1_row, rows, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy2D(d2.p, m2_row, m2, m2_step, m2_row, rows, hipMemcpyHostToDevice);
    if (e != hipSuccess) return status(e);
    const int rc = fixed ? tsm_remap_linear_fixed_device((const uint8_t*)ds.p, src_rows, src_cols, srow, C,
                                                         (const int16_t*)d1.p, m1_row, (const uint16_t*)d2.p,
                                                         m2_row, rows, cols, (uint8_t*)dd.p, drow, nullptr)
                         : tsm_remap_linear_float_device((const uint8_t*)ds.p, src_rows, src_cols, srow, C,
                                                         (const float*)d1.p, (const float*)d2.p, m1_row, rows,
                                                         cols, (uint8_t*)dd.p, drow, nullptr);
    if (rc != TSM_OK) return rc;
    e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy2D(dst, dst_step, dd.p, drow, drow, rows, hipMemcpyDeviceToHost);
    return status(e);
}

int tsm_remap_linear_fixed(const uint8_t* src, int src_rows, int src_cols, size_t src_step,
                           int channels, const int16_t* xy, size_t xy_step, const uint16_t* fxy,
                           size_t fxy_step, int rows, int cols, uint8_t* dst, size_t dst_step) {
    const int C = channels;
    if (!src || !xy || !fxy || !dst || bad_dims(rows, cols) || bad_dims(src_rows, src_cols) ||
        (C != 1 && C != 3 && C != 4) || src_step < (size_t)C * src_cols || xy_step < 4 * (size_t)cols ||
        fxy_step < 2 * (size_t)cols || dst_step < (size_t)C * cols)
        return TSM_ERR_ARGUMENT;
    return remap_host(src, src_rows, src_cols, src_step, C, xy, 4 * (size_t)cols, xy_step, fxy,
                      2 * (size_t)cols, fxy_step, rows, cols, dst, dst_step, true);
}

int tsm_remap_linear_float(const uint8_t* src, int src_rows, int src_cols, size_t src_step,
                           int channels, const float* mapx, const float* mapy, size_t map_step,
                           int rows, int cols, uint8_t* dst, size_t dst_step) {
    const int C = channels;
    if (!src || !mapx || !mapy || !dst || bad_dims(rows, cols) || bad_dims(src_rows, src_cols) ||
        (C != 1 && C != 3 && C != 4) || src_step < (size_t)C * src_cols || map_step < 4 * (size_t)cols ||
        dst_step < (size_t)C * cols)
        return TSM_ERR_ARGUMENT;
    return remap_host(src, src_rows, src_cols, src_step, C, mapx, 4 * (size_t)cols, map_step, mapy,
                      4 * (size_t)cols, map_step, rows, cols, dst, dst_step, false);
}

}  // extern "C"
