/* stereo_ops.c -- TEST INFRASTRUCTURE ONLY (parity checker, never shipped or measured).
 *
 * CPU restatement of the calls either side of the AD-Census path:
 *   f2  applyColorMap, both overloads            (source/stereo.cpp:94-134)
 *   f3  reprojectToDepth, reprojectTo3D x2       (source/stereo.cpp:136-202)
 *   f4  EpipolarRectify::rectify = cv::remap INTER_LINEAR, BORDER_CONSTANT 0
 *                                                (source/EpipolarRectify.cpp:87-101)
 *
 * f2/f3 follow the reference's own loops; the float -> unsigned char cast of the colour
 * index is pinned to x86 semantics (cvttss2si: out of int range / NaN -> 0x80000000,
 * low byte kept), which is what the reference's MSVC x64 build executes for the
 * undefined cases (range 0 when max == min, +inf disparities).  The Q overload's
 * product Q_float32 * [u v d 1]^T (cv::gemm, stereo.cpp:191) is summed here in index
 * order; OpenCV's own summation order is not in the reference -> tolerance, see tests.
 *
 * f4 restates OpenCV 4.x remapBilinear for 8-bit images (OpenCV 4.13 is not in the
 * image and no reference test or fixture exercises remap: PARITY UNPINNED).  The maps
 * are the reference's CV_16SC2 + CV_16UC1 pair (stereo_utils.cpp:164-167): integer
 * source (sx, sy) and a 10-bit fraction index f = fy * 32 + fx (INTER_BITS = 5).  Tap
 * weights are the exact products (32 - fx)(32 - fy), fx(32 - fy), (32 - fx)fy, fx fy
 * scaled to 2^15 (INTER_REMAP_COEF_BITS), the sum rounds by + 2^14 >> 15, taps outside
 * the source read the constant border value 0.  Float maps (CV_32FC1 x / y) are first
 * rounded to 1/32 pixel (cvRound(x * 32): nearest, ties to even; NaN / out of int
 * range -> INT_MIN as on x86), as OpenCV converts them.
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>

#include "adcensus_oracle.h"

/* (unsigned char)t for the reference's float index, x86 cvttss2si semantics */
static uint8_t cast_u8_x86(float t) {
    if (!(t > -2147483648.0f && t < 2147483648.0f)) return 0; /* NaN, +-inf, out of range */
    return (uint8_t)((int32_t)t & 0xff);
}

/* applyColorMap(src, dst, colorMap) stereo.cpp:94-118 (use_range = 0) and
 * applyColorMap(src, dst, minVal, maxVal, colorMap) stereo.cpp:120-134 (use_range = 1). */
void orc_apply_colormap_ex(const float* disp, int H, int W, size_t step_f, const uint8_t* lut,
                           int use_range, float minv, float maxv, uint8_t* bgr, size_t out_step) {
    float mn = INFINITY, mx = -INFINITY;
    if (use_range) {
        mn = minv;
        mx = maxv;
    } else {
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x) {
                const float v = disp[(size_t)y * step_f + x];
                if (v < 0 || isinf(v)) continue;
                mn = v < mn ? v : mn; /* std::min(minVal, v): NaN never replaces */
                mx = mx < v ? v : mx; /* std::max(maxVal, v) */
            }
    }
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const float v = disp[(size_t)y * step_f + x];
            uint8_t* o = bgr + (size_t)y * out_step + 3 * (size_t)x;
            const int black = use_range ? (v < mn || v > mx) : (v < 0);
            if (black) {
                o[0] = o[1] = o[2] = 0;
                continue;
            }
            const uint8_t idx = cast_u8_x86(((v - mn) / (mx - mn)) * 255);
            o[0] = lut[3 * idx + 0];
            o[1] = lut[3 * idx + 1];
            o[2] = lut[3 * idx + 2];
        }
}

/* reprojectToDepth stereo.cpp:136-148 */
void orc_reproject_depth(const float* disp, int H, int W, size_t step_f, float f, float b,
                         float* depth, size_t out_step_f) {
    const float fb = f * b;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const float d = disp[(size_t)y * step_f + x];
            depth[(size_t)y * out_step_f + x] = (d < 0 || isinf(d)) ? 0.f : fb / d;
        }
}

/* reprojectTo3D(disparity, f, b, cx, cy) stereo.cpp:150-169; xyz rows of 3*W floats */
void orc_reproject_3d(const float* disp, int H, int W, size_t step_f, float f, float b, float cx,
                      float cy, float* xyz, size_t out_step_f) {
    const float fb = f * b;
    for (int v = 0; v < H; ++v)
        for (int u = 0; u < W; ++u) {
            const float d = disp[(size_t)v * step_f + u];
            float* o = xyz + (size_t)v * out_step_f + 3 * (size_t)u;
            if (d < 0 || isinf(d)) {
                o[0] = o[1] = o[2] = 0.f;
                continue;
            }
            const float Z = fb / d;
            const float Zf = Z / f;
            o[0] = ((float)u - cx) * Zf;
            o[1] = ((float)v - cy) * Zf;
            o[2] = Z;
        }
}

/* reprojectTo3D(disparity, Q, XYZ) stereo.cpp:171-202: Q converted to fp32 (:190),
 * [x y z w] = Q [u v d 1], then x/w, y/w, z/w (no validity test) */
void orc_reproject_3d_q(const float* disp, int H, int W, size_t step_f, const double* Q,
                        float* xyz, size_t out_step_f) {
    float q[16];
    for (int i = 0; i < 16; ++i) q[i] = (float)Q[i];
    for (int v = 0; v < H; ++v)
        for (int u = 0; u < W; ++u) {
            const float d = disp[(size_t)v * step_f + u];
            const float p[4] = {(float)u, (float)v, d, 1.f};
            float r[4];
            for (int i = 0; i < 4; ++i) {
                float s = 0.f;
                for (int k = 0; k < 4; ++k) s += q[4 * i + k] * p[k];
                r[i] = s;
            }
            float* o = xyz + (size_t)v * out_step_f + 3 * (size_t)u;
            o[0] = r[0] / r[3];
            o[1] = r[1] / r[3];
            o[2] = r[2] / r[3];
        }
}

/* bilinear 8-bit remap of one pixel, C channels, source (sx, sy) + fraction (fx, fy) */
static void remap_px(const uint8_t* src, int sh, int sw, size_t sstep, int C, int sx, int sy,
                     int fx, int fy, uint8_t* o) {
    const int w[4] = {(32 - fx) * (32 - fy) * 32, fx * (32 - fy) * 32, (32 - fx) * fy * 32,
                      fx * fy * 32};
    const int tx[4] = {sx, sx + 1, sx, sx + 1}, ty[4] = {sy, sy, sy + 1, sy + 1};
    for (int c = 0; c < C; ++c) {
        int acc = 0;
        for (int t = 0; t < 4; ++t) {
            const int in = tx[t] >= 0 && tx[t] < sw && ty[t] >= 0 && ty[t] < sh;
            const int p = in ? src[(size_t)ty[t] * sstep + (size_t)tx[t] * C + c] : 0;
            acc += p * w[t];
        }
        int r = (acc + (1 << 14)) >> 15;
        o[c] = (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
    }
}

/* cv::remap(src, dst, map1 CV_16SC2, map2 CV_16UC1, INTER_LINEAR) */
void orc_remap_linear_fixed(const uint8_t* src, int sh, int sw, size_t sstep, int C,
                            const int16_t* xy, size_t xy_step_e, const uint16_t* fxy,
                            size_t fxy_step_e, int H, int W, uint8_t* dst, size_t dstep) {
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const int sx = xy[(size_t)y * xy_step_e + 2 * (size_t)x];
            const int sy = xy[(size_t)y * xy_step_e + 2 * (size_t)x + 1];
            const int f = fxy[(size_t)y * fxy_step_e + x] & 1023;
            remap_px(src, sh, sw, sstep, C, sx, sy, f & 31, f >> 5, dst + (size_t)y * dstep + (size_t)x * C);
        }
}

static int sat_s16(long v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : (int)v); }

/* cv::remap(src, dst, mapx CV_32FC1, mapy CV_32FC1, INTER_LINEAR) */
void orc_remap_linear_float(const uint8_t* src, int sh, int sw, size_t sstep, int C,
                            const float* mx, const float* my, size_t map_step_f, int H, int W,
                            uint8_t* dst, size_t dstep) {
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const float fxv = mx[(size_t)y * map_step_f + x], fyv = my[(size_t)y * map_step_f + x];
            /* saturate_cast<int>(v * INTER_TAB_SIZE) = cvRound: nearest-even, and x86's
             * "integer indefinite" INT_MIN for NaN / out-of-range values */
            const float ax = fxv * 32.f, ay = fyv * 32.f;
            const long ix = (ax >= -2147483648.0f && ax < 2147483648.0f) ? lrintf(ax) : -2147483648L;
            const long iy = (ay >= -2147483648.0f && ay < 2147483648.0f) ? lrintf(ay) : -2147483648L;
            const int sx = sat_s16(ix >> 5), sy = sat_s16(iy >> 5);
            remap_px(src, sh, sw, sstep, C, sx, sy, (int)(ix & 31), (int)(iy & 31),
                     dst + (size_t)y * dstep + (size_t)x * C);
        }
}
