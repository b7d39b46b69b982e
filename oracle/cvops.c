/*
 * cvops.c -- OpenCV 4.x semantics of the four imgproc calls on the AD-Census path,
 * restated for the oracle.  TEST INFRASTRUCTURE ONLY.
 *
 * The reference calls (source/ADCensus.cpp):
 *   cv::equalizeHist(dispU, dispU)                         :1252
 *   cv::blur(gray, edges, Size(3,3))  (BORDER_REFLECT_101) :1263
 *   cv::Canny(edges, edges, 30, 90, 3) (L1 gradient)       :1264
 *   cv::medianBlur(dispTemp, dispTemp, 3) on CV_32F         :1372
 *   cv::filter2D(hsi, median, -1, gauss3x3, ..., BORDER_CONSTANT)  HSI only, :1480
 * OpenCV 4.13.0 (README.md:39) is a third-party dependency absent from this image;
 * these are restatements of its published (non-IPP) algorithms.  Parity of this
 * boundary is unpinned beyond the reference's demo-output fixtures.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "adcensus_oracle.h"

/* saturate_cast<uchar>(float) = cvRound (round half to even) then clamp. */
static inline int round_half_even_f(float v) { return (int)lrintf(v); }
static inline uint8_t sat_u8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

/* imgproc/src/histogram.cpp equalizeHist: lut[i] = saturate_cast<uchar>(sum * scale),
 * scale = 255.f / (total - hist[first nonzero]). */
void orc_cv_equalize_hist(const uint8_t* src, uint8_t* dst, int H, int W) {
    int hist[256] = {0};
    int lut[256];
    const size_t n = (size_t)H * W;
    for (size_t i = 0; i < n; ++i) hist[src[i]]++;
    int i = 0;
    while (i < 256 && !hist[i]) ++i;
    if (i == 256) return;
    const int total = (int)n;
    if (hist[i] == total) {
        for (size_t k = 0; k < n; ++k) dst[k] = (uint8_t)i;
        return;
    }
    float scale = (256 - 1.f) / (float)(total - hist[i]);
    int sum = 0;
    for (int k = 0; k < 256; ++k) lut[k] = 0;
    for (lut[i++] = 0; i < 256; ++i) {
        sum += hist[i];
        lut[i] = sat_u8(round_half_even_f((float)sum * scale));
    }
    for (size_t k = 0; k < n; ++k) dst[k] = (uint8_t)lut[src[k]];
}

/* BORDER_REFLECT_101 index (gfedcb|abcdefgh|gfedcba). */
static inline int reflect101(int i, int n) {
    if (n == 1) return 0;
    while (i < 0 || i >= n) {
        if (i < 0) i = -i;
        if (i >= n) i = 2 * n - 2 - i;
    }
    return i;
}
static inline int clampi(int i, int n) { return i < 0 ? 0 : (i >= n ? n - 1 : i); }

/* boxFilter 3x3 normalised on CV_8U: RowSum<uchar,ushort> + ColumnSum<ushort,uchar> whose
 * fixed-point divide ((s + 4) * 932068) >> 23 equals round(s / 9) for every s in [0, 2295]. */
void orc_cv_blur3(const uint8_t* src, uint8_t* dst, int H, int W) {
    for (int h = 0; h < H; ++h) {
        for (int w = 0; w < W; ++w) {
            int s = 0;
            for (int dy = -1; dy <= 1; ++dy) {
                int hh = reflect101(h + dy, H);
                for (int dx = -1; dx <= 1; ++dx) s += src[(size_t)hh * W + reflect101(w + dx, W)];
            }
            dst[(size_t)h * W + w] = (uint8_t)(((s + 4) * 932068) >> 23);
        }
    }
}

/* imgproc/src/canny.cpp (aperture 3, L2gradient=false): Sobel 3x3 BORDER_REPLICATE to
 * CV_16S, L1 magnitude, TG22 fixed-point non-maximum suppression against a zero-padded
 * magnitude border, then 8-connected hysteresis from "strong" (m > high) pixels through
 * NMS survivors (m > low).  Output 0 / 255. */
void orc_cv_canny(const uint8_t* src, uint8_t* dst, int H, int W, double low_thresh,
                  double high_thresh) {
    if (low_thresh > high_thresh) { double t = low_thresh; low_thresh = high_thresh; high_thresh = t; }
    const int low = (int)floor(low_thresh), high = (int)floor(high_thresh);
    const int CANNY_SHIFT = 15;
    const int TG22 = (int)(0.4142135623730950488016887242097 * (1 << CANNY_SHIFT) + 0.5);
    const int MW = W + 2;
    short* dx = (short*)malloc((size_t)H * W * sizeof(short));
    short* dy = (short*)malloc((size_t)H * W * sizeof(short));
    int* mag = (int*)calloc((size_t)(H + 2) * MW, sizeof(int)); /* zero border */
    uint8_t* map = (uint8_t*)malloc((size_t)(H + 2) * MW);
    int* stack = (int*)malloc((size_t)(H + 2) * MW * sizeof(int));
#define S(hh, ww) ((int)src[(size_t)clampi(hh, H) * W + clampi(ww, W)])
    for (int h = 0; h < H; ++h) {
        for (int w = 0; w < W; ++w) {
            int gx = (S(h - 1, w + 1) + 2 * S(h, w + 1) + S(h + 1, w + 1)) -
                     (S(h - 1, w - 1) + 2 * S(h, w - 1) + S(h + 1, w - 1));
            int gy = (S(h + 1, w - 1) + 2 * S(h + 1, w) + S(h + 1, w + 1)) -
                     (S(h - 1, w - 1) + 2 * S(h - 1, w) + S(h - 1, w + 1));
            dx[(size_t)h * W + w] = (short)gx;
            dy[(size_t)h * W + w] = (short)gy;
            mag[(size_t)(h + 1) * MW + (w + 1)] = abs(gx) + abs(gy);
        }
    }
#undef S
    memset(map, 1, (size_t)(H + 2) * MW);
    size_t top = 0;
#define M(hh, ww) mag[(size_t)((hh) + 1) * MW + ((ww) + 1)]
    for (int h = 0; h < H; ++h) {
        for (int w = 0; w < W; ++w) {
            const int m = M(h, w);
            uint8_t* pm = &map[(size_t)(h + 1) * MW + (w + 1)];
            int keep = 0;
            if (m > low) {
                const int xs = dx[(size_t)h * W + w], ys = dy[(size_t)h * W + w];
                const int x = abs(xs);
                const int y = abs(ys) << CANNY_SHIFT;
                const int tg22x = x * TG22;
                if (y < tg22x) {
                    if (m > M(h, w - 1) && m >= M(h, w + 1)) keep = 1;
                } else {
                    const int tg67x = tg22x + (x << (CANNY_SHIFT + 1));
                    if (y > tg67x) {
                        if (m > M(h - 1, w) && m >= M(h + 1, w)) keep = 1;
                    } else {
                        const int s = (xs ^ ys) < 0 ? -1 : 1;
                        if (m > M(h - 1, w - s) && m > M(h + 1, w + s)) keep = 1;
                    }
                }
            }
            if (!keep) { *pm = 1; continue; }
            if (m > high) {
                *pm = 2;
                stack[top++] = (h + 1) * MW + (w + 1);
            } else {
                *pm = 0;
            }
        }
    }
#undef M
    while (top > 0) {
        const int q = stack[--top];
        const int nb[8] = {-1, 1, -MW - 1, -MW, -MW + 1, MW - 1, MW, MW + 1};
        for (int k = 0; k < 8; ++k) {
            const int r = q + nb[k];
            if (map[r] == 0) {
                map[r] = 2;
                stack[top++] = r;
            }
        }
    }
    for (int h = 0; h < H; ++h)
        for (int w = 0; w < W; ++w)
            dst[(size_t)h * W + w] = map[(size_t)(h + 1) * MW + (w + 1)] == 2 ? 255 : 0;
    free(dx); free(dy); free(mag); free(map); free(stack);
}

static int cmp_float(const void* a, const void* b) {
    float x = *(const float*)a, y = *(const float*)b;
    return (x > y) - (x < y);
}

/* medianBlur ksize 3 on CV_32F: median of the 3x3 neighbourhood, BORDER_REPLICATE. */
void orc_cv_median3f(const float* src, float* dst, int H, int W) {
    for (int h = 0; h < H; ++h) {
        for (int w = 0; w < W; ++w) {
            float v[9];
            int k = 0;
            for (int dy = -1; dy <= 1; ++dy)
                for (int dx = -1; dx <= 1; ++dx)
                    v[k++] = src[(size_t)clampi(h + dy, H) * W + clampi(w + dx, W)];
            qsort(v, 9, sizeof(float), cmp_float);
            dst[(size_t)h * W + w] = v[4];
        }
    }
}

/* filter2D with getGaussianKernel(3, -1) (= {0.25, 0.5, 0.25}, the fixed small-kernel
 * table) outer product, BORDER_CONSTANT 0, 3 channels: float accumulation of exactly
 * representable terms, then saturate_cast<uchar> (round half to even). */
void orc_cv_gauss3_filter2d(const uint8_t* src, uint8_t* dst, int H, int W) {
    static const int k[3] = {1, 2, 1};
    for (int h = 0; h < H; ++h) {
        for (int w = 0; w < W; ++w) {
            for (int c = 0; c < 3; ++c) {
                int s = 0;
                for (int dy = -1; dy <= 1; ++dy) {
                    int hh = h + dy;
                    if (hh < 0 || hh >= H) continue;
                    for (int dx = -1; dx <= 1; ++dx) {
                        int ww = w + dx;
                        if (ww < 0 || ww >= W) continue;
                        s += k[dy + 1] * k[dx + 1] * src[((size_t)hh * W + ww) * 3 + c];
                    }
                }
                int q = s >> 4, r = s & 15;
                if (r > 8 || (r == 8 && (q & 1))) q++;
                dst[((size_t)h * W + w) * 3 + c] = sat_u8(q);
            }
        }
    }
}

/* stereo.cpp:75-92 */
void orc_jet_colormap(uint8_t lut[256][3]) {
#define SET(i, b, g, r) do { lut[i][0] = (uint8_t)(b); lut[i][1] = (uint8_t)(g); lut[i][2] = (uint8_t)(r); } while (0)
    for (int i = 0; i < 32; ++i) SET(i, 128 + 4 * i, 0, 0);
    SET(32, 255, 0, 0);
    for (int i = 0; i < 63; ++i) SET(33 + i, 255, 4 + 4 * i, 0);
    SET(96, 254, 255, 2);
    for (int i = 0; i < 62; ++i) SET(97 + i, 250 - 4 * i, 255, 6 + 4 * i);
    SET(159, 1, 255, 254);
    for (int i = 0; i < 64; ++i) SET(160 + i, 0, 252 - 4 * i, 255);
    for (int i = 0; i < 32; ++i) SET(224 + i, 0, 0, 252 - 4 * i);
#undef SET
}

/* applyColorMap(src, dst, colorMap), stereo.cpp:94-118 */
void orc_apply_colormap(const float* disp, int H, int W, uint8_t* bgr) {
    uint8_t lut[256][3];
    orc_jet_colormap(lut);
    orc_apply_colormap_ex(disp, H, W, (size_t)W, &lut[0][0], 0, 0.f, 0.f, bgr, (size_t)W * 3);
}
