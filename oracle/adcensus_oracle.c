/*
 * adcensus_oracle.c -- CPU restatement of stereo::ADCensus (reference source/ADCensus.cpp).
 *
 * TEST INFRASTRUCTURE ONLY (see adcensus_oracle.h).  Not linked by the product.
 *
 * Semantics are the reference's, including its quirks (each one is cited where it is
 * restated).  The only deliberate deviation: the scanline passes run with serial
 * (intended) semantics by default; the reference parallelises them over the
 * recursion dimension (ADCensus.cpp:801-853), which is a data race.  Set
 * orc_params.scan_emulate_threads = T to reproduce the race's deterministic
 * lock-step outcome for T threads.
 *
 * Build: see oracle/Makefile.  Must be compiled with -ffp-contract=off (the
 * reference's MSVC /fp:precise build does not contract a*b+c into an FMA).
 */
#include "adcensus_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define DISP_OCCLUSION 1 /* ADCensus.cpp:294 */
#define DISP_MISMATCH 2  /* ADCensus.cpp:295 */

/* ------------------------------------------------------------------------- */
/* parameters                                                                */
/* ------------------------------------------------------------------------- */

void orc_default_params(orc_params* p, int color_model) {
    /* stereo_utils.cpp:271-326 */
    memset(p, 0, sizeof(*p));
    p->color_model = color_model;
    p->min_disparity = 0;  /* ADCensus.cpp:411 */
    p->max_disparity = 64; /* ADCensus.cpp:412 */
    p->lambda_ad = 10.f;
    p->census_win = ORC_CENSUSWIN_9x7;
    p->lambda_census = 30.f;
    p->lambda_hue = 1.f;
    p->lambda_saturation = 2.5f;
    p->lambda_intensity = 2.5f;
    p->iterations = 4;
    p->pi1 = 1.f;
    p->pi2 = 3.f;
    p->disp_tolerance = 0;
    p->voting_thresh = 20;
    p->voting_ratio_thresh = 0.4f;
    p->max_search_depth = 20;
    p->blur_kernel_size = 3;
    p->canny_thresh1 = 30;
    p->canny_thresh2 = 90;
    p->canny_kernel_size = 3;
    if (color_model == ORC_RGB) {
        p->color_thresh1 = 20;
        p->color_thresh2 = 6;
        p->max_length1 = 34;
        p->max_length2 = 17;
        p->color_diff = 15;
        p->saturation_thresh1 = p->saturation_thresh2 = 0; /* NULL */
        p->intensity_thresh1 = p->intensity_thresh2 = 0;
    } else {
        p->color_thresh1 = 5;
        p->color_thresh2 = 1;
        p->max_length1 = 17;
        p->max_length2 = 8;
        p->color_diff = 3;
        p->saturation_thresh1 = 10;
        p->saturation_thresh2 = 2;
        p->intensity_thresh1 = 12;
        p->intensity_thresh2 = 3;
    }
}

int orc_check_disparity_range(int mn, int mx) {
    /* ADCensus.cpp:309 -- note: int product, as in the reference */
    if ((long long)mn * (long long)mx < 0 || mn >= mx) return -2;
    return 0;
}

static int nthreads(const orc_params* p) {
#ifdef _OPENMP
    return p->num_threads > 0 ? p->num_threads : omp_get_max_threads();
#else
    (void)p;
    return 1;
#endif
}

/* ------------------------------------------------------------------------- */
/* pixel helpers                                                             */
/* ------------------------------------------------------------------------- */

typedef struct {
    const uint8_t* img[2]; /* dense [H][W][3] */
    int H, W;
} views_t;

static inline const uint8_t* px(const views_t* v, int k, int h, int w) {
    return v->img[k] + ((size_t)h * v->W + w) * 3;
}
static inline int is_black(const uint8_t* a) { return a[0] == 0 && a[1] == 0 && a[2] == 0; }
static inline int iabs(int x) { return x < 0 ? -x : x; }
static inline int imin(int a, int b) { return a < b ? a : b; }

/* colorDiff, ADCensus.cpp:583-602 */
static inline int color_diff(const orc_params* p, const uint8_t* a, const uint8_t* b) {
    if (p->color_model == ORC_RGB) {
        int diff = 0;
        for (int i = 0; i < 3; ++i) {
            int c = iabs((int)a[i] - (int)b[i]);
            diff = diff > c ? diff : c;
        }
        return diff;
    }
    int hd = iabs((int)a[0] - (int)b[0]);
    return imin(hd, 255 - hd);
}

/* ------------------------------------------------------------------------- */
/* Step 1: cost initialisation                                               */
/* ------------------------------------------------------------------------- */

/* computeRGBADCost, ADCensus.cpp:426-437 */
static inline float rgb_ad(const uint8_t* l, const uint8_t* r) {
    float ad = 0.f;
    for (int i = 0; i < 3; ++i) ad += (float)iabs((int)l[i] - (int)r[i]);
    return ad / 3.f;
}

/* computeHSIADCost, ADCensus.cpp:439-452 */
static inline float hsi_ad(const orc_params* p, const uint8_t* l, const uint8_t* r) {
    float ad = 0.f;
    int hd = iabs((int)l[0] - (int)r[0]);
    ad += (float)imin(hd, 255 - hd) * p->lambda_hue;
    ad += (float)iabs((int)l[1] - (int)r[1]) * p->lambda_saturation;
    ad += (float)iabs((int)l[2] - (int)r[2]) * p->lambda_intensity;
    return ad;
}

/* computeRGBCensusCost (ADCensus.cpp:454-474) and computeHSICensusCost (:476-498):
 * ternary sign-disagreement count; ties never count (:469). */
static inline float census(const orc_params* p, const views_t* v, int h1, int w1, int h2, int w2,
                           int wh, int ww) {
    const uint8_t* lp = px(v, 0, h1, w1);
    const uint8_t* rp = px(v, 1, h2, w2);
    if (p->mask_matching && (is_black(lp) || is_black(rp))) return INFINITY; /* :459-460 */
    float c = 0.f;
    for (int i = -wh / 2; i <= wh / 2; ++i) {
        for (int j = -ww / 2; j <= ww / 2; ++j) {
            const uint8_t* la = px(v, 0, h1 + i, w1 + j);
            const uint8_t* ra = px(v, 1, h2 + i, w2 + j);
            if (p->color_model == ORC_RGB) {
                for (int k = 0; k < 3; ++k)
                    c += (((int)la[k] - (int)lp[k]) * ((int)ra[k] - (int)rp[k]) < 0) ? 1.f : 0.f;
            } else {
                /* :489-494 -- hue bit is NAND of the two "positive" classes */
                int dl = (int)la[0] - (int)lp[0];
                int dr = (int)ra[0] - (int)rp[0];
                int posl = (dl <= -127) || (dl >= 0 && dl <= 127);
                int posr = (dr <= -127) || (dr >= 0 && dr <= 127);
                c += (posl && posr) ? 0.f : 1.f;
                c += (((int)la[1] - (int)lp[1]) * ((int)ra[1] - (int)rp[1]) < 0) ? 1.f : 0.f;
                c += (((int)la[2] - (int)lp[2]) * ((int)ra[2] - (int)rp[2]) < 0) ? 1.f : 0.f;
            }
        }
    }
    return c;
}

/* computeADCensusCost, ADCensus.cpp:500-520 */
static inline float adcensus_cost(const orc_params* p, const views_t* v, int h1, int w1, int h2,
                                  int w2, int wh, int ww) {
    float ad, cc;
    if (p->color_model == ORC_RGB)
        ad = rgb_ad(px(v, 0, h1, w1), px(v, 1, h2, w2));
    else
        ad = hsi_ad(p, px(v, 0, h1, w1), px(v, 1, h2, w2));
    cc = census(p, v, h1, w1, h2, w2, wh, ww);
    return 2.f - expf(-ad / p->lambda_ad) - expf(-cc / p->lambda_census);
}

static void census_dims(const orc_params* p, int* wh, int* ww) {
    /* ADCensus.cpp:525-537 */
    if (p->census_win == ORC_CENSUSWIN_7x5) {
        *ww = 7;
        *wh = 5;
    } else {
        *ww = 9;
        *wh = 7;
    }
}

static void cost_initialize(const orc_params* p, const views_t* v, float* vol) {
    /* costInitialize, ADCensus.cpp:522-581 */
    const int H = v->H, W = v->W;
    const int L = p->max_disparity - p->min_disparity + 1;
    int wh, ww;
    census_dims(p, &wh, &ww);
    const int hw = ww / 2, hh = wh / 2;
    const size_t plane = (size_t)H * W;
    for (int k = 0; k < 2; ++k) {
#pragma omp parallel for schedule(static) num_threads(nthreads(p))
        for (int d = 0; d < L; ++d) { /* :542-544 omp over d */
            float* dst = vol + ((size_t)k * L + d) * plane;
            for (int i = 0; i < H; ++i) {
                for (int j = 0; j < W; ++j) {
                    if (p->mask_matching && is_black(px(v, k, i, j))) { /* :551-555 */
                        dst[(size_t)i * W + j] = 2.f;
                        continue;
                    }
                    int colL = j - p->min_disparity; /* :556-561 */
                    int colR = j + p->min_disparity;
                    if (k == 0)
                        colR = j - d;
                    else
                        colL = j + d;
                    int out = colL - hw < 0 || colL + hw >= W || colR - hw < 0 || colR + hw >= W ||
                              i - hh < 0 || i + hh >= H; /* :562-564 */
                    dst[(size_t)i * W + j] =
                        out ? 2.f : adcensus_cost(p, v, i, colL, i, colR, wh, ww);
                }
            }
        }
    }
}

/* ------------------------------------------------------------------------- */
/* Step 2: cross arms + aggregation                                          */
/* ------------------------------------------------------------------------- */

/* computeLimit, ADCensus.cpp:604-659 */
static int compute_limit(const orc_params* p, const views_t* v, int height, int width, int dH,
                         int dW, int k) {
    const int H = v->H, W = v->W;
    const uint8_t* pp = px(v, k, height, width);
    int d = 1;
    int h1 = height + dH, w1 = width + dW;
    const uint8_t* p2 = pp;
    int inside = 0 <= h1 && h1 < H && 0 <= w1 && w1 < W;
    if (inside) {
        int colorCond = 1, wLimitCond = 1, fColorCond = 1;
        while (colorCond && wLimitCond && fColorCond && inside) {
            const uint8_t* p1 = px(v, k, h1, w1);
            if (p->mask_matching && is_black(p1)) { /* :625-629 */
                d++;
                break;
            }
            colorCond = color_diff(p, pp, p1) < p->color_thresh1 &&
                        color_diff(p, p1, p2) < p->color_thresh1; /* :631 */
            if (p->color_model == ORC_HSI) {
                /* :632-636 -- both assignments overwrite: only intensity survives */
                colorCond = iabs((int)pp[1] - (int)p1[1]) < p->saturation_thresh1 &&
                            iabs((int)p1[1] - (int)p2[1]) < p->saturation_thresh1;
                colorCond = iabs((int)pp[2] - (int)p1[2]) < p->intensity_thresh1 &&
                            iabs((int)p1[2] - (int)p2[2]) < p->intensity_thresh1;
            }
            wLimitCond = d < p->max_length1; /* :638 */
            fColorCond = (d <= p->max_length2) ||
                         (d > p->max_length2 && color_diff(p, pp, p1) < p->color_thresh2); /* :640 */
            if (p->color_model == ORC_HSI) {
                fColorCond = (d <= p->max_length2) ||
                             (d > p->max_length2 &&
                              iabs((int)pp[1] - (int)p1[1]) < p->saturation_thresh2);
                fColorCond = (d <= p->max_length2) ||
                             (d > p->max_length2 &&
                              iabs((int)pp[2] - (int)p1[2]) < p->intensity_thresh2);
            }
            p2 = p1;
            h1 += dH;
            w1 += dW;
            inside = 0 <= h1 && h1 < H && 0 <= w1 && w1 < W;
            d++;
        }
        d--; /* :656 */
    }
    return d - 1; /* :658 -- arm is one shorter when the walk ends at the image edge */
}

static void compute_limits(const orc_params* p, const views_t* v, int32_t* arms) {
    /* costAggregate :756-766 -> computeLimits :661-683 */
    static const int dirs[4][2] = {{-1, 0}, {1, 0}, {0, -1}, {0, 1}}; /* up, down, left, right */
    const int H = v->H, W = v->W;
    const size_t plane = (size_t)H * W;
    for (int k = 0; k < 2; ++k) {
        for (int a = 0; a < 4; ++a) {
            int32_t* dst = arms + ((size_t)k * 4 + a) * plane;
#pragma omp parallel for schedule(static) num_threads(nthreads(p))
            for (int h = 0; h < H; ++h) {
                for (int w = 0; w < W; ++w) {
                    if (p->mask_matching && is_black(px(v, k, h, w))) {
                        dst[(size_t)h * W + w] = 0;
                        continue;
                    }
                    dst[(size_t)h * W + w] = compute_limit(p, v, h, w, dirs[a][0], dirs[a][1], k);
                }
            }
        }
    }
}

/* aggregation1D, ADCensus.cpp:685-723: sequential fp32 sum from -arm to +arm. */
static void aggregation_1d(const float* in, float* out, const int32_t* armA, const int32_t* armB,
                           int dH, int dW, const int32_t* ws_in, int32_t* ws_out, int H, int W) {
    for (int h = 0; h < H; ++h) {
        for (int w = 0; w < W; ++w) {
            const size_t idx = (size_t)h * W + w;
            const int dmin = -armA[idx], dmax = armB[idx];
            float cost = 0;
            int wsum = 0;
            for (int d = dmin; d <= dmax; ++d) {
                const size_t j = (size_t)(h + d * dH) * W + (w + d * dW);
                cost += in[j];
                wsum += ws_in[j];
            }
            out[idx] = cost;
            ws_out[idx] = wsum;
        }
    }
}

static void cost_aggregate(const orc_params* p, int H, int W, const int32_t* arms, float* vol) {
    /* costAggregate, ADCensus.cpp:753-793; aggregation2D :725-751 */
    const int L = p->max_disparity - p->min_disparity + 1;
    const size_t plane = (size_t)H * W;
    for (int k = 0; k < 2; ++k) {
        const int32_t* up = arms + ((size_t)k * 4 + 0) * plane;
        const int32_t* down = arms + ((size_t)k * 4 + 1) * plane;
        const int32_t* left = arms + ((size_t)k * 4 + 2) * plane;
        const int32_t* right = arms + ((size_t)k * 4 + 3) * plane;
#pragma omp parallel num_threads(nthreads(p))
        {
            float* tmp = (float*)malloc(plane * sizeof(float));
            int32_t* wsA = (int32_t*)malloc(plane * sizeof(int32_t));
            int32_t* wsB = (int32_t*)malloc(plane * sizeof(int32_t));
#pragma omp for schedule(static)
            for (int d = 0; d < L; ++d) { /* :771-774 omp over d */
                float* c = vol + ((size_t)k * L + d) * plane;
                int horizontalFirst = 1; /* :776 */
                for (int it = 0; it < p->iterations; ++it) {
                    /* aggregation2D: directionH=1,directionW=0, swapped when horizontalFirst */
                    int dH = 1, dW = 0;
                    if (horizontalFirst) { dH = 0; dW = 1; }
                    for (size_t i = 0; i < plane; ++i) wsA[i] = 1; /* :733 */
                    for (int pass = 0; pass < 2; ++pass) {
                        if (dH == 0)
                            aggregation_1d(c, tmp, left, right, 0, 1, wsA, wsB, H, W);
                        else
                            aggregation_1d(c, tmp, up, down, 1, 0, wsA, wsB, H, W);
                        memcpy(c, tmp, plane * sizeof(float));
                        memcpy(wsA, wsB, plane * sizeof(int32_t));
                        int t = dH; dH = dW; dW = t;
                    }
                    for (size_t i = 0; i < plane; ++i) c[i] /= (float)wsA[i]; /* :743-749 */
                    horizontalFirst = !horizontalFirst;
                }
            }
            free(tmp);
            free(wsA);
            free(wsB);
        }
    }
}

/* ------------------------------------------------------------------------- */
/* Step 3: scanline optimisation                                             */
/* ------------------------------------------------------------------------- */

/* computeP1P2, ADCensus.cpp:915-981 */
static inline void compute_p1p2(const orc_params* p, const views_t* v, int h1, int h2, int w1,
                                int w2, int disparity, int rightFirst, float* p1, float* p2) {
    int k = 0, o = 1;
    if (rightFirst) { k = 1; o = 0; disparity = -disparity; } /* :919-924 */
    const int W = v->W;
    int d1 = color_diff(p, px(v, k, h1, w1), px(v, k, h2, w2));
    int d2 = p->color_diff + 1;
    if (0 <= w1 + disparity && w1 + disparity < W && 0 <= w2 + disparity && w2 + disparity < W)
        d2 = color_diff(p, px(v, o, h1, w1 + disparity), px(v, o, h2, w2 + disparity));
    if (d1 < p->color_diff) {
        if (d2 < p->color_diff) { *p1 = p->pi1; *p2 = p->pi2; }
        else { *p1 = p->pi1 / 4.f; *p2 = p->pi2 / 4.f; }
    } else {
        if (d2 < p->color_diff) { *p1 = p->pi1 / 4.f; *p2 = p->pi2 / 4.f; }
        else { *p1 = p->pi1 / 10.f; *p2 = p->pi2 / 10.f; }
    }
}

/* partialOptimization, ADCensus.cpp:869-913.  `cq` points at the predecessor's L values
 * (stride `qs`), `cp` at the current pixel's (stride `ps`).  In-place on cp. */
static void partial_optimization(const orc_params* p, const views_t* v, int h1, int h2, int w1,
                                 int w2, float* cp, size_t ps, const float* cq, size_t qs,
                                 int rightFirst) {
    const int L = p->max_disparity - p->min_disparity + 1;
    float minOpt = cq[0];
    for (int d = 1; d < L; ++d) {
        float t = cq[(size_t)d * qs];
        if (minOpt > t) minOpt = t;
    }
    if (minOpt == 0) return; /* :880-881 -- p left untouched */
    const float mink = minOpt;
    for (int d = 0; d < L; ++d) {
        float cost = cp[(size_t)d * ps] - mink;
        float p1 = 0.f, p2 = 0.f;
        compute_p1p2(p, v, h1, h2, w1, w2, d + p->min_disparity, rightFirst, &p1, &p2);
        float mo = mink + p2;
        float t = cq[(size_t)d * qs];
        if (mo > t) mo = t;
        if (d != 0) {
            t = cq[(size_t)(d - 1) * qs] + p1;
            if (mo > t) mo = t;
        }
        if (d != L - 1) {
            t = cq[(size_t)(d + 1) * qs] + p1;
            if (mo > t) mo = t;
        }
        cp[(size_t)d * ps] = (float)((cost + mo) / 2);
    }
}

/* OpenMP static schedule of n iterations over T threads (libgomp / vcomp): the first
 * n%T threads take q+1 iterations.  Returns 1 if iteration index `it` starts a chunk
 * other than the first. */
static int chunk_start(int it, int n, int T) {
    if (T <= 1 || n <= 0) return 0;
    int q = n / T, r = n % T, s = 0;
    for (int t = 0; t < T; ++t) {
        int len = q + (t < r ? 1 : 0);
        if (len == 0) break;
        if (it == s) return t > 0;
        s += len;
    }
    return 0;
}

/* One vertical pass (verticalComputation, ADCensus.cpp:795-818 + verticalOptimization
 * :820-829).  dir=+1: rows 1..H-1 reading row-1; dir=-1: rows H-2..0 reading row+1. */
static void vertical_pass(const orc_params* p, const views_t* v, float* vol, int rightFirst,
                          int dir) {
    const int H = v->H, W = v->W;
    const size_t plane = (size_t)H * W;
    const int L = p->max_disparity - p->min_disparity + 1;
    const int T = p->scan_emulate_threads;
    const int n = H - 1;
    /* snapshot of stale predecessor rows for the racy-schedule emulation */
    float* stale = NULL;
    if (T > 1) {
        stale = (float*)malloc((size_t)H * W * L * sizeof(float));
        for (int it = 0; it < n; ++it) {
            if (!chunk_start(it, n, T)) continue;
            int h1 = dir > 0 ? 1 + it : H - 2 - it;
            int h2 = h1 - dir;
            for (int w = 0; w < W; ++w)
                for (int d = 0; d < L; ++d)
                    stale[((size_t)h2 * W + w) * L + d] = vol[d * plane + (size_t)h2 * W + w];
        }
    }
    /* serial over rows; columns are independent within a row step */
#pragma omp parallel for schedule(static) num_threads(nthreads(p))
    for (int w = 0; w < W; ++w) {
        for (int it = 0; it < n; ++it) {
            int h1 = dir > 0 ? 1 + it : H - 2 - it;
            int h2 = h1 - dir;
            if (p->mask_matching && is_black(px(v, rightFirst, h2, w))) continue; /* :824 */
            float* cp = vol + (size_t)h1 * W + w;
            const float* cq = vol + (size_t)h2 * W + w;
            size_t qs = plane;
            if (T > 1 && chunk_start(it, n, T)) {
                cq = stale + ((size_t)h2 * W + w) * L;
                qs = 1;
            }
            partial_optimization(p, v, h1, h2, w, w, cp, plane, cq, qs, rightFirst);
        }
    }
    free(stale);
}

/* One horizontal pass (horizontalComputation :831-856 + horizontalOptimization :858-867). */
static void horizontal_pass(const orc_params* p, const views_t* v, float* vol, int rightFirst,
                            int dir) {
    const int H = v->H, W = v->W;
    const size_t plane = (size_t)H * W;
    const int L = p->max_disparity - p->min_disparity + 1;
    const int T = p->scan_emulate_threads;
    const int n = W - 1;
    float* stale = NULL;
    if (T > 1) {
        stale = (float*)malloc((size_t)H * W * L * sizeof(float));
        for (int it = 0; it < n; ++it) {
            if (!chunk_start(it, n, T)) continue;
            int w1 = dir > 0 ? 1 + it : W - 2 - it;
            int w2 = w1 - dir;
            for (int h = 0; h < H; ++h)
                for (int d = 0; d < L; ++d)
                    stale[((size_t)h * W + w2) * L + d] = vol[d * plane + (size_t)h * W + w2];
        }
    }
#pragma omp parallel for schedule(static) num_threads(nthreads(p))
    for (int h = 0; h < H; ++h) {
        for (int it = 0; it < n; ++it) {
            int w1 = dir > 0 ? 1 + it : W - 2 - it;
            int w2 = w1 - dir;
            if (p->mask_matching && is_black(px(v, rightFirst, h, w2))) continue; /* :862 */
            float* cp = vol + (size_t)h * W + w1;
            const float* cq = vol + (size_t)h * W + w2;
            size_t qs = plane;
            if (T > 1 && chunk_start(it, n, T)) {
                cq = stale + ((size_t)h * W + w2) * L;
                qs = 1;
            }
            partial_optimization(p, v, h, h, w1, w2, cp, plane, cq, qs, rightFirst);
        }
    }
    free(stale);
}

static void scanline_optimize(const orc_params* p, const views_t* v, float* vol) {
    /* scanlineOptimize :997-1011 -> scanline :983-995 (4 chained in-place passes) */
    const int L = p->max_disparity - p->min_disparity + 1;
    const size_t plane = (size_t)v->H * v->W;
    for (int k = 0; k < 2; ++k) {
        float* c = vol + (size_t)k * L * plane;
        vertical_pass(p, v, c, k == 1, +1);
        vertical_pass(p, v, c, k == 1, -1);
        horizontal_pass(p, v, c, k == 1, +1);
        horizontal_pass(p, v, c, k == 1, -1);
    }
}

/* ------------------------------------------------------------------------- */
/* Step 4: multi-step refinement                                             */
/* ------------------------------------------------------------------------- */

/* cost2disparity, ADCensus.cpp:1394-1413 (first minimum wins; stores the loop index d). */
void orc_cost2disparity(const orc_params* p, int H, int W, const float* c, int32_t* disp) {
    const size_t plane = (size_t)H * W;
    for (size_t i = 0; i < plane; ++i) {
        float low = FLT_MAX;
        int32_t best = p->min_disparity; /* reference leaves it uninitialised if nothing < FLT_MAX */
        for (int d = p->min_disparity; d <= p->max_disparity - p->min_disparity; ++d) {
            float t = c[(size_t)d * plane + i];
            if (low > t) { low = t; best = d; }
        }
        disp[i] = best;
    }
}

/* outlierElimination, ADCensus.cpp:1013-1044 */
static void outlier_elimination(const orc_params* p, int H, int W, const int32_t* dl,
                                const int32_t* dr, int32_t* out) {
    const int occ = 0 - DISP_OCCLUSION, mis = 0 - DISP_MISMATCH; /* :415-416 */
#pragma omp parallel for schedule(static) num_threads(nthreads(p))
    for (int h = 0; h < H; ++h) {
        for (int w = 0; w < W; ++w) {
            int d = dl[(size_t)h * W + w];
            if (w - d < 0 || iabs(d - dr[(size_t)h * W + (w - d)]) > p->disp_tolerance) {
                int occlusion = 1;
                for (int k = p->min_disparity; k <= p->max_disparity; ++k) {
                    if (w - k >= 0 && k == dr[(size_t)h * W + (w - k)]) { occlusion = 0; break; }
                }
                d = occlusion ? occ : mis;
            }
            out[(size_t)h * W + w] = d;
        }
    }
}

/* regionVoting, ADCensus.cpp:1046-1159.  Serial raster order; the vote histogram is only
 * cleared by an outlier with vote > votingThresh, so low-vote outliers' counts carry into
 * the next high-vote outlier (:1132-1151). */
static void region_voting(const orc_params* p, int H, int W, int32_t* disp, const int32_t* arms0,
                          int horizontalFirst) {
    const size_t plane = (size_t)H * W;
    const int L = p->max_disparity - p->min_disparity + 1;
    const int32_t *up = arms0, *down = arms0 + plane, *left = arms0 + 2 * plane,
                  *right = arms0 + 3 * plane;
    const int32_t *oA, *oB, *iA, *iB;
    if (horizontalFirst) { oA = up; oB = down; iA = left; iB = right; }
    else { oA = left; oB = right; iA = up; iB = down; }
    int32_t* tmp = (int32_t*)malloc(plane * sizeof(int32_t));
    int* hist = (int*)calloc((size_t)L, sizeof(int));
    const int mind = p->min_disparity;
    for (int h = 0; h < H; ++h) {
        for (int w = 0; w < W; ++w) {
            const size_t idx = (size_t)h * W + w;
            if (disp[idx] >= mind) { tmp[idx] = disp[idx]; continue; }
            int outerA = -oA[idx], outerB = oB[idx];
            int vote = 0;
            for (int outer = outerA; outer <= outerB; ++outer) {
                int innerA, innerB;
                if (horizontalFirst) {
                    innerA = -iA[(size_t)(h + outer) * W + w];
                    innerB = iB[(size_t)(h + outer) * W + w];
                } else {
                    innerA = -iA[(size_t)h * W + (w + outer)];
                    innerB = iB[(size_t)h * W + (w + outer)];
                }
                for (int inner = innerA; inner <= innerB; ++inner) {
                    int hh, ww;
                    if (horizontalFirst) { hh = h + outer; ww = w + inner; }
                    else { hh = h + inner; ww = w + outer; }
                    int dv = disp[(size_t)hh * W + ww];
                    if (dv >= mind) {
                        vote++;
                        hist[dv - mind] += 1;
                    }
                }
            }
            if (vote <= p->voting_thresh) {
                tmp[idx] = disp[idx];
            } else {
                int dsel = disp[idx];
                float ratioMax = 0;
                for (int d = p->min_disparity; d <= p->max_disparity; ++d) {
                    float ratio = hist[d - mind] / (float)vote;
                    if (ratio > ratioMax) {
                        ratioMax = ratio;
                        dsel = (ratioMax > p->voting_ratio_thresh) ? d : dsel;
                    }
                    hist[d - mind] = 0;
                }
                tmp[idx] = dsel;
            }
        }
    }
    memcpy(disp, tmp, plane * sizeof(int32_t));
    free(tmp);
    free(hist);
}

/* properInterpolation, ADCensus.cpp:1161-1239 */
static void proper_interpolation(const orc_params* p, int H, int W, int32_t* disp,
                                 const uint8_t* img0) {
    static const int dW[16] = {0, 2, 2, 2, 0, -2, -2, -2, 1, 2, 2, 1, -1, -2, -2, -1};
    static const int dHt[16] = {2, 2, 0, -2, -2, -2, 0, 2, 2, 1, -1, -2, -2, -1, 1, 2};
    const size_t plane = (size_t)H * W;
    int32_t* tmp = (int32_t*)malloc(plane * sizeof(int32_t));
    const int mind = p->min_disparity;
#pragma omp parallel for schedule(static) num_threads(nthreads(p))
    for (int h = 0; h < H; ++h) {
        for (int w = 0; w < W; ++w) {
            const size_t idx = (size_t)h * W + w;
            int cur = disp[idx];
            if (cur >= mind) { tmp[idx] = cur; continue; }
            int nd[16], ndiff[16];
            for (int k = 0; k < 16; ++k) { nd[k] = cur; ndiff[k] = -1; }
            for (int dir = 0; dir < 16; ++dir) {
                int hD = h, wD = w, inside = 1, got = 0;
                for (int s = 0; s < p->max_search_depth && inside && !got; ++s) {
                    if (s % 2 == 0) { hD += dHt[dir] / 2; wD += dW[dir] / 2; }
                    else { hD += dHt[dir] - dHt[dir] / 2; wD += dW[dir] - dW[dir] / 2; }
                    inside = hD >= 0 && hD < H && wD >= 0 && wD < W;
                    if (inside && disp[(size_t)hD * W + wD] >= mind) {
                        nd[dir] = disp[(size_t)hD * W + wD];
                        const uint8_t* a = img0 + idx * 3;
                        const uint8_t* b = img0 + ((size_t)hD * W + wD) * 3;
                        ndiff[dir] = color_diff(p, a, b);
                        got = 1;
                    }
                }
            }
            if (cur == mind - DISP_OCCLUSION) { /* :1209 */
                int m = nd[0];
                for (int k = 1; k < 16; ++k) if (m > nd[k]) m = nd[k];
                tmp[idx] = m;
            } else {
                int md = nd[0], mdiff = ndiff[0];
                for (int k = 1; k < 16; ++k) {
                    if (mdiff < 0 || (mdiff > ndiff[k] && ndiff[k] > 0)) { /* :1226 */
                        md = nd[k];
                        mdiff = ndiff[k];
                    }
                }
                tmp[idx] = md;
            }
        }
    }
    memcpy(disp, tmp, plane * sizeof(int32_t));
    free(tmp);
}

/* convertDisp2Gray, ADCensus.cpp:1241-1254 ((uchar) wraps values > 255). */
static void disp_to_gray(int H, int W, const int32_t* disp, uint8_t* gray) {
    const size_t plane = (size_t)H * W;
    uint8_t* tmp = (uint8_t*)malloc(plane);
    for (size_t i = 0; i < plane; ++i) tmp[i] = disp[i] < 0 ? 0 : (uint8_t)disp[i];
    orc_cv_equalize_hist(tmp, gray, H, W);
    free(tmp);
}

/* discontinuityAdjustment, ADCensus.cpp:1256-1342 */
static void discontinuity_adjustment(const orc_params* p, int H, int W, int32_t* disp,
                                     const float* cost0 /*[L][H][W]*/, uint8_t* gray_dump,
                                     uint8_t* edges_dump) {
    const size_t plane = (size_t)H * W;
    int32_t* tmp = (int32_t*)malloc(plane * sizeof(int32_t));
    memcpy(tmp, disp, plane * sizeof(int32_t));
    uint8_t* gray = (uint8_t*)malloc(plane);
    uint8_t* edges = (uint8_t*)malloc(plane);
    uint8_t* blurred = (uint8_t*)malloc(plane);
    disp_to_gray(H, W, disp, gray);
    orc_cv_blur3(gray, blurred, H, W); /* blurKernelSize = 3 */
    orc_cv_canny(blurred, edges, H, W, p->canny_thresh1, p->canny_thresh2);
    if (gray_dump) memcpy(gray_dump, gray, plane);
    if (edges_dump) memcpy(edges_dump, edges, plane);
    static const int dH[8] = {-1, 1, -1, 1, -1, 1, 0, 0};
    static const int dW[8] = {-1, 1, 0, 0, 1, -1, -1, 1};
    const int mind = p->min_disparity;
#define E(hh, ww) (edges[(size_t)(hh) * W + (ww)] != 0)
    for (int h = 1; h < H - 1; h++) {
        for (int w = 1; w < W - 1; w++) {
            if (!E(h, w)) continue;
            int direction = -1;
            if (E(h - 1, w - 1) && E(h + 1, w + 1)) direction = 0;
            else if (E(h - 1, w + 1) && E(h + 1, w - 1)) direction = 4;
            else if (E(h - 1, w) || E(h + 1, w)) {
                if (E(h - 1, w - 1) || E(h - 1, w) || E(h - 1, w + 1))
                    if (E(h + 1, w - 1) || E(h + 1, w) || E(h + 1, w + 1)) direction = 2;
            } else {
                if (E(h - 1, w - 1) || E(h, w - 1) || E(h + 1, w - 1))
                    if (E(h - 1, w + 1) || E(h, w + 1) || E(h + 1, w + 1)) direction = 6;
            }
            if (direction == -1) continue;
            int dsel = disp[(size_t)h * W + w];
            direction = (direction + 4) % 8;
            if (dsel >= mind) {
                float cost = cost0[(size_t)(dsel - mind) * plane + (size_t)h * W + w];
                int h1 = h + dH[direction], w1 = w + dW[direction];
                int h2 = h + dH[direction + 1], w2 = w + dW[direction + 1];
                int d1 = disp[(size_t)h1 * W + w1];
                int d2 = disp[(size_t)h2 * W + w2];
                float cost1 = d1 >= mind ? cost0[(size_t)(d1 - mind) * plane + (size_t)h1 * W + w1] : -1;
                float cost2 = d2 >= mind ? cost0[(size_t)(d2 - mind) * plane + (size_t)h2 * W + w2] : -1;
                if (cost1 != -1 && cost1 < cost) { dsel = d1; cost = cost1; }
                if (cost2 != -1 && cost2 < cost) { dsel = d2; }
            }
            tmp[(size_t)h * W + w] = dsel;
        }
    }
#undef E
    memcpy(disp, tmp, plane * sizeof(int32_t));
    free(tmp);
    free(gray);
    free(edges);
    free(blurred);
}

/* subpixelEnhancement, ADCensus.cpp:1344-1374 (median applied by the caller) */
static void subpixel_enhancement(const orc_params* p, int H, int W, const int32_t* disp,
                                 const float* cost0, float* out) {
    const size_t plane = (size_t)H * W;
    const int mind = p->min_disparity;
    for (size_t i = 0; i < plane; ++i) {
        int d = disp[i];
        float inter = (float)d;
        if (d > p->min_disparity && d < p->max_disparity) {
            float c = cost0[(size_t)(d - mind) * plane + i];
            float cp = cost0[(size_t)(d + 1 - mind) * plane + i];
            float cm = cost0[(size_t)(d - 1 - mind) * plane + i];
            float diff = (cp - cm) / (2 * (cp + cm - 2 * c));
            if (diff > -1 && diff < 1) inter -= diff;
        }
        out[i] = inter;
    }
}

/* ------------------------------------------------------------------------- */
/* HSI conversion (ADCensus.cpp:1429-1499)                                   */
/* ------------------------------------------------------------------------- */

#define ORC_CV_PI 3.1415926535897932384626433832795

static void bgr2hsi(const uint8_t* src, uint8_t* dst, int H, int W, int filter) {
    for (size_t i = 0; i < (size_t)H * W; ++i) {
        const uint8_t* s = src + i * 3;
        uint8_t* o = dst + i * 3;
        float b = s[0] / 255.f, g = s[1] / 255.f, r = s[2] / 255.f;
        float sum = b + g + r;
        float iv = sum / 3.0f;
        o[2] = (uint8_t)(iv * 255);
        float sv;
        if (sum == 0) sv = 0;
        else {
            float mn = b < g ? b : g; /* cv::min(cv::min(b,g),r) */
            mn = mn < r ? mn : r;
            sv = 1 - 3 * mn / sum;
        }
        o[1] = (uint8_t)(sv * 255);
        float den = sqrtf((r - g) * (r - g) + (r - b) * (g - b));
        float num = (2 * r - g - b) / 2.f;
        float hv;
        if (den == 0.f || den <= num || sv < 0.05f) hv = 0;
        else {
            float theta = acosf(num / den);
            hv = b <= g ? (float)(theta / (2 * ORC_CV_PI)) : (float)(1 - theta / (2 * ORC_CV_PI));
        }
        o[0] = (uint8_t)(hv * 255);
    }
    if (filter) {
        for (size_t i = 0; i < (size_t)H * W; ++i) {
            uint8_t* o = dst + i * 3;
            if (o[0] >= 60 || o[0] <= 10) o[0] = o[1] = o[2] = 0;
        }
    }
}

/* exported for the HSI conversion test (tests/test_gpu_parity.py) */
void orc_bgr2hsi(const uint8_t* src, uint8_t* dst, int H, int W, int filter) { bgr2hsi(src, dst, H, W, filter); }

static void gauss_median(const uint8_t* src, uint8_t* dst, int H, int W) {
    /* computeGaussMedian, ADCensus.cpp:1475-1499 */
    const size_t n = (size_t)H * W * 3;
    uint8_t* med = (uint8_t*)malloc(n);
    orc_cv_gauss3_filter2d(src, med, H, W);
    memcpy(dst, src, n);
    for (size_t i = 0; i < (size_t)H * W; ++i) {
        const uint8_t* s = src + i * 3;
        const uint8_t* m = med + i * 3;
        uint8_t* o = dst + i * 3;
        int hd = iabs((int)s[0] - (int)m[0]);
        hd = imin(hd, 255 - hd);
        if (hd >= 2) o[0] = m[0];
        for (int c = 1; c < 3; ++c)
            if (!(iabs((int)s[c] - (int)m[c]) < 3)) o[c] = m[c];
    }
    free(med);
}

/* ------------------------------------------------------------------------- */
/* public stage wrappers                                                     */
/* ------------------------------------------------------------------------- */

void orc_cost_initialize(const orc_params* p, const uint8_t* img0, const uint8_t* img1, int H,
                         int W, float* vol) {
    views_t v = {{img0, img1}, H, W};
    cost_initialize(p, &v, vol);
}

void orc_compute_limits(const orc_params* p, const uint8_t* img0, const uint8_t* img1, int H,
                        int W, int32_t* arms) {
    views_t v = {{img0, img1}, H, W};
    compute_limits(p, &v, arms);
}

void orc_cost_aggregate(const orc_params* p, int H, int W, const int32_t* arms, float* vol) {
    cost_aggregate(p, H, W, arms, vol);
}

void orc_scanline_optimize(const orc_params* p, const uint8_t* img0, const uint8_t* img1, int H,
                           int W, float* vol) {
    views_t v = {{img0, img1}, H, W};
    scanline_optimize(p, &v, vol);
}

/* ------------------------------------------------------------------------- */
/* ADCensus::compute                                                         */
/* ------------------------------------------------------------------------- */

int orc_compute(const orc_params* pin, const uint8_t* left, const uint8_t* right, int rows,
                int cols, size_t step, float* out, orc_dump* dump) {
    if (!left || !right || rows <= 0 || cols <= 0) return -1; /* :332-333 */
    orc_params P = *pin;
    orc_params* p = &P;
    const int H = rows, W = cols;
    const size_t plane = (size_t)H * W;
    if (p->roi_matching || p->mask_matching) p->max_disparity = W / 2; /* :339-340 */
    const int L = p->max_disparity - p->min_disparity + 1;
    if (L <= 0) return -2;

    /* dense BGR copies (clone, :336-337) */
    uint8_t* orig[2];
    uint8_t* img[2];
    for (int k = 0; k < 2; ++k) {
        const uint8_t* src = k == 0 ? left : right;
        orig[k] = (uint8_t*)malloc(plane * 3);
        img[k] = (uint8_t*)malloc(plane * 3);
        for (int h = 0; h < H; ++h) memcpy(orig[k] + (size_t)h * W * 3, src + (size_t)h * step, (size_t)W * 3);
        memcpy(img[k], orig[k], plane * 3);
    }
    if (p->color_model == ORC_HSI) { /* :351-371 */
        for (int k = 0; k < 2; ++k) {
            if (p->mask_matching || p->roi_matching) {
                bgr2hsi(orig[k], img[k], H, W, 1);
            } else {
                uint8_t* hsi = (uint8_t*)malloc(plane * 3);
                bgr2hsi(orig[k], hsi, H, W, 0);
                gauss_median(hsi, img[k], H, W);
                free(hsi);
            }
        }
    }
    if (dump && dump->images) {
        memcpy(dump->images, img[0], plane * 3);
        memcpy(dump->images + plane * 3, img[1], plane * 3);
    }
    views_t v = {{img[0], img[1]}, H, W};

    float* vol = (float*)malloc((size_t)2 * L * plane * sizeof(float));
    int32_t* arms = (int32_t*)malloc((size_t)8 * plane * sizeof(int32_t));
    if (!vol || !arms) {
        free(vol); free(arms);
        for (int k = 0; k < 2; ++k) { free(orig[k]); free(img[k]); }
        return -3;
    }

    cost_initialize(p, &v, vol);
    if (dump && dump->cost_init) memcpy(dump->cost_init, vol, (size_t)2 * L * plane * sizeof(float));
    compute_limits(p, &v, arms);
    if (dump && dump->arms) memcpy(dump->arms, arms, (size_t)8 * plane * sizeof(int32_t));
    cost_aggregate(p, H, W, arms, vol);
    if (dump && dump->cost_agg) memcpy(dump->cost_agg, vol, (size_t)2 * L * plane * sizeof(float));
    scanline_optimize(p, &v, vol);
    if (dump && dump->cost_scan) memcpy(dump->cost_scan, vol, (size_t)2 * L * plane * sizeof(float));

    /* multiOptimize, ADCensus.cpp:1376-1392 */
    int32_t* d0 = (int32_t*)malloc(plane * sizeof(int32_t));
    int32_t* d1 = (int32_t*)malloc(plane * sizeof(int32_t));
    int32_t* dm = (int32_t*)malloc(plane * sizeof(int32_t));
    orc_cost2disparity(p, H, W, vol, d0);
    orc_cost2disparity(p, H, W, vol + (size_t)L * plane, d1);
    if (dump && dump->wta) {
        memcpy(dump->wta, d0, plane * sizeof(int32_t));
        memcpy(dump->wta + plane, d1, plane * sizeof(int32_t));
    }
    outlier_elimination(p, H, W, d0, d1, dm);
    if (dump && dump->outlier) memcpy(dump->outlier, dm, plane * sizeof(int32_t));
    int hf = 0;
    for (int i = 0; i < 5; i++) {
        region_voting(p, H, W, dm, arms, hf);
        hf = !hf;
    }
    if (dump && dump->voting) memcpy(dump->voting, dm, plane * sizeof(int32_t));
    proper_interpolation(p, H, W, dm, img[0]);
    if (dump && dump->interp) memcpy(dump->interp, dm, plane * sizeof(int32_t));
    discontinuity_adjustment(p, H, W, dm, vol, dump ? dump->gray : NULL, dump ? dump->edges : NULL);
    if (dump && dump->adjusted) memcpy(dump->adjusted, dm, plane * sizeof(int32_t));
    float* sub = (float*)malloc(plane * sizeof(float));
    subpixel_enhancement(p, H, W, dm, vol, sub);
    if (dump && dump->subpix) memcpy(dump->subpix, sub, plane * sizeof(float));
    orc_cv_median3f(sub, out, H, W); /* :1372 */

    if (p->roi_matching || p->mask_matching) {
        for (size_t i = 0; i < plane; ++i) /* disparityOffset :1415-1427 */
            if (out[i] > 0) out[i] = out[i] + p->offset;
        for (size_t i = 0; i < plane; ++i) { /* :392-403 */
            if ((is_black(orig[0] + i * 3) && out[i] > 0) || out[i] == 0) out[i] = -1.f;
        }
    }

    free(sub); free(d0); free(d1); free(dm); free(vol); free(arms);
    for (int k = 0; k < 2; ++k) { free(orig[k]); free(img[k]); }
    return 0;
}
