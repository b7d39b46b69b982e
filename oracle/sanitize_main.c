/*
 * sanitize_main.c -- TEST INFRASTRUCTURE ONLY: drives the oracle (adcensus_oracle.c,
 * cvops.c) through every mode on small synthetic pairs so it can be built and run once
 * under AddressSanitizer + UndefinedBehaviorSanitizer and under ThreadSanitizer
 * (SURVEY.md §5 "Race detection / sanitizers"; `make -C oracle sanitize`).  The pairs come
 * from a fixed LCG (a textured left view, the right view a 5-px shift of it).  Every run
 * must finish with the same disparity checksum whatever the thread count: the OpenMP
 * stages are data-parallel and the racy scanline schedule is emulated deterministically.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "adcensus_oracle.h"

static void make_pair(int H, int W, uint8_t* l, uint8_t* r, int black) {
    uint32_t s = 2024u;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x)
            for (int c = 0; c < 3; ++c) {
                s = s * 1664525u + 1013904223u;
                l[(y * W + x) * 3 + c] = (uint8_t)(48 + ((x / 5 + y / 4 + 3 * c) * 29 + (s >> 27)) % 160);
            }
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x)
            for (int c = 0; c < 3; ++c) r[(y * W + x) * 3 + c] = l[(y * W + (x + 5 < W ? x + 5 : W - 1)) * 3 + c];
    if (black)  /* a black band and block: the ROI / mask rules */
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x)
                if (x < 6 || (y > H / 3 && y < H / 2 && x > W / 2 && x < W / 2 + 7))
                    for (int c = 0; c < 3; ++c) l[(y * W + x) * 3 + c] = r[(y * W + x) * 3 + c] = 0;
}

static double checksum(const float* d, int n) {
    double s = 0;
    for (int i = 0; i < n; ++i) s += (double)d[i] * (double)((i % 97) + 1);
    return s;
}

int main(int argc, char** argv) {
    const int threads = argc > 1 ? atoi(argv[1]) : 4;
    const int H = 40, W = 72;
    uint8_t* l = malloc((size_t)H * W * 3);
    uint8_t* r = malloc((size_t)H * W * 3);
    float* out = malloc((size_t)H * W * sizeof(float));
    struct { int model, roi, mask, minD, maxD, emu, win; } cases[] = {
        {ORC_RGB, 0, 0, 0, 16, 0, ORC_CENSUSWIN_9x7},
        {ORC_RGB, 0, 0, 3, 20, 5, ORC_CENSUSWIN_9x7},   /* minD > 0, racy-schedule emulation */
        {ORC_HSI, 0, 0, 0, 24, 0, ORC_CENSUSWIN_9x7},
        {ORC_RGB, 0, 0, 0, 12, 0, ORC_CENSUSWIN_7x5},
        {ORC_RGB, 1, 0, 0, 0, 0, ORC_CENSUSWIN_9x7},    /* ROI: maxD := W/2 */
        {ORC_HSI, 0, 1, 0, 0, 3, ORC_CENSUSWIN_9x7},    /* mask, HSI, emulation */
    };
    int fails = 0;
    for (size_t k = 0; k < sizeof(cases) / sizeof(cases[0]); ++k) {
        orc_params p;
        orc_default_params(&p, cases[k].model);
        p.roi_matching = cases[k].roi;
        p.mask_matching = cases[k].mask;
        p.min_disparity = cases[k].minD;
        p.max_disparity = cases[k].maxD ? cases[k].maxD : W / 2;
        p.scan_emulate_threads = cases[k].emu;
        p.census_win = cases[k].win;
        p.num_threads = threads;
        make_pair(H, W, l, r, cases[k].roi || cases[k].mask);
        const int L = p.max_disparity - p.min_disparity + 1;
        /* every stage dump as well: the dump paths are sanitized too */
        orc_dump d;
        memset(&d, 0, sizeof d);
        d.images = malloc((size_t)2 * H * W * 3);
        d.cost_init = malloc((size_t)2 * L * H * W * sizeof(float));
        d.arms = malloc((size_t)8 * H * W * sizeof(int32_t));
        d.cost_agg = malloc((size_t)2 * L * H * W * sizeof(float));
        d.cost_scan = malloc((size_t)2 * L * H * W * sizeof(float));
        d.wta = malloc((size_t)2 * H * W * sizeof(int32_t));
        d.outlier = malloc((size_t)H * W * sizeof(int32_t));
        d.voting = malloc((size_t)H * W * sizeof(int32_t));
        d.interp = malloc((size_t)H * W * sizeof(int32_t));
        d.gray = malloc((size_t)H * W);
        d.edges = malloc((size_t)H * W);
        d.adjusted = malloc((size_t)H * W * sizeof(int32_t));
        d.subpix = malloc((size_t)H * W * sizeof(float));
        const int rc = orc_compute(&p, l, r, H, W, (size_t)W * 3, out, &d);
        float* again = malloc((size_t)H * W * sizeof(float));
        const int rc2 = orc_compute(&p, l, r, H, W, (size_t)W * 3, again, NULL);
        const int same = rc == 0 && rc2 == 0 && memcmp(out, again, (size_t)H * W * sizeof(float)) == 0;
        printf("case %zu: rc=%d checksum=%.6f repeat=%s\n", k, rc, checksum(out, H * W), same ? "same" : "DIFF");
        fails += !same;
        free(again);
        free(d.images); free(d.cost_init); free(d.arms); free(d.cost_agg); free(d.cost_scan);
        free(d.wta); free(d.outlier); free(d.voting); free(d.interp); free(d.gray); free(d.edges);
        free(d.adjusted); free(d.subpix);
    }
    /* the setters' checks and an image error */
    fails += orc_check_disparity_range(-2, 5) != -2;
    fails += orc_check_disparity_range(0, 5) != 0;
    {
        orc_params p;
        orc_default_params(&p, ORC_RGB);
        fails += orc_compute(&p, l, r, 0, W, (size_t)W * 3, out, NULL) != -1;
    }
    free(l);
    free(r);
    free(out);
    printf("%s (%d failures)\n", fails ? "FAILED" : "OK", fails);
    return fails ? 1 : 0;
}
