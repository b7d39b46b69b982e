/*
 * tsm_adcensus.h -- C ABI of the MI355X-native AD-Census stereo matcher.
 *
 * This is the drop-in boundary for the reference's one hot path,
 * stereo::ADCensus (YYpasser/tea_stereo_matching include/stereo.h:388-422,
 * source/ADCensus.cpp).  Every entry point below names the reference member it
 * replaces.  Plain pointers and sizes only; no exceptions, no C++ or torch types
 * cross this boundary.  The C++ class in include/stereo.h and the Python mirror in
 * tea_stereo_matching_amd/ are thin layers over it.
 *
 * Images are BGR u8 interleaved (cv::Mat CV_8UC3) with a row `step` in bytes;
 * disparities are fp32 (CV_32FC1) with an `out_step` in bytes.  Invalid pixels
 * carry the reference's codes (-1 occlusion, -2 mismatch, possibly median-mixed).
 *
 * Threading: a handle is not thread-safe (as the reference's mutable PIMPL,
 * ADCensus.cpp:9-296).  Handles on different devices run concurrently.
 */
#ifndef TSM_ADCENSUS_H
#define TSM_ADCENSUS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TSM_ADC_ABI_VERSION 1

typedef struct tsm_adc tsm_adc;

/* Status codes.  The messages of the three validation errors are the reference's
 * thrown std::string texts (ADCensus.cpp:310, :326, :333). */
enum tsm_status {
    TSM_OK = 0,
    TSM_ERR_ARGUMENT = -1,        /* NULL handle/pointer, bad enum */
    TSM_ERR_DISPARITY_RANGE = -2, /* "[ADCensus] Set MinMaxDisparity error." */
    TSM_ERR_OFFSET = -3,          /* "[ADCensus] Offset must be positive." */
    TSM_ERR_IMAGE = -4,           /* "[ADCensus] Image error." */
    TSM_ERR_DEVICE = -5,          /* HIP runtime failure / no device */
    TSM_ERR_OUT_OF_MEMORY = -6,
    TSM_ERR_UNSUPPORTED = -7      /* configuration outside what the kernels support */
};

/* stereo::ColorModel (stereo_utils.h:191-195) */
enum tsm_color_model { TSM_COLOR_RGB = 0, TSM_COLOR_HSI = 1 };

/* stereo::ADCensusParams (stereo_utils.h:209-244); defaults from
 * setADCensusParams (stereo_utils.cpp:271-326). */
typedef struct tsm_adc_params {
    float lambda_ad;
    int census_win; /* 0 = 9x7, 1 = 7x5 (stereo_utils.h:200-204) */
    float lambda_census;
    float lambda_hue, lambda_saturation, lambda_intensity;
    int color_thresh1, color_thresh2;
    int saturation_thresh1, saturation_thresh2;
    int intensity_thresh1, intensity_thresh2;
    int max_length1, max_length2;
    int iterations;
    int color_diff;
    float pi1, pi2;
    int disp_tolerance;
    int voting_thresh;
    float voting_ratio_thresh;
    int max_search_depth;
    int blur_kernel_size;
    int canny_thresh1, canny_thresh2, canny_kernel_size;
} tsm_adc_params;

/* Per-stage host dumps in the REFERENCE layout (NULL = skip); test/debug only.
 * L = max - min + 1.  Volumes [view][d][H][W] fp32; arms [view][up,down,left,right][H][W]. */
typedef struct tsm_adc_dump {
    uint8_t* images;   /* [2][H][W][3] matched images (HSI-converted in HSI mode) */
    float* cost_init;  /* [2][L][H][W] costInitialize, ADCensus.cpp:522 */
    int32_t* arms;     /* [2][4][H][W] computeLimits, :661 */
    float* cost_agg;   /* [2][L][H][W] costAggregate, :753 */
    float* cost_scan;  /* [2][L][H][W] scanlineOptimize, :997 (view 1 not kept: see note) */
    int32_t* wta;      /* [2][H][W] cost2disparity, :1394 */
    int32_t* outlier;  /* [H][W] outlierElimination, :1013 */
    int32_t* voting;   /* [H][W] after 5x regionVoting, :1046 */
    int32_t* interp;   /* [H][W] properInterpolation, :1161 */
    uint8_t* gray;     /* [H][W] convertDisp2Gray, :1241 */
    uint8_t* edges;    /* [H][W] Canny edges, :1264 */
    int32_t* adjusted; /* [H][W] discontinuityAdjustment, :1256 */
    float* subpix;     /* [H][W] subpixelEnhancement before medianBlur, :1344 */
} tsm_adc_dump;

/* Stage ids for tsm_adc_stage_times. */
enum tsm_stage {
    TSM_STAGE_PREP = 0,      /* image packing / HSI conversion, census descriptors */
    TSM_STAGE_COST = 1,      /* cost-volume build (costInitialize) */
    TSM_STAGE_ARMS = 2,      /* cross arms + window sizes */
    TSM_STAGE_AGGREGATE = 3, /* 2*iterations 1-D aggregation passes */
    TSM_STAGE_SCANLINE = 4,  /* 4 chained passes x 2 views + fused WTA */
    TSM_STAGE_REFINE = 5,    /* outlier .. median */
    TSM_STAGE_COUNT = 6
};

/* ---- lifetime -------------------------------------------------------------- */

/* stereo::ADCensus::ADCensus() (ADCensus.cpp:298-301, Impl defaults :409-420:
 * HSI model, disparity [0, 64]).  `device` is a HIP ordinal. */
int tsm_adc_create(int device, tsm_adc** out);
/* stereo::ADCensus::~ADCensus() (ADCensus.cpp:303-305) */
int tsm_adc_destroy(tsm_adc* h);

/* ---- setters (reference API) -------------------------------------------- */

/* setMinMaxDisparity (stereo.h:399, ADCensus.cpp:307-313); inclusive range. */
int tsm_adc_set_disparity_range(tsm_adc* h, int min_disparity, int max_disparity);
/* setMatchingStrategy (stereo.h:406, ADCensus.cpp:315-321); resets params to the model's set. */
int tsm_adc_set_strategy(tsm_adc* h, int color_model, int roi_matching, int mask_matching);
/* setOffset (stereo.h:411, ADCensus.cpp:323-328). */
int tsm_adc_set_offset(tsm_adc* h, int offset);

/* ---- compute ----------------------------------------------------------------- */

/* compute(left, right, disparity) (stereo.h:418, ADCensus.cpp:330-407), host buffers,
 * synchronous.  out: rows x cols fp32 with out_step bytes per row. */
int tsm_adc_compute(tsm_adc* h, const uint8_t* left, const uint8_t* right, int rows, int cols,
                    size_t step, float* out, size_t out_step);
/* Same on device-resident buffers (HBM); enqueued on `hip_stream` (NULL = the handle's
 * stream) and NOT synchronised.  The handle's first workspace serves every call: a caller
 * stream first waits for the workspace's earlier work, and the workspace's stream then
 * waits for this pipeline, so calls on different streams never race on the workspace and
 * tsm_adc_synchronize also covers work enqueued on caller streams. */
int tsm_adc_compute_device(tsm_adc* h, const uint8_t* d_left, const uint8_t* d_right, int rows,
                           int cols, size_t step, float* d_out, size_t out_step, void* hip_stream);
/* Batch form, the precedent being ONNXRuntimeInference::compute(vector<Mat>...) (stereo.h:381).
 * Pairs run in groups of tsm_adc_set_concurrency pairs (one pipeline per group); synchronous.
 * On an error every stream is drained before returning, so no queued copy still touches
 * the caller's buffers. */
int tsm_adc_compute_batch(tsm_adc* h, int n, const uint8_t* const* lefts,
                          const uint8_t* const* rights, int rows, int cols, size_t step,
                          float* const* outs, size_t out_step);
int tsm_adc_compute_batch_device(tsm_adc* h, int n, const uint8_t* const* d_lefts,
                                 const uint8_t* const* d_rights, int rows, int cols, size_t step,
                                 float* const* d_outs, size_t out_step);
/* Wait for everything the handle enqueued. */
int tsm_adc_synchronize(tsm_adc* h);

/* ---- extensions (no reference counterpart) ------------------------------ */

int tsm_adc_get_params(const tsm_adc* h, tsm_adc_params* out);
int tsm_adc_set_params(tsm_adc* h, const tsm_adc_params* in);
int tsm_adc_get_disparity_range(const tsm_adc* h, int* min_disparity, int* max_disparity);
/* Pairs per group in the batch entry points (default 2, at most 64): a group of K pairs
 * runs as one pipeline whose every launch covers the K pairs (K pair slots in one arena),
 * and consecutive groups alternate between two streams.  Lowering it releases the HBM of
 * larger arenas (reallocated for the new group size on next use). */
int tsm_adc_set_concurrency(tsm_adc* h, int n_streams);
/* 0/1 (default): serial scanline semantics.  T > 1: reproduce the deterministic
 * lock-step outcome of the reference's racy omp-static scanline schedule on T threads
 * (ADCensus.cpp:801-853); T = 20 reproduces the shipped demo outputs bit-for-bit. */
int tsm_adc_set_omp_emulation(tsm_adc* h, int threads);
/* Debug run with per-stage dumps (reference layout); synchronous. */
int tsm_adc_compute_debug(tsm_adc* h, const uint8_t* left, const uint8_t* right, int rows,
                          int cols, size_t step, float* out, size_t out_step, tsm_adc_dump* dump);
/* Per-stage HIP-event timing (enable, then read accumulated ms and call counts). */
int tsm_adc_set_profiling(tsm_adc* h, int enable);
int tsm_adc_stage_times(tsm_adc* h, double* ms_sum, int* counts, int n);
int tsm_adc_reset_stage_times(tsm_adc* h);
/* Device bytes of ONE pair slot for a rows x cols pair at the current range and colour
 * model.  A handle holds up to two group arenas of `concurrency` slots each (batches),
 * plus input / output staging of the same count; single-frame calls use one slot. */
size_t tsm_adc_workspace_bytes(const tsm_adc* h, int rows, int cols);
/* bgr2hsi (ADCensus.cpp:1429-1473; filter != 0: the mask / ROI hue-band filter,
 * :1463-1470) on the device, BGR u8 in, H S I u8 out; synchronous.  The conversion the
 * HSI model runs before the census (test hook for its bit-exactness). */
int tsm_adc_convert_hsi(tsm_adc* h, const uint8_t* bgr, int rows, int cols, size_t step, int filter,
                        uint8_t* out, size_t out_step);
/* Last error message of the handle ("" if none). */
const char* tsm_adc_last_error(const tsm_adc* h);
/* Number of visible HIP devices (0 if none / no runtime). */
int tsm_device_count(void);
const char* tsm_version(void);

#ifdef __cplusplus
}
#endif
#endif /* TSM_ADCENSUS_H */
