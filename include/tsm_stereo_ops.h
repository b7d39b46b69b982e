/*
 * tsm_stereo_ops.h -- C ABI of the gfx950 operators either side of the AD-Census path
 * (SURVEY §8f rows f2-f4): the JET colour map that renders a disparity, the
 * reprojections that turn it into depth / points (+ the PCD/PLY writers), and the
 * INTER_LINEAR remap that rectifies the input pair.  Same library as tsm_adcensus.h.
 *
 * Every operator has a host form (host buffers in and out, synchronous; the device
 * buffers are the library's) and a _device form (device buffers, enqueued on
 * `hip_stream`, NULL = the null stream, not synchronised).  Strides are in BYTES.
 * Status codes are tsm_adcensus.h's (TSM_OK, TSM_ERR_ARGUMENT, TSM_ERR_DEVICE, ...).
 *
 * Values follow the reference's loops bit for bit (fp32, no contraction); the float ->
 * u8 colour index cast follows x86 (out-of-range / NaN -> 0), what the reference's
 * MSVC x64 build executes for its undefined cases.
 */
#ifndef TSM_STEREO_OPS_H
#define TSM_STEREO_OPS_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- f2: colour map (source/stereo.cpp:75-134) ------------------------------ */

/* stereo::JETColorMap() (stereo.cpp:75-92): 256 BGR entries, lut[3*i + c]. */
int tsm_jet_colormap(uint8_t* lut768);

/* stereo::applyColorMap(src, dst, colorMap) (stereo.cpp:94-118) when use_range = 0:
 * range = min / max over pixels that are >= 0 and not inf, pixels < 0 black; and
 * applyColorMap(src, dst, minVal, maxVal, colorMap) (stereo.cpp:120-134) when
 * use_range = 1: pixels outside [min_val, max_val] black.  lut768: host BGR table,
 * NULL = JET.  disp: rows x cols fp32; bgr: rows x cols x 3 u8. */
int tsm_apply_colormap(const float* disp, int rows, int cols, size_t step, const uint8_t* lut768,
                       int use_range, float min_val, float max_val, uint8_t* bgr, size_t out_step);
int tsm_apply_colormap_device(const float* d_disp, int rows, int cols, size_t step,
                              const uint8_t* lut768, int use_range, float min_val, float max_val,
                              uint8_t* d_bgr, size_t out_step, void* hip_stream);

/* Group form: n maps of one size (n <= any; launched 64 maps at a time), e.g. a batch's
 * outputs straight from tsm_adc_compute_batch_device.  Per map, the same result as the
 * single call (auto range: each map's own min / max). */
int tsm_apply_colormap_batch_device(int n, const float* const* d_disps, int rows, int cols, size_t step,
                                    const uint8_t* lut768, int use_range, float min_val, float max_val,
                                    uint8_t* const* d_bgrs, size_t out_step, void* hip_stream);

/* ---- f3: reprojection and point clouds (source/stereo.cpp:136-356) --------- */

/* stereo::reprojectToDepth (stereo.cpp:136-148): depth = f*b / d, 0 where d < 0 or inf. */
int tsm_reproject_to_depth(const float* disp, int rows, int cols, size_t step, float focal,
                           float baseline, float* depth, size_t out_step);
int tsm_reproject_to_depth_device(const float* d_disp, int rows, int cols, size_t step, float focal,
                                  float baseline, float* d_depth, size_t out_step, void* hip_stream);

/* Group form (n maps of one size, 64 a launch). */
int tsm_reproject_to_depth_batch_device(int n, const float* const* d_disps, int rows, int cols, size_t step,
                                        float focal, float baseline, float* const* d_depths, size_t out_step,
                                        void* hip_stream);

/* stereo::reprojectTo3D(disparity, f, b, cx, cy, XYZ) (stereo.cpp:150-169): xyz is
 * rows x cols x 3 fp32 (CV_32FC3), 0 where d < 0 or inf. */
int tsm_reproject_to_3d(const float* disp, int rows, int cols, size_t step, float focal,
                        float baseline, float cx, float cy, float* xyz, size_t out_step);
int tsm_reproject_to_3d_device(const float* d_disp, int rows, int cols, size_t step, float focal,
                               float baseline, float cx, float cy, float* d_xyz, size_t out_step,
                               void* hip_stream);

/* Group form (n maps of one size, 64 a launch). */
int tsm_reproject_to_3d_batch_device(int n, const float* const* d_disps, int rows, int cols, size_t step,
                                     float focal, float baseline, float cx, float cy, float* const* d_xyzs,
                                     size_t out_step, void* hip_stream);

/* stereo::reprojectTo3D(disparity, Q, XYZ) (stereo.cpp:171-202): [x y z w] = Q [u v d 1]
 * with Q (row-major 4x4, CV_64F) converted to fp32, then x/w, y/w, z/w. */
int tsm_reproject_to_3d_q(const float* disp, int rows, int cols, size_t step, const double* q16,
                          float* xyz, size_t out_step);
int tsm_reproject_to_3d_q_device(const float* d_disp, int rows, int cols, size_t step,
                                 const double* q16, float* d_xyz, size_t out_step, void* hip_stream);

/* stereo::writePointCloudToPCD / writePointCloudToPLY (stereo.cpp:204-356): host only.
 * bgr rows x cols x 3 u8 (the colour image), xyz rows x cols x 3 fp32; points with a
 * +inf coordinate are skipped.  TSM_ERR_ARGUMENT on empty input (the reference logs and
 * returns, :252-256), TSM_ERR_IMAGE if the file cannot be written. */
int tsm_write_point_cloud_pcd(const uint8_t* bgr, size_t bgr_step, const float* xyz, size_t xyz_step,
                              int rows, int cols, const char* path);
int tsm_write_point_cloud_ply(const uint8_t* bgr, size_t bgr_step, const float* xyz, size_t xyz_step,
                              int rows, int cols, const char* path);

/* ---- f4: rectification remap (source/EpipolarRectify.cpp:87-101) ----------- */

/* cv::remap(src, dst, map1, map2, INTER_LINEAR) with the reference's CV_16SC2 +
 * CV_16UC1 maps (stereo_utils.cpp:164-167): xy = int16 (sx, sy) pairs, fxy = u16
 * fraction index fy*32 + fx.  src: src_rows x src_cols x channels u8 (1, 3 or 4);
 * dst: rows x cols x channels.  Border: constant 0. */
int tsm_remap_linear_fixed(const uint8_t* src, int src_rows, int src_cols, size_t src_step,
                           int channels, const int16_t* xy, size_t xy_step, const uint16_t* fxy,
                           size_t fxy_step, int rows, int cols, uint8_t* dst, size_t dst_step);
int tsm_remap_linear_fixed_device(const uint8_t* d_src, int src_rows, int src_cols, size_t src_step,
                                  int channels, const int16_t* d_xy, size_t xy_step,
                                  const uint16_t* d_fxy, size_t fxy_step, int rows, int cols,
                                  uint8_t* d_dst, size_t dst_step, void* hip_stream);
/* Group form: n images of one size through the same maps (every left view of a batch
 * through the left maps, EpipolarRectify.cpp:99), 64 a launch. */
int tsm_remap_linear_fixed_batch_device(int n, const uint8_t* const* d_srcs, int src_rows, int src_cols,
                                        size_t src_step, int channels, const int16_t* d_xy, size_t xy_step,
                                        const uint16_t* d_fxy, size_t fxy_step, int rows, int cols,
                                        uint8_t* const* d_dsts, size_t dst_step, void* hip_stream);
/* Same with CV_32FC1 x / y maps (rounded to 1/32 pixel, as cv::remap converts them). */
int tsm_remap_linear_float(const uint8_t* src, int src_rows, int src_cols, size_t src_step,
                           int channels, const float* mapx, const float* mapy, size_t map_step,
                           int rows, int cols, uint8_t* dst, size_t dst_step);
int tsm_remap_linear_float_device(const uint8_t* d_src, int src_rows, int src_cols, size_t src_step,
                                  int channels, const float* d_mapx, const float* d_mapy,
                                  size_t map_step, int rows, int cols, uint8_t* d_dst,
                                  size_t dst_step, void* hip_stream);

/* Wait for the work enqueued on `hip_stream` (NULL = the null stream) by the _device
 * forms. */
int tsm_stream_synchronize(void* hip_stream);

#ifdef __cplusplus
}
#endif
#endif /* TSM_STEREO_OPS_H */
