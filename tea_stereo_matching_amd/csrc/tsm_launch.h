// tsm_launch.h -- host-side launchers of the gfx950 kernels (one per .hip file), called
// by the engine.  Each .hip file owns its kernels; no relocatable device code needed.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tsm_device.h"

namespace tsm {

// Debug hook (engine.cpp): with TSM_TRACE=1 in the environment, synchronise the stream
// after every launch and log the kernel name + status to stderr.  No-op otherwise.
void trace_point(const char* what, hipStream_t st);
// With TSM_TRACE=1: a zeroed two-word device flag of the current device and stream `st` that checked kernel
// variants set on a protocol violation ([0] = kind, [1] = detail) instead of addressing
// outside their buffers; trace_point reports and clears it.  nullptr when tracing is off.
uint32_t* trace_flag(hipStream_t st);

// Raise `kernel`'s dynamic-LDS limit to `bytes` on the current device, once per (kernel,
// device) and thread-safe (engine.cpp): handles on several threads may launch at once, and
// the attribute is a per-device property.  Launchers of kernels that may ask for more than
// 64 KB of dynamic LDS call it before every launch (a lookup under a mutex after the first).
void ensure_lds_limit(const void* kernel, size_t bytes);

// k_cost.hip
// Every launcher runs its stage for the group's P.npairs pairs (DevParams.pstride apart).
void launch_pack(const PairIn& in, size_t step, uint32_t* img, const DevParams& P, hipStream_t st);
// table: the 2^24-entry BGR -> HSI table (engine.cpp hsi_table)
void launch_hsi(const uint32_t* src, uint32_t* tmp, uint32_t* dst, int filter, const uint32_t* table,
                const DevParams& P, hipStream_t st);
// n packed pixels through bgr2hsi alone (tsm_adc_convert_hsi)
void launch_hsi_convert(const uint32_t* src, uint32_t* dst, int n, int filter, const uint32_t* table, hipStream_t st);
void launch_census(const uint32_t* img, uint32_t* desc, const DevParams& P, hipStream_t st);
size_t cost_volume_lds_bytes(const DevParams& P);
int launch_cost_volume(const uint32_t* desc, const float* lutA, int lutA_n, const float* lutB, float* vol,
                       const DevParams& P, hipStream_t st);

// k_aggregate.hip
void launch_arms(const uint32_t* img, uint32_t* arms, const DevParams& P, hipStream_t st);
void launch_window_sizes(const uint32_t* arms, int32_t* ws, const DevParams& P, hipStream_t st);
void launch_color_grad(const uint32_t* img, uint8_t* gv, uint8_t* gh, const DevParams& P,
                       hipStream_t st);
// One 1-D aggregation pass (fused: this pass and the next same-direction one) in place.
// ws: window sizes of a dividing pass (nullptr: no divide); ws_base: the window-size
// workspace (reciprocals, packed descriptors; k_window_sizes).  Arms longer than
// agg_max_streamer_arm() run one pass a launch (fused returns -1).  Returns 0 or -1.
int agg_max_streamer_arm();
int launch_aggregation_pass(float* vol, const uint32_t* arms, const int32_t* ws, const int32_t* ws_base,
                            int horizontal, bool fused, const DevParams& P, hipStream_t st);

// k_scanline.hip
// infvec: >= 16 bytes of +inf (the vector lanes past the label axis read)
int launch_scan_vertical(float* vol, const uint8_t* gv, const uint32_t* img, int dir,
                         const float* infvec, const DevParams& P, hipStream_t st);
int launch_scan_horizontal(float* vol, const uint8_t* gh, const uint32_t* img, int dir,
                           int32_t* wta, int store_view1, const float* infvec, const DevParams& P,
                           hipStream_t st);
// largest padded label count the scanline handles (label vectors a lane)
int scan_max_lp();

// k_refine.hip
struct RefineBufs {
    int32_t* disp0;   // WTA view 0           [H][W]
    int32_t* disp1;   // WTA view 1           [H][W]
    int32_t* dm;      // working disparity    [H][W]
    int32_t* dtmp;    // Jacobi scratch       [H][W]
    int32_t* out_list;// [H][W]
    int32_t* cvote;   // [H][W] vote count by outlier rank (out_pos order)
    uint16_t* csamp;  // [H][W][20] low-vote samples by outlier rank
    uint64_t* flags;  // single-pass scan flags (epoch << 32 | count), refine_flag_words
    int32_t* hv_list; // [H][W] ranks of the high-vote outliers of a voting pass, in rank order
    int32_t* long_list; // [H][W] list positions of the high-vote ranks with long carries
    int32_t* counts;  // [4]
    uint8_t* gray;    // [H][W]
    int32_t* hist;    // [256] histogram (+ 64 spare ints)
    uint8_t* gray_eq; // [H][W] equalised gray (debug dump)
    uint8_t* map;     // [H][W]
    int32_t* label;   // [H][W]
    uint8_t* strong;  // [H][W]
    uint8_t* edges;   // [H][W]
    float* subpix;    // [H][W]
    int32_t* vpre;    // valid-pixel prefix counts of a voting pass (refine_vpre_ints)
    uint32_t epoch = 0;  // voting launches so far on this workspace (tags the scan flags)
};
// ints of RefineBufs.vpre: raster ranks (H W + 1), column prefixes ((H+1) W + chunk prefixes)
size_t refine_vpre_ints(int H, int W);
size_t refine_scan_blocks(int n);
// 64-bit words of RefineBufs.flags
size_t refine_flag_words(int H, int W);
void launch_outlier(RefineBufs& B, const DevParams& P, hipStream_t st);
void launch_region_voting(RefineBufs& B, const uint32_t* arms0, int horizontal_first,
                          const DevParams& P, hipStream_t st);
void launch_interpolation(RefineBufs& B, const uint32_t* img0, const DevParams& P,
                          hipStream_t st);
void launch_discontinuity(RefineBufs& B, const float* vol0, const DevParams& P,
                          hipStream_t st);
// edge map, discontinuity adjustment, subpixel step, median + store (one launch); dm then
// holds the adjusted map
void launch_refine_tail(RefineBufs& B, const float* vol0, const uint32_t* orig_left, const PairOut& outs,
                        size_t out_step, int roi_or_mask, int offset, const DevParams& P, hipStream_t st);

// debug helpers (pair 0 of the group)
void launch_vol_to_ref(const float* vol, float* ref, int views, const DevParams& P,
                       hipStream_t st);
void launch_arms_to_ref(const uint32_t* arms, int32_t* ref, const DevParams& P, hipStream_t st);

}  // namespace tsm
