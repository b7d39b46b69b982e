// engine.cpp -- host orchestration of the AD-Census pipeline on one MI355X and the
// C ABI declared in include/tsm_adcensus.h.
//
// A handle (tsm_adc) holds the reference's matcher state (ADCensusImpl members,
// ADCensus.cpp:276-295) plus up to two group workspaces, each with its own HIP stream and
// one HBM arena of K pair slots sized for (H, W, L).  A group of K pairs runs as ONE
// pipeline: every launch covers all K pairs (blockIdx.z = pair, slots DevParams.pstride
// bytes apart), so the latency-bound stages (the row-serial scanline passes, the
// refinement chain) and the launch gaps are paid once per group rather than once per
// pair.  Batches alternate their groups between the two workspaces, so one group's tail
// overlaps the next group's head.  No host synchronisation inside a pipeline.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <limits>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <unistd.h>

#include "../../include/tsm_adcensus.h"
#include "copy_pool.h"
#include "tsm_launch.h"

using namespace tsm;

namespace tsm {
static bool trace_enabled() {
    static const bool trace = [] {  // read once (thread-safe static initialisation)
        const char* e = std::getenv("TSM_TRACE");
        return e && e[0] == '1';
    }();
    return trace;
}

// one flag per (device, stream): concurrent pipelines never report or clear each other's
// violations; read and cleared in stream order on the stream being traced
uint32_t* trace_flag(hipStream_t st) {
    if (!trace_enabled()) return nullptr;
    static std::mutex mu;
    static std::map<std::pair<int, hipStream_t>, uint32_t*> per_stream;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> g(mu);
    uint32_t*& f = per_stream[{dev, st}];
    if (!f && hipMalloc((void**)&f, 64) == hipSuccess) (void)hipMemset(f, 0, 64);
    return f;
}

void trace_point(const char* what, hipStream_t st) {
    if (!trace_enabled()) return;
    hipError_t le = hipGetLastError();
    hipError_t se = hipStreamSynchronize(st);
    std::fprintf(stderr, "[tsm] %-40s launch=%s sync=%s\n", what, hipGetErrorString(le), hipGetErrorString(se));
    if (uint32_t* f = trace_flag(st)) {
        uint32_t v[2] = {0, 0};
        if (hipMemcpyAsync(v, f, 8, hipMemcpyDeviceToHost, st) == hipSuccess && hipStreamSynchronize(st) == hipSuccess &&
            v[0] != 0) {
            std::fprintf(stderr, "[tsm] %-40s PROTOCOL CHECK FAILED: kind=%u detail=0x%08x\n", what, v[0], v[1]);
            (void)hipMemsetAsync(f, 0, 8, st);
            (void)hipStreamSynchronize(st);
        }
    }
    std::fflush(stderr);
}

void ensure_lds_limit(const void* kernel, size_t bytes) {
    static std::mutex mu;
    static std::map<std::pair<const void*, int>, size_t> set;  // (kernel, device) -> limit set
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> g(mu);
    size_t& cur = set[{kernel, dev}];
    if (bytes <= cur) return;
    if (hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) == hipSuccess)
        cur = bytes;
}
}  // namespace tsm

namespace {

const char* kMsgRange = "[ADCensus] Set MinMaxDisparity error.";  // ADCensus.cpp:310
const char* kMsgOffset = "[ADCensus] Offset must be positive.";    // ADCensus.cpp:326
const char* kMsgImage = "[ADCensus] Image error.";                 // ADCensus.cpp:333

// setADCensusParams, stereo_utils.cpp:271-326
void default_params(tsm_adc_params* p, int model) {
    std::memset(p, 0, sizeof(*p));
    p->lambda_ad = 10.f;
    p->census_win = 0;
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
    if (model == TSM_COLOR_RGB) {
        p->color_thresh1 = 20;
        p->color_thresh2 = 6;
        p->max_length1 = 34;
        p->max_length2 = 17;
        p->color_diff = 15;
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

struct Workspace {
    hipStream_t stream = nullptr;
    int H = 0, W = 0, L = 0, Lp = 0, model = -1, maxD = -1;
    float lambda_ad = 0, lambda_census = 0;
    int cap = 0;          // pair slots in the arena
    size_t slot = 0;      // bytes per pair slot (DevParams.pstride)
    size_t bytes = 0;
    // host-API staging: `cap` slots of in_cap bytes per input, H*W floats per output
    uint8_t* in_left = nullptr;
    uint8_t* in_right = nullptr;
    size_t in_cap = 0;
    int in_slots = 0;
    float* out_dev = nullptr;
    // host-batch staging in pinned memory (tsm_adc_compute_batch): the caller's pageable
    // images are copied in by the host and its outputs copied out once the group's stream
    // has drained, so every device copy is asynchronous and groups overlap
    uint8_t* h_in = nullptr;       // [2][slots][rows * cols * 3]: left images, then right
    float* h_out = nullptr;        // [slots][rows * cols]
    size_t h_in_bytes = 0, h_out_bytes = 0;
    std::vector<float*> pend_out;  // the caller's outputs of the group in flight
    int pend_rows = 0, pend_cols = 0;
    size_t pend_step = 0;
    // pair 0's buffers in the arena (pair p: + p * slot)
    uint32_t* img_orig = nullptr;  // [2][H][W] packed BGR
    uint32_t* img = nullptr;       // [2][H][W] matched images (== img_orig for RGB)
    uint32_t* img_tmp = nullptr;   // HSI scratch
    uint32_t* desc = nullptr;      // [2][H][W][16]
    float* vol = nullptr;          // [2][H][W][Lp]
    uint32_t* arms = nullptr;      // [2][H][W]
    int32_t* ws = nullptr;         // [2][2][H][W] window sizes, reciprocals, descriptors
    uint8_t* gv = nullptr;         // [2][H][gstride] (sentinel margins)
    uint8_t* gh = nullptr;         // [2][H][gstride]
    RefineBufs rb{};
    // shared by the group's pairs
    float* infvec = nullptr;       // 64 x +inf (scanline lanes past the label axis)
    float* lutA = nullptr;
    float* lutB = nullptr;
    int lutA_n = 0;
    std::vector<void*> allocs;
    // profiling: per group, its stage events and pair count
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::pair<std::vector<hipEvent_t>, int>> pending;
};

}  // namespace

struct tsm_adc {
    int device = 0;
    int min_disparity = 0;   // ADCensus.cpp:411
    int max_disparity = 64;  // ADCensus.cpp:412
    int color_model = TSM_COLOR_HSI;  // ADCensus.cpp:413
    int roi = 0, mask = 0, offset = 0;
    tsm_adc_params params{};
    int omp_threads = 0;
    int concurrency = 2;
    int ncu = 256;           // compute units of `device` (persistent-grid sizes)
    bool profiling = false;
    double stage_ms[TSM_STAGE_COUNT] = {};
    int stage_cnt[TSM_STAGE_COUNT] = {};
    std::vector<Workspace*> ws;
    std::string err;
};

namespace {

int fail(tsm_adc* h, int code, const std::string& msg) {
    if (h) h->err = msg;
    return code;
}

#define HIP_OK(expr)                                                                      \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return fail(h, TSM_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

int round_up4(int x) { return (x + 3) / 4 * 4; }

// Supported label range: the scanline holds a pixel's label vector in one wave, up to
// scan_max_lp() labels (8 float4 a lane); every other stage has no label limit.
int max_labels() { return scan_max_lp(); }

// BGR -> HSI conversion table (bgr2hsi, ADCensus.cpp:1429-1473): entry b | g << 8 | r << 16
// holds H | S << 8 | I << 16, computed with the reference's float expressions (no
// contraction: the library builds with -ffp-contract=off) and this host's libm acosf, so
// the device conversion is a lookup and bit-identical to the host's.  Built once per
// process (2^24 entries, 64 MiB, threads over the red channel), uploaded once per device.
const std::vector<uint32_t>& hsi_host_table() {
    static std::vector<uint32_t> tab;
    static std::once_flag once;
    std::call_once(once, [] {
        tab.resize((size_t)1 << 24);
        auto fill = [](uint32_t* t, int r0, int r1) {
            const double tp = 2 * 3.1415926535897932384626433832795;  // 2 * CV_PI
            for (int ri = r0; ri < r1; ++ri)
                for (int gi = 0; gi < 256; ++gi)
                    for (int bi = 0; bi < 256; ++bi) {
                        const float b = bi / 255.f, g = gi / 255.f, r = ri / 255.f;
                        const float sum = b + g + r;
                        const float iv = sum / 3.0f;
                        const uint32_t I = (uint8_t)(iv * 255);
                        float sv;
                        if (sum == 0) sv = 0;
                        else {
                            float mn = b < g ? b : g;  // cv::min(cv::min(b, g), r)
                            mn = mn < r ? mn : r;
                            sv = 1 - 3 * mn / sum;
                        }
                        const uint32_t S = (uint8_t)(sv * 255);
                        const float den = std::sqrt((r - g) * (r - g) + (r - b) * (g - b));
                        const float num = (2 * r - g - b) / 2.f;
                        float hv;
                        if (den == 0.f || den <= num || sv < 0.05f) hv = 0;
                        else {
                            const float theta = std::acos(num / den);  // float overload: acosf
                            hv = b <= g ? (float)(theta / tp) : (float)(1 - theta / tp);
                        }
                        const uint32_t Hh = (uint8_t)(hv * 255);
                        t[(size_t)bi | ((size_t)gi << 8) | ((size_t)ri << 16)] = Hh | (S << 8) | (I << 16);
                    }
        };
        const int nt = std::max(1, std::min(16, (int)std::thread::hardware_concurrency()));
        std::vector<std::thread> th;
        for (int k = 0; k < nt; ++k) th.emplace_back(fill, tab.data(), 256 * k / nt, 256 * (k + 1) / nt);
        for (auto& t : th) t.join();
    });
    return tab;
}

// The table in HBM of `device` (kept for the process; shared by every handle).
const uint32_t* hsi_device_table(int device) {
    static std::mutex mu;
    static std::vector<uint32_t*> per_dev;
    std::lock_guard<std::mutex> lk(mu);
    if ((int)per_dev.size() <= device) per_dev.resize(device + 1, nullptr);
    if (!per_dev[device]) {
        const std::vector<uint32_t>& t = hsi_host_table();
        uint32_t* d = nullptr;
        if (hipMalloc((void**)&d, t.size() * 4) != hipSuccess) return nullptr;
        if (hipMemcpy(d, t.data(), t.size() * 4, hipMemcpyHostToDevice) != hipSuccess) { hipFree(d); return nullptr; }
        per_dev[device] = d;
    }
    return per_dev[device];
}

void free_ws(Workspace* w) {
    for (void* p : w->allocs) hipFree(p);
    w->allocs.clear();
    w->bytes = 0;
    w->H = w->W = w->L = 0;
    w->cap = 0;
    w->slot = 0;
}

int alloc(tsm_adc* h, Workspace* w, void** p, size_t bytes) {
    bytes = (bytes + 255) & ~(size_t)255;
    hipError_t e = hipMalloc(p, bytes);
    if (e != hipSuccess) return fail(h, TSM_ERR_OUT_OF_MEMORY, std::string("hipMalloc: ") + hipGetErrorString(e));
    w->allocs.push_back(*p);
    w->bytes += bytes;
    return TSM_OK;
}

// Per-pair slot of the arena: every buffer a pair owns, at 256-B aligned offsets.  With
// `base` null it only measures (the offsets are what the pointers become).
struct SlotLayout {
    size_t off = 0;
    char* base = nullptr;
    template <class T>
    void take(T*& p, size_t bytes) {
        p = reinterpret_cast<T*>(base + off);
        off += (bytes + 255) & ~(size_t)255;
    }
};

void layout_slot(Workspace* w, SlotLayout& S, int H, int W, int L, int model) {
    const size_t N = (size_t)H * W;
    const int Lp = round_up4(L);
    S.take(w->img_orig, 2 * N * 4);
    if (model == TSM_COLOR_HSI) {
        S.take(w->img, 2 * N * 4);
        S.take(w->img_tmp, 2 * N * 4);
    } else {
        w->img = w->img_orig;
        w->img_tmp = nullptr;
    }
    S.take(w->desc, 2 * N * 16 * 4);
    S.take(w->vol, 2 * N * (size_t)Lp * 4);
    S.take(w->arms, 2 * N * 4);
    S.take(w->ws, 12 * N * 4);  // window sizes, reciprocals, packed descriptors (k_window_sizes)
    RefineBufs& B = w->rb;
    S.take(B.disp0, 2 * N * 4);  // [2][H][W]: the fused WTA writes view v at disp0 + v*N
    B.disp1 = B.disp0 + N;
    S.take(B.dm, N * 4);
    S.take(B.dtmp, N * 4);
    S.take(B.out_list, N * 4);
    S.take(B.cvote, N * 4);
    S.take(B.csamp, N * 20 * 2);
    S.take(B.flags, refine_flag_words(H, W) * 8 + 64);
    S.take(B.hv_list, N * 4);
    S.take(B.long_list, N * 4);
    S.take(B.counts, 16);
    S.take(B.gray, N);
    S.take(B.gray_eq, N);
    S.take(B.hist, (256 + 64) * 4);
    S.take(B.map, N);
    S.take(B.label, N * 4);
    S.take(B.strong, N);
    S.take(B.edges, N);
    S.take(B.subpix, N * 4);
    S.take(B.vpre, refine_vpre_ints(H, W) * 4);
}

// Bytes of one pair slot (the per-pair part of a workspace arena), as ensure_workspace
// lays it out for this range and colour model.
size_t slot_bytes(int H, int W, int L, int maxD, int model) {
    Workspace tmp;
    SlotLayout S;
    layout_slot(&tmp, S, H, W, L, model);
    const size_t gs = (size_t)(((W + 2 * grad_pad(maxD) + 15) / 16) * 16);
    S.take(tmp.gv, 2 * (size_t)H * gs + 64);
    S.take(tmp.gh, 2 * (size_t)H * gs + 64);
    return (S.off + 4095) & ~(size_t)4095;
}

// Host-built exp tables: the exact float arguments the reference hands to std::exp
// (ADCensus.cpp:518 with :426-452), evaluated by the host libm once.
void build_luts(const tsm_adc_params& p, int model, std::vector<float>& A, std::vector<float>& B) {
    if (model == TSM_COLOR_RGB) {
        A.resize(766);
        for (int s = 0; s < 766; ++s) {
            float ad = 0.f;
            ad = (float)s;  // exact integer sum of |dB|+|dG|+|dR|
            ad = ad / 3.f;
            A[s] = std::exp(-ad / p.lambda_ad);
        }
    } else {
        // ad = hueDiff*lambdaHue + satDiff*lambdaSat + intDiff*lambdaInt with the default
        // lambdas (1, 2.5, 2.5) is exactly k/2 for k = 2*hue + 5*(sat+int).
        A.resize(2805);
        for (int k = 0; k < 2805; ++k) {
            const float ad = (float)k / 2.f;
            A[k] = std::exp(-ad / p.lambda_ad);
        }
    }
    B.resize(188);
    for (int c = 0; c < 187; ++c) {
        const float cc = (float)c;
        B[c] = std::exp(-cc / p.lambda_census);
    }
    B[187] = 0.f;  // exp(-inf): mask-mode census of a black centre (:459-460)
}

DevParams make_params(const tsm_adc* h, int H, int W) {
    const tsm_adc_params& p = h->params;
    DevParams P{};
    P.H = H;
    P.W = W;
    P.minD = h->min_disparity;
    P.maxD = h->max_disparity;
    P.L = P.maxD - P.minD + 1;
    P.Lp = round_up4(P.L);
    P.ncu = h->ncu;
    P.color_model = h->color_model;
    P.mask = h->mask;
    P.censusW = p.census_win == 1 ? 7 : 9;
    P.censusH = p.census_win == 1 ? 5 : 7;
    P.color_thresh1 = p.color_thresh1;
    P.color_thresh2 = p.color_thresh2;
    P.sat_thresh1 = p.saturation_thresh1;
    P.sat_thresh2 = p.saturation_thresh2;
    P.int_thresh1 = p.intensity_thresh1;
    P.int_thresh2 = p.intensity_thresh2;
    P.max_length1 = p.max_length1;
    P.max_length2 = p.max_length2;
    P.color_diff = p.color_diff;
    P.pi1 = p.pi1;
    P.pi2 = p.pi2;
    // computeP1P2 :954-979 (float divisions as written)
    P.p1t[2] = p.pi1;
    P.p2t[2] = p.pi2;
    P.p1t[1] = p.pi1 / 4.f;
    P.p2t[1] = p.pi2 / 4.f;
    P.p1t[0] = p.pi1 / 10.f;
    P.p2t[0] = p.pi2 / 10.f;
    P.disp_tolerance = p.disp_tolerance;
    P.voting_thresh = p.voting_thresh;
    P.voting_ratio = p.voting_ratio_thresh;
    P.max_search_depth = p.max_search_depth;
    // Canny(…, low, high): cvFloor of the (swapped if needed) thresholds
    double lo = p.canny_thresh1, hi = p.canny_thresh2;
    if (lo > hi) std::swap(lo, hi);
    P.canny_low = (int)std::floor(lo);
    P.canny_high = (int)std::floor(hi);
    P.omp_threads = h->omp_threads;
    P.gpad = grad_pad(P.maxD);
    P.gstride = ((W + 2 * P.gpad + 15) / 16) * 16;
    return P;
}

// A group stream on a hardware queue of its own.  Plain streams share the process's
// GPU_MAX_HW_QUEUES hardware queues (4 by default), and once those are taken a new stream
// joins an existing queue: measured on the box, a handle created while another handle
// held its two streams got both of its group streams on ONE queue, so its two groups ran
// one after the other (385 against 420 pairs/s on the bench batch, tools/headline_ab.py,
// profiles/r06_stream_queues.txt).  A stream created with a CU mask always gets a new
// queue; the mask names every CU, so nothing else changes.
hipError_t create_group_stream(const tsm_adc* h, hipStream_t* s) {
    std::vector<uint32_t> mask((size_t)(h->ncu + 31) / 32, 0xffffffffu);
    if (h->ncu % 32) mask.back() = (1u << (h->ncu % 32)) - 1u;
    if (hipExtStreamCreateWithCUMask(s, (uint32_t)mask.size(), mask.data()) == hipSuccess) return hipSuccess;
    (void)hipGetLastError();
    return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}

// Workspace for groups of up to K pairs of H x W at the current range and model.
int ensure_workspace(tsm_adc* h, Workspace* w, int H, int W, int K) {
    const int L = h->max_disparity - h->min_disparity + 1;
    if (w->stream == nullptr) HIP_OK(create_group_stream(h, &w->stream));
    const tsm_adc_params& p = h->params;
    if (w->H == H && w->W == W && w->L == L && w->maxD == h->max_disparity && w->model == h->color_model &&
        w->lambda_ad == p.lambda_ad && w->lambda_census == p.lambda_census && w->cap >= K)
        return TSM_OK;
    HIP_OK(hipStreamSynchronize(w->stream));
    // a geometry / parameter change reallocates anyway: size the arena for the group the
    // caller needs now (a growing K on the same geometry keeps nothing to preserve either)
    const int cap = K;
    free_ws(w);
    if (w->in_left) { hipFree(w->in_left); w->in_left = nullptr; }
    if (w->in_right) { hipFree(w->in_right); w->in_right = nullptr; }
    if (w->out_dev) { hipFree(w->out_dev); w->out_dev = nullptr; }
    w->in_cap = 0;
    w->in_slots = 0;
    const size_t N = (size_t)H * W;
    const int Lp = round_up4(L);
    int rc;
#define A(ptr, bytes)                                                      \
    if ((rc = alloc(h, w, (void**)&(ptr), (bytes))) != TSM_OK) { free_ws(w); return rc; }
    // one arena of `cap` slots; pair 0's pointers are the slot offsets from its base
    SlotLayout S;
    layout_slot(w, S, H, W, L, h->color_model);
    const int gp = grad_pad(h->max_disparity);
    const size_t gs = (size_t)(((W + 2 * gp + 15) / 16) * 16);
    S.take(w->gv, 2 * (size_t)H * gs + 64);
    S.take(w->gh, 2 * (size_t)H * gs + 64);
    const size_t slot = (S.off + 4095) & ~(size_t)4095;
    char* arena = nullptr;
    A(arena, slot * (size_t)cap);
    S.off = 0;
    S.base = arena;
    layout_slot(w, S, H, W, L, h->color_model);
    S.take(w->gv, 2 * (size_t)H * gs + 64);
    S.take(w->gh, 2 * (size_t)H * gs + 64);
    A(w->infvec, 256);
    std::vector<float> la, lb;
    build_luts(p, h->color_model, la, lb);
    A(w->lutA, la.size() * 4);
    A(w->lutB, lb.size() * 4);
#undef A
    w->lutA_n = (int)la.size();
    HIP_OK(hipMemcpy(w->lutA, la.data(), la.size() * 4, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(w->lutB, lb.data(), lb.size() * 4, hipMemcpyHostToDevice));
    // padded lanes of the volumes are never read as labels; keep the arena defined anyway
    HIP_OK(hipMemset(arena, 0, slot * (size_t)cap));
    {
        std::vector<float> inf(64, std::numeric_limits<float>::infinity());
        HIP_OK(hipMemcpy(w->infvec, inf.data(), 256, hipMemcpyHostToDevice));
    }
    (void)N;
    (void)Lp;
    w->cap = cap;
    w->slot = slot;
    w->H = H;
    w->W = W;
    w->L = L;
    w->Lp = Lp;
    w->maxD = h->max_disparity;
    w->model = h->color_model;
    w->lambda_ad = p.lambda_ad;
    w->lambda_census = p.lambda_census;
    return TSM_OK;
}

// Host-API staging for K pairs: K input slots of H * step bytes per view, K outputs.
int ensure_input_staging(tsm_adc* h, Workspace* w, int H, size_t step, int W, int K) {
    const size_t need = (size_t)H * step;
    if (w->in_cap < need || w->in_slots < K) {
        if (w->in_left) { hipFree(w->in_left); w->in_left = nullptr; }
        if (w->in_right) { hipFree(w->in_right); w->in_right = nullptr; }
        if (w->out_dev) { hipFree(w->out_dev); w->out_dev = nullptr; }
        const size_t cap = std::max(need, w->in_cap);
        const int slots = std::max(K, w->in_slots);
        HIP_OK(hipMalloc((void**)&w->in_left, cap * slots));
        HIP_OK(hipMalloc((void**)&w->in_right, cap * slots));
        HIP_OK(hipMalloc((void**)&w->out_dev, (size_t)H * W * 4 * slots + 256));
        w->in_cap = cap;
        w->in_slots = slots;
    }
    return TSM_OK;
}

// Validation shared by every compute entry (ADCensus.cpp:332-340).
int validate(tsm_adc* h, const void* l, const void* r, int rows, int cols, size_t step) {
    if (!h) return TSM_ERR_ARGUMENT;
    if (!l || !r || rows <= 0 || cols <= 0 || step < (size_t)cols * 3)
        return fail(h, TSM_ERR_IMAGE, kMsgImage);
    if (h->roi || h->mask) h->max_disparity = cols / 2;  // :339-340 (persists, as in the reference)
    const int L = h->max_disparity - h->min_disparity + 1;
    if (L <= 1 || round_up4(L) > max_labels())
        return fail(h, TSM_ERR_UNSUPPORTED, "disparity range of " + std::to_string(L) + " labels is outside [2, " + std::to_string(max_labels()) + "]");
    if (h->min_disparity < 0)
        return fail(h, TSM_ERR_UNSUPPORTED, "negative minimum disparity (reference indexes its volume out of bounds, ADCensus.cpp:1398-1404)");
    // build_luts indexes the HSI AD table by 2*hue + 5*(sat + int), exact only for the
    // default weights (ADCensus.cpp:444-451); any census window, any other weights: refuse
    if (h->color_model == TSM_COLOR_HSI && (h->params.lambda_hue != 1.f || h->params.lambda_saturation != 2.5f ||
                                            h->params.lambda_intensity != 2.5f))
        return fail(h, TSM_ERR_UNSUPPORTED, "HSI AD lambdas other than (1, 2.5, 2.5)");
    return TSM_OK;
}

struct Prof {
    Workspace* w;
    std::vector<hipEvent_t> ev;
};

hipEvent_t take_event(Workspace* w) {
    if (!w->ev_pool.empty()) {
        hipEvent_t e = w->ev_pool.back();
        w->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    hipEventCreate(&e);
    return e;
}

// Enqueue the full pipeline for a group of K pairs on workspace w (K <= w->cap).
// in: device BGR images with `step`; outs: device fp32 maps with out_step.  Every launch
// covers the K pairs.  No host synchronisation (dumps, K = 1 only, synchronise).
int run_pipeline(tsm_adc* h, Workspace* w, int K, const PairIn& in, size_t step, const PairOut& outs,
                 size_t out_step, const tsm_adc_dump* dump, hipStream_t st) {
    const int H = w->H, W = w->W;
    DevParams P = make_params(h, H, W);
    P.pstride = w->slot;
    P.npairs = K;
    if (K < 1 || K > w->cap || K > kMaxGroup || (dump && K != 1))
        return fail(h, TSM_ERR_ARGUMENT, "pair group size");
    const size_t N = (size_t)H * W;
    std::vector<hipEvent_t> ev;
    auto mark = [&]() {
        if (!h->profiling) return;
        hipEvent_t e = take_event(w);
        hipEventRecord(e, st);
        ev.push_back(e);
    };
    auto dump_vol = [&](float* dst, int views) -> int {
        float* tmp = nullptr;
        HIP_OK(hipMalloc((void**)&tmp, (size_t)views * P.L * N * 4));
        launch_vol_to_ref(w->vol, tmp, views, P, st);
        HIP_OK(hipMemcpyAsync(dst, tmp, (size_t)views * P.L * N * 4, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        hipFree(tmp);
        return TSM_OK;
    };
    auto d2h = [&](void* dst, const void* src, size_t bytes) -> int {
        HIP_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        return TSM_OK;
    };
    int rc;
    auto mark_stage = [&]() { mark(); };

    mark_stage();
    // --- prep: pack (+HSI), census descriptors -------------------------------------
    launch_pack(in, step, w->img_orig, P, st);
    if (h->color_model == TSM_COLOR_HSI) {
        const uint32_t* tab = hsi_device_table(h->device);
        if (!tab) return fail(h, TSM_ERR_OUT_OF_MEMORY, "HSI conversion table");
        launch_hsi(w->img_orig, w->img_tmp, w->img, (h->roi || h->mask) ? 1 : 0, tab, P, st);
    }
    launch_census(w->img, w->desc, P, st);
    mark_stage();
    // --- cost volume -------------------------------------------------------------
    if (launch_cost_volume(w->desc, w->lutA, w->lutA_n, w->lutB, w->vol, P, st) != 0)
        return fail(h, TSM_ERR_UNSUPPORTED, "cost volume: label count");
    mark_stage();
    if (dump && dump->images) {
        std::vector<uint32_t> tmp(2 * N);
        if ((rc = d2h(tmp.data(), w->img, 2 * N * 4)) != TSM_OK) return rc;
        for (size_t i = 0; i < 2 * N; ++i) {
            dump->images[3 * i + 0] = tmp[i] & 0xff;
            dump->images[3 * i + 1] = (tmp[i] >> 8) & 0xff;
            dump->images[3 * i + 2] = (tmp[i] >> 16) & 0xff;
        }
    }
    if (dump && dump->cost_init && (rc = dump_vol(dump->cost_init, 2)) != TSM_OK) return rc;
    // --- arms, window sizes, colour gradients ----------------------------------------
    launch_arms(w->img, w->arms, P, st);
    launch_window_sizes(w->arms, w->ws, P, st);
    launch_color_grad(w->img, w->gv, w->gh, P, st);
    mark_stage();
    if (dump && dump->arms) {
        int32_t* tmp = nullptr;
        HIP_OK(hipMalloc((void**)&tmp, 8 * N * 4));
        launch_arms_to_ref(w->arms, tmp, P, st);
        rc = d2h(dump->arms, tmp, 8 * N * 4);
        hipFree(tmp);
        if (rc != TSM_OK) return rc;
    }
    // --- aggregation: iterations x (1-D pass, 1-D pass + divide) -----------------------
    {
        // costAggregate :776-782: iteration it runs (first orientation, no divide) then
        // (other orientation, divide by ws[hf]); hf alternates T,F,T,F.  Consecutive
        // same-direction passes (2nd of an iteration + 1st of the next) run fused.
        struct Pass { int horizontal; const int32_t* ws; };
        std::vector<Pass> passes;
        bool hf = true;
        for (int it = 0; it < h->params.iterations; ++it) {
            const int32_t* wsel = w->ws + (hf ? 0 : N);  // ws[v][hf?0:1] via the per-view stride 2N
            passes.push_back({hf ? 1 : 0, nullptr});
            passes.push_back({hf ? 0 : 1, wsel});
            hf = !hf;
        }
        // the persistent line streamers fuse each same-direction pass pair into one launch;
        // arms past their rings run one pass a launch
        const bool can_fuse = P.max_length1 - 1 <= agg_max_streamer_arm();
        for (size_t i = 0; i < passes.size(); ++i) {
            const Pass& a = passes[i];
            const bool pair = can_fuse && i + 1 < passes.size() && a.ws && !passes[i + 1].ws &&
                              passes[i + 1].horizontal == a.horizontal;
            if (launch_aggregation_pass(w->vol, w->arms, a.ws, w->ws, a.horizontal, pair, P, st) != 0)
                return fail(h, TSM_ERR_UNSUPPORTED, "aggregation: image too wide for the long-arm pass");
            if (pair) ++i;
        }
    }
    mark_stage();
    if (dump && dump->cost_agg && (rc = dump_vol(dump->cost_agg, 2)) != TSM_OK) return rc;
    // --- scanline, then WTA of both final volumes --------------------------------------
    const bool keep_view1 = dump && dump->cost_scan;
    // WTA fused into the leftward pass, which then never stores view 1's final volume
    // (only its argmin is used) unless a debug dump asks for it
    const bool ok = launch_scan_vertical(w->vol, w->gv, w->img, +1, w->infvec, P, st) == 0 &&
                    launch_scan_vertical(w->vol, w->gv, w->img, -1, w->infvec, P, st) == 0 &&
                    launch_scan_horizontal(w->vol, w->gh, w->img, +1, nullptr, 1, w->infvec, P, st) == 0 &&
                    launch_scan_horizontal(w->vol, w->gh, w->img, -1, w->rb.disp0, keep_view1 ? 1 : 0,
                                           w->infvec, P, st) == 0;
    if (!ok) return fail(h, TSM_ERR_UNSUPPORTED, "scanline: label count");
    mark_stage();
    if (keep_view1 && (rc = dump_vol(dump->cost_scan, 2)) != TSM_OK) return rc;
    if (dump && dump->wta && (rc = d2h(dump->wta, w->rb.disp0, 2 * N * 4)) != TSM_OK) return rc;
    // --- refinement --------------------------------------------------------------------
    launch_outlier(w->rb, P, st);
    if (dump && dump->outlier && (rc = d2h(dump->outlier, w->rb.dm, N * 4)) != TSM_OK) return rc;
    {
        int hf = 0;  // multiOptimize :1382-1387
        for (int i = 0; i < 5; ++i) {
            launch_region_voting(w->rb, w->arms, hf, P, st);
            hf = !hf;
        }
    }
    if (dump && dump->voting && (rc = d2h(dump->voting, w->rb.dm, N * 4)) != TSM_OK) return rc;
    launch_interpolation(w->rb, w->img, P, st);
    if (dump && dump->interp && (rc = d2h(dump->interp, w->rb.dm, N * 4)) != TSM_OK) return rc;
    launch_discontinuity(w->rb, w->vol, P, st);
    launch_refine_tail(w->rb, w->vol, w->img_orig, outs, out_step, (h->roi || h->mask) ? 1 : 0, h->offset, P, st);
    if (dump && dump->gray && (rc = d2h(dump->gray, w->rb.gray_eq, N)) != TSM_OK) return rc;
    if (dump && dump->edges && (rc = d2h(dump->edges, w->rb.edges, N)) != TSM_OK) return rc;
    if (dump && dump->adjusted && (rc = d2h(dump->adjusted, w->rb.dm, N * 4)) != TSM_OK) return rc;
    if (dump && dump->subpix && (rc = d2h(dump->subpix, w->rb.subpix, N * 4)) != TSM_OK) return rc;
    mark_stage();
    HIP_OK(hipGetLastError());
    if (h->profiling) w->pending.emplace_back(ev, K);
    return TSM_OK;
}

// Fold finished groups' events into the handle's stage totals (call after sync): a
// group's stage span counts once per pair it carried, so ms / count is per pair.
void collect_profile(tsm_adc* h, Workspace* w) {
    for (auto& [ev, K] : w->pending) {
        for (size_t k = 0; k + 1 < ev.size() && k < TSM_STAGE_COUNT; ++k) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, ev[k], ev[k + 1]) == hipSuccess) {
                h->stage_ms[k] += ms;
                h->stage_cnt[k] += K;
            }
        }
        for (hipEvent_t e : ev) w->ev_pool.push_back(e);
    }
    w->pending.clear();
}

int ensure_pool(tsm_adc* h, int n) {
    while ((int)h->ws.size() < n) h->ws.push_back(new Workspace());
    return TSM_OK;
}

int set_device(tsm_adc* h) {
    HIP_OK(hipSetDevice(h->device));
    return TSM_OK;
}

// Make stream `after` wait for everything enqueued so far on stream `before`.
int stream_after(tsm_adc* h, Workspace* w, hipStream_t before, hipStream_t after) {
    if (before == after) return TSM_OK;
    hipEvent_t e = take_event(w);
    HIP_OK(hipEventRecord(e, before));
    HIP_OK(hipStreamWaitEvent(after, e, 0));
    w->ev_pool.push_back(e);  // reusable: the wait captured the recorded state
    return TSM_OK;
}

// Pinned output staging of the group that ran on w -> the caller's buffers (row by row
// when the caller's row step is wider).  The stream must have drained.
void copy_out_pending(Workspace* w) {
    const size_t rowb = (size_t)w->pend_cols * 4, img = (size_t)w->pend_rows * w->pend_cols;
    for (size_t j = 0; j < w->pend_out.size(); ++j)
        copy_rows(w->pend_out[j], w->pend_step, w->h_out + j * img, rowb, rowb, w->pend_rows);
    w->pend_out.clear();
}

// After an error in a batch, queued copies may still read/write caller buffers: drain
// every workspace stream before handing the error back (keeps the first error message).
int drain_after_error(tsm_adc* h, int rc) {
    const std::string msg = h->err;
    for (Workspace* w : h->ws) {
        // groups already enqueued by a failing host batch still hand their outputs over
        // (they were validated and ran); nothing is left pending for a later call
        if (w->stream && hipStreamSynchronize(w->stream) == hipSuccess) copy_out_pending(w);
        w->pend_out.clear();
    }
    h->err = msg;
    return rc;
}

}  // namespace

// ============================================================================
// C ABI
// ============================================================================
extern "C" {

int tsm_adc_create(int device, tsm_adc** out) {
    if (!out) return TSM_ERR_ARGUMENT;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return TSM_ERR_DEVICE;
    if (device < 0 || device >= n) return TSM_ERR_ARGUMENT;
    tsm_adc* h = new tsm_adc();
    h->device = device;
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0)
        h->ncu = ncu;
    default_params(&h->params, h->color_model);
    *out = h;
    return TSM_OK;
}

int tsm_adc_destroy(tsm_adc* h) {
    if (!h) return TSM_ERR_ARGUMENT;
    hipSetDevice(h->device);
    for (Workspace* w : h->ws) {
        if (w->stream) hipStreamSynchronize(w->stream);
        free_ws(w);
        if (w->in_left) hipFree(w->in_left);
        if (w->in_right) hipFree(w->in_right);
        if (w->out_dev) hipFree(w->out_dev);
        if (w->h_in) hipHostFree(w->h_in);
        if (w->h_out) hipHostFree(w->h_out);
        for (auto& pe : w->pending) for (hipEvent_t e : pe.first) hipEventDestroy(e);
        for (hipEvent_t e : w->ev_pool) hipEventDestroy(e);
        if (w->stream) hipStreamDestroy(w->stream);
        delete w;
    }
    delete h;
    return TSM_OK;
}

int tsm_adc_set_disparity_range(tsm_adc* h, int mn, int mx) {
    if (!h) return TSM_ERR_ARGUMENT;
    if ((long long)mn * (long long)mx < 0 || mn >= mx) return fail(h, TSM_ERR_DISPARITY_RANGE, kMsgRange);
    h->min_disparity = mn;
    h->max_disparity = mx;
    return TSM_OK;
}

int tsm_adc_get_disparity_range(const tsm_adc* h, int* mn, int* mx) {
    if (!h || !mn || !mx) return TSM_ERR_ARGUMENT;
    *mn = h->min_disparity;
    *mx = h->max_disparity;
    return TSM_OK;
}

int tsm_adc_set_strategy(tsm_adc* h, int model, int roi, int mask) {
    if (!h) return TSM_ERR_ARGUMENT;
    if (model != TSM_COLOR_RGB && model != TSM_COLOR_HSI) return fail(h, TSM_ERR_ARGUMENT, "unknown color model");
    h->color_model = model;
    default_params(&h->params, model);  // m_paMatching = ADCensusParams(colorModel)
    h->roi = roi ? 1 : 0;
    h->mask = mask ? 1 : 0;
    return TSM_OK;
}

int tsm_adc_set_offset(tsm_adc* h, int offset) {
    if (!h) return TSM_ERR_ARGUMENT;
    if (offset < 0) return fail(h, TSM_ERR_OFFSET, kMsgOffset);
    h->offset = offset;
    return TSM_OK;
}

int tsm_adc_get_params(const tsm_adc* h, tsm_adc_params* out) {
    if (!h || !out) return TSM_ERR_ARGUMENT;
    *out = h->params;
    return TSM_OK;
}

int tsm_adc_set_params(tsm_adc* h, const tsm_adc_params* in) {
    if (!h || !in) return TSM_ERR_ARGUMENT;
    if (in->census_win != 0 && in->census_win != 1) return fail(h, TSM_ERR_ARGUMENT, "census_win must be 0 (9x7) or 1 (7x5)");
    // arms are packed as bytes (arm <= maxLength1 - 1 <= 255)
    if (in->max_length1 < 1 || in->max_length1 > 256) return fail(h, TSM_ERR_UNSUPPORTED, "max_length1 outside [1, 256]");
    // the refinement keeps at most 20 carried samples per low-vote outlier
    if (in->voting_thresh > 20 || in->voting_thresh < 0) return fail(h, TSM_ERR_UNSUPPORTED, "voting_thresh outside [0, 20]");
    // colorDiff + 1 is the byte sentinel of the scanline's colour-difference maps
    if (in->color_diff < 0 || in->color_diff > 254) return fail(h, TSM_ERR_UNSUPPORTED, "color_diff outside [0, 254]");
    if (in->iterations < 0) return fail(h, TSM_ERR_ARGUMENT, "iterations must be >= 0");
    // k_eq_blur / k_sobel are the fixed 3x3 cv::blur / cv::Canny apertures (ADCensus.cpp:1263-1264)
    if (in->blur_kernel_size != 3) return fail(h, TSM_ERR_UNSUPPORTED, "blur_kernel_size other than 3");
    if (in->canny_kernel_size != 3) return fail(h, TSM_ERR_UNSUPPORTED, "canny_kernel_size other than 3");
    h->params = *in;
    return TSM_OK;
}

int tsm_adc_set_concurrency(tsm_adc* h, int n) {
    if (!h || n < 1 || n > kMaxGroup) return TSM_ERR_ARGUMENT;
    h->concurrency = n;
    // a smaller group size gives back the HBM of larger arenas (reallocated on next use)
    if (set_device(h) != TSM_OK) return TSM_ERR_DEVICE;
    for (Workspace* w : h->ws) {
        if (w->cap <= n) continue;
        if (w->stream && hipStreamSynchronize(w->stream) == hipSuccess) copy_out_pending(w);
        w->pend_out.clear();
        collect_profile(h, w);
        free_ws(w);
    }
    return TSM_OK;
}

int tsm_adc_set_omp_emulation(tsm_adc* h, int threads) {
    if (!h || threads < 0) return TSM_ERR_ARGUMENT;
    h->omp_threads = threads;
    return TSM_OK;
}

int tsm_adc_set_profiling(tsm_adc* h, int enable) {
    if (!h) return TSM_ERR_ARGUMENT;
    h->profiling = enable != 0;
    return TSM_OK;
}

int tsm_adc_stage_times(tsm_adc* h, double* ms, int* counts, int n) {
    if (!h) return TSM_ERR_ARGUMENT;
    for (int k = 0; k < n && k < TSM_STAGE_COUNT; ++k) {
        if (ms) ms[k] = h->stage_ms[k];
        if (counts) counts[k] = h->stage_cnt[k];
    }
    return TSM_OK;
}

int tsm_adc_reset_stage_times(tsm_adc* h) {
    if (!h) return TSM_ERR_ARGUMENT;
    for (int k = 0; k < TSM_STAGE_COUNT; ++k) { h->stage_ms[k] = 0; h->stage_cnt[k] = 0; }
    return TSM_OK;
}

size_t tsm_adc_workspace_bytes(const tsm_adc* h, int rows, int cols) {
    if (!h || rows <= 0 || cols <= 0) return 0;
    const int maxd = (h->roi || h->mask) ? cols / 2 : h->max_disparity;
    return slot_bytes(rows, cols, maxd - h->min_disparity + 1, maxd, h->color_model);
}

const char* tsm_adc_last_error(const tsm_adc* h) { return h ? h->err.c_str() : "null handle"; }

int tsm_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char* tsm_version(void) { return "tea_stereo_matching_amd 0.1.0 (gfx950)"; }

int tsm_adc_synchronize(tsm_adc* h) {
    if (!h) return TSM_ERR_ARGUMENT;
    int rc;
    if ((rc = set_device(h)) != TSM_OK) return rc;
    for (Workspace* w : h->ws) {
        if (!w->stream) continue;
        HIP_OK(hipStreamSynchronize(w->stream));
        collect_profile(h, w);
    }
    return TSM_OK;
}

int tsm_adc_compute_device(tsm_adc* h, const uint8_t* dl, const uint8_t* dr, int rows, int cols,
                           size_t step, float* dout, size_t out_step, void* stream) {
    int rc = validate(h, dl, dr, rows, cols, step);
    if (rc != TSM_OK) return rc;
    if (!dout || out_step < (size_t)cols * 4) return fail(h, TSM_ERR_ARGUMENT, "output buffer");
    if ((rc = set_device(h)) != TSM_OK) return rc;
    ensure_pool(h, 1);
    Workspace* w = h->ws[0];
    if ((rc = ensure_workspace(h, w, rows, cols, 1)) != TSM_OK) return rc;
    hipStream_t st = stream ? (hipStream_t)stream : w->stream;
    // The workspace buffers belong to w->stream: the caller's stream first waits for
    // the workspace's earlier work, and w->stream then waits for this pipeline, so
    // later calls on any stream (and tsm_adc_synchronize) are ordered after it.
    if ((rc = stream_after(h, w, w->stream, st)) != TSM_OK) return rc;
    PairIn in{};
    PairOut out{};
    in.left[0] = dl;
    in.right[0] = dr;
    out.out[0] = dout;
    if ((rc = run_pipeline(h, w, 1, in, step, out, out_step, nullptr, st)) != TSM_OK) return rc;
    return stream_after(h, w, st, w->stream);
}

// H2D of pair i of a host batch into staging slot k of w (device step 3 * cols).
static int ensure_pinned(tsm_adc* h, Workspace* w, int rows, int cols, int K);
static int stage_pinned_pair(tsm_adc* h, Workspace* w, int K, int j, const uint8_t* l, const uint8_t* r,
                             int rows, int cols, size_t step, PairIn& in);

static int compute_host(tsm_adc* h, const uint8_t* l, const uint8_t* r, int rows, int cols,
                        size_t step, float* out, size_t out_step, const tsm_adc_dump* dump) {
    int rc = validate(h, l, r, rows, cols, step);
    if (rc != TSM_OK) return rc;
    if (!out || out_step < (size_t)cols * 4) return fail(h, TSM_ERR_ARGUMENT, "output buffer");
    if ((rc = set_device(h)) != TSM_OK) return rc;
    ensure_pool(h, 1);
    Workspace* w = h->ws[0];
    if ((rc = ensure_workspace(h, w, rows, cols, 1)) != TSM_OK) return rc;
    if ((rc = ensure_input_staging(h, w, rows, (size_t)cols * 3, cols, 1)) != TSM_OK) return rc;
    if ((rc = ensure_pinned(h, w, rows, cols, 1)) != TSM_OK) return rc;
    PairIn in{};
    PairOut po{};
    // pageable caller buffers go through pinned staging (a pageable copy costs ~6 ms a
    // config-B frame, the whole pipeline ~4)
    if ((rc = stage_pinned_pair(h, w, 1, 0, l, r, rows, cols, step, in)) != TSM_OK) return drain_after_error(h, rc);
    po.out[0] = w->out_dev;
    if ((rc = run_pipeline(h, w, 1, in, (size_t)cols * 3, po, (size_t)cols * 4, dump, w->stream)) != TSM_OK)
        return drain_after_error(h, rc);
    HIP_OK(hipMemcpyAsync(w->h_out, w->out_dev, (size_t)rows * cols * 4, hipMemcpyDeviceToHost, w->stream));
    w->pend_out.assign(1, out);
    w->pend_rows = rows;
    w->pend_cols = cols;
    w->pend_step = out_step;
    if (hipStreamSynchronize(w->stream) != hipSuccess) {
        w->pend_out.clear();
        return fail(h, TSM_ERR_DEVICE, "hipStreamSynchronize");
    }
    copy_out_pending(w);
    collect_profile(h, w);
    return TSM_OK;
}

int tsm_adc_convert_hsi(tsm_adc* h, const uint8_t* bgr, int rows, int cols, size_t step, int filter,
                        uint8_t* out, size_t out_step) {
    if (!h || !bgr || !out || rows <= 0 || cols <= 0 || step < (size_t)cols * 3 || out_step < (size_t)cols * 3)
        return TSM_ERR_ARGUMENT;
    int rc;
    if ((rc = set_device(h)) != TSM_OK) return rc;
    const uint32_t* tab = hsi_device_table(h->device);
    if (!tab) return fail(h, TSM_ERR_OUT_OF_MEMORY, "HSI conversion table");
    const size_t n = (size_t)rows * cols;
    if (n > (size_t)1 << 30) return fail(h, TSM_ERR_ARGUMENT, "image too large");
    std::vector<uint32_t> packed(n);
    for (int y = 0; y < rows; ++y)
        for (int x = 0; x < cols; ++x) {
            const uint8_t* s = bgr + (size_t)y * step + (size_t)x * 3;
            packed[(size_t)y * cols + x] = s[0] | (s[1] << 8) | (s[2] << 16);
        }
    uint32_t* d = nullptr;
    HIP_OK(hipMalloc((void**)&d, 2 * n * 4));
    hipStream_t st = nullptr;
    rc = TSM_OK;
    if (hipMemcpy(d, packed.data(), n * 4, hipMemcpyHostToDevice) != hipSuccess) rc = TSM_ERR_DEVICE;
    if (rc == TSM_OK) {
        launch_hsi_convert(d, d + n, (int)n, filter ? 1 : 0, tab, st);
        if (hipMemcpy(packed.data(), d + n, n * 4, hipMemcpyDeviceToHost) != hipSuccess) rc = TSM_ERR_DEVICE;
    }
    hipFree(d);
    if (rc != TSM_OK) return fail(h, rc, "bgr2hsi on the device");
    for (int y = 0; y < rows; ++y)
        for (int x = 0; x < cols; ++x) {
            const uint32_t v = packed[(size_t)y * cols + x];
            uint8_t* o = out + (size_t)y * out_step + (size_t)x * 3;
            o[0] = v & 0xff;
            o[1] = (v >> 8) & 0xff;
            o[2] = (v >> 16) & 0xff;
        }
    return TSM_OK;
}

int tsm_adc_compute(tsm_adc* h, const uint8_t* l, const uint8_t* r, int rows, int cols, size_t step,
                    float* out, size_t out_step) {
    return compute_host(h, l, r, rows, cols, step, out, out_step, nullptr);
}

int tsm_adc_compute_debug(tsm_adc* h, const uint8_t* l, const uint8_t* r, int rows, int cols,
                          size_t step, float* out, size_t out_step, tsm_adc_dump* dump) {
    return compute_host(h, l, r, rows, cols, step, out, out_step, dump);
}

// Batches run in groups of K = concurrency pairs, alternating between two group
// workspaces (two streams) when there is more than one group (three measured no faster:
// DESIGN §7).  K = 1 keeps one workspace: pairs then run strictly one after another
// (per-stage timing alone).
static int group_plan(tsm_adc* h, int n, int& K, int& nws) {
    constexpr int kGroupStreams = 2;
    K = std::min(h->concurrency, kMaxGroup);
    nws = (n > K && K > 1) ? std::min(kGroupStreams, (n + K - 1) / K) : 1;
    return ensure_pool(h, nws);
}

// Pinned host staging of a group of K pairs (grown, never shrunk).
static int ensure_pinned(tsm_adc* h, Workspace* w, int rows, int cols, int K) {
    const size_t in_need = (size_t)2 * K * rows * cols * 3, out_need = (size_t)K * rows * cols * 4;
    if (w->h_in_bytes < in_need) {
        if (w->h_in) hipHostFree(w->h_in);
        w->h_in = nullptr;
        w->h_in_bytes = 0;
        HIP_OK(hipHostMalloc((void**)&w->h_in, in_need, hipHostMallocDefault));
        w->h_in_bytes = in_need;
    }
    if (w->h_out_bytes < out_need) {
        if (w->h_out) hipHostFree(w->h_out);
        w->h_out = nullptr;
        w->h_out_bytes = 0;
        HIP_OK(hipHostMalloc((void**)&w->h_out, out_need, hipHostMallocDefault));
        w->h_out_bytes = out_need;
    }
    return TSM_OK;
}

// Pair j of a group of K: the caller's (pageable) images -> pinned staging on the host,
// then an async copy into the workspace's device input slot.
static int stage_pinned_pair(tsm_adc* h, Workspace* w, int K, int j, const uint8_t* l, const uint8_t* r,
                             int rows, int cols, size_t step, PairIn& in) {
    const size_t rowb = (size_t)cols * 3, img = rowb * rows;
    for (int side = 0; side < 2; ++side) {
        const uint8_t* src = side ? r : l;
        uint8_t* pin = w->h_in + ((size_t)side * K + j) * img;
        copy_rows(pin, rowb, src, step, rowb, rows);
        uint8_t* dst = (side ? w->in_right : w->in_left) + (size_t)j * w->in_cap;
        HIP_OK(hipMemcpyAsync(dst, pin, img, hipMemcpyHostToDevice, w->stream));
        (side ? in.right[j] : in.left[j]) = dst;
    }
    return TSM_OK;
}

// Wait for the group in flight on w and hand its outputs over.
static int flush_outputs(tsm_adc* h, Workspace* w) {
    if (w->pend_out.empty()) return TSM_OK;
    HIP_OK(hipStreamSynchronize(w->stream));
    copy_out_pending(w);
    return TSM_OK;
}

int tsm_adc_compute_batch_device(tsm_adc* h, int n, const uint8_t* const* dls,
                                 const uint8_t* const* drs, int rows, int cols, size_t step,
                                 float* const* douts, size_t out_step) {
    if (!h || n < 0 || (n > 0 && (!dls || !drs || !douts))) return TSM_ERR_ARGUMENT;
    int rc;
    if ((rc = set_device(h)) != TSM_OK) return rc;
    for (int i = 0; i < n; ++i) {  // everything is checked before anything is enqueued
        if ((rc = validate(h, dls[i], drs[i], rows, cols, step)) != TSM_OK) return rc;
        if (!douts[i] || out_step < (size_t)cols * 4) return fail(h, TSM_ERR_ARGUMENT, "output buffer");
    }
    int K, nws;
    group_plan(h, n, K, nws);
    for (int g = 0, i0 = 0; i0 < n; ++g, i0 += K) {
        const int k = std::min(K, n - i0);
        Workspace* w = h->ws[g % nws];
        if ((rc = ensure_workspace(h, w, rows, cols, K)) != TSM_OK) return drain_after_error(h, rc);
        PairIn in{};
        PairOut out{};
        for (int j = 0; j < k; ++j) {
            in.left[j] = dls[i0 + j];
            in.right[j] = drs[i0 + j];
            out.out[j] = douts[i0 + j];
        }
        if ((rc = run_pipeline(h, w, k, in, step, out, out_step, nullptr, w->stream)) != TSM_OK)
            return drain_after_error(h, rc);
    }
    return tsm_adc_synchronize(h);
}

int tsm_adc_compute_batch(tsm_adc* h, int n, const uint8_t* const* ls, const uint8_t* const* rs,
                          int rows, int cols, size_t step, float* const* outs, size_t out_step) {
    if (!h || n < 0 || (n > 0 && (!ls || !rs || !outs))) return TSM_ERR_ARGUMENT;
    int rc;
    if ((rc = set_device(h)) != TSM_OK) return rc;
    int K, nws;
    group_plan(h, n, K, nws);
    for (int g = 0, i0 = 0; i0 < n; ++g, i0 += K) {
        const int k = std::min(K, n - i0);
        Workspace* w = h->ws[g % nws];
        for (int j = 0; j < k; ++j) {
            const int i = i0 + j;
            if ((rc = validate(h, ls[i], rs[i], rows, cols, step)) != TSM_OK) return drain_after_error(h, rc);
            if (!outs[i] || out_step < (size_t)cols * 4)
                return drain_after_error(h, fail(h, TSM_ERR_ARGUMENT, "output buffer"));
        }
        // the group before on this workspace hands its outputs over first (its pinned
        // staging is reused below); the other workspace's group keeps running meanwhile
        if ((rc = flush_outputs(h, w)) != TSM_OK) return drain_after_error(h, rc);
        if ((rc = ensure_workspace(h, w, rows, cols, K)) != TSM_OK) return drain_after_error(h, rc);
        if ((rc = ensure_input_staging(h, w, rows, (size_t)cols * 3, cols, K)) != TSM_OK)
            return drain_after_error(h, rc);
        if ((rc = ensure_pinned(h, w, rows, cols, K)) != TSM_OK) return drain_after_error(h, rc);
        PairIn in{};
        PairOut po{};
        for (int j = 0; j < k; ++j) {  // pageable -> pinned (host), pinned -> HBM (async)
            if ((rc = stage_pinned_pair(h, w, K, j, ls[i0 + j], rs[i0 + j], rows, cols, step, in)) != TSM_OK)
                return drain_after_error(h, rc);
            po.out[j] = w->out_dev + (size_t)j * rows * cols;
        }
        if ((rc = run_pipeline(h, w, k, in, (size_t)cols * 3, po, (size_t)cols * 4, nullptr, w->stream)) != TSM_OK)
            return drain_after_error(h, rc);
        rc = hipMemcpyAsync(w->h_out, w->out_dev, (size_t)k * rows * cols * 4, hipMemcpyDeviceToHost, w->stream) ==
                     hipSuccess ? TSM_OK : TSM_ERR_DEVICE;
        if (rc != TSM_OK) return drain_after_error(h, fail(h, rc, "hipMemcpyAsync (output)"));
        w->pend_out.assign(outs + i0, outs + i0 + k);
        w->pend_rows = rows;
        w->pend_cols = cols;
        w->pend_step = out_step;
    }
    for (Workspace* w : h->ws)
        if ((rc = flush_outputs(h, w)) != TSM_OK) return drain_after_error(h, rc);
    return tsm_adc_synchronize(h);
}

}  // extern "C"
