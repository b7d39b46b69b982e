// stereo.h -- C++20 drop-in for the reference's stereo::ADCensus (YYpasser/
// tea_stereo_matching include/stereo.h:325-331 StereoMatching, :388-422 ADCensus),
// backed by the MI355X kernels through the C ABI in tsm_adcensus.h.
//
// Same namespace, class and method names, argument meaning and error behaviour:
//   setMinMaxDisparity / setOffset throw std::string with the reference's messages
//   (ADCensus.cpp:310, :326); compute throws std::string("[ADCensus] Image error.")
//   on empty / size-mismatched inputs (:332-333) and std::runtime_error on internal
//   failures (:383-387).
// Images are BGR u8 (CV_8UC3); the disparity is fp32 (CV_32FC1).  When OpenCV headers are
// found (<opencv2/core/mat.hpp>), StereoMatching's pure virtual is the reference's
// compute(const cv::Mat&, const cv::Mat&, cv::Mat&) and ADCensus overrides it; the light
// ImageView / DisparityMap form is then an overload (and the virtual without OpenCV).
// StereoMatching and ADCensus are header-only over the C ABI (link libtsm_adcensus.so).
#pragma once
#include <algorithm>
#include <array>
#include <cstddef>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "tsm_adcensus.h"
#include "tsm_stereo_ops.h"

// Which form is built is the includer's choice: -DTSM_WITH_OPENCV forces the cv::Mat form,
// -DTSM_NO_OPENCV the light form; with neither, the cv::Mat form when the OpenCV header is
// found.  Each form lives in its own inline namespace (stereo::cvmat_v1 / stereo::light_v1):
// callers still write stereo::ADCensus, but a program whose translation units were compiled
// in different forms fails to link (different mangled names) instead of mixing two vtable
// layouts of one class at run time.
#if defined(TSM_WITH_OPENCV) && defined(TSM_NO_OPENCV)
#error "define at most one of TSM_WITH_OPENCV and TSM_NO_OPENCV"
#endif
#if defined(TSM_WITH_OPENCV) || (!defined(TSM_NO_OPENCV) && __has_include(<opencv2/core/mat.hpp>))
#include <opencv2/core/mat.hpp>
#define TSM_HAVE_OPENCV 1
#endif

namespace stereo {
#ifdef TSM_HAVE_OPENCV
inline namespace cvmat_v1 {
#else
inline namespace light_v1 {
#endif

/** stereo_utils.h:191-195 */
enum class ColorModel { RGB = 0, HSI = 1 };
/** stereo_utils.h:200-204 */
enum class CensusWin { CENSUSWIN_9x7 = 0, CENSUSWIN_7x5 = 1 };

/** stereo_utils.h:206-244, defaults stereo_utils.cpp:271-326: the (Selective)
 *  AD-Census(-HSI) parameter set, member for member.  The reference keeps one inside
 *  ADCensus (ADCensus.cpp:278), set from the colour model by setMatchingStrategy; here
 *  ADCensus::getParams / setParams also exchange it (extensions). */
class ADCensusParams {
public:
    ADCensusParams() { setADCensusParams(ColorModel::RGB); }
    ADCensusParams(const ColorModel& colorModel) { setADCensusParams(colorModel); }
    ~ADCensusParams() {}

    void setADCensusParams(const ColorModel& colorModel) {
        lambdaAD = 10.f;
        censusWin = CensusWin::CENSUSWIN_9x7;
        lambdaCensus = 30.f;
        lambdaHue = 1.f;
        lambdaSaturation = 2.5f;
        lambdaIntensity = 2.5f;
        iterations = 4;
        pi1 = 1.f;
        pi2 = 3.f;
        dispTolerance = 0;
        votingThresh = 20;
        votingRatioThresh = 0.4f;
        maxSearchDepth = 20;
        blurKernelSize = 3;
        cannyThresh1 = 30;
        cannyThresh2 = 90;
        cannyKernelSize = 3;
        if (colorModel == ColorModel::RGB) {
            colorThresh1 = 20;
            colorThresh2 = 6;
            maxLength1 = 34;
            maxLength2 = 17;
            colorDiff = 15;
            saturationThresh1 = saturationThresh2 = 0;  // the reference assigns NULL
            intensityThresh1 = intensityThresh2 = 0;
        } else {  // HSI (and the reference's default branch)
            colorThresh1 = 5;
            colorThresh2 = 1;
            maxLength1 = 17;
            maxLength2 = 8;
            colorDiff = 3;
            saturationThresh1 = 10;
            saturationThresh2 = 2;
            intensityThresh1 = 12;
            intensityThresh2 = 3;
        }
    }

    float lambdaAD;
    CensusWin censusWin;
    float lambdaCensus;
    float lambdaHue;
    float lambdaSaturation;
    float lambdaIntensity;
    int colorThresh1;
    int colorThresh2;
    int saturationThresh1;
    int saturationThresh2;
    int intensityThresh1;
    int intensityThresh2;
    int maxLength1;
    int maxLength2;
    int iterations;
    int colorDiff;
    float pi1;
    float pi2;
    int dispTolerance;
    int votingThresh;
    float votingRatioThresh;
    int maxSearchDepth;
    int blurKernelSize;
    int cannyThresh1;
    int cannyThresh2;
    int cannyKernelSize;

    /** The C ABI's form (include/tsm_adcensus.h tsm_adc_params), and back. */
    tsm_adc_params toC() const {
        tsm_adc_params c{};
        c.lambda_ad = lambdaAD;
        c.census_win = (int)censusWin;
        c.lambda_census = lambdaCensus;
        c.lambda_hue = lambdaHue;
        c.lambda_saturation = lambdaSaturation;
        c.lambda_intensity = lambdaIntensity;
        c.color_thresh1 = colorThresh1;
        c.color_thresh2 = colorThresh2;
        c.saturation_thresh1 = saturationThresh1;
        c.saturation_thresh2 = saturationThresh2;
        c.intensity_thresh1 = intensityThresh1;
        c.intensity_thresh2 = intensityThresh2;
        c.max_length1 = maxLength1;
        c.max_length2 = maxLength2;
        c.iterations = iterations;
        c.color_diff = colorDiff;
        c.pi1 = pi1;
        c.pi2 = pi2;
        c.disp_tolerance = dispTolerance;
        c.voting_thresh = votingThresh;
        c.voting_ratio_thresh = votingRatioThresh;
        c.max_search_depth = maxSearchDepth;
        c.blur_kernel_size = blurKernelSize;
        c.canny_thresh1 = cannyThresh1;
        c.canny_thresh2 = cannyThresh2;
        c.canny_kernel_size = cannyKernelSize;
        return c;
    }
    static ADCensusParams fromC(const tsm_adc_params& c) {
        ADCensusParams p;
        p.lambdaAD = c.lambda_ad;
        p.censusWin = (CensusWin)c.census_win;
        p.lambdaCensus = c.lambda_census;
        p.lambdaHue = c.lambda_hue;
        p.lambdaSaturation = c.lambda_saturation;
        p.lambdaIntensity = c.lambda_intensity;
        p.colorThresh1 = c.color_thresh1;
        p.colorThresh2 = c.color_thresh2;
        p.saturationThresh1 = c.saturation_thresh1;
        p.saturationThresh2 = c.saturation_thresh2;
        p.intensityThresh1 = c.intensity_thresh1;
        p.intensityThresh2 = c.intensity_thresh2;
        p.maxLength1 = c.max_length1;
        p.maxLength2 = c.max_length2;
        p.iterations = c.iterations;
        p.colorDiff = c.color_diff;
        p.pi1 = c.pi1;
        p.pi2 = c.pi2;
        p.dispTolerance = c.disp_tolerance;
        p.votingThresh = c.voting_thresh;
        p.votingRatioThresh = c.voting_ratio_thresh;
        p.maxSearchDepth = c.max_search_depth;
        p.blurKernelSize = c.blur_kernel_size;
        p.cannyThresh1 = c.canny_thresh1;
        p.cannyThresh2 = c.canny_thresh2;
        p.cannyKernelSize = c.canny_kernel_size;
        return p;
    }
};

/** Non-owning BGR u8 image (the fields of a CV_8UC3 cv::Mat the matcher uses). */
struct ImageView {
    const std::uint8_t* data = nullptr;
    int rows = 0;
    int cols = 0;
    std::size_t step = 0; // bytes per row (>= 3*cols)
    bool empty() const { return data == nullptr || rows <= 0 || cols <= 0; }
};

/** Owning fp32 disparity map (CV_32FC1 equivalent, dense rows). */
struct DisparityMap {
    int rows = 0;
    int cols = 0;
    std::vector<float> data;
    float& at(int r, int c) { return data[(std::size_t)r * cols + c]; }
    float at(int r, int c) const { return data[(std::size_t)r * cols + c]; }
    bool empty() const { return data.empty(); }
};

/** stereo.h:325-331.  With OpenCV the one pure virtual is the reference's cv::Mat form, so
 *  a caller holding a StereoMatching& (or a subclass written against the reference, e.g.
 *  TensorRTInference) compiles unchanged; without OpenCV it is the ImageView form.  The
 *  class and ADCensus are header-only over the C ABI, so their vtables are laid out by the
 *  including translation unit and never depend on how the library was built. */
class StereoMatching {
public:
    virtual ~StereoMatching() = 0;
#ifdef TSM_HAVE_OPENCV
    virtual void compute(const cv::Mat& leftImage, const cv::Mat& rightImage, cv::Mat& disparity) = 0;
#else
    virtual void compute(const ImageView& leftImage, const ImageView& rightImage,
                         DisparityMap& disparity) = 0;
#endif
};
inline StereoMatching::~StereoMatching() {}  // stereo.cpp:413

/** stereo.h:388-422 -- AD-Census on one MI355X (HIP device `device`). */
class ADCensus : public StereoMatching {
public:
    ADCensus() : ADCensus(0) {}
    explicit ADCensus(int device) {
        const int rc = tsm_adc_create(device, &h_);
        if (rc != TSM_OK)
            throw std::runtime_error("[ADCensus] no usable HIP device (tsm_adc_create " + std::to_string(rc) + ")");
    }
    ~ADCensus() override {
        if (h_) tsm_adc_destroy(h_);
    }
    ADCensus(const ADCensus&) = delete;
    ADCensus& operator=(const ADCensus&) = delete;

    /** Inclusive disparity range; throws std::string on min*max < 0 or min >= max. */
    void setMinMaxDisparity(const int& minDisparity, const int& maxDisparity) {
        check(tsm_adc_set_disparity_range(h_, minDisparity, maxDisparity));
    }
    /** Colour model (resets the model's parameter set), ROI and mask modes. */
    void setMatchingStrategy(const ColorModel& colorModel = ColorModel::RGB,
                             const bool& roiMatching = false, const bool& maskMatching = false) {
        check(tsm_adc_set_strategy(h_, (int)colorModel, roiMatching ? 1 : 0, maskMatching ? 1 : 0));
    }
    /** ROI/mask disparity offset; throws std::string when negative. */
    void setOffset(const int& offset) { check(tsm_adc_set_offset(h_, offset)); }

#ifdef TSM_HAVE_OPENCV
    /** ADCensus.cpp:330-407: CV_8UC3 views in (any row step, ROIs included), a freshly
     *  allocated CV_32FC1 disparity out (`disparity = m_floatDisparityMap.clone()`, :391:
     *  a Mat that shared the old buffer keeps its data). */
    void compute(const cv::Mat& leftImage, const cv::Mat& rightImage, cv::Mat& disparity) override {
        if (leftImage.empty() || rightImage.empty() || leftImage.size() != rightImage.size())
            throw(std::string("[ADCensus] Image error."));  // the reference's check (:332-333)
        // a deliberate tightening: the reference reads any type as 3-byte BGR pixels; here a
        // non-CV_8UC3 input is refused as an internal-error type, so callers catching the
        // reference's std::string cases see them unchanged
        if (leftImage.type() != CV_8UC3 || rightImage.type() != CV_8UC3)
            throw std::runtime_error("[ADCensus] images must be CV_8UC3 (BGR u8)");
        cv::Mat out(leftImage.rows, leftImage.cols, CV_32FC1);
        run(view(leftImage), view(rightImage), out.ptr<float>(0), (std::size_t)out.step[0]);
        disparity = out;
    }
    /** Batch form over cv::Mat (ONNXRuntimeInference::compute(vector...) precedent, stereo.h:381). */
    void compute(const std::vector<cv::Mat>& leftImages, const std::vector<cv::Mat>& rightImages,
                 std::vector<cv::Mat>& disparities) {
        if (leftImages.size() != rightImages.size()) throw(std::string("[ADCensus] Image error."));
        std::vector<ImageView> ls, rs;
        for (std::size_t i = 0; i < leftImages.size(); ++i) {
            const cv::Mat& l = leftImages[i];
            const cv::Mat& r = rightImages[i];
            if (l.empty() || r.empty() || l.size() != r.size()) throw(std::string("[ADCensus] Image error."));
            if (l.type() != CV_8UC3 || r.type() != CV_8UC3)
                throw std::runtime_error("[ADCensus] images must be CV_8UC3 (BGR u8)");
            ls.push_back(view(l));
            rs.push_back(view(r));
        }
        std::vector<cv::Mat> out(ls.size());
        std::vector<float*> op(ls.size());
        for (std::size_t i = 0; i < ls.size(); ++i) {
            out[i] = cv::Mat(ls[i].rows, ls[i].cols, CV_32FC1);
            op[i] = out[i].ptr<float>(0);
        }
        if (!ls.empty()) run_batch(ls, rs, op, 0);  // fresh Mats are dense
        disparities = std::move(out);
    }
#endif
    /** Disparity of the left view (the form without OpenCV; an overload with it). */
    void compute(const ImageView& leftImage, const ImageView& rightImage, DisparityMap& disparity)
#ifndef TSM_HAVE_OPENCV
        override
#endif
    {
        if (leftImage.empty() || rightImage.empty() || leftImage.rows != rightImage.rows ||
            leftImage.cols != rightImage.cols)
            throw(std::string("[ADCensus] Image error."));
        DisparityMap out;
        out.rows = leftImage.rows;
        out.cols = leftImage.cols;
        out.data.resize((std::size_t)out.rows * out.cols);
        run(leftImage, rightImage, out.data.data(), (std::size_t)out.cols * 4);
        disparity = std::move(out);  // output reassigned, as :391
    }
    /** Batch form (ONNXRuntimeInference::compute(vector...) precedent, stereo.h:381). */
    void compute(const std::vector<ImageView>& leftImages, const std::vector<ImageView>& rightImages,
                 std::vector<DisparityMap>& disparities) {
        if (leftImages.size() != rightImages.size()) throw(std::string("[ADCensus] Image error."));
        std::vector<DisparityMap> out(leftImages.size());
        std::vector<float*> op(out.size());
        for (std::size_t i = 0; i < out.size(); ++i) {
            const ImageView& l = leftImages[i];
            const ImageView& r = rightImages[i];
            if (l.empty() || r.empty() || l.rows != r.rows || l.cols != r.cols)
                throw(std::string("[ADCensus] Image error."));
            out[i].rows = l.rows;
            out[i].cols = l.cols;
            out[i].data.resize((std::size_t)l.rows * l.cols);
            op[i] = out[i].data.data();
        }
        if (!out.empty()) run_batch(leftImages, rightImages, op, 0);
        disparities = std::move(out);
    }

    /** Extension: the active parameter set (the reference's m_paMatching). */
    ADCensusParams getParams() const {
        tsm_adc_params c{};
        check(tsm_adc_get_params(h_, &c));
        return ADCensusParams::fromC(c);
    }
    /** Extension: replace the parameter set (setMatchingStrategy resets it to the model's). */
    void setParams(const ADCensusParams& params) {
        const tsm_adc_params c = params.toC();
        check(tsm_adc_set_params(h_, &c));
    }
    /** Extension: reproduce the reference's racy omp-static scanline on T threads. */
    void setOmpEmulation(int threads) { check(tsm_adc_set_omp_emulation(h_, threads)); }
    /** Extension: number of concurrent pair pipelines for the batch form. */
    void setConcurrency(int streams) { check(tsm_adc_set_concurrency(h_, streams)); }

private:
    tsm_adc* h_ = nullptr;

    /** Status code -> the reference's exception: std::string for the three validation
     *  errors (ADCensus.cpp:309-310, :325-326, :332-333), std::runtime_error otherwise (:383-387). */
    void check(int rc) const {
        if (rc == TSM_OK) return;
        const std::string msg = tsm_adc_last_error(h_);
        if (rc == TSM_ERR_DISPARITY_RANGE || rc == TSM_ERR_OFFSET || rc == TSM_ERR_IMAGE) throw(msg);
        throw std::runtime_error(msg.empty() ? std::string("tsm_adc error ") + std::to_string(rc) : msg);
    }
#ifdef TSM_HAVE_OPENCV
    static ImageView view(const cv::Mat& m) {
        return ImageView{m.data, m.rows, m.cols, (std::size_t)m.step[0]};
    }
#endif
    /** Dense copy of a view at step cols*3 (the C ABI takes one step for both views). */
    static std::vector<std::uint8_t> dense(const ImageView& v) {
        const std::size_t row = (std::size_t)v.cols * 3;
        std::vector<std::uint8_t> a((std::size_t)v.rows * row);
        for (int y = 0; y < v.rows; ++y)
            std::copy(v.data + (std::size_t)y * v.step, v.data + (std::size_t)y * v.step + row, a.data() + y * row);
        return a;
    }
    void run(const ImageView& l, const ImageView& r, float* out, std::size_t out_step) {
        int rc;
        if (l.step == r.step) {
            rc = tsm_adc_compute(h_, l.data, r.data, l.rows, l.cols, l.step, out, out_step);
        } else {
            const std::vector<std::uint8_t> a = dense(l), b = dense(r);
            rc = tsm_adc_compute(h_, a.data(), b.data(), l.rows, l.cols, (std::size_t)l.cols * 3, out, out_step);
        }
        check(rc);
    }
    /** One tsm_adc_compute_batch when every pair has the first one's geometry and step;
     *  otherwise pair by pair.  out_step 0 = dense rows (cols * 4). */
    void run_batch(const std::vector<ImageView>& ls, const std::vector<ImageView>& rs,
                   const std::vector<float*>& outs, std::size_t out_step) {
        const ImageView& f = ls[0];
        const std::size_t os = out_step ? out_step : (std::size_t)f.cols * 4;
        bool uniform = true;
        for (std::size_t i = 0; i < ls.size(); ++i)
            uniform = uniform && ls[i].rows == f.rows && ls[i].cols == f.cols && ls[i].step == f.step &&
                      rs[i].step == f.step;
        if (!uniform) {
            for (std::size_t i = 0; i < ls.size(); ++i)
                run(ls[i], rs[i], outs[i], out_step ? out_step : (std::size_t)ls[i].cols * 4);
            return;
        }
        std::vector<const std::uint8_t*> lp, rp;
        for (std::size_t i = 0; i < ls.size(); ++i) {
            lp.push_back(ls[i].data);
            rp.push_back(rs[i].data);
        }
        check(tsm_adc_compute_batch(h_, (int)ls.size(), lp.data(), rp.data(), f.rows, f.cols, f.step,
                                    outs.data(), os));
    }
};

// ---- the calls either side of the matcher, gfx950 kernels through
// include/tsm_stereo_ops.h, header-only like the matcher.  Device failures throw
// std::runtime_error; the reference's "log and return" cases (empty inputs, maps not
// loaded) return without output.  With OpenCV the reference's cv::Mat signatures
// (reference include/stereo.h:194-296) are declared as well, and JETColorMap() returns the
// reference's 1 x 256 CV_8UC3 cv::Mat; JETColorMapTable() returns the light table either way.

namespace detail {
inline void ops_check(int rc, const char* what) {
    if (rc != TSM_OK) throw std::runtime_error(std::string(what) + " failed (status " + std::to_string(rc) + ")");
}
}  // namespace detail

/** Owning BGR u8 image (CV_8UC3 equivalent, dense rows). */
struct ColorImage {
    int rows = 0;
    int cols = 0;
    std::vector<std::uint8_t> data;  // rows * cols * 3
    bool empty() const { return data.empty(); }
    ImageView view() const { return ImageView{data.data(), rows, cols, (std::size_t)cols * 3}; }
};

/** Owning fp32 point image (CV_32FC3 equivalent): X, Y, Z per pixel. */
struct PointImage {
    int rows = 0;
    int cols = 0;
    std::vector<float> data;  // rows * cols * 3
    bool empty() const { return data.empty(); }
};

/** A colour table as stereo::JETColorMap returns it (1 x 256 CV_8UC3): lut[3*i + c], BGR. */
using ColorMapTable = std::array<std::uint8_t, 768>;

/** stereo.cpp:75-92, as a light table */
inline ColorMapTable JETColorMapTable() {
    ColorMapTable t{};
    detail::ops_check(tsm_jet_colormap(t.data()), "JETColorMap");
    return t;
}

namespace detail {
inline void color_map(const DisparityMap& src, ColorImage& dst, int use_range, float mn, float mx,
                      const ColorMapTable& lut) {
    if (src.empty()) return;
    dst.rows = src.rows;
    dst.cols = src.cols;
    dst.data.assign((std::size_t)src.rows * src.cols * 3, 0);
    ops_check(tsm_apply_colormap(src.data.data(), src.rows, src.cols, (std::size_t)src.cols * 4, lut.data(),
                                 use_range, mn, mx, dst.data.data(), (std::size_t)src.cols * 3),
              "applyColorMap");
}
}  // namespace detail

/** stereo.cpp:94-118: range from the pixels >= 0 and not inf; pixels < 0 black. */
inline void applyColorMap(const DisparityMap& src, ColorImage& dst, const ColorMapTable& colorMap) {
    detail::color_map(src, dst, 0, 0.f, 0.f, colorMap);
}
/** stereo.cpp:120-134: pixels outside [minVal, maxVal] black. */
inline void applyColorMap(const DisparityMap& src, ColorImage& dst, float minVal, float maxVal,
                          const ColorMapTable& colorMap) {
    detail::color_map(src, dst, 1, minVal, maxVal, colorMap);
}
/** stereo.cpp:136-148: depth = f*b / d (0 where d < 0 or inf); `depth` is a fp32 map. */
inline void reprojectToDepth(const DisparityMap& d, float focalLength, float baseline, DisparityMap& depth) {
    if (d.empty()) return;
    depth.rows = d.rows;
    depth.cols = d.cols;
    depth.data.assign(d.data.size(), 0.f);
    detail::ops_check(tsm_reproject_to_depth(d.data.data(), d.rows, d.cols, (std::size_t)d.cols * 4, focalLength,
                                             baseline, depth.data.data(), (std::size_t)d.cols * 4),
                      "reprojectToDepth");
}
/** stereo.cpp:150-169 */
inline void reprojectTo3D(const DisparityMap& d, float focalLength, float baseline, float cx, float cy,
                          PointImage& xyz) {
    if (d.empty()) return;
    xyz.rows = d.rows;
    xyz.cols = d.cols;
    xyz.data.assign(d.data.size() * 3, 0.f);
    detail::ops_check(tsm_reproject_to_3d(d.data.data(), d.rows, d.cols, (std::size_t)d.cols * 4, focalLength,
                                          baseline, cx, cy, xyz.data.data(), (std::size_t)d.cols * 12),
                      "reprojectTo3D");
}
/** stereo.cpp:171-202: Q is the 4x4 reprojection matrix, row-major (CV_64F). */
inline void reprojectTo3D(const DisparityMap& d, const std::array<double, 16>& Q, PointImage& xyz) {
    if (d.empty()) return;
    xyz.rows = d.rows;
    xyz.cols = d.cols;
    xyz.data.assign(d.data.size() * 3, 0.f);
    detail::ops_check(tsm_reproject_to_3d_q(d.data.data(), d.rows, d.cols, (std::size_t)d.cols * 4, Q.data(),
                                            xyz.data.data(), (std::size_t)d.cols * 12),
                      "reprojectTo3D");
}
/** stereo.cpp:250-278 (RGBImage is BGR-ordered, as the reference's cv::Mat) */
inline void writePointCloudToPCD(const ImageView& img, const PointImage& xyz, const std::string& path) {
    if (img.empty() || xyz.empty() || path.empty()) return;  // "Empty input." (stereo.cpp:252-256)
    detail::ops_check(tsm_write_point_cloud_pcd(img.data, img.step, xyz.data.data(), (std::size_t)xyz.cols * 12,
                                                xyz.rows, xyz.cols, path.c_str()),
                      "writePointCloudToPCD");
}
/** stereo.cpp:328-356 */
inline void writePointCloudToPLY(const ImageView& img, const PointImage& xyz, const std::string& path) {
    if (img.empty() || xyz.empty() || path.empty()) return;
    detail::ops_check(tsm_write_point_cloud_ply(img.data, img.step, xyz.data.data(), (std::size_t)xyz.cols * 12,
                                                xyz.rows, xyz.cols, path.c_str()),
                      "writePointCloudToPLY");
}

/** cv::Size */
struct Size {
    int width = 0;
    int height = 0;
};

#ifndef TSM_HAVE_OPENCV
/** stereo.cpp:75-92 */
inline ColorMapTable JETColorMap() { return JETColorMapTable(); }

/** stereo::EpipolarRectifyMap (stereo_utils.cpp:88-174), the remap pairs in the form
 *  initUndistortRectifyMap(..., CV_16SC2, ...) makes them (stereo_utils.cpp:164-167):
 *  map00 / map10 = int16 (x, y) per pixel, map01 / map11 = u16 fraction index fy*32+fx.
 *  R1, R2, P1, P2 are carried along (3x3 / 3x4, row-major) and not used by rectify. */
struct EpipolarRectifyMap {
    std::vector<double> R1, R2, P1, P2;
    int rows = 0, cols = 0;  // map size (= rectified image size)
    std::vector<std::int16_t> map00, map10;   // rows * cols * 2
    std::vector<std::uint16_t> map01, map11;  // rows * cols
    bool empty() const { return map00.empty() || map01.empty() || map10.empty() || map11.empty(); }
};
#else
/** stereo.cpp:75-92: the reference's 1 x 256 CV_8UC3 table */
inline cv::Mat JETColorMap() {
    cv::Mat m(1, 256, CV_8UC3);
    detail::ops_check(tsm_jet_colormap(m.ptr<std::uint8_t>(0)), "JETColorMap");
    return m;
}

namespace detail {
inline void need(bool ok, const char* what) {
    if (!ok) throw std::runtime_error(what);
}
inline ColorMapTable table_of(const cv::Mat& colorMap) {
    need(colorMap.type() == CV_8UC3 && colorMap.rows * colorMap.cols >= 256, "colorMap must be 256 CV_8UC3 entries");
    ColorMapTable t{};
    for (int i = 0; i < 256; ++i) {  // row-major over the table (1 x 256 or 256 x 1)
        const std::uint8_t* e = colorMap.ptr<std::uint8_t>(i / colorMap.cols) + (std::size_t)(i % colorMap.cols) * 3;
        t[3 * i] = e[0];
        t[3 * i + 1] = e[1];
        t[3 * i + 2] = e[2];
    }
    return t;
}
inline void color_map(const cv::Mat& src, cv::Mat& dst, int use_range, float mn, float mx, const cv::Mat& colorMap) {
    if (src.empty()) { dst = cv::Mat(); return; }
    need(src.type() == CV_32FC1, "applyColorMap: src must be CV_32FC1");
    const ColorMapTable lut = table_of(colorMap);
    cv::Mat out(src.rows, src.cols, CV_8UC3);  // dst = cv::Mat::zeros(src.size(), CV_8UC3) (:106)
    ops_check(tsm_apply_colormap(src.ptr<float>(0), src.rows, src.cols, (std::size_t)src.step[0], lut.data(), use_range,
                                 mn, mx, out.ptr<std::uint8_t>(0), (std::size_t)out.step[0]),
              "applyColorMap");
    dst = out;
}
}  // namespace detail

/** stereo.cpp:94-118 */
inline void applyColorMap(const cv::Mat& src, cv::Mat& dst, const cv::Mat& colorMap) {
    detail::color_map(src, dst, 0, 0.f, 0.f, colorMap);
}
/** stereo.cpp:120-134 */
inline void applyColorMap(const cv::Mat& src, cv::Mat& dst, float minVal, float maxVal, const cv::Mat& colorMap) {
    detail::color_map(src, dst, 1, minVal, maxVal, colorMap);
}
/** stereo.cpp:136-148 */
inline void reprojectToDepth(const cv::Mat& disparity, float focalLength, float baseline, cv::Mat& depth) {
    if (disparity.empty()) { depth = cv::Mat(); return; }
    detail::need(disparity.type() == CV_32FC1, "reprojectToDepth: disparity must be CV_32FC1");
    cv::Mat out(disparity.rows, disparity.cols, CV_32FC1);
    detail::ops_check(tsm_reproject_to_depth(disparity.ptr<float>(0), disparity.rows, disparity.cols,
                                             (std::size_t)disparity.step[0], focalLength, baseline,
                                             out.ptr<float>(0), (std::size_t)out.step[0]),
                      "reprojectToDepth");
    depth = out;
}
/** stereo.cpp:150-169 */
inline void reprojectTo3D(const cv::Mat& disparity, float focalLength, float baseline, float cx, float cy,
                          cv::Mat& XYZPoints) {
    if (disparity.empty()) { XYZPoints = cv::Mat(); return; }
    detail::need(disparity.type() == CV_32FC1, "reprojectTo3D: disparity must be CV_32FC1");
    cv::Mat out(disparity.rows, disparity.cols, CV_32FC3);
    detail::ops_check(tsm_reproject_to_3d(disparity.ptr<float>(0), disparity.rows, disparity.cols,
                                          (std::size_t)disparity.step[0], focalLength, baseline, cx, cy,
                                          out.ptr<float>(0), (std::size_t)out.step[0]),
                      "reprojectTo3D");
    XYZPoints = out;
}
/** stereo.cpp:171-202: Q 4 x 4, CV_32FC1 or CV_64FC1 */
inline void reprojectTo3D(const cv::Mat& disparity, const cv::Mat& Q, cv::Mat& XYZPoints) {
    if (disparity.empty()) { XYZPoints = cv::Mat(); return; }
    detail::need(disparity.type() == CV_32FC1, "reprojectTo3D: disparity must be CV_32FC1");
    detail::need(Q.rows == 4 && Q.cols == 4 && (Q.type() == CV_64FC1 || Q.type() == CV_32FC1),
                 "reprojectTo3D: Q must be 4 x 4 CV_32FC1 / CV_64FC1");
    double q[16];
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c)
            q[4 * r + c] = Q.type() == CV_64FC1 ? Q.ptr<double>(r)[c] : (double)Q.ptr<float>(r)[c];
    cv::Mat out(disparity.rows, disparity.cols, CV_32FC3);
    detail::ops_check(tsm_reproject_to_3d_q(disparity.ptr<float>(0), disparity.rows, disparity.cols,
                                            (std::size_t)disparity.step[0], q, out.ptr<float>(0),
                                            (std::size_t)out.step[0]),
                      "reprojectTo3D");
    XYZPoints = out;
}
/** stereo.cpp:250-278 */
inline void writePointCloudToPCD(const cv::Mat& RGBImage, const cv::Mat& XYZPoints, const std::string& pcdPath) {
    if (RGBImage.empty() || XYZPoints.empty() || pcdPath.empty()) return;  // "Empty input." (:252-256)
    detail::need(RGBImage.type() == CV_8UC3 && XYZPoints.type() == CV_32FC3 && RGBImage.size() == XYZPoints.size(),
                 "writePointCloudToPCD: CV_8UC3 image and CV_32FC3 points of one size");
    detail::ops_check(tsm_write_point_cloud_pcd(RGBImage.ptr<std::uint8_t>(0), (std::size_t)RGBImage.step[0],
                                                XYZPoints.ptr<float>(0), (std::size_t)XYZPoints.step[0],
                                                XYZPoints.rows, XYZPoints.cols, pcdPath.c_str()),
                      "writePointCloudToPCD");
}
/** stereo.cpp:328-356 */
inline void writePointCloudToPLY(const cv::Mat& RGBImage, const cv::Mat& XYZPoints, const std::string& plyPath) {
    if (RGBImage.empty() || XYZPoints.empty() || plyPath.empty()) return;
    detail::need(RGBImage.type() == CV_8UC3 && XYZPoints.type() == CV_32FC3 && RGBImage.size() == XYZPoints.size(),
                 "writePointCloudToPLY: CV_8UC3 image and CV_32FC3 points of one size");
    detail::ops_check(tsm_write_point_cloud_ply(RGBImage.ptr<std::uint8_t>(0), (std::size_t)RGBImage.step[0],
                                                XYZPoints.ptr<float>(0), (std::size_t)XYZPoints.step[0],
                                                XYZPoints.rows, XYZPoints.cols, plyPath.c_str()),
                      "writePointCloudToPLY");
}

/** stereo_utils.h:109-148: the rectification maps as initUndistortRectifyMap makes them
 *  (map00 / map10 CV_16SC2 + map01 / map11 CV_16UC1, or CV_32FC1 x / y map pairs).  The
 *  YAML loader and compute() (calibration) are out of scope. */
class EpipolarRectifyMap {
public:
    cv::Mat R1, R2, P1, P2;
    cv::Mat map00, map01, map10, map11;
    EpipolarRectifyMap() = default;
    EpipolarRectifyMap(const cv::Mat& R1_, const cv::Mat& R2_, const cv::Mat& P1_, const cv::Mat& P2_,
                       const cv::Mat& m00, const cv::Mat& m01, const cv::Mat& m10, const cv::Mat& m11)
        : R1(R1_), R2(R2_), P1(P1_), P2(P2_), map00(m00), map01(m01), map10(m10), map11(m11) {}
    bool empty() const { return map00.empty() || map01.empty() || map10.empty() || map11.empty(); }
};
#endif

/** stereo.h:254-296 / EpipolarRectify.cpp -- INTER_LINEAR remap of both views. */
class EpipolarRectify {
public:
    EpipolarRectify() = default;
#ifdef TSM_HAVE_OPENCV
    EpipolarRectify(const EpipolarRectifyMap& rectifyMap, const cv::Size& imgsz) {
        loadEpipolarRectifyMap(rectifyMap, imgsz);
    }
    /** Throws std::runtime_error("stereo params is empty, please load it first") on empty maps. */
    void loadEpipolarRectifyMap(const EpipolarRectifyMap& rectifyMap, const cv::Size& imgsz) {
        if (rectifyMap.empty()) throw std::runtime_error("stereo params is empty, please load it first");
        m_rectifyMap = rectifyMap;
        m_imgsz = Size{imgsz.width, imgsz.height};
    }
    /** Side-by-side stereo image in, side-by-side rectified image out (:46-64). */
    void rectify(const cv::Mat& stereoImage, cv::Mat& rectifiedStereoImage) {
        cv::Mat l, r;
        rectify(stereoImage, l, r);
        if (l.empty()) return;
        cv::Mat out(l.rows, l.cols + r.cols, l.type());  // cv::hconcat
        const std::size_t lb = (std::size_t)l.cols * l.elemSize(), rb = (std::size_t)r.cols * r.elemSize();
        for (int y = 0; y < out.rows; ++y) {
            std::copy_n(l.ptr<std::uint8_t>(y), lb, out.ptr<std::uint8_t>(y));
            std::copy_n(r.ptr<std::uint8_t>(y), rb, out.ptr<std::uint8_t>(y) + lb);
        }
        rectifiedStereoImage = out;
    }
    /** Side-by-side stereo image in, both rectified views out (:66-82). */
    void rectify(const cv::Mat& stereoImage, cv::Mat& rectifyLeftImage, cv::Mat& rectifiedRightImage) {
        if (m_rectifyMap.empty() || stereoImage.empty()) return;  // logged and returned (:68-77)
        const int w = m_imgsz.width, h = m_imgsz.height;
        const cv::Mat left = stereoImage(cv::Rect(0, 0, w, h)), right = stereoImage(cv::Rect(w, 0, w, h));
        rectify(left, right, rectifyLeftImage, rectifiedRightImage);
    }
    /** Both views in, both rectified views out (:84-101). */
    void rectify(const cv::Mat& leftImage, const cv::Mat& rightImage, cv::Mat& rectifyLeftImage,
                 cv::Mat& rectifiedRightImage) {
        if (m_rectifyMap.empty() || leftImage.empty() || rightImage.empty()) return;  // :89-98
        rectifyLeftImage = remap_mat(leftImage, m_rectifyMap.map00, m_rectifyMap.map01);
        rectifiedRightImage = remap_mat(rightImage, m_rectifyMap.map10, m_rectifyMap.map11);
    }
#endif
    EpipolarRectify(const EpipolarRectifyMap& rectifyMap, const Size& imgsz) { loadEpipolarRectifyMap(rectifyMap, imgsz); }
    /** Throws std::runtime_error("stereo params is empty, please load it first") on empty maps. */
    void loadEpipolarRectifyMap(const EpipolarRectifyMap& rectifyMap, const Size& imgsz) {
        if (rectifyMap.empty()) throw std::runtime_error("stereo params is empty, please load it first");
        m_rectifyMap = rectifyMap;
        m_imgsz = imgsz;
    }
#ifndef TSM_HAVE_OPENCV
    /** Side-by-side stereo image in, side-by-side rectified image out (:46-64). */
    void rectify(const ImageView& stereoImage, ColorImage& out) {
        ColorImage l, r;
        rectify(stereoImage, l, r);
        if (l.empty()) return;
        out.rows = l.rows;
        out.cols = l.cols + r.cols;
        out.data.resize((std::size_t)out.rows * out.cols * 3);
        for (int y = 0; y < out.rows; ++y) {  // cv::hconcat
            std::uint8_t* o = out.data.data() + (std::size_t)y * out.cols * 3;
            std::copy_n(l.data.data() + (std::size_t)y * l.cols * 3, (std::size_t)l.cols * 3, o);
            std::copy_n(r.data.data() + (std::size_t)y * r.cols * 3, (std::size_t)r.cols * 3, o + (std::size_t)l.cols * 3);
        }
    }
    /** Side-by-side stereo image in, both rectified views out (:66-82). */
    void rectify(const ImageView& stereoImage, ColorImage& outL, ColorImage& outR) {
        if (m_rectifyMap.empty() || stereoImage.empty()) return;  // logged and returned (:68-77)
        const int w = m_imgsz.width, h = m_imgsz.height;
        const ImageView left{stereoImage.data, h, w, stereoImage.step};
        const ImageView right{stereoImage.data + (std::size_t)w * 3, h, w, stereoImage.step};
        rectify(left, right, outL, outR);
    }
    /** Both views in, both rectified views out (:84-101). */
    void rectify(const ImageView& leftImage, const ImageView& rightImage, ColorImage& outL, ColorImage& outR) {
        if (m_rectifyMap.empty() || leftImage.empty() || rightImage.empty()) return;  // :89-98
        const EpipolarRectifyMap& m = m_rectifyMap;
        remap_view(leftImage, m.map00, m.map01, m.rows, m.cols, outL);
        remap_view(rightImage, m.map10, m.map11, m.rows, m.cols, outR);
    }
#endif

private:
    EpipolarRectifyMap m_rectifyMap;
    Size m_imgsz;
#ifdef TSM_HAVE_OPENCV
    /** cv::remap(src, dst, map1, map2, INTER_LINEAR) with BORDER_CONSTANT 0 (:99-100) */
    static cv::Mat remap_mat(const cv::Mat& src, const cv::Mat& map1, const cv::Mat& map2) {
        const int C = src.channels();
        detail::need((src.type() & 7) == CV_8U && (C == 1 || C == 3 || C == 4), "rectify: 8-bit images of 1, 3 or 4 channels");
        detail::need(map1.size() == map2.size(), "rectify: map sizes differ");
        cv::Mat out(map1.rows, map1.cols, src.type());
        int rc;
        if (map1.type() == CV_16SC2 && (map2.type() == CV_16UC1 || map2.type() == CV_16SC1)) {
            rc = tsm_remap_linear_fixed(src.ptr<std::uint8_t>(0), src.rows, src.cols, (std::size_t)src.step[0], C,
                                        map1.ptr<std::int16_t>(0), (std::size_t)map1.step[0],
                                        map2.ptr<std::uint16_t>(0), (std::size_t)map2.step[0], map1.rows, map1.cols,
                                        out.ptr<std::uint8_t>(0), (std::size_t)out.step[0]);
        } else {
            detail::need(map1.type() == CV_32FC1 && map2.type() == CV_32FC1 && map1.step[0] == map2.step[0],
                         "rectify: maps must be CV_16SC2 + CV_16UC1 or two CV_32FC1 of one step");
            rc = tsm_remap_linear_float(src.ptr<std::uint8_t>(0), src.rows, src.cols, (std::size_t)src.step[0], C,
                                        map1.ptr<float>(0), map2.ptr<float>(0), (std::size_t)map1.step[0],
                                        map1.rows, map1.cols, out.ptr<std::uint8_t>(0), (std::size_t)out.step[0]);
        }
        detail::ops_check(rc, "rectify");
        return out;
    }
#else
    static void remap_view(const ImageView& src, const std::vector<std::int16_t>& xy, const std::vector<std::uint16_t>& f,
                           int rows, int cols, ColorImage& dst) {
        dst.rows = rows;
        dst.cols = cols;
        dst.data.assign((std::size_t)rows * cols * 3, 0);
        detail::ops_check(tsm_remap_linear_fixed(src.data, src.rows, src.cols, src.step, 3, xy.data(),
                                                 (std::size_t)cols * 4, f.data(), (std::size_t)cols * 2, rows, cols,
                                                 dst.data.data(), (std::size_t)cols * 3),
                          "rectify");
    }
#endif
};

}  // inline namespace cvmat_v1 / light_v1
}  // namespace stereo
