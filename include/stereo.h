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
#include <array>
#include <cstddef>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "tsm_adcensus.h"

#if __has_include(<opencv2/core/mat.hpp>)
#include <opencv2/core/mat.hpp>
#define TSM_HAVE_OPENCV 1
#endif

namespace stereo {

/** stereo_utils.h:191-195 */
enum class ColorModel { RGB = 0, HSI = 1 };
/** stereo_utils.h:200-204 */
enum class CensusWin { CENSUSWIN_9x7 = 0, CENSUSWIN_7x5 = 1 };

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
        if (leftImage.empty() || rightImage.empty() || leftImage.size() != rightImage.size() ||
            leftImage.type() != CV_8UC3 || rightImage.type() != CV_8UC3)
            throw(std::string("[ADCensus] Image error."));
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
            if (l.empty() || r.empty() || l.size() != r.size() || l.type() != CV_8UC3 || r.type() != CV_8UC3)
                throw(std::string("[ADCensus] Image error."));
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
// include/tsm_stereo_ops.h.  Device failures throw std::runtime_error; the reference's
// "log and return" cases (empty inputs, maps not loaded) return without output.

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

/** stereo.cpp:75-92 */
ColorMapTable JETColorMap();
/** stereo.cpp:94-118: range from the pixels >= 0 and not inf; pixels < 0 black. */
void applyColorMap(const DisparityMap& src, ColorImage& dst, const ColorMapTable& colorMap);
/** stereo.cpp:120-134: pixels outside [minVal, maxVal] black. */
void applyColorMap(const DisparityMap& src, ColorImage& dst, float minVal, float maxVal,
                   const ColorMapTable& colorMap);
/** stereo.cpp:136-148: depth = f*b / d (0 where d < 0 or inf); `depth` is a fp32 map. */
void reprojectToDepth(const DisparityMap& disparity, float focalLength, float baseline, DisparityMap& depth);
/** stereo.cpp:150-169 */
void reprojectTo3D(const DisparityMap& disparity, float focalLength, float baseline, float cx, float cy,
                   PointImage& XYZPoints);
/** stereo.cpp:171-202: Q is the 4x4 reprojection matrix, row-major (CV_64F). */
void reprojectTo3D(const DisparityMap& disparity, const std::array<double, 16>& Q, PointImage& XYZPoints);
/** stereo.cpp:250-278 (RGBImage is BGR-ordered, as the reference's cv::Mat) */
void writePointCloudToPCD(const ImageView& RGBImage, const PointImage& XYZPoints, const std::string& pcdPath);
/** stereo.cpp:328-356 */
void writePointCloudToPLY(const ImageView& RGBImage, const PointImage& XYZPoints, const std::string& plyPath);

/** cv::Size */
struct Size {
    int width = 0;
    int height = 0;
};

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

/** stereo.h:254-296 / EpipolarRectify.cpp -- INTER_LINEAR remap of both views. */
class EpipolarRectify {
public:
    EpipolarRectify();
    EpipolarRectify(const EpipolarRectifyMap& rectifyMap, const Size& imgsz);
    ~EpipolarRectify();
    /** Throws std::runtime_error("stereo params is empty, please load it first") on empty maps. */
    void loadEpipolarRectifyMap(const EpipolarRectifyMap& rectifyMap, const Size& imgsz);
    /** Side-by-side stereo image in, side-by-side rectified image out (:46-64). */
    void rectify(const ImageView& stereoImage, ColorImage& rectifiedStereoImage);
    /** Side-by-side stereo image in, both rectified views out (:66-82). */
    void rectify(const ImageView& stereoImage, ColorImage& rectifyLeftImage, ColorImage& rectifiedRightImage);
    /** Both views in, both rectified views out (:84-101). */
    void rectify(const ImageView& leftImage, const ImageView& rightImage, ColorImage& rectifyLeftImage,
                 ColorImage& rectifiedRightImage);

private:
    EpipolarRectifyMap m_rectifyMap;
    Size m_imgsz;
};

}  // namespace stereo
