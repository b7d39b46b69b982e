// stereo.h -- C++20 drop-in for the reference's stereo::ADCensus (YYpasser/
// tea_stereo_matching include/stereo.h:325-331 StereoMatching, :388-422 ADCensus),
// backed by the MI355X kernels through the C ABI in tsm_adcensus.h.
//
// Same namespace, class and method names, argument meaning and error behaviour:
//   setMinMaxDisparity / setOffset throw std::string with the reference's messages
//   (ADCensus.cpp:310, :326); compute throws std::string("[ADCensus] Image error.")
//   on empty / size-mismatched inputs (:332-333) and std::runtime_error on internal
//   failures (:383-387).
// Images are BGR u8 (CV_8UC3); the disparity is fp32 (CV_32FC1).  Without OpenCV the
// class takes a light ImageView and fills a DisparityMap; when OpenCV headers are
// available a cv::Mat overload is compiled in (header-only adapter).
#pragma once
#include <cstddef>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

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

/** stereo.h:325-331 */
class StereoMatching {
public:
    virtual ~StereoMatching() = 0;
    virtual void compute(const ImageView& leftImage, const ImageView& rightImage,
                         DisparityMap& disparity) = 0;
};

/** stereo.h:388-422 -- AD-Census on one MI355X (HIP device `device`). */
class ADCensus : public StereoMatching {
public:
    ADCensus();
    explicit ADCensus(int device);
    ~ADCensus();
    ADCensus(const ADCensus&) = delete;
    ADCensus& operator=(const ADCensus&) = delete;

    /** Inclusive disparity range; throws std::string on min*max < 0 or min >= max. */
    void setMinMaxDisparity(const int& minDisparity, const int& maxDisparity);
    /** Colour model (resets the model's parameter set), ROI and mask modes. */
    void setMatchingStrategy(const ColorModel& colorModel = ColorModel::RGB,
                             const bool& roiMatching = false, const bool& maskMatching = false);
    /** ROI/mask disparity offset; throws std::string when negative. */
    void setOffset(const int& offset);
    /** Disparity of the left view. */
    void compute(const ImageView& leftImage, const ImageView& rightImage,
                 DisparityMap& disparity) override;
    /** Batch form (ONNXRuntimeInference::compute(vector...) precedent, stereo.h:381). */
    void compute(const std::vector<ImageView>& leftImages, const std::vector<ImageView>& rightImages,
                 std::vector<DisparityMap>& disparities);

    /** Extension: reproduce the reference's racy omp-static scanline on T threads. */
    void setOmpEmulation(int threads);
    /** Extension: number of concurrent pair pipelines for the batch form. */
    void setConcurrency(int streams);

#ifdef TSM_HAVE_OPENCV
    void compute(const cv::Mat& leftImage, const cv::Mat& rightImage, cv::Mat& disparity) {
        if (leftImage.empty() || rightImage.empty() || leftImage.size() != rightImage.size() ||
            leftImage.type() != CV_8UC3 || rightImage.type() != CV_8UC3)
            throw(std::string("[ADCensus] Image error."));
        ImageView l{leftImage.data, leftImage.rows, leftImage.cols, leftImage.step};
        ImageView r{rightImage.data, rightImage.rows, rightImage.cols, rightImage.step};
        DisparityMap d;
        compute(l, r, d);
        disparity.create(d.rows, d.cols, CV_32F);
        std::copy(d.data.begin(), d.data.end(), disparity.ptr<float>(0));
    }
#endif

private:
    class ADCensusImpl;
    std::unique_ptr<ADCensusImpl> impl;
};

}  // namespace stereo
