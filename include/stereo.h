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
#include <array>
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
