// stereo_ops_api.cpp -- the C++ mirror (include/stereo.h) of the reference's free
// functions and EpipolarRectify class around the matcher, over the
// C ABI of include/tsm_stereo_ops.h.
#include <stdexcept>
#include <string>

#include "stereo.h"
#include "tsm_adcensus.h"
#include "tsm_stereo_ops.h"

namespace stereo {
namespace {

void check(int rc, const char* what) {
    if (rc != TSM_OK) throw std::runtime_error(std::string(what) + " failed (status " + std::to_string(rc) + ")");
}

void color_map(const DisparityMap& src, ColorImage& dst, int use_range, float mn, float mx,
               const ColorMapTable& lut) {
    if (src.empty()) return;
    dst.rows = src.rows;
    dst.cols = src.cols;
    dst.data.assign((std::size_t)src.rows * src.cols * 3, 0);
    check(tsm_apply_colormap(src.data.data(), src.rows, src.cols, (std::size_t)src.cols * 4, lut.data(),
                             use_range, mn, mx, dst.data.data(), (std::size_t)src.cols * 3),
          "applyColorMap");
}

void remap_view(const ImageView& src, const std::vector<std::int16_t>& xy, const std::vector<std::uint16_t>& f,
                int rows, int cols, ColorImage& dst) {
    dst.rows = rows;
    dst.cols = cols;
    dst.data.assign((std::size_t)rows * cols * 3, 0);
    check(tsm_remap_linear_fixed(src.data, src.rows, src.cols, src.step, 3, xy.data(), (std::size_t)cols * 4,
                                 f.data(), (std::size_t)cols * 2, rows, cols, dst.data.data(),
                                 (std::size_t)cols * 3),
          "rectify");
}

}  // namespace

ColorMapTable JETColorMap() {
    ColorMapTable t{};
    check(tsm_jet_colormap(t.data()), "JETColorMap");
    return t;
}

void applyColorMap(const DisparityMap& src, ColorImage& dst, const ColorMapTable& colorMap) {
    color_map(src, dst, 0, 0.f, 0.f, colorMap);
}

void applyColorMap(const DisparityMap& src, ColorImage& dst, float minVal, float maxVal,
                   const ColorMapTable& colorMap) {
    color_map(src, dst, 1, minVal, maxVal, colorMap);
}

void reprojectToDepth(const DisparityMap& d, float focalLength, float baseline, DisparityMap& depth) {
    if (d.empty()) return;
    depth.rows = d.rows;
    depth.cols = d.cols;
    depth.data.assign(d.data.size(), 0.f);
    check(tsm_reproject_to_depth(d.data.data(), d.rows, d.cols, (std::size_t)d.cols * 4, focalLength, baseline,
                                 depth.data.data(), (std::size_t)d.cols * 4),
          "reprojectToDepth");
}

void reprojectTo3D(const DisparityMap& d, float focalLength, float baseline, float cx, float cy,
                   PointImage& xyz) {
    if (d.empty()) return;
    xyz.rows = d.rows;
    xyz.cols = d.cols;
    xyz.data.assign(d.data.size() * 3, 0.f);
    check(tsm_reproject_to_3d(d.data.data(), d.rows, d.cols, (std::size_t)d.cols * 4, focalLength, baseline, cx,
                              cy, xyz.data.data(), (std::size_t)d.cols * 12),
          "reprojectTo3D");
}

void reprojectTo3D(const DisparityMap& d, const std::array<double, 16>& Q, PointImage& xyz) {
    if (d.empty()) return;
    xyz.rows = d.rows;
    xyz.cols = d.cols;
    xyz.data.assign(d.data.size() * 3, 0.f);
    check(tsm_reproject_to_3d_q(d.data.data(), d.rows, d.cols, (std::size_t)d.cols * 4, Q.data(),
                                xyz.data.data(), (std::size_t)d.cols * 12),
          "reprojectTo3D");
}

void writePointCloudToPCD(const ImageView& img, const PointImage& xyz, const std::string& path) {
    if (img.empty() || xyz.empty() || path.empty()) return;  // "Empty input." (stereo.cpp:252-256)
    check(tsm_write_point_cloud_pcd(img.data, img.step, xyz.data.data(), (std::size_t)xyz.cols * 12, xyz.rows,
                                    xyz.cols, path.c_str()),
          "writePointCloudToPCD");
}

void writePointCloudToPLY(const ImageView& img, const PointImage& xyz, const std::string& path) {
    if (img.empty() || xyz.empty() || path.empty()) return;
    check(tsm_write_point_cloud_ply(img.data, img.step, xyz.data.data(), (std::size_t)xyz.cols * 12, xyz.rows,
                                    xyz.cols, path.c_str()),
          "writePointCloudToPLY");
}

EpipolarRectify::EpipolarRectify() = default;

EpipolarRectify::EpipolarRectify(const EpipolarRectifyMap& rectifyMap, const Size& imgsz) {
    loadEpipolarRectifyMap(rectifyMap, imgsz);
}

EpipolarRectify::~EpipolarRectify() = default;

void EpipolarRectify::loadEpipolarRectifyMap(const EpipolarRectifyMap& rectifyMap, const Size& imgsz) {
    if (rectifyMap.empty()) throw std::runtime_error("stereo params is empty, please load it first");
    m_rectifyMap = rectifyMap;
    m_imgsz = imgsz;
}

void EpipolarRectify::rectify(const ImageView& stereoImage, ColorImage& out) {
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

void EpipolarRectify::rectify(const ImageView& stereoImage, ColorImage& outL, ColorImage& outR) {
    if (m_rectifyMap.empty() || stereoImage.empty()) return;  // logged and returned (:68-77)
    const int w = m_imgsz.width, h = m_imgsz.height;
    const ImageView left{stereoImage.data, h, w, stereoImage.step};
    const ImageView right{stereoImage.data + (std::size_t)w * 3, h, w, stereoImage.step};
    rectify(left, right, outL, outR);
}

void EpipolarRectify::rectify(const ImageView& leftImage, const ImageView& rightImage, ColorImage& outL,
                              ColorImage& outR) {
    if (m_rectifyMap.empty() || leftImage.empty() || rightImage.empty()) return;  // :89-98
    const EpipolarRectifyMap& m = m_rectifyMap;
    remap_view(leftImage, m.map00, m.map01, m.rows, m.cols, outL);
    remap_view(rightImage, m.map10, m.map11, m.rows, m.cols, outR);
}

}  // namespace stereo
