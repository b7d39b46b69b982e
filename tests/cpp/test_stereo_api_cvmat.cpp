// The reference's own interface, compiled and run: stereo::StereoMatching's pure virtual
// compute(const cv::Mat&, const cv::Mat&, cv::Mat&) (reference include/stereo.h:325-331)
// overridden by stereo::ADCensus (:388-422), called through a StereoMatching& as the
// reference's callers do (README.md:177-191).  Built with tests/cpp/cvshim on the include
// path (a minimal cv::Mat; OpenCV is not in the image), so include/stereo.h takes its
// TSM_HAVE_OPENCV branch.  Run by tests/test_gpu_cpp_api.py on the GPU box, which compares
// the disparity with the oracle bit for bit.
#include <cstdio>
#include <array>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "stereo.h"

#ifndef TSM_HAVE_OPENCV
#error "the cv::Mat path of include/stereo.h was not selected"
#endif

static int fails = 0;
#define CHECK(c)                                                    \
    do {                                                            \
        if (!(c)) { std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); ++fails; } \
    } while (0)

template <typename F>
static std::string thrown_string(F f) {
    try { f(); } catch (const std::string& s) { return s; } catch (...) { return "<other>"; }
    return "<none>";
}

static bool same_bits(const cv::Mat& a, const cv::Mat& b) {
    if (a.rows != b.rows || a.cols != b.cols || a.type() != b.type()) return false;
    for (int y = 0; y < a.rows; ++y)
        if (std::memcmp(a.ptr(y), b.ptr(y), (size_t)a.cols * a.elemSize()) != 0) return false;
    return true;
}

// A matcher written against the reference's interface only (as TensorRTInference,
// stereo.h:334-355): it must compile against this header unchanged.
class ConstantMatcher : public stereo::StereoMatching {
public:
    void compute(const cv::Mat& leftImage, const cv::Mat&, cv::Mat& disparity) override {
        disparity.create(leftImage.rows, leftImage.cols, CV_32FC1);
        for (int y = 0; y < disparity.rows; ++y)
            for (int x = 0; x < disparity.cols; ++x) disparity.ptr<float>(y)[x] = 7.f;
    }
};

static void dump(const char* dir, const char* name, const cv::Mat& m) {
    const std::string path = std::string(dir) + "/" + name;
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) { std::printf("FAIL cannot write %s\n", path.c_str()); ++fails; return; }
    for (int y = 0; y < m.rows; ++y)
        if (std::fwrite(m.ptr(y), 1, (size_t)m.cols * m.elemSize(), f) != (size_t)m.cols * m.elemSize()) ++fails;
    std::fclose(f);
}

int main(int argc, char** argv) {
    const int H = 48, W = 80, PAD = 13;  // inputs are ROIs of wider parents (odd row step)
    cv::Mat lp(H + 2, W + PAD, CV_8UC3), rp(H + 2, W + PAD, CV_8UC3);
    std::memset(lp.data, 0, (size_t)lp.rows * lp.step[0]);
    std::memset(rp.data, 0, (size_t)rp.rows * rp.step[0]);
    cv::Mat L = lp(cv::Rect(5, 1, W, H)), R = rp(cv::Rect(5, 1, W, H));
    unsigned s = 12345;  // the pair of tests/cpp/test_stereo_api.cpp
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x)
            for (int c = 0; c < 3; ++c) {
                s = s * 1664525u + 1013904223u;
                L.ptr<unsigned char>(y)[x * 3 + c] = (unsigned char)(64 + ((x / 4 + y / 4 + c) * 37 + (s >> 28)) % 128);
            }
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x)
            for (int c = 0; c < 3; ++c)
                R.ptr<unsigned char>(y)[x * 3 + c] = L.ptr<unsigned char>(y)[std::min(W - 1, x + 6) * 3 + c];
    CHECK(!L.isContinuous() && L.step[0] == (size_t)(W + PAD) * 3);

    stereo::ADCensus adcensus;
    adcensus.setMatchingStrategy(stereo::ColorModel::RGB, false, false);
    adcensus.setMinMaxDisparity(0, 16);

    // the reference's call, through the abstract base
    stereo::StereoMatching& sm = adcensus;
    cv::Mat D;
    sm.compute(L, R, D);
    CHECK(D.rows == H && D.cols == W && D.type() == CV_32FC1 && D.isContinuous());

    // the same pair as dense Mats and through the ImageView overload: identical bits
    cv::Mat Lc = L.clone(), Rc = R.clone(), Dc;
    adcensus.compute(Lc, Rc, Dc);
    CHECK(same_bits(D, Dc));
    stereo::DisparityMap dv;
    adcensus.compute(stereo::ImageView{L.data, H, W, L.step[0]}, stereo::ImageView{R.data, H, W, R.step[0]}, dv);
    CHECK(dv.rows == H && dv.cols == W &&
          std::memcmp(dv.data.data(), D.ptr(0), (size_t)H * W * 4) == 0);
    // one ROI step and one dense step (the library is handed a dense copy of both)
    cv::Mat Dm;
    adcensus.compute(L, Rc, Dm);
    CHECK(same_bits(D, Dm));

    // the output is reassigned (disparity = m_floatDisparityMap.clone(), ADCensus.cpp:391):
    // a Mat that shared the caller's old buffer keeps its contents
    cv::Mat alias = D;
    const float before = alias.ptr<float>(0)[0];
    alias.ptr<float>(0)[1] = -123.f;
    sm.compute(L, R, D);
    CHECK(alias.data != D.data && alias.ptr<float>(0)[0] == before && alias.ptr<float>(0)[1] == -123.f);
    CHECK(same_bits(D, Dc));

    int six = 0, valid = 0;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const float v = D.ptr<float>(y)[x];
            if (v >= 0) { ++valid; if (v > 5.5f && v < 6.5f) ++six; }
        }
    CHECK(valid > H * W / 2 && six > valid * 8 / 10);
    if (argc > 1) {
        dump(argv[1], "left.bgr", L);
        dump(argv[1], "right.bgr", R);
        dump(argv[1], "disp.f32", D);
    }

    // batch over cv::Mat (ONNXRuntimeInference::compute(vector...) precedent, stereo.h:381)
    std::vector<cv::Mat> ls{L, Lc}, rs{R, Rc}, ds;
    adcensus.compute(ls, rs, ds);
    CHECK(ds.size() == 2 && same_bits(ds[0], D) && same_bits(ds[1], D));

    // the reference's exception types and messages (ADCensus.cpp:309-310, :325-326, :332-333)
    cv::Mat empty, narrow = L(cv::Rect(0, 0, W - 1, H)), gray(H, W, CV_8UC1);
    CHECK(thrown_string([&] { sm.compute(empty, R, D); }) == "[ADCensus] Image error.");
    CHECK(thrown_string([&] { sm.compute(L, narrow, D); }) == "[ADCensus] Image error.");
    {  // a non-CV_8UC3 input: a deliberate tightening, refused as std::runtime_error
        bool rt = false;
        try { sm.compute(gray, gray, D); } catch (const std::runtime_error&) { rt = true; } catch (...) {}
        CHECK(rt);
    }
    CHECK(thrown_string([&] { adcensus.setMinMaxDisparity(5, 2); }) == "[ADCensus] Set MinMaxDisparity error.");
    CHECK(thrown_string([&] { adcensus.setOffset(-4); }) == "[ADCensus] Offset must be positive.");

    // a subclass written against the reference's interface, used polymorphically
    ConstantMatcher cm;
    stereo::StereoMatching* matchers[2] = {&adcensus, &cm};
    cv::Mat out;
    matchers[1]->compute(L, R, out);
    CHECK(out.ptr<float>(H - 1)[W - 1] == 7.f);
    matchers[0]->compute(L, R, out);
    CHECK(same_bits(out, Dc));

    // ---- the calls either side of the matcher in the reference's cv::Mat signatures
    // (reference stereo.h:194-296), each equal to the light form on the same data
    const cv::Mat jet = stereo::JETColorMap();
    const stereo::ColorMapTable jt = stereo::JETColorMapTable();
    CHECK(jet.rows == 1 && jet.cols == 256 && jet.type() == CV_8UC3 &&
          std::memcmp(jet.ptr(0), jt.data(), 768) == 0);
    stereo::DisparityMap dl;  // the light copy of D
    dl.rows = H;
    dl.cols = W;
    dl.data.assign(D.ptr<float>(0), D.ptr<float>(0) + (size_t)H * W);
    auto same_bytes = [](const cv::Mat& m, const void* p, size_t rowb) {
        for (int y = 0; y < m.rows; ++y)
            if (std::memcmp(m.ptr(y), (const char*)p + (size_t)y * rowb, rowb) != 0) return false;
        return true;
    };
    cv::Mat vis, vis2;
    stereo::applyColorMap(D, vis, jet);
    stereo::ColorImage cvis;
    stereo::applyColorMap(dl, cvis, jt);
    CHECK(vis.type() == CV_8UC3 && vis.rows == H && same_bytes(vis, cvis.data.data(), (size_t)W * 3));
    stereo::applyColorMap(D, vis2, 2.f, 12.f, jet);
    stereo::applyColorMap(dl, cvis, 2.f, 12.f, jt);
    CHECK(same_bytes(vis2, cvis.data.data(), (size_t)W * 3));
    cv::Mat depth;
    stereo::reprojectToDepth(D, 700.f, 0.1f, depth);
    stereo::DisparityMap ldepth;
    stereo::reprojectToDepth(dl, 700.f, 0.1f, ldepth);
    CHECK(depth.type() == CV_32FC1 && same_bytes(depth, ldepth.data.data(), (size_t)W * 4));
    cv::Mat xyz, xyzq, xyzq32;
    stereo::reprojectTo3D(D, 700.f, 0.1f, W / 2.f, H / 2.f, xyz);
    stereo::PointImage lxyz;
    stereo::reprojectTo3D(dl, 700.f, 0.1f, W / 2.f, H / 2.f, lxyz);
    CHECK(xyz.type() == CV_32FC3 && same_bytes(xyz, lxyz.data.data(), (size_t)W * 12));
    const std::array<double, 16> q = {1, 0, 0, -W / 2.0, 0, 1, 0, -H / 2.0, 0, 0, 0, 700, 0, 0, 10, 0};
    cv::Mat Q(4, 4, CV_64FC1), Q32(4, 4, CV_32FC1);
    for (int i = 0; i < 16; ++i) {
        Q.ptr<double>(i / 4)[i % 4] = q[i];
        Q32.ptr<float>(i / 4)[i % 4] = (float)q[i];
    }
    stereo::reprojectTo3D(D, Q, xyzq);
    stereo::reprojectTo3D(D, Q32, xyzq32);
    stereo::reprojectTo3D(dl, q, lxyz);
    CHECK(same_bytes(xyzq, lxyz.data.data(), (size_t)W * 12) && same_bytes(xyzq32, lxyz.data.data(), (size_t)W * 12));
    // point clouds: the cv::Mat writers' files are byte-identical to the light writers'
    auto slurp = [](const char* path) {
        std::string s;
        if (FILE* f = std::fopen(path, "rb")) {
            char buf[4096];
            size_t n;
            while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, n);
            std::fclose(f);
        }
        return s;
    };
    stereo::reprojectTo3D(dl, 700.f, 0.1f, W / 2.f, H / 2.f, lxyz);
    stereo::writePointCloudToPLY(L, xyz, "/tmp/tsm_cvmat_cloud.ply");
    stereo::writePointCloudToPLY(stereo::ImageView{L.data, H, W, L.step[0]}, lxyz, "/tmp/tsm_light_cloud.ply");
    stereo::writePointCloudToPCD(L, xyz, "/tmp/tsm_cvmat_cloud.pcd");
    stereo::writePointCloudToPCD(stereo::ImageView{L.data, H, W, L.step[0]}, lxyz, "/tmp/tsm_light_cloud.pcd");
    const std::string ply = slurp("/tmp/tsm_cvmat_cloud.ply"), pcd = slurp("/tmp/tsm_cvmat_cloud.pcd");
    CHECK(ply.size() > 100 && ply == slurp("/tmp/tsm_light_cloud.ply"));
    CHECK(pcd.size() > 100 && pcd == slurp("/tmp/tsm_light_cloud.pcd"));
    // rectification with the reference's map types: identity CV_16SC2 + CV_16UC1 maps and
    // identity CV_32FC1 map pairs return their inputs
    cv::Mat m00(H, W, CV_16SC2), m01(H, W, CV_16UC1), fx(H, W, CV_32FC1), fy(H, W, CV_32FC1);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            m00.ptr<int16_t>(y)[2 * x] = (int16_t)x;
            m00.ptr<int16_t>(y)[2 * x + 1] = (int16_t)y;
            m01.ptr<uint16_t>(y)[x] = 0;
            fx.ptr<float>(y)[x] = (float)x;
            fy.ptr<float>(y)[x] = (float)y;
        }
    const cv::Mat empty_mat;
    stereo::EpipolarRectifyMap rm(empty_mat, empty_mat, empty_mat, empty_mat, m00, m01, m00, m01);
    stereo::EpipolarRectify rect(rm, cv::Size(W, H));
    cv::Mat rl, rr, side;
    rect.rectify(Lc, Rc, rl, rr);
    CHECK(same_bits(rl, Lc) && same_bits(rr, Rc));
    cv::Mat sbs(H, 2 * W, CV_8UC3);  // side by side: left | right
    for (int y = 0; y < H; ++y) {
        std::memcpy(sbs.ptr(y), Lc.ptr(y), (size_t)W * 3);
        std::memcpy(sbs.ptr(y) + (size_t)W * 3, Rc.ptr(y), (size_t)W * 3);
    }
    rect.rectify(sbs, side);
    CHECK(same_bits(side, sbs));
    stereo::EpipolarRectify rectf(stereo::EpipolarRectifyMap(empty_mat, empty_mat, empty_mat, empty_mat, fx, fy, fx, fy),
                                  cv::Size(W, H));
    rectf.rectify(Lc, Rc, rl, rr);
    CHECK(same_bits(rl, Lc) && same_bits(rr, Rc));
    bool threw = false;
    try { stereo::EpipolarRectify().loadEpipolarRectifyMap(stereo::EpipolarRectifyMap{}, cv::Size(W, H)); }
    catch (const std::runtime_error& e) { threw = std::string(e.what()) == "stereo params is empty, please load it first"; }
    CHECK(threw);

    std::printf("%s (%d failures)\n", fails ? "FAILED" : "OK", fails);
    return fails ? 1 : 0;
}
