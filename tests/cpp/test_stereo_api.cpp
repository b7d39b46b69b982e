// C++ API check (run by tests/test_gpu_cpp_api.py on the GPU box): the reference's
// usage pattern (README.md:177-191) against stereo::ADCensus from include/stereo.h,
// including the reference's exception types and messages.
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "stereo.h"

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

// argv[1] (optional): a directory where the pair and its disparity are written (raw
// left/right BGR bytes, fp32 disparity) for the Python driver to compare with the oracle
static void dump(const char* dir, const char* name, const void* p, size_t n) {
    const std::string path = std::string(dir) + "/" + name;
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) { std::printf("FAIL cannot write %s\n", path.c_str()); ++fails; return; }
    if (std::fwrite(p, 1, n, f) != n) { std::printf("FAIL short write %s\n", path.c_str()); ++fails; }
    std::fclose(f);
}

int main(int argc, char** argv) {
    const int H = 48, W = 80;
    std::vector<unsigned char> l(H * W * 3), r(H * W * 3);
    unsigned s = 12345;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x)
            for (int c = 0; c < 3; ++c) {
                s = s * 1664525u + 1013904223u;
                l[(y * W + x) * 3 + c] = (unsigned char)(64 + ((x / 4 + y / 4 + c) * 37 + (s >> 28)) % 128);
            }
    for (int y = 0; y < H; ++y)  // right view = left shifted by 6 px
        for (int x = 0; x < W; ++x)
            for (int c = 0; c < 3; ++c) r[(y * W + x) * 3 + c] = l[(y * W + std::min(W - 1, x + 6)) * 3 + c];

    stereo::ADCensus adcensus;
    // the parameter set: the engine's per-model defaults are the reference's
    // (stereo_utils.cpp:271-326; a new matcher is in the HSI model, ADCensus.cpp:409-420)
    auto same = [](const stereo::ADCensusParams& a, const stereo::ADCensusParams& b) {
        const tsm_adc_params x = a.toC(), y = b.toC();
        return std::memcmp(&x, &y, sizeof x) == 0;
    };
    CHECK(same(adcensus.getParams(), stereo::ADCensusParams(stereo::ColorModel::HSI)));
    adcensus.setMatchingStrategy(stereo::ColorModel::RGB, false, false);
    CHECK(same(adcensus.getParams(), stereo::ADCensusParams(stereo::ColorModel::RGB)));
    {
        stereo::ADCensusParams p(stereo::ColorModel::RGB);
        p.maxLength1 = 30;
        p.votingRatioThresh = 0.5f;
        adcensus.setParams(p);
        CHECK(same(adcensus.getParams(), p));
        adcensus.setParams(stereo::ADCensusParams(stereo::ColorModel::RGB));
    }
    adcensus.setMinMaxDisparity(0, 16);
    stereo::ImageView L{l.data(), H, W, (size_t)W * 3}, R{r.data(), H, W, (size_t)W * 3};
    stereo::DisparityMap d;
    adcensus.compute(L, R, d);
    CHECK(d.rows == H && d.cols == W && (int)d.data.size() == H * W);
    int six = 0, valid = 0;
    for (float v : d.data) { if (v >= 0) { ++valid; if (v > 5.5f && v < 6.5f) ++six; } }
    CHECK(valid > H * W / 2);
    CHECK(six > valid * 8 / 10);
    if (argc > 1) {
        dump(argv[1], "left.bgr", l.data(), l.size());
        dump(argv[1], "right.bgr", r.data(), r.size());
        dump(argv[1], "disp.f32", d.data.data(), d.data.size() * sizeof(float));
    }

    CHECK(thrown_string([&] { adcensus.setMinMaxDisparity(-3, 3); }) == "[ADCensus] Set MinMaxDisparity error.");
    CHECK(thrown_string([&] { adcensus.setMinMaxDisparity(9, 9); }) == "[ADCensus] Set MinMaxDisparity error.");
    CHECK(thrown_string([&] { adcensus.setOffset(-1); }) == "[ADCensus] Offset must be positive.");
    stereo::ImageView bad{l.data(), H, W - 1, (size_t)W * 3};
    CHECK(thrown_string([&] { adcensus.compute(L, bad, d); }) == "[ADCensus] Image error.");
    stereo::ImageView empty{};
    CHECK(thrown_string([&] { adcensus.compute(empty, R, d); }) == "[ADCensus] Image error.");

    std::vector<stereo::ImageView> ls{L, L}, rs{R, R};
    std::vector<stereo::DisparityMap> ds;
    adcensus.compute(ls, rs, ds);
    CHECK(ds.size() == 2 && ds[0].data == d.data && ds[1].data == d.data);

    // StereoMatching polymorphism, as the reference's callers use it
    stereo::StereoMatching* sm = &adcensus;
    stereo::DisparityMap d2;
    sm->compute(L, R, d2);
    CHECK(d2.data == d.data);

    // the calls around the matcher (stereo.cpp:75-356, EpipolarRectify.cpp), as a caller
    // chains them: colour map, depth, points, point cloud, rectification
    const stereo::ColorMapTable jet = stereo::JETColorMap();
    CHECK(jet[0] == 128 && jet[1] == 0 && jet[3 * 255 + 2] == 128);
    stereo::ColorImage vis;
    stereo::applyColorMap(d, vis, jet);
    CHECK(vis.rows == H && vis.cols == W && (int)vis.data.size() == H * W * 3);
    stereo::ColorImage vis2;
    stereo::applyColorMap(d, vis2, 0.f, 16.f, jet);
    CHECK(vis2.data.size() == vis.data.size());
    stereo::DisparityMap depth;
    stereo::reprojectToDepth(d, 700.f, 0.1f, depth);
    bool depth_ok = true;
    for (int i = 0; i < H * W; ++i)
        if (d.data[i] > 0 && depth.data[i] != (700.f * 0.1f) / d.data[i]) depth_ok = false;
    CHECK(depth_ok);
    stereo::PointImage xyz;
    stereo::reprojectTo3D(d, 700.f, 0.1f, W / 2.f, H / 2.f, xyz);
    CHECK(xyz.rows == H && (int)xyz.data.size() == H * W * 3);
    CHECK(xyz.data[2 * 3 * W + 3 * 40 + 2] == depth.at(2, 40));
    stereo::writePointCloudToPLY(L, xyz, "/tmp/tsm_cpp_api_cloud.ply");
    FILE* f = std::fopen("/tmp/tsm_cpp_api_cloud.ply", "rb");
    CHECK(f != nullptr);
    if (f) {
        char head[4] = {0};
        CHECK(std::fread(head, 1, 3, f) == 3 && std::string(head) == "ply");
        std::fclose(f);
    }
    stereo::EpipolarRectifyMap rm;  // identity maps: rectify returns its inputs
    rm.rows = H;
    rm.cols = W;
    rm.map00.resize((size_t)H * W * 2);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            rm.map00[(size_t)(y * W + x) * 2] = (int16_t)x;
            rm.map00[(size_t)(y * W + x) * 2 + 1] = (int16_t)y;
        }
    rm.map10 = rm.map00;
    rm.map01.assign((size_t)H * W, 0);
    rm.map11 = rm.map01;
    stereo::EpipolarRectify rect(rm, stereo::Size{W, H});
    stereo::ColorImage rl, rr;
    rect.rectify(L, R, rl, rr);
    CHECK(rl.data == l && rr.data == r);
    bool threw = false;
    try { stereo::EpipolarRectify().loadEpipolarRectifyMap(stereo::EpipolarRectifyMap{}, stereo::Size{W, H}); }
    catch (const std::runtime_error& e) { threw = std::string(e.what()) == "stereo params is empty, please load it first"; }
    CHECK(threw);
    std::printf("%s (%d failures)\n", fails ? "FAILED" : "OK", fails);
    return fails ? 1 : 0;
}
