// stereo_ops.cpp -- host side of f3: stereo::writePointCloudToPCD / writePointCloudToPLY
// (source/stereo.cpp:204-356).  The points come from the gfx950 reprojection
// (k_stereo_ops.hip); formatting a text file is host work.  Same output bytes as the
// reference: std::to_chars shortest floats, the same headers, points with a +inf
// coordinate skipped, PCD colour packed as r<<16 | g<<8 | b | 1<<24.
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

#include "tsm_adcensus.h"
#include "tsm_stereo_ops.h"

namespace {

struct Point {
    float x, y, z;
    uint8_t b, g, r;
};

std::vector<Point> gather_points(const uint8_t* bgr, size_t bgr_step, const float* xyz, size_t xyz_step,
                                 int rows, int cols) {
    std::vector<Point> pts;
    pts.reserve((size_t)rows * cols);
    const float inf = std::numeric_limits<float>::infinity();
    for (int y = 0; y < rows; ++y) {
        const float* p = reinterpret_cast<const float*>(reinterpret_cast<const uint8_t*>(xyz) + (size_t)y * xyz_step);
        const uint8_t* c = bgr + (size_t)y * bgr_step;
        for (int x = 0; x < cols; ++x) {
            const float X = p[3 * x], Y = p[3 * x + 1], Z = p[3 * x + 2];
            if (X == inf || Y == inf || Z == inf) continue;  // stereo.cpp:268-270
            pts.push_back(Point{X, Y, Z, c[3 * x], c[3 * x + 1], c[3 * x + 2]});
        }
    }
    return pts;
}

template <class T>
char* put(char* cur, char* end, T v) {
    return std::to_chars(cur, end, v).ptr;
}

int write_file(const std::string& body, const char* path) {
    FILE* f = std::fopen(path, "wb");  // binary: no newline translation (stereo.cpp:245)
    if (!f) return TSM_ERR_IMAGE;
    const size_t n = std::fwrite(body.data(), 1, body.size(), f);
    const int rc = std::fclose(f);
    return n == body.size() && rc == 0 ? TSM_OK : TSM_ERR_IMAGE;
}

bool bad(const uint8_t* bgr, const float* xyz, int rows, int cols, const char* path) {
    return !bgr || !xyz || rows <= 0 || cols <= 0 || !path || !*path;
}

}  // namespace

extern "C" {

int tsm_write_point_cloud_pcd(const uint8_t* bgr, size_t bgr_step, const float* xyz, size_t xyz_step,
                              int rows, int cols, const char* path) {
    if (bad(bgr, xyz, rows, cols, path)) return TSM_ERR_ARGUMENT;
    const std::vector<Point> p = gather_points(bgr, bgr_step, xyz, xyz_step, rows, cols);
    std::string out = "# .PCD v0.7 - Point Cloud Data file format\nVERSION 0.7\nFIELDS x y z rgb\n"
                      "SIZE 4 4 4 4\nTYPE F F F U\nCOUNT 1 1 1 1\n";
    out += "WIDTH " + std::to_string(p.size()) + "\nHEIGHT 1\nVIEWPOINT 0 0 0 1 0 0 0\n";
    out += "POINTS " + std::to_string(p.size()) + "\nDATA ascii\n";
    const size_t head = out.size();
    out.resize(head + 64 * p.size());  // the reference's per-point budget (:220)
    char* cur = out.data() + head;
    char* end = out.data() + out.size();
    for (const Point& q : p) {
        cur = put(cur, end, q.x);
        *cur++ = ' ';
        cur = put(cur, end, q.y);
        *cur++ = ' ';
        cur = put(cur, end, q.z);
        *cur++ = ' ';
        const unsigned rgb = (unsigned)q.r << 16 | (unsigned)q.g << 8 | (unsigned)q.b | 1u << 24;
        cur = put(cur, end, rgb);
        *cur++ = '\n';
    }
    out.resize((size_t)(cur - out.data()));
    return write_file(out, path);
}

int tsm_write_point_cloud_ply(const uint8_t* bgr, size_t bgr_step, const float* xyz, size_t xyz_step,
                              int rows, int cols, const char* path) {
    if (bad(bgr, xyz, rows, cols, path)) return TSM_ERR_ARGUMENT;
    const std::vector<Point> p = gather_points(bgr, bgr_step, xyz, xyz_step, rows, cols);
    std::string out = "ply\nformat ascii 1.0\n";
    out += "element vertex " + std::to_string(p.size()) + "\n";
    out += "property float x\nproperty float y\nproperty float z\n"
           "property uchar red\nproperty uchar green\nproperty uchar blue\nend_header\n";
    const size_t head = out.size();
    out.resize(head + 128 * p.size());  // :295
    char* cur = out.data() + head;
    char* end = out.data() + out.size();
    for (const Point& q : p) {
        cur = put(cur, end, q.x);
        *cur++ = ' ';
        cur = put(cur, end, q.y);
        *cur++ = ' ';
        cur = put(cur, end, q.z);
        *cur++ = ' ';
        cur = put(cur, end, (int)q.r);
        *cur++ = ' ';
        cur = put(cur, end, (int)q.g);
        *cur++ = ' ';
        cur = put(cur, end, (int)q.b);
        *cur++ = '\n';
    }
    out.resize((size_t)(cur - out.data()));
    return write_file(out, path);
}

}  // extern "C"
