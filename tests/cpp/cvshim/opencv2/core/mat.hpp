// Test-only minimal cv::Mat (tests/cpp): the handful of cv::Mat members that
// include/stereo.h's OpenCV path uses (data, rows, cols, step[0], type, empty, size,
// create, ptr, isContinuous, ROI views, shared reference-counted storage as OpenCV 4.x
// has it), so that path is compiled and run without OpenCV in the image.  Not a general
// OpenCV replacement and not used to build any reference source.
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <memory>
#include <vector>

#define CV_8U 0
#define CV_8S 1
#define CV_16U 2
#define CV_16S 3
#define CV_32S 4
#define CV_32F 5
#define CV_64F 6
#define CV_CN_SHIFT 3
#define CV_MAKETYPE(depth, cn) ((depth) + (((cn) - 1) << CV_CN_SHIFT))
#define CV_8UC1 CV_MAKETYPE(CV_8U, 1)
#define CV_8UC3 CV_MAKETYPE(CV_8U, 3)
#define CV_16UC1 CV_MAKETYPE(CV_16U, 1)
#define CV_16SC1 CV_MAKETYPE(CV_16S, 1)
#define CV_16SC2 CV_MAKETYPE(CV_16S, 2)
#define CV_32FC1 CV_MAKETYPE(CV_32F, 1)
#define CV_32FC3 CV_MAKETYPE(CV_32F, 3)
#define CV_64FC1 CV_MAKETYPE(CV_64F, 1)

namespace cv {

typedef unsigned char uchar;

struct Size {
    int width = 0, height = 0;
    Size() = default;
    Size(int w, int h) : width(w), height(h) {}
    bool operator==(const Size& o) const { return width == o.width && height == o.height; }
    bool operator!=(const Size& o) const { return !(*this == o); }
};

struct Rect {
    int x = 0, y = 0, width = 0, height = 0;
    Rect(int x_, int y_, int w, int h) : x(x_), y(y_), width(w), height(h) {}
};

struct MatStep {
    std::size_t p[2] = {0, 0};
    std::size_t operator[](int i) const { return p[i]; }
    std::size_t& operator[](int i) { return p[i]; }
    operator std::size_t() const { return p[0]; }
};

class Mat {
public:
    int rows = 0, cols = 0;
    uchar* data = nullptr;
    MatStep step;

    Mat() = default;
    Mat(int r, int c, int t) { create(r, c, t); }
    Mat(Size s, int t) { create(s.height, s.width, t); }
    /** Mat over user memory (no ownership), as cv::Mat(rows, cols, type, data, step). */
    Mat(int r, int c, int t, void* d, std::size_t s) : rows(r), cols(c), data((uchar*)d), type_(t) {
        step.p[0] = s;
        step.p[1] = elemSize();
    }
    Mat(const Mat& m, const Rect& roi) : Mat(m) {
        data = m.data + (std::size_t)roi.y * m.step.p[0] + (std::size_t)roi.x * m.elemSize();
        rows = roi.height;
        cols = roi.width;
    }
    Mat operator()(const Rect& roi) const { return Mat(*this, roi); }

    void create(int r, int c, int t) {
        if (data && rows == r && cols == c && type_ == t) return;  // OpenCV reuses a matching buffer
        rows = r;
        cols = c;
        type_ = t;
        step.p[1] = elemSize();
        step.p[0] = (std::size_t)c * step.p[1];
        store_ = std::make_shared<std::vector<uchar>>((std::size_t)r * step.p[0]);
        data = store_->data();
    }
    void create(Size s, int t) { create(s.height, s.width, t); }
    Mat clone() const {
        Mat m(rows, cols, type_);
        for (int y = 0; y < rows; ++y) std::memcpy(m.ptr(y), ptr(y), (std::size_t)cols * elemSize());
        return m;
    }
    int type() const { return type_; }
    int channels() const { return 1 + (type_ >> CV_CN_SHIFT); }
    std::size_t elemSize1() const {
        static const std::size_t sz[8] = {1, 1, 2, 2, 4, 4, 8, 2};
        return sz[type_ & 7];
    }
    std::size_t elemSize() const { return (std::size_t)channels() * elemSize1(); }
    bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
    Size size() const { return Size(cols, rows); }
    bool isContinuous() const { return step.p[0] == (std::size_t)cols * elemSize(); }
    uchar* ptr(int y = 0) { return data + (std::size_t)y * step.p[0]; }
    const uchar* ptr(int y = 0) const { return data + (std::size_t)y * step.p[0]; }
    template <typename T> T* ptr(int y = 0) { return (T*)ptr(y); }
    template <typename T> const T* ptr(int y = 0) const { return (const T*)ptr(y); }
    /** shared owners of the storage (the refcount OpenCV keeps in u->refcount) */
    long use_count() const { return store_ ? store_.use_count() : 0; }

private:
    int type_ = 0;
    std::shared_ptr<std::vector<uchar>> store_;
};

}  // namespace cv
