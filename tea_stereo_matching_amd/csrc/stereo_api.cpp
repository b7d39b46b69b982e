// stereo_api.cpp -- stereo::ADCensus (include/stereo.h) over the C ABI.
// Maps status codes back to the reference's exception types and messages
// (ADCensus.cpp:307-333, :383-387).
#include "../../include/stereo.h"

#include "../../include/tsm_adcensus.h"

namespace stereo {

StereoMatching::~StereoMatching() {}

class ADCensus::ADCensusImpl {
public:
    tsm_adc* h = nullptr;
};

namespace {
[[noreturn]] void raise(tsm_adc* h, int rc) {
    const std::string msg = tsm_adc_last_error(h);
    switch (rc) {
        case TSM_ERR_DISPARITY_RANGE:
        case TSM_ERR_OFFSET:
        case TSM_ERR_IMAGE:
            throw(msg);  // the reference throws std::string here
        default:
            throw std::runtime_error(msg.empty() ? std::string("tsm_adc error ") + std::to_string(rc) : msg);
    }
}
}  // namespace

ADCensus::ADCensus() : ADCensus(0) {}

ADCensus::ADCensus(int device) : impl(std::make_unique<ADCensusImpl>()) {
    const int rc = tsm_adc_create(device, &impl->h);
    if (rc != TSM_OK) throw std::runtime_error("[ADCensus] no usable HIP device (tsm_adc_create " + std::to_string(rc) + ")");
}

ADCensus::~ADCensus() {
    if (impl && impl->h) tsm_adc_destroy(impl->h);
}

void ADCensus::setMinMaxDisparity(const int& minDisparity, const int& maxDisparity) {
    const int rc = tsm_adc_set_disparity_range(impl->h, minDisparity, maxDisparity);
    if (rc != TSM_OK) raise(impl->h, rc);
}

void ADCensus::setMatchingStrategy(const ColorModel& colorModel, const bool& roiMatching,
                                   const bool& maskMatching) {
    const int rc = tsm_adc_set_strategy(impl->h, (int)colorModel, roiMatching ? 1 : 0, maskMatching ? 1 : 0);
    if (rc != TSM_OK) raise(impl->h, rc);
}

void ADCensus::setOffset(const int& offset) {
    const int rc = tsm_adc_set_offset(impl->h, offset);
    if (rc != TSM_OK) raise(impl->h, rc);
}

void ADCensus::setOmpEmulation(int threads) {
    const int rc = tsm_adc_set_omp_emulation(impl->h, threads);
    if (rc != TSM_OK) raise(impl->h, rc);
}

void ADCensus::setConcurrency(int streams) {
    const int rc = tsm_adc_set_concurrency(impl->h, streams);
    if (rc != TSM_OK) raise(impl->h, rc);
}

void ADCensus::compute(const ImageView& l, const ImageView& r, DisparityMap& d) {
    if (l.empty() || r.empty() || l.rows != r.rows || l.cols != r.cols)
        throw(std::string("[ADCensus] Image error."));
    DisparityMap out;
    out.rows = l.rows;
    out.cols = l.cols;
    out.data.resize((size_t)l.rows * l.cols);
    int rc;
    if (l.step == r.step) {
        rc = tsm_adc_compute(impl->h, l.data, r.data, l.rows, l.cols, l.step, out.data.data(),
                             (size_t)l.cols * 4);
    } else {  // the C ABI takes one step for both views
        std::vector<std::uint8_t> a((size_t)l.rows * l.cols * 3), b(a.size());
        for (int y = 0; y < l.rows; ++y) {
            std::copy(l.data + y * l.step, l.data + y * l.step + (size_t)l.cols * 3, a.data() + (size_t)y * l.cols * 3);
            std::copy(r.data + y * r.step, r.data + y * r.step + (size_t)r.cols * 3, b.data() + (size_t)y * r.cols * 3);
        }
        rc = tsm_adc_compute(impl->h, a.data(), b.data(), l.rows, l.cols, (size_t)l.cols * 3,
                             out.data.data(), (size_t)l.cols * 4);
    }
    if (rc != TSM_OK) raise(impl->h, rc);
    d = std::move(out);  // output reassigned, as disparity = m_floatDisparityMap.clone() (:391)
}

void ADCensus::compute(const std::vector<ImageView>& ls, const std::vector<ImageView>& rs,
                       std::vector<DisparityMap>& ds) {
    if (ls.size() != rs.size()) throw(std::string("[ADCensus] Image error."));
    if (ls.empty()) { ds.clear(); return; }
    const ImageView& f = ls[0];
    std::vector<const std::uint8_t*> lp, rp;
    std::vector<float*> op;
    std::vector<DisparityMap> out(ls.size());
    bool uniform = true;
    for (size_t i = 0; i < ls.size(); ++i) {
        const ImageView& l = ls[i];
        const ImageView& r = rs[i];
        if (l.empty() || r.empty() || l.rows != r.rows || l.cols != r.cols)
            throw(std::string("[ADCensus] Image error."));
        uniform = uniform && l.rows == f.rows && l.cols == f.cols && l.step == f.step && r.step == f.step;
    }
    if (!uniform) {  // mixed geometry: one pair at a time
        for (size_t i = 0; i < ls.size(); ++i) compute(ls[i], rs[i], out[i]);
        ds = std::move(out);
        return;
    }
    for (size_t i = 0; i < ls.size(); ++i) {
        out[i].rows = f.rows;
        out[i].cols = f.cols;
        out[i].data.resize((size_t)f.rows * f.cols);
        lp.push_back(ls[i].data);
        rp.push_back(rs[i].data);
        op.push_back(out[i].data.data());
    }
    const int rc = tsm_adc_compute_batch(impl->h, (int)ls.size(), lp.data(), rp.data(), f.rows, f.cols,
                                         f.step, op.data(), (size_t)f.cols * 4);
    if (rc != TSM_OK) raise(impl->h, rc);
    ds = std::move(out);
}

}  // namespace stereo
