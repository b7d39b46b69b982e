// include/stereo.h's ADCensusParams against the reference's defaults (stereo_utils.h:206-244,
// stereo_utils.cpp:271-326), header-only: no library, no GPU.
#include <cstdio>
#include <cstring>

#include "stereo.h"

#define CHECK(c)                                                    \
    do {                                                            \
        if (!(c)) {                                                 \
            std::fprintf(stderr, "CHECK failed: %s (line %d)\n", #c, __LINE__); \
            return 1;                                               \
        }                                                           \
    } while (0)

int main() {
    const stereo::ADCensusParams d;  // the reference's default constructor: RGB
    CHECK(d.lambdaAD == 10.f && d.censusWin == stereo::CensusWin::CENSUSWIN_9x7 && d.lambdaCensus == 30.f);
    CHECK(d.lambdaHue == 1.f && d.lambdaSaturation == 2.5f && d.lambdaIntensity == 2.5f);
    CHECK(d.colorThresh1 == 20 && d.colorThresh2 == 6 && d.maxLength1 == 34 && d.maxLength2 == 17);
    CHECK(d.colorDiff == 15 && d.saturationThresh1 == 0 && d.intensityThresh2 == 0);
    CHECK(d.iterations == 4 && d.pi1 == 1.f && d.pi2 == 3.f && d.dispTolerance == 0);
    CHECK(d.votingThresh == 20 && d.votingRatioThresh == 0.4f && d.maxSearchDepth == 20);
    CHECK(d.blurKernelSize == 3 && d.cannyThresh1 == 30 && d.cannyThresh2 == 90 && d.cannyKernelSize == 3);
    stereo::ADCensusParams h(stereo::ColorModel::HSI);
    CHECK(h.colorThresh1 == 5 && h.colorThresh2 == 1 && h.maxLength1 == 17 && h.maxLength2 == 8);
    CHECK(h.colorDiff == 3 && h.saturationThresh1 == 10 && h.saturationThresh2 == 2);
    CHECK(h.intensityThresh1 == 12 && h.intensityThresh2 == 3 && h.lambdaAD == 10.f);
    h.setADCensusParams(stereo::ColorModel::RGB);  // re-set: every member rewritten
    const tsm_adc_params a = h.toC(), b = d.toC();
    CHECK(std::memcmp(&a, &b, sizeof a) == 0);
    h.pi2 = 7.5f;
    h.censusWin = stereo::CensusWin::CENSUSWIN_7x5;
    const stereo::ADCensusParams back = stereo::ADCensusParams::fromC(h.toC());
    CHECK(back.pi2 == 7.5f && back.censusWin == stereo::CensusWin::CENSUSWIN_7x5 && back.maxLength1 == 34);
    std::printf("params ok\n");
    return 0;
}
