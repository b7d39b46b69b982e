"""The C++ boundary compiles and links on the CPU (no GPU needed): include/stereo.h
without OpenCV (ImageView virtual) and with a cv::Mat on the include path
(tests/cpp/cvshim), where StereoMatching's pure virtual must be the reference's
compute(const cv::Mat&, const cv::Mat&, cv::Mat&) (reference include/stereo.h:325-331)."""
import os
import shutil

import pytest

from test_gpu_cpp_api import compile_program, LIB


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
@pytest.mark.parametrize("src,opencv", [("test_stereo_api.cpp", False),
                                        ("test_stereo_api_cvmat.cpp", True)])
def test_cpp_api_compiles_and_links(tmp_path, src, opencv):
    if not os.path.exists(os.path.join(LIB, "libtsm_adcensus.so")):
        pytest.skip("library not built (make lib)")
    exe = str(tmp_path / "prog")
    compile_program(src, exe, opencv)
    assert os.path.getsize(exe) > 0
