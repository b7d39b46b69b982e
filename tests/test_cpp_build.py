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


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_mixed_opencv_modes_fail_to_link(tmp_path):
    """One program, two translation units that include stereo.h in different forms (light
    ImageView vs cv::Mat): the forms live in different inline namespaces, so passing an
    ADCensus across them is a link error, not a silent ODR violation at run time."""
    import subprocess

    from conftest import ROOT

    inc = os.path.join(ROOT, "include")
    shim = os.path.join(ROOT, "tests", "cpp", "cvshim")
    (tmp_path / "a.cpp").write_text('#include "stereo.h"\nvoid use(stereo::ADCensus& m) { m.setOffset(1); }\n')
    (tmp_path / "b.cpp").write_text('#include "stereo.h"\nvoid use(stereo::ADCensus& m);\n'
                                    'void call(stereo::ADCensus& m) { use(m); }\nint main() { return 0; }\n')
    objs = []
    for name, extra in (("a", ["-DTSM_NO_OPENCV"]), ("b", ["-I", shim])):
        o = str(tmp_path / f"{name}.o")
        subprocess.run(["g++", "-std=c++20", "-c", "-I", inc, *extra, str(tmp_path / f"{name}.cpp"), "-o", o],
                       check=True)
        objs.append(o)
    # same form on both sides links
    o2 = str(tmp_path / "a2.o")
    subprocess.run(["g++", "-std=c++20", "-c", "-I", inc, "-I", shim, str(tmp_path / "a.cpp"), "-o", o2], check=True)
    nm = subprocess.run(["nm", "-C", objs[0], o2], capture_output=True, text=True, check=True).stdout
    assert "stereo::light_v1::ADCensus" in nm and "stereo::cvmat_v1::ADCensus" in nm
    r = subprocess.run(["g++", objs[0], objs[1], "-o", str(tmp_path / "mixed")], capture_output=True, text=True)
    assert r.returncode != 0 and "undefined reference" in r.stderr, r.stderr


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_adcensus_params_defaults_match_reference(tmp_path):
    """include/stereo.h's ADCensusParams (reference stereo_utils.h:206-244) carries the
    reference's per-model defaults (stereo_utils.cpp:271-326) and converts to the C ABI's
    tsm_adc_params and back; header-only, so it runs without the library or a GPU."""
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "params")
    subprocess.run(["g++", "-std=c++20", "-Wall", "-Werror", "-I", os.path.join(root, "include"),
                    os.path.join(root, "tests", "cpp", "test_params.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert "params ok" in r.stdout
