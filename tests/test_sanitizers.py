"""Once-only sanitizer runs (SURVEY.md §5 "Race detection / sanitizers"), on the CPU:

* the oracle (the C restatement, oracle/) through every mode under AddressSanitizer +
  UndefinedBehaviorSanitizer and under ThreadSanitizer over its OpenMP stages (LLVM's
  OpenMP runtime with the Archer tool, so the runtime's synchronisation is visible):
  `make -C oracle sanitize`, oracle/sanitize_main.c;
* the product's host threading, the row-band copy pool the host entry points use
  (tea_stereo_matching_amd/csrc/copy_pool.h), under ThreadSanitizer and AddressSanitizer,
  four caller threads at once (tests/cpp/test_copy_pool.cpp).
GPU code is not sanitized (no GPU ASan / XNACK on this pool)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

CSRC = os.path.join(ROOT, "tea_stereo_matching_amd", "csrc")


@pytest.mark.skipif(shutil.which("gcc") is None or not os.path.exists("/opt/rocm/lib/llvm/lib/libarcher.so"),
                    reason="needs gcc and ROCm's LLVM (libarcher)")
def test_oracle_under_asan_ubsan_and_tsan():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize"], capture_output=True,
                       text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert out.count("OK (0 failures)") == 2, out[-4000:]
    assert "ThreadSanitizer" not in out and "AddressSanitizer" not in out and "runtime error" not in out


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_copy_pool_under_sanitizer(tmp_path, san):
    exe = str(tmp_path / "copy_pool")
    subprocess.run(["g++", "-std=c++20", "-O1", "-g", f"-fsanitize={san}", "-fno-sanitize-recover=all",
                    "-I", CSRC, os.path.join(ROOT, "tests", "cpp", "test_copy_pool.cpp"), "-o", exe, "-pthread"],
                   check=True)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "OK (0 failures)" in r.stdout, r.stdout + r.stderr[-4000:]
