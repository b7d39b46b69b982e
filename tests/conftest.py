import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running oracle case")


def load_bgr(path: str) -> np.ndarray:
    from PIL import Image

    return np.ascontiguousarray(np.array(Image.open(path).convert("RGB"))[:, :, ::-1])


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O

    O.build()
    return O


@pytest.fixture(scope="session")
def demo_pair_0600():
    d = os.path.join(GOLDEN, "demo")
    return load_bgr(os.path.join(d, "0600-Left.png")), load_bgr(os.path.join(d, "0600-Right.png"))


@pytest.fixture(scope="session")
def demo_pair_0045():
    d = os.path.join(GOLDEN, "demo")
    return load_bgr(os.path.join(d, "0045-Left.png")), load_bgr(os.path.join(d, "0045-Right.png"))


def host_threads() -> int:
    # the GPU box reports the whole machine's cores; keep to its share
    return max(1, min(16, os.cpu_count() or 1))
