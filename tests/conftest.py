import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); parity tests through the C ABI")


@pytest.fixture(scope="session")
def native_lib():
    from bugcar_image_segmentation_amd.build import build_native
    build_native()
    from bugcar_image_segmentation_amd import _native
    return _native.load_library()


@pytest.fixture(scope="session")
def blocks():
    from bugcar_image_segmentation_amd import enet_spec
    return enet_spec.build_enet()


@pytest.fixture(scope="session")
def gpu(native_lib):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible HIP device")
    torch.cuda.set_device(0)
    return torch.device("cuda", 0)
