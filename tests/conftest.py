import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the C-ABI on the GPU)")


@pytest.fixture(scope="session")
def native_lib():
    from pathtracer_gaussiansplatting_amd import build as B
    B.build()
    from pathtracer_gaussiansplatting_amd import _abi
    return _abi.load_library()


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def renderer(native_lib):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from pathtracer_gaussiansplatting_amd import Renderer
    r = Renderer(0, publish_splat_buffers=True)
    yield r
    r.close()


@pytest.fixture(params=["megakernel", "wavefront"])
def pt(renderer, request):
    """The renderer with either path tracer selected (both must give the oracle's image)."""
    renderer.set_wavefront(request.param == "wavefront")
    yield renderer
    renderer.set_wavefront(False)
