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
    # the library is built beforehand (__graft_entry__.build(), in this tree); it is rebuilt here only
    # when missing: a GPU box receives the built libptgs.so without the object files, and a rebuild
    # there would run the tests on a library other than the one profiled and benchmarked
    from pathtracer_gaussiansplatting_amd import _abi
    from pathtracer_gaussiansplatting_amd import build as B
    if not os.path.exists(B.LIB):
        B.build()
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
