"""Shared fixtures.  `-m "not gpu"` runs on CPU; `-m gpu` needs an MI355X."""
import os
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
for p in (os.path.join(ROOT, "oracle"), os.path.join(ROOT, "reed-solomon-novelpoly_amd", "python"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "default_stream: runs on torch's default stream (no per-test stream; "
                            "tests/test_gpu_default_stream.py)")
    config.addinivalue_line("markers", "pin_in_place: NP_PAGEABLE=pin cases, run in a child process "
                            "(test_gpu_pin_isolated.py) so that the rest of the suite never shares a "
                            "process with buffers the engine registered in place")


def pytest_collection_modifyitems(config, items):
    if os.environ.get("NP_PIN_CHILD"):
        return
    skip = pytest.mark.skip(reason="NP_PAGEABLE=pin case: runs in the child process of test_gpu_pin_isolated.py")
    for it in items:
        if it.get_closest_marker("pin_in_place"):
            it.add_marker(skip)


@pytest.fixture(scope="session")
def oracle():
    import np_oracle

    return np_oracle.Oracle()


@pytest.fixture(scope="session")
def refc():
    import np_oracle

    if not np_oracle.ref_available():
        pytest.skip("oracle/_ref/librsec_ref.so not built (reference tree absent)")
    return np_oracle.RefC()


@pytest.fixture(scope="session")
def golden_vectors():
    import numpy as np

    return np.load(os.path.join(GOLDEN, "vectors.npz"), allow_pickle=False)


@pytest.fixture(scope="session")
def golden_json():
    import json

    def load(name):
        with open(os.path.join(GOLDEN, name)) as f:
            return json.load(f)

    return load


@pytest.fixture(scope="session")
def gpu():
    """A device context on cuda:0 through the product library (fails loudly)."""
    import novelpoly_amd as npa
    import torch

    assert torch.cuda.is_available(), "GPU test run without a visible GPU"
    torch.cuda.init()
    ctx = npa.default_context(0)
    return ctx


@pytest.fixture(autouse=True)
def _own_stream(request):
    """GPU tests run on a non-default torch stream, and the tests hand that
    stream to the library: torch's fills and copies and our kernels are then
    ordered on one queue.  (A NULL stream is the legacy null stream, torch's
    default stream: tests marked `default_stream` run there.)"""
    if request.node.get_closest_marker("gpu") is None or request.node.get_closest_marker("default_stream"):
        yield
        return
    import torch

    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        yield
    torch.cuda.synchronize()


@pytest.fixture(autouse=True)
def _bounds_checked(request):
    """In the checked-build child of tests/test_gpu_bounds.py (NP_BOUNDS_CHILD,
    NP_LIB_PATH = lib/libnovelpoly_hip_chk.so): after every GPU test, no global
    access of the instrumented kernels fell outside its buffer."""
    yield
    if not os.environ.get("NP_BOUNDS_CHILD") or request.node.get_closest_marker("gpu") is None:
        return
    import novelpoly_amd as npa

    r = npa.debug_bounds_check(npa.default_context(0))
    assert r is not None, "NP_BOUNDS_CHILD set but the library is not the checked build"
    assert r["count"] == 0, f"out-of-extent global accesses: {r}"
