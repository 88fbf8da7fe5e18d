"""The product's kernels in the checked build (lib/libnovelpoly_hip_chk.so,
-DNP_BOUNDS_CHECK=1, device_common.hpp): the global accesses of
the kernels of round 5's probe p11 window (k_error_locator, k_prefix_locator /
k_locator_records, k_reconstruct_res) and of the encode and decode kernels'
shared row, payload and output helpers (fast, resident, small, big and
sub-transform kernels) are compared with the extent of their buffer implied
by the kernel's arguments (payloads, shards, present flags, locators, decode
records, outputs, statuses, the zero page); an access outside is counted,
recorded and redirected, so the kernel completes and the host reads the
record.

One child process runs every GPU test file but the pin-in-place child's and
the multi-context one (p11's shape [2048-1024-540] among them) against the
checked library, one launch at a time, and
conftest.py's `_bounds_checked` fixture asserts after every test that no
access fell outside.  The child first checks the checker:
with NP_BOUNDS_SELFTEST the out extent is shortened, and the last payload's
output writes must be caught."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
CHK_LIB = os.path.join(ROOT, "reed-solomon-novelpoly_amd", "lib", "libnovelpoly_hip_chk.so")


def _child_env():
    # The checked kernels keep their extents in one record per code object and
    # device, so the child runs one launch at a time: the host pipeline on one
    # stream (NP_PIPE_SLOTS=1), and no multi-context file (test_gpu_multi.py
    # runs contexts from several threads at once).
    return dict(os.environ, NP_LIB_PATH=CHK_LIB, NP_BOUNDS_CHILD="1", NP_PIPE_SLOTS="1")


def test_checked_library_built():
    assert os.path.exists(CHK_LIB), "run `make -C reed-solomon-novelpoly_amd chk` (__graft_entry__.build does)"


@pytest.mark.skipif(bool(os.environ.get("NP_BOUNDS_CHILD")), reason="the product library's answer")
def test_product_library_has_no_checks(gpu):
    """The product library reports that it is not a checked build (its code
    objects carry no checks: the macros are the plain expressions)."""
    import novelpoly_amd as npa

    assert npa.debug_bounds_check(gpu) is None


@pytest.mark.skipif(not os.environ.get("NP_BOUNDS_CHILD"), reason="runs in the checked child process")
def test_checker_catches_a_short_out_extent(gpu, monkeypatch):
    """NP_BOUNDS_SELFTEST=64: the kernels see an out extent 64 bytes short, so
    the copy-out of the last payload's last column must be flagged."""
    import numpy as np
    import torch

    import novelpoly_amd as npa
    from novelpoly_amd import synth

    p = npa.CodeParams.derive_parameters(2048, 1024)
    n, k, sl, batch = p.n(), p.k(), 540, 2
    rows = torch.randint(0, 256, (batch, n, sl), dtype=torch.uint8, device="cuda")
    pres = torch.from_numpy(np.stack([synth.present_mask(b, n, 600) for b in range(batch)]).astype(np.uint8)).cuda()
    olen = (sl // 2) * 2 * k
    out = torch.empty((batch, olen), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    assert npa.debug_bounds_check(gpu)["count"] == 0
    monkeypatch.setenv("NP_BOUNDS_SELFTEST", "64")
    npa.reconstruct_batch_dev2(p, rows.data_ptr(), sl, n * sl, pres.data_ptr(), 0, batch, out.data_ptr(), olen,
                               ctx=gpu, stream=s)
    r = npa.debug_bounds_check(gpu)
    assert r["count"] > 0 and r["kind"] == "out", r
    assert r["offset"] + r["bytes"] > batch * olen - 64, r
    monkeypatch.delenv("NP_BOUNDS_SELFTEST")
    npa.reconstruct_batch_dev2(p, rows.data_ptr(), sl, n * sl, pres.data_ptr(), 0, batch, out.data_ptr(), olen,
                               ctx=gpu, stream=s)
    assert npa.debug_bounds_check(gpu)["count"] == 0


@pytest.mark.skipif(bool(os.environ.get("NP_BOUNDS_CHILD")), reason="the parent of the checked child")
@pytest.mark.timeout(1100)
def test_p11_window_kernels_in_bounds():
    assert os.path.exists(CHK_LIB)
    files = ["tests/test_gpu_bounds.py", "tests/test_gpu_noncodeword.py", "tests/test_gpu_parity.py",
             "tests/test_gpu_fuzz.py", "tests/test_gpu_default_stream.py", "tests/test_gpu_huge.py",
             "tests/test_gpu_slices.py", "tests/test_gpu_host_guard.py"]
    r = subprocess.run([sys.executable, "-u", "-m", "pytest", *files, "-m", "gpu and not pin_in_place", "-x", "-q",
                        "-p", "no:cacheprovider", "--timeout", "120", "--timeout-method", "thread"],
                       cwd=ROOT, env=_child_env(), capture_output=True, text=True, timeout=1080)
    tail = "\n".join((r.stdout + r.stderr).splitlines()[-30:])
    assert r.returncode == 0, tail
    assert " passed" in tail and "failed" not in tail and " error" not in tail, tail
