"""The NP_PAGEABLE=pin cases (marker pin_in_place: pageable host buffers
pinned in place for a call through engine.cpp's PinRegistry) in one child
process.  Pinning in place is opt-in since round 5: one GPU run saw an illegal
address in a process that had registered and unregistered numpy buffers
earlier, so the rest of the suite never shares a process with
such buffers.  One child for all the cases (not one per case)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


@pytest.mark.timeout(900)  # the child's own cases are limited to 120 s each
def test_pin_in_place_cases_in_child_process():
    env = dict(os.environ, NP_PIN_CHILD="1")
    files = ["tests/test_gpu_host_guard.py", "tests/test_gpu_parity.py", "tests/test_gpu_multi.py"]
    r = subprocess.run([sys.executable, "-u", "-m", "pytest", *files, "-m", "gpu and pin_in_place", "-x", "-q",
                        "-p", "no:cacheprovider", "--timeout", "120", "--timeout-method", "thread"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    tail = "\n".join((r.stdout + r.stderr).splitlines()[-25:])
    assert r.returncode == 0, tail
    assert " passed" in tail and "failed" not in tail, tail
