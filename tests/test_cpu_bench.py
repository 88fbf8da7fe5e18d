"""CPU baseline harness (oracle/cpu_bench.c): whole-payload encode + reconstruct
through the crate glue round-trips for the restatement and, where it was built,
for the reference's own C implementation (oracle/_ref)."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PORT = os.path.join(ROOT, "oracle", "cpu_bench_port")
REF = os.path.join(ROOT, "oracle", "_ref", "cpu_bench_ref")


def _run(exe, n, k, plen, erase, threads=2):
    out = subprocess.run([exe, str(n), str(k), str(plen), str(erase), str(threads), "0.2"],
                         check=False, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr + out.stdout
    return json.loads(out.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("exe", [PORT, REF], ids=["port", "reference"])
@pytest.mark.parametrize("n,k,plen,erase", [(16, 8, 4096, 8), (256, 64, 4097, 192), (1024, 256, 65536, 342)])
def test_cpu_bench_roundtrip(exe, n, k, plen, erase):
    if not os.path.exists(exe):
        pytest.skip(f"{exe} not built")
    r = _run(exe, n, k, plen, erase)
    assert r["failures"] == 0 and r["payloads"] >= 1
    assert r["kind"] == ("reference" if exe == REF else "port")


def test_cpu_bench_rejects_bad_arguments():
    if not os.path.exists(PORT):
        pytest.skip("not built")
    out = subprocess.run([PORT, "16", "8", "0", "0", "1", "0.1"], capture_output=True, text=True)
    assert out.returncode == 2
