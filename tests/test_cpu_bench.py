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


def _build_sanitized():
    """Builds the restatement under ASan + UBSan (oracle/Makefile `san`); skips
    where gcc or its sanitizer runtimes are missing."""
    out = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "san"], capture_output=True, text=True,
                         timeout=300)
    if out.returncode != 0:
        pytest.skip("sanitizer build unavailable: " + out.stderr[-300:])


_SAN_ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")


@pytest.mark.parametrize("n,k,plen,erase", [(16, 8, 4096, 8), (256, 64, 65537, 170), (1024, 256, 1048576, 342),
                                            (512, 64, 100000, 300)])
def test_oracle_bench_sanitized(n, k, plen, erase):
    """The whole-payload encode / locator / decode loop of the restatement runs
    clean under AddressSanitizer + UBSan and round-trips."""
    _build_sanitized()
    exe = os.path.join(ROOT, "oracle", "_ref", "cpu_bench_port_san")
    out = subprocess.run([exe, str(n), str(k), str(plen), str(erase), "2", "0.2"], capture_output=True, text=True,
                         timeout=300, env=_SAN_ENV)
    assert out.returncode == 0, out.stderr[-3000:]
    assert json.loads(out.stdout.strip().splitlines()[-1])["failures"] == 0


def test_oracle_api_sanitized():
    """The crate glue of the restatement (derive_parameters, encode, reconstruct
    incl. the fuzz target's arbitrary shards, reconstruct_from_systematic) runs
    clean under AddressSanitizer + UBSan (oracle/san_api.c)."""
    _build_sanitized()
    exe = os.path.join(ROOT, "oracle", "_ref", "san_api")
    out = subprocess.run([exe, "7", "200"], capture_output=True, text=True, timeout=300, env=_SAN_ENV)
    assert out.returncode == 0, out.stderr[-3000:]
    assert json.loads(out.stdout.strip().splitlines()[-1])["failures"] == 0
