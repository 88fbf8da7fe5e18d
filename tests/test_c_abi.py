"""The drop-in boundary from C: tests/c_abi/abi_check.c is compiled as strict
C99 (-pedantic -Wall -Wextra -Werror) against include/novelpoly.h and linked
to the product library, as a bindgen-built binding would use it
(/root/reference/reed-solomon-novelpoly/build.rs:18-41, src/cxx.rs:13-31).
CPU: it compiles and links.  GPU: it runs np_encode, np_reconstruct,
np_encode_batch_dev and np_reconstruct_batch_dev2 on BASELINE config 2 and its
digests equal tests/golden/digests.json (made from the reference C build)."""
import json
import os
import subprocess

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
LIBDIR = os.path.join(ROOT, "reed-solomon-novelpoly_amd", "lib")
SRC = os.path.join(ROOT, "tests", "c_abi", "abi_check.c")


def build(tmp_path):
    exe = str(tmp_path / "abi_check")
    cmd = ["gcc", "-std=c99", "-pedantic", "-Wall", "-Wextra", "-Werror", "-D__HIP_PLATFORM_AMD__",
           "-isystem", "/opt/rocm/include", "-I", os.path.join(ROOT, "include"), SRC, "-o", exe,
           "-L" + LIBDIR, "-lnovelpoly_hip", "-L/opt/rocm/lib", "-lamdhip64",
           "-Wl,-rpath," + LIBDIR, "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def test_c_abi_compiles_and_links(tmp_path):
    if not os.path.exists(os.path.join(LIBDIR, "libnovelpoly_hip.so")):
        pytest.skip("product library not built")
    build(tmp_path)


@pytest.mark.gpu
def test_c_abi_program_matches_golden(tmp_path):
    exe = build(tmp_path)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.stdout, r.stderr)
    got = dict(line.split(" ", 1) for line in r.stdout.strip().splitlines() if " " in line)
    with open(os.path.join(ROOT, "tests", "golden", "digests.json")) as f:
        d = json.load(f)["cfg2"]
    assert got["payload"] == d["payload_sha256"]
    assert got["present"] == d["present_sha256"]
    assert got["np_encode"] == d["encode_sha256"]
    assert got["np_encode_batch_dev"] == d["encode_sha256"]
    assert got["np_reconstruct"] == d["reconstruct_sha256"]
    assert got["np_reconstruct_batch_dev2"] == d["reconstruct_sha256"]
    assert got["need_more_shards"] == "have=63 min=64 all=256"
    assert got["params"].startswith("n=256 k=64 wanted_n=256 shard_len=1024 fast=1")
