"""The resident kernels' LDS swizzles (res_common.hpp rsw<K>) are conflict-free
for every sweep the kernels make (tools/res_swizzle.py models the CQ, HA and
HD reads and writes and the payload tile's writes under the guide's bank
rules), and rsw<K> in the source is the swizzle the model checks; the
encode's quad items (res_common.hpp Qi, pi(p) = p ^ bit 4 of p) are
conflict-free for its CQ, HA' and HD' sweeps."""
import os
import re
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import res_swizzle  # noqa: E402


def source_rows(K):
    src = open(os.path.join(ROOT, "reed-solomon-novelpoly_amd", "csrc", "res_common.hpp")).read()
    body = src[src.index("__host__ __device__ constexpr uint32_t rsw(uint32_t c) {"):]
    branch = body.split("else")[0] if K == 1024 else body.split("else")[1]
    vals = re.findall(r"\(c & (\d+)u\) \? (\d+)u : 0u", branch)
    return [int(v) for b, v in sorted(vals, key=lambda t: int(t[0]))]


@pytest.mark.parametrize("K", [1024, 512])
def test_resident_swizzle_conflict_free(K):
    rows = source_rows(K)
    assert rows == res_swizzle.PRODUCT[K]
    assert res_swizzle.conflicts(K, res_swizzle.rsw_of(rows)) == 0


def test_model_sees_conflicts():
    # the k = 1024 swizzle under the k = 512 HD geometry conflicts (why K = 512 has its own)
    assert res_swizzle.conflicts(512, res_swizzle.rsw_of(res_swizzle.PRODUCT[1024])) > 0
    assert res_swizzle.conflicts(1024, res_swizzle.rsw_of([0] * 6)) > 0


@pytest.mark.parametrize("K", [1024, 512])
def test_encode_quad_items_conflict_free(K):
    src = open(os.path.join(ROOT, "reed-solomon-novelpoly_amd", "csrc", "res_common.hpp")).read()
    assert "q.hd = 128u * (ph ^ ((ph >> 4) & 1u))" in src  # the pi of the model
    assert res_swizzle.qi_conflicts(K) == 0
    assert res_swizzle.qi_conflicts(K, pi_bit=None) > 0  # without pi the CQ reads conflict
