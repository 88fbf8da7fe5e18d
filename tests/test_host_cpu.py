"""CPU tests of the product library's host side: it loads, exports every
symbol include/novelpoly.h declares, and its parameter logic matches the
reference's known answers (no GPU compute here)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import novelpoly_amd as npa
from novelpoly_amd import synth

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "novelpoly.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(np_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = npa.lib()
    names = declared_functions()
    assert len(names) >= 28
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_status_messages():
    L = npa.lib()
    for st in range(0, 9):
        assert L.np_status_message(st)
    assert "gfx950" in npa.version()


def test_recoverability_subset_size():
    # util.rs:44-59 three_f_plus_1
    kat = {0: 1, 1: 1, 2: 1, 3: 1, 4: 2, 5: 2, 6: 2, 8: 3, 11: 4, 173: 58, 174: 58, 175: 59}
    for n, want in kat.items():
        assert npa.recoverablity_subset_size(n) == want


def test_code_params_kat():
    # tests.rs:421-446 test_code_params
    with pytest.raises(npa.Error):
        npa.CodeParams.derive_parameters(0, npa.recoverablity_subset_size(0))
    with pytest.raises(npa.WantedShardCountTooLow):
        npa.CodeParams.derive_parameters(1, npa.recoverablity_subset_size(1))
    for nw, n, k in ((2, 2, 1), (3, 4, 1), (4, 4, 2), (100, 128, 32)):
        p = npa.CodeParams.derive_parameters(nw, npa.recoverablity_subset_size(nw))
        assert (p.n(), p.k(), p.wanted_n) == (n, k, nw)
    with pytest.raises(npa.WantedPayloadShardCountTooLow):
        npa.CodeParams.derive_parameters(10, 0)
    with pytest.raises(npa.WantedShardCountTooHigh) as ei:
        npa.CodeParams.derive_parameters(65537, 3)
    assert ei.value.fields == (65537,)
    assert npa.CodeParams.derive_parameters(65536, 21846).n() == 65536


def test_k_n_construction():
    # tests.rs:50-64
    for vc in range(3, 8201):
        p = npa.CodeParams.derive_parameters(vc, npa.recoverablity_subset_size(vc))
        assert p.wanted_n == vc and vc <= p.n()
        assert vc // 3 >= p.k() - 1 and vc >= (p.k() - 1) * 3


def test_shard_len_kat():
    # tests.rs:448-466 shard_len_is_reasonable (n16 k4 wanted 5)
    p = npa._Params(16, 4, 5)
    L = npa.lib()
    for size, want in ((100, 26), (99, 26), (95, 24), (94, 24), (90, 24), (19, 6)):
        assert L.np_shard_len(C.byref(p), size) == want


def test_params_new_power_of_two_rule():
    # mod.rs:109-115: only fails when neither n nor k is a power of two
    p = npa._Params()
    assert npa.lib().np_params_new(12, 3, 12, C.byref(p)) == 6
    assert npa.lib().np_params_new(16, 3, 12, C.byref(p)) == 0


def test_wrapped_shard_pads_odd():
    # wrapped_shard.rs:33-39
    assert npa.WrappedShard(b"abc").into_inner() == b"abc\x00"
    assert npa.WrappedShard(b"ab").into_inner() == b"ab"


def test_baseline_configs_effective_params():
    # SURVEY F10
    for cid, cfg in synth.CONFIGS.items():
        p = npa.CodeParams.derive_parameters(cfg["n_wanted"], cfg["k_wanted"])
        assert (p.n(), p.k()) == (cfg["n"], cfg["k"]), cid


def test_synth_is_deterministic():
    a = synth.payload(7, 1000)
    assert a == synth.payload(7, 1000) and a != synth.payload(8, 1000)
    e = synth.erasure_indices(3, 1024, 342)
    assert len(set(e.tolist())) == 342 and e.max() < 1024
    assert np.array_equal(e, synth.erasure_indices(3, 1024, 342))


def test_fast_path_table():
    """np_is_fast_path (the crate's is_faster8 slot, mod.rs:64-71) reports the
    kernel families the engine dispatches to (engine.cpp rec_path): small
    (k <= 32), fast (64-256), resident (512, 1024), big (2048) and huge
    (4096-16384, 1 MiB payloads) serve both directions at n/k in {2, 4, 8};
    explicit n/k >= 16 reconstructs on the generic kernels."""
    for cfg in synth.CONFIGS.values():
        p = npa.CodeParams.derive_parameters(cfg["n_wanted"], cfg["k_wanted"])
        assert p.is_faster8(), cfg
    served = [(2, 1), (3, 1), (10, 4), (16, 8), (100, 34), (256, 86), (1024, 342), (2000, 667), (4096, 1366),
              (8192, 2731), (10000, 3334), (16384, 5462), (30000, 10000), (65536, 21846)]
    for nw, kw in served:
        assert npa.CodeParams.derive_parameters(nw, kw).is_faster8(), (nw, kw)
    for nw, kw in [(4096, 256), (8192, 512), (32768, 1024)]:  # n / k >= 16: generic reconstruct
        assert not npa.CodeParams.derive_parameters(nw, kw).is_faster8(), (nw, kw)


def test_ctx_without_gpu_reports_no_device():
    import torch

    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(npa.DeviceError):
        npa.Context(0)


def test_payload_batch_dev_matches_splitmix():
    """bench.py's torch generator of the §8(d) payloads equals synth.payload
    (splitmix64, seed 0x5EED_0000 + index), here on the CPU device."""
    import torch

    for lo, hi, nbytes in ((0, 3, 64), (1022, 1024, 1 << 12), (5, 7, 1001)):
        got = synth.payload_batch_dev(lo, hi, nbytes, torch.device("cpu")).numpy()
        for i in range(lo, hi):
            assert got[i - lo].tobytes() == synth.payload(i, nbytes), (lo, hi, nbytes, i)



def test_batch_split_contiguous_ranges():
    """np_batch_split: contiguous, disjoint ranges covering the
    batch, sizes differing by at most one, the larger ones first."""
    for batch in (0, 1, 7, 8, 1000, 8192):
        for ndev in (1, 2, 3, 8):
            rng = [npa.batch_split(batch, ndev, i) for i in range(ndev)]
            assert rng[0][0] == 0
            assert all(a[0] + a[1] == b[0] for a, b in zip(rng, rng[1:]))
            assert rng[-1][0] + rng[-1][1] == batch
            sizes = [c for _, c in rng]
            assert max(sizes) - min(sizes) <= 1 and sizes == sorted(sizes, reverse=True)
    assert npa.batch_split(10, 2, 5) == (10, 0)  # out-of-range device: empty
