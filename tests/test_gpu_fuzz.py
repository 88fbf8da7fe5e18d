"""Randomised GPU parity (seeded): device-batch encode and reconstruct through
the C ABI against the oracle, over random code parameters, payload lengths,
batch sizes, payload/shard/output strides, wanted_n, erasure patterns of every
decode-prefix mode and tile-per-workgroup counts (NP_ENC_TPW / NP_REC_TPW pin
the multi-tile kernels' split).  Complements the fixed shapes of
test_gpu_parity.py; like the reference's quickcheck round trips
(novel_poly_basis/tests.rs), every case is checked bit for bit -- including
received rows that are not a codeword (a corrupted present row), as the
reference's reconstruct fuzz target feeds (fuzzit/src/reconstruct.rs:15-43)."""
import numpy as np
import pytest

import novelpoly_amd as npa
from novelpoly_amd import synth

pytestmark = pytest.mark.gpu

# (n_wanted, k_wanted) -> effective k in {64, 128, 256}, n in {2k, 4k, 8k}
SHAPES = [(1024, 342), (512, 256), (2048, 300), (256, 86), (512, 128), (256, 128), (768, 256), (300, 100),
          (700, 234)]
# k in {512, 1024} (kernels_big.hip), n in {2k, 4k, 8k}; shorter payloads (the
# oracle's size-8192 transforms are slow)
SHAPES_BIG = [(2000, 667), (1024, 512), (2500, 834), (4096, 1366), (5000, 1667), (2048, 1024), (7000, 2334),
              (4096, 2048)]
# k in {8, 16, 32} (kernels_small.hip)
SHAPES_SMALL = [(100, 34), (150, 50), (60, 20), (90, 30), (40, 14), (16, 8), (30, 10), (64, 32), (190, 63)]


def _erasures(rng, n, k, mode):
    pres = np.ones(n, np.uint8)
    if mode == "random":
        pres[rng.choice(n, rng.integers(0, n - k + 1), replace=False)] = 0
    elif mode == "systematic_kept":
        pres[k + rng.choice(n - k, rng.integers(0, n - k + 1), replace=False)] = 0
    elif mode == "heavy":  # exactly k rows left
        pres[rng.choice(n, n - k, replace=False)] = 0
    return pres


@pytest.mark.parametrize("case", range(24))
def test_fuzz_device_batch_roundtrip(gpu, oracle, monkeypatch, case):
    _fuzz(gpu, oracle, monkeypatch, case, SHAPES, [3, 300, 900], 10)


@pytest.mark.parametrize("case", range(24))
def test_fuzz_big_device_batch_roundtrip(gpu, oracle, monkeypatch, case):
    _fuzz(gpu, oracle, monkeypatch, 100 + case, SHAPES_BIG, [1, 3, 24], 5)


@pytest.mark.parametrize("case", range(24))
def test_fuzz_small_device_batch_roundtrip(gpu, oracle, monkeypatch, case):
    _fuzz(gpu, oracle, monkeypatch, 200 + case, SHAPES_SMALL, [3, 300, 900], 10)


def _fuzz(gpu, oracle, monkeypatch, case, shapes, chunk_counts, max_batch):
    import torch

    rng = np.random.default_rng(1000 + case)
    nw, kw = shapes[case % len(shapes)]
    p = npa.CodeParams.derive_parameters(nw, kw)
    n, k = p.n(), p.k()
    wanted = n if case % 3 else int(rng.integers(n // 2 + 1, n + 1))
    monkeypatch.setenv("NP_ENC_TPW", str(int(rng.integers(1, 6))))
    monkeypatch.setenv("NP_REC_TPW", str(int(rng.integers(1, 6))))
    batch = int(rng.integers(1, max_batch))
    plen = int(rng.integers(1, 2 * k * int(rng.choice(chunk_counts))))
    pstride = plen + int(rng.choice([0, 0, 1, 8, 13]))
    sl = p.make_encoder(gpu).shard_len(plen)
    # device encode writes the n-row layout; rows >= wanted are not produced
    sstride = n * sl + int(rng.choice([0, 0, 8, 16, 2]))
    pls = np.zeros((batch, pstride), np.uint8)
    for b in range(batch):
        pls[b, :plen] = np.frombuffer(synth.payload(case * 100 + b, plen), dtype=np.uint8)
    dp = dev(pls)
    ds = torch.zeros((batch, sstride), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    p_enc = npa.CodeParams(n, k, wanted)
    npa.encode_batch_dev(p_enc, dp.data_ptr(), plen, pstride, batch, ds.data_ptr(), sstride, ctx=gpu, stream=s)
    torch.cuda.synchronize()
    hs = ds.cpu().numpy()
    rows = []
    for b in range(batch):
        st, want = oracle.encode(pls[b, :plen].tobytes(), n, k, wanted)
        assert st == 0
        got = hs[b, : n * sl].reshape(n, sl)
        bad = [v for v in range(wanted) if got[v].tobytes() != want[v]]
        assert not bad, ("encode", case, b, len(bad), bad[:4])
        rows.append(got)
    if wanted != n:
        return  # reconstruct needs every codeword row
    modes = ["random", "systematic_kept", "heavy"]
    pres = np.stack([_erasures(rng, n, k, modes[(case + b) % 3]) for b in range(batch)])
    # half the payloads get a corrupted present row (not a codeword any more):
    # the decode must still equal the reference's linear map of every present row
    for b in range(batch):
        if rng.random() < 0.5:
            v = int(rng.choice(np.flatnonzero(pres[b])))
            rows[b][v] ^= rng.integers(1, 256, sl, dtype=np.uint8)
            ds[b, v * sl:(v + 1) * sl] = torch.from_numpy(rows[b][v].copy()).cuda()
    dpres = dev(pres)
    olen = (sl // 2) * 2 * k
    ostride = olen + int(rng.choice([0, 0, 8, 3]))
    out = torch.zeros((batch, ostride), dtype=torch.uint8, device="cuda")
    npa.reconstruct_batch_dev2(p, ds.data_ptr(), sl, sstride, dpres.data_ptr(), 0, batch, out.data_ptr(), ostride,
                               ctx=gpu, stream=s)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    for b in range(batch):
        recv = [rows[b][i].tobytes() if pres[b, i] else None for i in range(n)]
        st, want = oracle.reconstruct(recv, n, k)
        assert st == 0
        assert o[b, :olen].tobytes() == want, ("reconstruct", case, b)


def dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a)).cuda()
