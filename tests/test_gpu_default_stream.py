"""`_dev` calls on torch's DEFAULT stream (cuda_stream == 0), with no
synchronisation between torch's producers and the library's kernels.

A NULL stream is HIP's legacy null stream, the caller's default stream
(include/novelpoly.h conventions).  So the torch
generators, fills and copies queued there before a call are finished before
the library's kernels read the buffers, and the fills of the outputs and
statuses land before the kernels write them.  Until round 5 NULL meant the
context's non-blocking stream: round 5's probe p17 (gpurun_out/r05/
pytest_huge_p17.log) saw status rows left at the -1 of a `torch.full` that
landed after the kernel had written them.  These tests run without the
autouse stream fixture of conftest.py (marker `default_stream`), so the
whole test is on torch's default stream.

Reference semantics: the crate's calls are synchronous
(src/novel_poly_basis/mod.rs:117-239), so its callers assume exactly this
ordering."""
import numpy as np
import pytest

import novelpoly_amd as npa
from novelpoly_amd import synth

pytestmark = [pytest.mark.gpu, pytest.mark.default_stream]


def test_default_stream_is_torch_default(gpu):
    import torch

    assert torch.cuda.current_stream().cuda_stream == 0  # no fixture stream here


# p17's shape: 65,536 validators (n 65536, k 16384), 1 MiB payloads, a batch
# that spans two scratch slices with paired tiles (tests/test_gpu_slices.py).
@pytest.mark.parametrize("batch", [1801])
def test_huge_round_trip_on_default_stream(gpu, batch):
    import torch

    p = npa.CodeParams.derive_parameters(65536, 21846)
    n, k = p.n(), p.k()
    plen = 1 << 20
    sl = p.make_encoder(gpu).shard_len(plen)
    g = torch.Generator(device="cuda")
    g.manual_seed(batch)
    pays = torch.randint(0, 256, (batch, plen), dtype=torch.uint8, device="cuda", generator=g)
    shards = torch.empty((batch, n, sl), dtype=torch.uint8, device="cuda")
    npa.encode_batch_dev(p, pays.data_ptr(), plen, plen, batch, shards.data_ptr(), n * sl, ctx=gpu, stream=0)
    keep = torch.rand((batch, n), device="cuda", generator=g) >= 1 / 3
    keep[:, :k] &= torch.rand((batch, k), device="cuda", generator=g) >= 0.5
    pres = keep.to(torch.uint8)
    out = torch.full((batch, plen), 0xA5, dtype=torch.uint8, device="cuda")
    st = torch.full((batch, 2), -1, dtype=torch.int32, device="cuda")
    npa.reconstruct_batch_dev2(p, shards.data_ptr(), sl, n * sl, pres.data_ptr(), 0, batch, out.data_ptr(), plen,
                               ctx=gpu, stream=0, d_status=st.data_ptr())  # np_reconstruct_batch_dev3
    # no synchronisation: torch's default-stream reads below queue after the kernels
    have = pres.sum(dim=1, dtype=torch.int32)
    wrong = torch.nonzero((st[:, 0] != 0) | (st[:, 1] != have)).flatten().cpu().numpy()
    assert wrong.size == 0, (wrong.size, wrong[:5], st[wrong[:5]].cpu().numpy())
    bad = torch.nonzero((out != pays).any(dim=1)).flatten().cpu().numpy()
    assert bad.size == 0, f"{bad.size} payloads differ, first {bad[:5]}"


# p11's shape: n 2048, k 1024 (the resident decode), shard_len 540 (a full
# 64-column tile and a partial one of 14), non-codeword rows; device
# locators, then the caller's locators, each right after torch fills.
def test_noncodeword_locators_on_default_stream(gpu, oracle):
    import torch

    p = npa.CodeParams.derive_parameters(2048, 1024)
    n, k, sl, batch = p.n(), p.k(), 540, 3
    rng = np.random.default_rng(2048 + sl)
    rows = rng.integers(0, 256, (batch, n, sl), dtype=np.uint8)
    pres = np.stack([synth.present_mask(7 + b, n, (n - k) // 3 + b) for b in range(batch)]).astype(np.uint8)
    want = []
    for b in range(batch):
        st, w = oracle.reconstruct([rows[b, i].tobytes() if pres[b, i] else None for i in range(n)], n, k)
        assert st == 0
        want.append(w)
    olen = (sl // 2) * 2 * k
    ds = torch.from_numpy(rows).to("cuda", non_blocking=True)
    dpres = torch.from_numpy(pres).to("cuda", non_blocking=True)
    loc = torch.full((batch, n), 0x7FFF, dtype=torch.int16, device="cuda")
    npa.error_locator_dev(n, dpres.data_ptr(), batch, loc.data_ptr(), ctx=gpu, stream=0)
    for lp in (0, loc.data_ptr()):
        out = torch.full((batch, olen), 0x5A, dtype=torch.uint8, device="cuda")
        st_d = torch.full((batch, 2), -1, dtype=torch.int32, device="cuda")
        npa.reconstruct_batch_dev2(p, ds.data_ptr(), sl, n * sl, dpres.data_ptr(), lp, batch, out.data_ptr(), olen,
                                   ctx=gpu, stream=0, d_status=st_d.data_ptr())
        o, stat = out.cpu().numpy(), st_d.cpu().numpy()
        for b in range(batch):
            assert o[b].tobytes() == want[b], ("caller" if lp else "device", b)
            assert tuple(stat[b]) == (0, int(pres[b].sum())), b


# config 3's code on torch's default stream through the NULL stream of the
# ctypes wrapper (stream argument omitted), encode -> reconstruct round trip.
def test_config3_round_trip_null_stream(gpu):
    import torch

    p = npa.CodeParams.derive_parameters(1024, 342)
    n, plen, batch = p.n(), 1 << 20, 64
    sl = p.make_encoder(gpu).shard_len(plen)
    olen = (sl // 2) * 2 * p.k()
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    pays = torch.randint(0, 256, (batch, plen), dtype=torch.uint8, device="cuda", generator=g)
    shards = torch.full((batch, n, sl), 0xEE, dtype=torch.uint8, device="cuda")
    npa.encode_batch_dev(p, pays.data_ptr(), plen, plen, batch, shards.data_ptr(), n * sl, ctx=gpu)
    pres = (torch.rand((batch, n), device="cuda", generator=g) >= 342 / 1024).to(torch.uint8)
    pres[:, :8] = 0  # always a decode
    out = torch.full((batch, olen), 0x11, dtype=torch.uint8, device="cuda")
    npa.reconstruct_batch_dev2(p, shards.data_ptr(), sl, n * sl, pres.data_ptr(), 0, batch, out.data_ptr(), olen,
                               ctx=gpu)
    assert torch.equal(out[:, :plen], pays)
