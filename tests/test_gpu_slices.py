"""Batches larger than one slice of the context scratch (engine.cpp
launch_reconstruct: per-payload records are made for a slice of the batch at
a time, the decode then runs over that slice): tiny payloads (one chunk, shard
length 2) in batches that need two or three slices, on the fast path
(n = 1024, k = 256), the k = 512 path (n = 2048) and the k = 1024 path
(n = 4096).  Random erasures at a rate that leaves some payloads with fewer
than k present rows: those get NeedMoreShards{have, k, n} and keep their
output bytes; every other payload must come back as its payload (the shards
are codewords), and a sample of both kinds is checked against the oracle.
Also the sub-transform path (k >= 4096) over two and three slices with paired
tiles: full-size round trips."""
import numpy as np
import pytest

import novelpoly_amd as npa

pytestmark = pytest.mark.gpu


# (n_wanted, k_wanted, batch, present rate): the batch exceeds one slice of the
# 8 GiB scratch (fast: ~51k payloads of n = 1024; k = 512: ~172k of n = 2048;
# k = 1024: ~86k of n = 4096)
CASES = [(1024, 342, 104000, 0.27), (2000, 667, 180000, 0.272), (4096, 1366, 90000, 0.262)]


@pytest.mark.parametrize("nw,kw,batch,rate", CASES)
def test_reconstruct_record_slices(gpu, oracle, nw, kw, batch, rate):
    import torch

    p = npa.CodeParams.derive_parameters(nw, kw)
    n, k = p.n(), p.k()
    plen = 2 * k  # one chunk: shard length 2
    sl = p.make_encoder(gpu).shard_len(plen)
    assert sl == 2
    rng = np.random.default_rng(nw + batch)
    s = torch.cuda.current_stream().cuda_stream
    pays = torch.from_numpy(rng.integers(0, 256, (batch, plen), dtype=np.uint8)).cuda()
    shards = torch.empty((batch, n, sl), dtype=torch.uint8, device="cuda")
    npa.encode_batch_dev(p, pays.data_ptr(), plen, plen, batch, shards.data_ptr(), n * sl, ctx=gpu, stream=s)
    pres = (torch.rand((batch, n), device="cuda") < rate).to(torch.uint8)
    pres[:, nw:] = 0  # rows >= wanted_n were never produced
    have = pres.sum(dim=1).cpu().numpy()
    short = have < k
    assert short.any() and (~short).sum() > batch // 2
    out = torch.full((batch, plen), 0xA5, dtype=torch.uint8, device="cuda")
    st = torch.full((batch, 2), -1, dtype=torch.int32, device="cuda")
    npa.reconstruct_batch_dev2(p, shards.data_ptr(), sl, n * sl, pres.data_ptr(), 0, batch, out.data_ptr(), plen,
                               ctx=gpu, stream=s, d_status=st.data_ptr())
    torch.cuda.synchronize()
    o, stat, pay = out.cpu().numpy(), st.cpu().numpy(), pays.cpu().numpy()
    assert (stat[~short, 0] == 0).all()
    assert (stat[short, 0] == npa.NeedMoreShards.code).all()
    assert (stat[:, 1] == have).all()
    ok = np.nonzero(~short)[0]
    bad = ok[(o[ok] != pay[ok]).any(axis=1)]
    assert bad.size == 0, f"{bad.size} payloads differ, first {bad[:5]}"
    assert (o[short] == 0xA5).all()
    # oracle on a sample spread over the slices
    hs, hp = shards.cpu().numpy(), pres.cpu().numpy()
    for b in list(ok[:: max(1, ok.size // 6)][:6]) + list(np.nonzero(short)[0][:2]):
        recv = [hs[b, v].tobytes() if hp[b, v] else None for v in range(n)]
        code, want = oracle.reconstruct(recv, n, k)
        if short[b]:
            assert code == npa.NeedMoreShards.code
        else:
            assert code == 0 and o[b].tobytes() == want[:plen], b


# 65,536 validators, 1 MiB payloads (32 columns: two per tile): the encode's
# slots take 4 MiB per payload (2 slices of the 8 GiB scratch for 2,501
# payloads), the decode's 5 MiB + 128 KiB (2 slices); slices hold whole pairs,
# and the odd last payload has a tile of its own.
@pytest.mark.parametrize("batch", [2501])
def test_huge_paired_slices_round_trip(gpu, batch):
    import torch

    p = npa.CodeParams.derive_parameters(65536, 21846)
    n, k = p.n(), p.k()
    plen = 1 << 20
    sl = p.make_encoder(gpu).shard_len(plen)
    assert k == 16384 and sl // 2 == 32
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cuda")
    g.manual_seed(batch)
    pays = torch.randint(0, 256, (batch, plen), dtype=torch.uint8, device="cuda", generator=g)
    shards = torch.empty((batch, n, sl), dtype=torch.uint8, device="cuda")
    npa.encode_batch_dev(p, pays.data_ptr(), plen, plen, batch, shards.data_ptr(), n * sl, ctx=gpu, stream=s)
    keep = torch.rand((batch, n), device="cuda", generator=g) >= 1 / 3
    keep[:, :k] &= torch.rand((batch, k), device="cuda", generator=g) >= 0.5  # systematic rows lost too
    pres = keep.to(torch.uint8)
    out = torch.full((batch, plen), 0xA5, dtype=torch.uint8, device="cuda")
    st = torch.full((batch, 2), -1, dtype=torch.int32, device="cuda")
    npa.reconstruct_batch_dev2(p, shards.data_ptr(), sl, n * sl, pres.data_ptr(), 0, batch, out.data_ptr(), plen,
                               ctx=gpu, stream=s, d_status=st.data_ptr())
    torch.cuda.synchronize()
    stat = st.cpu().numpy()
    have = pres.sum(dim=1).cpu().numpy()
    wrong = np.nonzero((stat[:, 0] != 0) | (stat[:, 1] != have))[0]
    assert wrong.size == 0, (wrong.size, wrong[:5], stat[wrong[:5]], have[wrong[:5]])
    bad = torch.nonzero((out != pays).any(dim=1)).flatten().cpu().numpy()
    assert bad.size == 0, f"{bad.size} payloads differ, first {bad[:5]}"
