"""Batches larger than one slice of the context scratch (engine.cpp
launch_reconstruct: per-payload records are made for a slice of the batch at
a time, the decode then runs over that slice): tiny payloads (one chunk, shard
length 2) in batches that need two or three slices, on the fast path
(n = 1024, k = 256), the k = 512 path (n = 2048) and the k = 1024 path
(n = 4096).  Random erasures at a rate that leaves some payloads with fewer
than k present rows: those get NeedMoreShards{have, k, n} and keep their
output bytes; every other payload must come back as its payload (the shards
are codewords), and a sample of both kinds is checked against the oracle."""
import numpy as np
import pytest

import novelpoly_amd as npa

pytestmark = pytest.mark.gpu


# (n_wanted, k_wanted, batch, present rate): the batch exceeds one slice
# (fast: ~12.7k payloads of n = 1024; big: ~43k of n = 2048, ~21k of n = 4096)
CASES = [(1024, 342, 26000, 0.27), (2000, 667, 45000, 0.272), (4096, 1366, 22500, 0.262)]


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
