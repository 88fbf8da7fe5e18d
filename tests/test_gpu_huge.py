"""k = 2048 .. 16384 as size-1024 sub-transforms plus top levels
(kernels_huge.hip; more than 12,288 validators: n = 16384 .. 65536): encode
and reconstruct bit-exact against the oracle over every n / k the crate
derives there, full and partial 64-column tiles, odd payload tails, wanted_n
< n, random / worst-case / no erasures.  Reference: inc_encode.rs:15-48,
inc_reconstruct.rs:1-113, mod.rs:43-61 / :117-239."""
import numpy as np
import pytest

import novelpoly_amd as npa
from novelpoly_amd import synth

pytestmark = pytest.mark.gpu

# (n_wanted, k_wanted, payload bytes): n16384 k4096 (NQ 4), n32768 k4096 (8),
# n32768 k8192 (4), n65536 k8192 (8), n65536 k16384 (4); tiles of 64 columns
ENC = [(16384, 5462, 2 * 4096 * 64), (16384, 5462, 2 * 4096 * 70 + 3), (12289, 4097, 2 * 4096 * 3 + 1),
       (20000, 6667, 2 * 4096 * 65), (24000, 8000, 999), (30000, 10000, 2 * 8192 * 64 + 5),
       (32768, 10923, 2 * 8192 * 2), (40000, 13334, 2 * 8192 * 66), (65536, 21846, 2 * 16384 * 65 + 7),
       (50000, 16667, 2 * 16384 * 3)]


@pytest.mark.parametrize("nw,kw,plen", ENC)
def test_huge_encode(gpu, oracle, nw, kw, plen):
    p = npa.CodeParams.derive_parameters(nw, kw)
    assert p.k() >= 4096
    pl = synth.payload(nw + plen, plen)
    got = p.make_encoder(gpu).encode(pl)
    st, want = oracle.encode(pl, p.n(), p.k(), nw)
    assert st == 0
    bad = [v for v in range(nw) if got[v] != want[v]]
    assert not bad, f"{len(bad)} shards differ, first {bad[:5]}"


# erase: number of random erasures; -1: every systematic shard lost; 0: none (copy);
# -2: whole 1024-row blocks (0, 3 and the second k-row segment: k_huge_rec_inv
# skips blocks without a present row, k_huge_rec_top reads them as zero)
REC = [(20000, 6667, 2 * 4096 * 65, -2), (40000, 13334, 2 * 8192 * 66 + 1, -2), (16384, 5462, 2 * 4096 * 64, -2),
       (16384, 5462, 2 * 4096 * 64, 8000), (16384, 5462, 2 * 4096 * 70 + 3, -1), (20000, 6667, 2 * 4096 * 65, 13333),
       (20000, 6667, 2 * 4096 * 2, 0), (30000, 10000, 2 * 8192 * 64 + 5, 20000), (30000, 10000, 2 * 8192 * 3, -1),
       (40000, 13334, 2 * 8192 * 66, 26666), (65536, 21846, 2 * 16384 * 65 + 7, 43690),
       (65536, 21846, 2 * 16384 * 2, -1)]


@pytest.mark.parametrize("nw,kw,plen,erase", REC)
def test_huge_reconstruct(gpu, oracle, nw, kw, plen, erase):
    p = npa.CodeParams.derive_parameters(nw, kw)
    n, k = p.n(), p.k()
    assert k >= 4096 and n in (2 * k, 4 * k, 8 * k)
    pl = synth.payload(3 * nw + plen, plen)
    shards = p.make_encoder(gpu).encode(pl)
    if erase == -1:
        gone = set(range(k))
    elif erase == -2:
        gone = set(range(1024)) | set(range(3072, 4096)) | set(range(k, 2 * k))
    else:
        gone = set(synth.erasure_indices(plen + erase, nw, min(erase, nw - k)).tolist())
    recv = [None if i in gone else s for i, s in enumerate(shards[:nw])]
    assert sum(r is not None for r in recv) >= k
    got = p.make_encoder(gpu).reconstruct(recv)
    st, want = oracle.reconstruct(recv, n, k)
    assert st == 0 and got == want
    assert got[:plen] == pl


# k = 16384 payloads of at most 32 columns: the sub-transform encode packs two
# payloads into one 64-column tile (kernels_huge.hip HugeArgs::pair): odd and
# even batches (the last tile half empty), whole and partial 32-column halves,
# wanted_n < n; every payload against the oracle.
PAIR = [(65536, 21846, 2 * 16384 * 32, 4), (65536, 21846, 2 * 16384 * 17 + 3, 3), (50000, 16667, 2 * 16384 * 5, 5)]


@pytest.mark.parametrize("nw,kw,plen,batch", PAIR)
def test_huge_encode_paired_batch(gpu, oracle, nw, kw, plen, batch):
    import torch

    p = npa.CodeParams.derive_parameters(nw, kw)
    n, k = p.n(), p.k()
    assert k == 16384
    sl = p.make_encoder(gpu).shard_len(plen)
    assert sl // 2 <= 32
    pls = np.stack([np.frombuffer(synth.payload(nw + plen + b, plen), np.uint8) for b in range(batch)])
    dp = torch.from_numpy(pls).cuda()
    bstride = nw * sl + 6
    ds = torch.full((batch, bstride), 0xA5, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    npa.encode_batch_dev(p, dp.data_ptr(), plen, plen, batch, ds.data_ptr(), bstride, ctx=gpu,
                         stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    hs = ds.cpu().numpy()
    for b in range(batch):
        st, want = oracle.encode(pls[b].tobytes(), n, k, nw)
        assert st == 0
        bad = [v for v in range(nw) if hs[b, v * sl:(v + 1) * sl].tobytes() != want[v]]
        assert not bad, (b, len(bad), bad[:5])
        assert (hs[b, nw * sl:] == 0xA5).all()


# The same pairing in the sub-transform decode: a tile runs the larger of its
# two payloads' modes, each lane half merges and writes for its own payload.
# Mixed modes per pair: random erasures (decode), only parity lost (copy),
# every systematic shard lost, fewer than k shards (NeedMoreShards: status
# set, output untouched), a non-codeword (a corrupted present shard), and
# whole 1024-row blocks erased (a pair's blocks are skipped where neither
# payload has a present row).
PAIR_REC = [(65536, 21846, 2 * 16384 * 32, ["rand", "copy", "nosys", "rand"]),
            (65536, 21846, 2 * 16384 * 9, ["blocks", "blocks2", "blocks", "rand", "blocks2"]),
            (65536, 21846, 2 * 16384 * 17 + 3, ["copy", "rand", "few", "corrupt", "rand"]),
            (50000, 16667, 2 * 16384 * 5, ["few", "rand", "rand"])]


@pytest.mark.parametrize("nw,kw,plen,kinds", PAIR_REC)
def test_huge_reconstruct_paired_batch(gpu, oracle, nw, kw, plen, kinds):
    import torch

    p = npa.CodeParams.derive_parameters(nw, kw)
    n, k = p.n(), p.k()
    assert k == 16384
    sl = p.make_encoder(gpu).shard_len(plen)
    assert sl // 2 <= 32
    batch = len(kinds)
    pls = np.stack([np.frombuffer(synth.payload(2 * nw + plen + b, plen), np.uint8) for b in range(batch)])
    dp = torch.from_numpy(pls).cuda()
    ds = torch.zeros((batch, n * sl), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    npa.encode_batch_dev(p, dp.data_ptr(), plen, plen, batch, ds.data_ptr(), n * sl, ctx=gpu,
                         stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    hs = ds.cpu().numpy()
    rng = np.random.default_rng(plen + batch)
    pres = np.zeros((batch, n), np.uint8)
    for b, kind in enumerate(kinds):
        pres[b, :nw] = 1
        if kind in ("rand", "corrupt"):
            pres[b, rng.choice(nw, nw - k, replace=False)] = 0
        elif kind == "copy":
            pres[b, k + rng.choice(nw - k, (nw - k) // 2, replace=False)] = 0
        elif kind == "nosys":
            pres[b, :k] = 0
        elif kind == "few":
            pres[b, rng.choice(nw, nw - k + 1, replace=False)] = 0
        elif kind == "blocks":  # blocks 0, 5, 17-20 and 40-63
            for u in [0, 5, 17, 18, 19, 20] + list(range(40, n // 1024)):
                pres[b, 1024 * u:1024 * (u + 1)] = 0
        elif kind == "blocks2":  # blocks 5, 6 and 33-63, and random rows
            for u in [5, 6] + list(range(33, n // 1024)):
                pres[b, 1024 * u:1024 * (u + 1)] = 0
            pres[b, rng.choice(1024 * 30, 5000, replace=False)] = 0
        if kind == "corrupt":
            v = int(rng.choice(np.flatnonzero(pres[b])))
            hs[b, v * sl:(v + 1) * sl] ^= 0x3C
    ds = torch.from_numpy(hs).cuda()
    dpres = torch.from_numpy(pres).cuda()
    olen = (sl // 2) * 2 * k
    dout = torch.full((batch, olen), 0x77, dtype=torch.uint8, device="cuda")
    dst = torch.full((batch, 2), -1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    npa.reconstruct_batch_dev2(p, ds.data_ptr(), sl, n * sl, dpres.data_ptr(), 0, batch, dout.data_ptr(), olen,
                               ctx=gpu, stream=torch.cuda.current_stream().cuda_stream, d_status=dst.data_ptr())
    torch.cuda.synchronize()
    o, stat = dout.cpu().numpy(), dst.cpu().numpy()
    for b, kind in enumerate(kinds):
        have = int(pres[b].sum())
        if kind == "few":
            assert have < k and stat[b, 0] != 0 and stat[b, 1] == have, (b, stat[b])
            assert (o[b] == 0x77).all(), b  # a NeedMoreShards payload's output is left untouched
            continue
        assert tuple(stat[b]) == (0, have), (b, stat[b])
        recv = [hs[b, i * sl:(i + 1) * sl].tobytes() if pres[b, i] else None for i in range(n)]
        st, want = oracle.reconstruct(recv, n, k)
        assert st == 0 and o[b].tobytes() == want, (b, kind)
        if kind != "corrupt":
            assert want[:plen] == pls[b].tobytes()
