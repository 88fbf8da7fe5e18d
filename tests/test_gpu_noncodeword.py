"""Reconstruct on received shards that are NOT a codeword, through every
crate-equivalent entry point, byte for byte against the oracle.

The reference's reconstruct (mod.rs:162-239 -> inc_reconstruct.rs:1-85) is a
fixed linear map of every present shard: it never checks that the shards form
a codeword, and its fuzz target feeds it arbitrary bytes
(reed-solomon-novelpoly-fuzzit/src/reconstruct.rs:15-43).  So the GPU decode
must equal that map for any input, not only for encoder output.  Two inputs per
shape: random bytes in every row, and a valid codeword with one present row
>= 2k corrupted (a row a decoder from a 2k-row prefix would never read).
Entries: np_reconstruct, np_rs_reconstruct, np_reconstruct_batch_dev,
np_reconstruct_batch_dev2 (device locators and caller locators) and
np_reconstruct_batch_host.  Also: the device-side NeedMoreShards status of
np_reconstruct_batch_dev2 and the opt-in codeword entry."""
import numpy as np
import pytest

import novelpoly_amd as npa
from novelpoly_amd import synth

pytestmark = pytest.mark.gpu

# (n_wanted, k_wanted, shard_len): config 2 (n256 k64), config 3 (n1024 k256),
# config 4 (n4096 k1024), n/k = 8 (n512 k64, n1024 k128, n2048 k256), n/k = 2
# (n1024 k256 with wanted_n 600; n2048 k1024), k = 512 (n1024, n2048, n4096)
# and n/k = 8 at k = 1024 (n8192); k in {8, 16, 32} (n128 k32, n256 k32, n64
# k16, n64 k8, n16 k8, n64 k32); shard lengths of one full 256-column tile
# plus a partial one
SHAPES = [(256, 86, 2 * 300), (1024, 342, 2 * 300), (4096, 1366, 2 * 260), (300, 100, 2 * 270),
          (700, 234, 2 * 300), (1200, 400, 2 * 290), (600, 256, 2 * 280), (2048, 1024, 2 * 270),
          (1024, 512, 2 * 270), (2000, 667, 2 * 260), (2500, 834, 2 * 270), (5000, 1667, 2 * 260),
          (100, 34, 2 * 300), (150, 50, 2 * 270), (60, 20, 2 * 260), (40, 14, 2 * 280), (16, 8, 2 * 300),
          (64, 32, 2 * 257), (7000, 2334, 2 * 260), (4096, 2048, 2 * 257), (10000, 3334, 2 * 260),
          # k = 4096 .. 16384 (kernels_huge.hip): n16384 k4096, n32768 k4096 / k8192,
          # n65536 k8192 / k16384; one full 64-column tile plus a partial one
          (16384, 5462, 2 * 70), (20000, 6667, 2 * 66), (30000, 10000, 2 * 65), (40000, 13334, 2 * 64 + 2),
          (65536, 21846, 2 * 67)]


def _dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _host(t):
    import torch

    torch.cuda.synchronize()
    return t.cpu().numpy()


def _inputs(p, sl, seed, gpu):
    """Three payloads' received rows (batch x n x sl) and present masks:
    random bytes; a codeword with a present row >= 2k corrupted; a codeword
    whose k systematic rows are present and every other present row random."""
    n, k = p.n(), p.k()
    rng = np.random.default_rng(seed)
    rows = np.zeros((3, n, sl), np.uint8)
    pres = np.zeros((3, n), np.uint8)
    # 0: random bytes, random erasures (about a third)
    rows[0] = rng.integers(0, 256, (n, sl), dtype=np.uint8)
    pres[0] = synth.present_mask(seed, n, (n - k) // 2 if n > 2 * k else (n - k) // 3)
    # 1: codeword, one present row >= 2k flipped (or >= k for n = 2k)
    plen = sl // 2 * 2 * k - 3
    shards = p.make_encoder(gpu).encode(synth.payload(seed, plen))  # wanted_n rows
    rows[1, : len(shards)] = np.stack([np.frombuffer(s, np.uint8) for s in shards])
    pres[1] = synth.present_mask(seed + 1, n, (n - k) // 3)
    pres[1, len(shards):] = 0
    lo = 2 * k if n > 2 * k else k
    cand = [v for v in range(lo, n) if pres[1, v]]
    victim = cand[len(cand) // 2]
    rows[1, victim] ^= rng.integers(1, 256, sl, dtype=np.uint8)
    # 2: all systematic rows present, the rest random: the output is those rows
    rows[2] = rng.integers(0, 256, (n, sl), dtype=np.uint8)
    pres[2] = 1
    pres[2, k + rng.choice(n - k, (n - k) // 2, replace=False)] = 0
    return rows, pres


def _recv(rows, pres):
    return [rows[i].tobytes() if pres[i] else None for i in range(len(pres))]


@pytest.mark.parametrize("nw,kw,sl", SHAPES)
def test_noncodeword_all_entries(gpu, oracle, nw, kw, sl):
    import torch

    p = npa.CodeParams.derive_parameters(nw, kw)
    n, k = p.n(), p.k()
    rows, pres = _inputs(p, sl, nw + sl, gpu)
    batch = rows.shape[0]
    want = []
    for b in range(batch):
        st, w = oracle.reconstruct(_recv(rows[b], pres[b]), n, k)
        assert st == 0
        want.append(w)
    olen = (sl // 2) * 2 * k
    rs = p.make_encoder(gpu)
    for b in range(batch):
        recv = _recv(rows[b], pres[b])
        # np_rs_reconstruct (mod.rs:162-239) and np_reconstruct (reconstruct.rs:4-9)
        assert rs.reconstruct(recv) == want[b], ("np_rs_reconstruct", b)
        if kw == npa.recoverablity_subset_size(nw):  # the validator count derives the same code
            assert npa.reconstruct(recv, nw, ctx=gpu) == want[b], ("np_reconstruct", b)
    ds = _dev(rows)
    s = torch.cuda.current_stream().cuda_stream
    # np_reconstruct_batch_dev (host present mask)
    out = torch.full((batch, olen), 0x5A, dtype=torch.uint8, device="cuda")
    npa.reconstruct_batch_dev(p, ds.data_ptr(), sl, n * sl, pres.tobytes(), batch, out.data_ptr(), olen, ctx=gpu,
                              stream=s)
    o = _host(out)
    for b in range(batch):
        assert o[b].tobytes() == want[b], ("np_reconstruct_batch_dev", b)
    # np_reconstruct_batch_dev2: device locators, then the caller's locators
    dpres = _dev(pres)
    loc = torch.empty((batch, n), dtype=torch.int16, device="cuda")
    npa.error_locator_dev(n, dpres.data_ptr(), batch, loc.data_ptr(), ctx=gpu, stream=s)
    for lp in (0, loc.data_ptr()):
        out = torch.full((batch, olen), 0x5A, dtype=torch.uint8, device="cuda")
        st_d = torch.full((batch, 2), -1, dtype=torch.int32, device="cuda")
        npa.reconstruct_batch_dev2(p, ds.data_ptr(), sl, n * sl, dpres.data_ptr(), lp, batch, out.data_ptr(), olen,
                                   ctx=gpu, stream=s, d_status=st_d.data_ptr())
        o = _host(out)
        stat = _host(st_d)
        for b in range(batch):
            assert o[b].tobytes() == want[b], ("np_reconstruct_batch_dev2", "caller" if lp else "device", b)
            assert tuple(stat[b]) == (0, int(pres[b].sum())), b
    # np_reconstruct_batch_host (host buffers, pipelined)
    hout = np.zeros((batch, olen), np.uint8)
    hrows = np.ascontiguousarray(rows)
    npa.reconstruct_batch_host(p, hrows.ctypes.data, sl, n * sl, pres.ctypes.data, batch, hout.ctypes.data, olen,
                               ctx=gpu)
    for b in range(batch):
        assert hout[b].tobytes() == want[b], ("np_reconstruct_batch_host", b)


@pytest.mark.parametrize("nw,kw,sl", SHAPES)
def test_device_need_more_shards_status(gpu, oracle, nw, kw, sl):
    """np_reconstruct_batch_dev2 reports NeedMoreShards{have, k, n} per payload
    (mod.rs:178-180) and leaves that payload's output untouched, while the other
    payloads of the batch decode as the reference."""
    import torch

    p = npa.CodeParams.derive_parameters(nw, kw)
    n, k = p.n(), p.k()
    rng = np.random.default_rng(sl + nw)
    batch = 4
    rows = rng.integers(0, 256, (batch, n, sl), dtype=np.uint8)
    pres = np.ones((batch, n), np.uint8)
    pres[0, rng.choice(n, n - k, replace=False)] = 0      # exactly k present: decodes
    pres[1, rng.choice(n, n - k + 1, replace=False)] = 0  # k - 1 present
    pres[2, k // 2:] = 0                                  # k/2 present, all systematic
    pres[3] = 0                                           # nothing received
    olen = (sl // 2) * 2 * k
    out = torch.full((batch, olen), 0x5A, dtype=torch.uint8, device="cuda")
    st_d = torch.full((batch, 2), -1, dtype=torch.int32, device="cuda")
    ds, dpres = _dev(rows), _dev(pres)
    npa.reconstruct_batch_dev2(p, ds.data_ptr(), sl, n * sl, dpres.data_ptr(), 0, batch, out.data_ptr(), olen,
                               ctx=gpu, stream=torch.cuda.current_stream().cuda_stream, d_status=st_d.data_ptr())
    o, stat = _host(out), _host(st_d)
    errs = npa.payload_errors(p, stat)
    assert errs[0] is None
    st, want = oracle.reconstruct(_recv(rows[0], pres[0]), n, k)
    assert st == 0 and o[0].tobytes() == want
    for b in (1, 2, 3):
        have = int(pres[b].sum())
        assert errs[b] == npa.NeedMoreShards(have, k, n), b
        assert (o[b] == 0x5A).all(), b  # not decoded
        st, _ = oracle.reconstruct(_recv(rows[b], pres[b]), n, k)
        assert st == npa.NeedMoreShards.code
    # without a status buffer the short payloads are skipped all the same
    out2 = torch.full((batch, olen), 0x5A, dtype=torch.uint8, device="cuda")
    npa.reconstruct_batch_dev2(p, ds.data_ptr(), sl, n * sl, dpres.data_ptr(), 0, batch, out2.data_ptr(), olen,
                               ctx=gpu, stream=torch.cuda.current_stream().cuda_stream)
    o2 = _host(out2)
    assert o2[0].tobytes() == want and (o2[1:] == 0x5A).all()


@pytest.mark.parametrize("nw,kw,plen", [(1024, 342, 512 * 300 + 1), (256, 86, 128 * 256), (512, 128, 256 * 257),
                                        (100, 34, 64 * 300 + 1), (60, 20, 32 * 257)])
def test_codewords_entry_on_codewords(gpu, oracle, nw, kw, plen):
    """The opt-in np_reconstruct_codewords_batch_dev (2k-row prefix decode on
    n = 4k shapes) equals the reference on unmodified codewords, in every
    erasure mode (copy, 2k prefix, full)."""
    import torch

    p = npa.CodeParams.derive_parameters(nw, kw)
    n, k = p.n(), p.k()
    rng = np.random.default_rng(plen)
    pats = []
    pres = np.ones(n, np.uint8)
    pres[k + rng.choice(n - k, (n - k) // 2, replace=False)] = 0
    pats.append(pres)
    pres = np.ones(n, np.uint8)
    pres[rng.choice(k, k // 3, replace=False)] = 0
    pres[2 * k + rng.choice(n - 2 * k, (n - 2 * k) // 2, replace=False)] = 0
    pats.append(pres)
    pres = np.ones(n, np.uint8)
    pres[rng.choice(2 * k, k + 1, replace=False)] = 0
    pats.append(pres)
    for pres in pats:
        pres[nw:] = 0  # rows >= wanted_n were never produced
    batch = len(pats)
    sl = p.make_encoder(gpu).shard_len(plen)
    pls = np.stack([np.frombuffer(synth.payload(77 + b, plen), np.uint8) for b in range(batch)])
    dp = _dev(pls)
    ds = torch.empty((batch, n, sl), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    npa.encode_batch_dev(p, dp.data_ptr(), plen, plen, batch, ds.data_ptr(), n * sl, ctx=gpu, stream=s)
    pres = np.stack(pats)
    olen = (sl // 2) * 2 * k
    out = torch.empty((batch, olen), dtype=torch.uint8, device="cuda")
    npa.reconstruct_codewords_batch_dev(p, ds.data_ptr(), sl, n * sl, _dev(pres).data_ptr(), batch, out.data_ptr(),
                                        olen, ctx=gpu, stream=s)
    o, hs = _host(out), _host(ds)
    for b in range(batch):
        st, want = oracle.reconstruct(_recv(hs[b], pres[b]), n, k)
        assert st == 0 and o[b].tobytes() == want, b
        assert want[:plen] == pls[b].tobytes()


@pytest.mark.parametrize("case", range(16))
def test_fuzzit_reconstruct_feed(gpu, oracle, case):
    """The reference's fuzz target (reed-solomon-novelpoly-fuzzit/src/reconstruct.rs:15-43):
    validator_count in 0..=2200, a random drop count, arbitrary bytes per shard,
    the list truncated to validator_count - 1 entries and optionally a last shard
    holding the remaining bytes (possibly of another length).  The GPU's result
    (bytes or error variant) equals the oracle's."""
    rng = np.random.default_rng(4200 + case)
    vc = int(rng.integers(0, 2201)) if case % 4 else int(rng.integers(2, 40))
    drop = int(rng.integers(0, vc + 1))
    n_chunks = vc - drop
    total = int(rng.integers(0, 20000))
    per = total // n_chunks if n_chunks > 0 else 0
    data = rng.integers(0, 256, total, dtype=np.uint8).tobytes()
    gone = set(rng.choice(vc, vc - n_chunks, replace=False).tolist()) if vc else set()
    pos = 0
    received = []
    for idx in range(vc):
        if idx in gone:
            received.append(None)
        else:
            received.append(data[pos:pos + per])
            pos += per
    received = received[: max(0, vc - 1)]
    rest = data[pos:]
    if not rest or len(rest) > per // 2:
        received.append(rest)
    try:
        got = ("ok", npa.reconstruct(received, vc, ctx=gpu))
    except npa.Error as e:
        got = ("err", type(e).__name__, e.fields)
    try:
        p = npa.CodeParams.derive_parameters(vc, npa.recoverablity_subset_size(vc))
    except npa.Error as e:
        assert got == ("err", type(e).__name__, e.fields)
        return
    padded = [None if s is None else (s + b"\x00" if len(s) & 1 else s) for s in received]
    st, want = oracle.reconstruct(padded, p.n(), p.k())
    if st == 0:
        assert got == ("ok", want)
    else:
        assert got[0] == "err" and got[1] == npa._BY_CODE[st].__name__, (got, st)
