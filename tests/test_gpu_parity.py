"""GPU parity tests: the HIP path (through the C ABI) against the oracle and
the golden fixtures generated from the reference's own C build.  Bit-exact
everywhere (integer arithmetic)."""
import hashlib
import os

import numpy as np
import pytest

import novelpoly_amd as npa
from novelpoly_amd import synth

pytestmark = pytest.mark.gpu


def dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    import torch

    torch.cuda.synchronize()
    return t.cpu().numpy()


def stream():
    import torch

    return torch.cuda.current_stream().cuda_stream


def to_dev_u16(a):
    return dev(np.ascontiguousarray(a, dtype=np.uint16).view(np.int16))


def from_dev_u16(t):
    return host(t).view(np.uint16)


def sha(b):
    return hashlib.sha256(b).hexdigest()


# ------------------------------------------------------------- primitives ----
def test_mul_dev_golden(gpu, golden_vectors):
    import torch

    g = golden_vectors
    a, m = to_dev_u16(g["mul_a"]), to_dev_u16(g["mul_m"])
    out = torch.empty_like(a)
    npa.mul_dev(a.data_ptr(), m.data_ptr(), out.data_ptr(), a.numel(), ctx=gpu, stream=stream())
    assert np.array_equal(from_dev_u16(out), g["mul_out"])


def test_afft_dev_golden(gpu, golden_vectors):
    g = golden_vectors
    for size, index in g["transform_cases"]:
        key = f"s{size}_i{index}"
        for inverse, suffix in ((False, "_afft"), (True, "_ifft")):
            t = to_dev_u16(g[key + "_in"])
            npa.afft_dev(t.data_ptr(), int(size), int(index), 1, inverse=inverse, ctx=gpu, stream=stream())
            assert np.array_equal(from_dev_u16(t), g[key + suffix]), key + suffix


def test_afft_dev_many_columns(gpu, oracle):
    rng = np.random.default_rng(5)
    for size, index, cols in ((64, 128, 37), (256, 0, 70), (1024, 3072, 9)):
        x = rng.integers(0, 65536, (cols, size), dtype=np.uint16)
        t = to_dev_u16(x)
        npa.afft_dev(t.data_ptr(), size, index, cols, inverse=False, ctx=gpu, stream=stream())
        got = from_dev_u16(t)
        for c in range(cols):
            assert np.array_equal(got[c], oracle.afft(x[c], size, index))


def test_walsh_dev_golden(gpu, golden_vectors):
    g = golden_vectors
    for size in (2, 16, 256, 4096):
        t = to_dev_u16(g[f"walsh{size}_in"])
        npa.walsh_dev(t.data_ptr(), size, ctx=gpu, stream=stream())
        assert np.array_equal(from_dev_u16(t), g[f"walsh{size}_out"])


def test_encode_low_and_decode_main_dev_golden(gpu, golden_vectors, oracle):
    import torch

    g = golden_vectors
    for n, k in g["codec_cases"]:
        n, k = int(n), int(k)
        key = f"n{n}_k{k}"
        d = to_dev_u16(g[key + "_data"])
        cw = torch.zeros(n, dtype=torch.int16, device="cuda")
        npa.encode_low_dev(d.data_ptr(), k, cw.data_ptr(), n, 1, ctx=gpu, stream=stream())
        assert np.array_equal(from_dev_u16(cw), g[key + "_codeword"]), key
        pres = dev(g[key + "_present"])
        loc = torch.zeros(n, dtype=torch.int16, device="cuda")
        npa.error_locator_dev(n, pres.data_ptr(), 1, loc.data_ptr(), ctx=gpu, stream=stream())
        assert np.array_equal(from_dev_u16(loc), g[key + "_locator"]), key
        c = g[key + "_codeword"].copy()
        c[g[key + "_present"] == 0] = 0
        ct = to_dev_u16(c)
        npa.decode_main_dev(ct.data_ptr(), k, pres.data_ptr(), loc.data_ptr(), n, 1, ctx=gpu, stream=stream())
        assert np.array_equal(from_dev_u16(ct), g[key + "_decoded"]), key


@pytest.mark.parametrize("n", [2, 16, 256, 1024, 4096, 16384, 32768, 65536])
def test_error_locator_dev_vs_oracle(gpu, oracle, n):
    """np_error_locator_dev (kernels_generic.hip k_error_locator: the two
    65536-point Walsh transforms in registers, three layouts) against the
    oracle's eval_error_polynomial (inc_reconstruct.rs:90-113), including the
    patterns whose zero residues read 65535 (no erasure, every row erased)."""
    import torch

    rng = np.random.default_rng(n)
    pats = [np.ones(n, np.uint8), np.zeros(n, np.uint8)]
    for frac in (0.5, 0.1, 0.9):
        pats.append((rng.random(n) >= frac).astype(np.uint8))
    one = np.ones(n, np.uint8)
    one[n // 2] = 0
    pats.append(one)
    half = np.ones(n, np.uint8)
    half[: n // 2] = 0
    pats.append(half)
    pres = np.stack(pats)
    dpres = dev(pres)
    loc = torch.empty((len(pats), n), dtype=torch.int16, device="cuda")
    npa.error_locator_dev(n, dpres.data_ptr(), len(pats), loc.data_ptr(), ctx=gpu, stream=stream())
    got = host(loc).view(np.uint16)
    for b, p in enumerate(pats):
        want = oracle.eval_error_polynomial(1 - p)[:n]
        assert np.array_equal(got[b], want), (b, np.flatnonzero(got[b] != want)[:5])


# ---------------------------------------------------------- crate surface ----
def test_api_cases_golden(gpu, golden_json):
    for case in golden_json("api_cases.json"):
        nw = case["n_wanted"]
        pl = bytes.fromhex(case["payload"])
        shards = npa.encode(pl, nw, ctx=gpu)
        assert [s.hex() for s in shards] == case["shards"], nw
        keep = set(case["kept"])
        recv = [shards[i] if i in keep else None for i in range(nw)]
        rec = npa.reconstruct(recv, nw, ctx=gpu)
        assert rec.hex() == case["reconstructed"], nw
        assert rec[: len(pl)] == pl


@pytest.mark.parametrize("nw,plen", [(2, 1), (3, 10), (4, 100), (10, 16), (100, 1), (123, 1337), (2003, 17),
                                     (2003, 0), (4, 2), (770, 5120), (1000, 100_000), (65535, 40_000),
                                     (300, 77_777), (33, 3)])
def test_roundtrip_vs_oracle(gpu, oracle, nw, plen):
    # simplicissimus! cases (tests.rs:291-307) and larger shapes
    pl = synth.payload(nw * 7 + plen, plen)
    if plen == 0:
        with pytest.raises(npa.PayloadSizeIsZero):
            npa.encode(pl, nw, ctx=gpu)
        return
    p = npa.CodeParams.derive_parameters(nw, npa.recoverablity_subset_size(nw))
    shards = npa.encode(pl, nw, ctx=gpu)
    st, want = oracle.encode(pl, p.n(), p.k(), nw)
    assert st == 0 and shards == want
    # drop the first half of the redundancy and (if possible) some data shards
    rng = np.random.default_rng(nw + plen)
    ndrop = max(0, min(nw, p.n()) - p.k())
    drop = set(rng.choice(nw, size=min(ndrop, nw - 1 if nw > 1 else 0), replace=False).tolist())
    recv = [None if i in drop else shards[i] for i in range(nw)]
    if sum(s is not None for s in recv) < p.k():
        with pytest.raises(npa.NeedMoreShards):
            npa.reconstruct(recv, nw, ctx=gpu)
        return
    rec = npa.reconstruct(recv, nw, ctx=gpu)
    st, want_rec = oracle.reconstruct(recv, p.n(), p.k())
    assert st == 0 and rec == want_rec
    assert rec[:plen] == pl


def test_reconstruct_inconsistent_input_matches_oracle(gpu, oracle):
    # arbitrary (non-codeword) shards: the decoder must compute the same linear map
    nw = 300
    p = npa.CodeParams.derive_parameters(nw, npa.recoverablity_subset_size(nw))
    rng = np.random.default_rng(11)
    shards = [rng.integers(0, 256, 64, dtype=np.uint8).tobytes() for _ in range(nw)]
    recv = [s if rng.random() < 0.7 else None for s in shards]
    st, want = oracle.reconstruct(recv, p.n(), p.k())
    assert st == 0 and npa.reconstruct(recv, nw, ctx=gpu) == want


def test_errors(gpu):
    shards = npa.encode(bytes(range(100)), 16, ctx=gpu)
    with pytest.raises(npa.NeedMoreShards) as e:
        npa.reconstruct([shards[0]] + [None] * 15, 16, ctx=gpu)
    assert e.value.fields == (1, 4, 16)
    with pytest.raises(npa.EmptyShard):
        npa.reconstruct([b""] * 8 + [None] * 8, 16, ctx=gpu)
    with pytest.raises(npa.InconsistentShardLengths):
        npa.reconstruct([shards[0], shards[1], shards[2][:-2], shards[3]] + [None] * 12, 16, ctx=gpu)
    rs = npa.CodeParams.derive_parameters(16, npa.recoverablity_subset_size(16)).make_encoder(gpu)
    with pytest.raises(npa.NeedMoreShards):
        rs.reconstruct_from_systematic(shards[:1])
    with pytest.raises(npa.PayloadSizeIsZero):
        rs.encode(b"")


def test_reconstruct_from_systematic(gpu):
    # tests.rs:482-497 round_trip_systematic_quickcheck (a few fixed draws)
    for nw, plen in ((2, 5), (100, 1234), (1000, 70_001)):
        rs = npa.CodeParams.derive_parameters(nw, (nw - 1) // 3 + 1).make_encoder(gpu)
        pl = synth.payload(plen, plen)
        chunks = rs.encode(pl)
        assert rs.reconstruct_from_systematic(chunks[: rs.k])[:plen] == pl


def test_round_trip_first_wanted_k(gpu):
    # tests.rs:499-512 round_trip_quickcheck: reconstruct from the first wanted_k shards
    rng = np.random.default_rng(499)
    for _ in range(12):
        nw = int(rng.integers(2, 65536))
        plen = int(rng.integers(2, 200_000))
        wk = (nw - 1) // 3 + 1
        rs = npa.CodeParams.derive_parameters(nw, wk).make_encoder(gpu)
        pl = synth.payload(nw, plen)
        chunks = rs.encode(pl)
        res = rs.reconstruct([c for c in chunks[:wk]])
        assert res[:plen] == pl, (nw, plen)


# ------------------------------------------------- BASELINE-size digests ----
@pytest.mark.parametrize("cid", [1, 2, 3, 4])
def test_config_digests_device_batch(gpu, golden_json, cid):
    import torch

    d = golden_json("digests.json")[f"cfg{cid}"]
    p = npa.CodeParams.derive_parameters(d["n_wanted"], d["k_wanted"])
    n, k, nw = p.n(), p.k(), p.wanted_n
    plen = d["payload_len"]
    pl = np.frombuffer(synth.payload(0, plen), dtype=np.uint8)
    sl = d["shard_len"]
    dp = dev(pl)
    ds = torch.empty(nw * sl, dtype=torch.uint8, device="cuda")
    npa.encode_batch_dev(p, dp.data_ptr(), plen, plen, 1, ds.data_ptr(), nw * sl, ctx=gpu, stream=stream())
    shards = host(ds).tobytes()
    assert sha(shards) == d["encode_sha256"]
    pres = synth.present_mask(0, n, d["erase"])
    out = torch.empty((sl // 2) * 2 * k, dtype=torch.uint8, device="cuda")
    npa.reconstruct_batch_dev(p, ds.data_ptr(), sl, n * sl, pres.tobytes(), 1, out.data_ptr(), out.numel(),
                              ctx=gpu, stream=stream())
    assert sha(host(out).tobytes()) == d["reconstruct_sha256"]


@pytest.mark.parametrize("cid", [2, 3, 4])
def test_full_size_batch_properties(gpu, oracle, cid):
    """At BASELINE shapes, with a batch: per-payload digests against the oracle
    on a sample, and encode->erase->reconstruct round trip on every payload."""
    import torch

    cfg = synth.CONFIGS[cid]
    p = npa.CodeParams.derive_parameters(cfg["n_wanted"], cfg["k_wanted"])
    n, k = p.n(), p.k()
    batch = {2: 64, 3: 16, 4: 4}[cid]
    plen = cfg["payload"]
    pls = np.stack([np.frombuffer(synth.payload(100 + b, plen), dtype=np.uint8) for b in range(batch)])
    sl = p.make_encoder(gpu).shard_len(plen)
    dp = dev(pls)
    ds = torch.empty((batch, n, sl), dtype=torch.uint8, device="cuda")
    npa.encode_batch_dev(p, dp.data_ptr(), plen, plen, batch, ds.data_ptr(), n * sl, ctx=gpu, stream=stream())
    hs = host(ds)
    for b in (0, batch - 1):
        st, want = oracle.encode(pls[b].tobytes(), n, k, n)
        assert st == 0 and hs[b].tobytes() == b"".join(want), b
    erase = cfg["erase"] if cfg["erase"] is not None else n - k
    pres = np.stack([synth.present_mask(100 + b, n, erase) for b in range(batch)])
    # poison erased rows: the kernel must never read them
    ds2 = ds.clone()
    ds2[torch.from_numpy(pres == 0).cuda()] = 0xA5
    out = torch.empty((batch, (sl // 2) * 2 * k), dtype=torch.uint8, device="cuda")
    npa.reconstruct_batch_dev(p, ds2.data_ptr(), sl, n * sl, pres.tobytes(), batch, out.data_ptr(),
                              out.shape[1], ctx=gpu, stream=stream())
    ho = host(out)
    for b in range(batch):
        assert ho[b, :plen].tobytes() == pls[b].tobytes(), b


@pytest.mark.parametrize("batch,plen", [(40, 4 << 20), (33, 2048 * 256 * 9 - 5)])
def test_big_path_launch_rounds(gpu, oracle, batch, plen):
    """k = 1024 (config 4 shape, the resident kernels of kernels_res.hip; with
    NP_RES=0 the scratch kernels of kernels_big.hip, test_host_pipeline_all_
    systematic_switched) over many tiles: 320 tiles with an XCD-major batch and
    297 tiles with a ragged last tile and batch % 8 != 0.  The last payload
    against the oracle; every payload round-trips."""
    import torch

    p = npa.CodeParams.derive_parameters(4096, 1366)
    n, k = p.n(), p.k()
    assert (n, k) == (4096, 1024)
    pls = np.stack([np.frombuffer(synth.payload(300 + b, plen), dtype=np.uint8) for b in range(batch)])
    sl = p.make_encoder(gpu).shard_len(plen)
    dp = dev(pls)
    ds = torch.empty((batch, n, sl), dtype=torch.uint8, device="cuda")
    npa.encode_batch_dev(p, dp.data_ptr(), plen, plen, batch, ds.data_ptr(), n * sl, ctx=gpu, stream=stream())
    hs = host(ds)
    st, want = oracle.encode(pls[-1].tobytes(), n, k, n)
    assert st == 0 and hs[-1].tobytes() == b"".join(want)
    pres = np.stack([synth.present_mask(500 + b, n, 2730) for b in range(batch)])
    out = torch.empty((batch, (sl // 2) * 2 * k), dtype=torch.uint8, device="cuda")
    npa.reconstruct_batch_dev(p, ds.data_ptr(), sl, n * sl, pres.tobytes(), batch, out.data_ptr(),
                              out.shape[1], ctx=gpu, stream=stream())
    ho = host(out)
    bad = [b for b in range(batch) if ho[b, :plen].tobytes() != pls[b].tobytes()]
    assert not bad, bad


@pytest.mark.parametrize("nw,kw,plen", [(256, 86, 128 * 256), (256, 86, 128 * 300 + 5), (256, 86, 1280),
                                        (512, 100, 128 * 700), (1024, 342, 512 * 256), (1024, 342, 5121),
                                        (1024, 342, 512 * 512 + 77), (300, 100, 77777), (512, 128, 256 * 600),
                                        (600, 256, 512 * 300), (2048, 300, 512 * 260),
                                        (4096, 1366, 2048 * 256), (4096, 1366, 2048 * 300 + 3),
                                        (2048, 1024, 2048 * 100), (3000, 1024, 5000),
                                        (1024, 512, 1024 * 100 + 3), (2000, 667, 1024 * 256),
                                        (2000, 667, 1024 * 300 + 5), (2500, 834, 1024 * 256 + 1),
                                        (5000, 1667, 2048 * 64 + 1), (1500, 512, 999),
                                        (7000, 2334, 4096 * 256 + 3), (4096, 2048, 4096 * 40),
                                        (6144, 2048, 4096 * 300 + 1), (9000, 3000, 4096 * 3 + 5)])
def test_fast_encode_shapes(gpu, oracle, nw, kw, plen):
    """Specialised encode kernels (k in {64,128,256}; k in {512,1024,2048} in
    kernels_big.hip): single/multi/partial tiles, odd payload tails, wanted_n < n
    and n/k in {2,4,8}."""
    p = npa.CodeParams.derive_parameters(nw, kw)
    assert p.is_faster8()
    pl = synth.payload(nw + plen, plen)
    got = p.make_encoder(gpu).encode(pl)
    st, want = oracle.encode(pl, p.n(), p.k(), nw)
    assert st == 0
    bad = [v for v in range(nw) if got[v] != want[v]]
    assert not bad, f"{len(bad)} shards differ, first {bad[:5]}"


@pytest.mark.parametrize("nw,kw,plen,erase", [(256, 86, 128 * 256, 170), (256, 86, 128 * 300 + 5, 100),
                                              (128, 64, 128 * 256, 64), (128, 64, 999, 1),
                                              (512, 128, 256 * 300, 300), (256, 128, 256 * 256 + 3, 128),
                                              (1024, 342, 512 * 256, 342), (1024, 342, 512 * 300 + 1, 768),
                                              (512, 256, 512 * 257, 256), (1000, 256, 4097, 0),
                                              (1024, 342, 512 * 256, -1), (4096, 1366, 2048 * 256, 2730),
                                              (4096, 1366, 2048 * 260 + 1, 3072), (2048, 1024, 2048 * 100, 1024),
                                              (4096, 1366, 2048 * 256, -1), (3000, 1024, 7777, 1000),
                                              (300, 100, 128 * 256, 200), (300, 100, 128 * 300 + 7, -1),
                                              (700, 234, 256 * 256 + 1, 500), (1200, 400, 512 * 256, 900),
                                              (1200, 400, 512 * 257, -1), (512, 64, 128 * 64, 448),
                                              (1024, 512, 1024 * 100, 512), (2000, 667, 1024 * 256, 1333),
                                              (2000, 667, 1024 * 257 + 9, -1), (2500, 834, 1024 * 260 + 1, 1666),
                                              (2500, 834, 1024 * 256, -1), (5000, 1667, 2048 * 40 + 3, 3333),
                                              (5000, 1667, 2048 * 33, -1), (2000, 667, 1024 * 256 + 5, 0),
                                              (4096, 1366, 2048 * 256, 0), (7000, 2334, 4096 * 256 + 3, 4666),
                                              (7000, 2334, 4096 * 100, -1), (4096, 2048, 4096 * 40, 2048),
                                              (8192, 2731, 4096 * 257, 5461), (7000, 2334, 4096 * 30, 0),
                                              (9000, 3000, 4096 * 3 + 5, 6000), (12288, 4095, 4096 * 20, 8000),
                                              (10000, 3334, 4096 * 2, -1), (9000, 3000, 4096 * 2 + 1, 0)])
def test_fast_reconstruct_shapes(gpu, oracle, nw, kw, plen, erase):
    """Specialised reconstruct kernels (k in {64,128,256} fast, {512,1024,2048}
    big with n in {2k,4k,8k}; 8,193-12,288 validators: n = 16384, k = 2048): full
    and partial column tiles, random and worst-case erasure sets (erase = -1:
    every systematic shard lost), bit-exact against the oracle."""
    p = npa.CodeParams.derive_parameters(nw, kw)
    n, k = p.n(), p.k()
    assert n in (2 * k, 4 * k, 8 * k) and k in (64, 128, 256, 512, 1024, 2048)
    pl = synth.payload(7 * nw + plen, plen)
    shards = p.make_encoder(gpu).encode(pl)
    if erase == -1:
        gone = set(range(k))
    else:
        gone = set(synth.erasure_indices(plen + erase, n, min(erase, n - k)).tolist())
    recv = [None if i in gone else s for i, s in enumerate(shards[:nw])]
    assert sum(r is not None for r in recv) >= k
    got = p.make_encoder(gpu).reconstruct(recv)
    st, want = oracle.reconstruct(recv, n, k)
    assert st == 0 and got == want
    assert got[:plen] == pl


# k in {8, 16, 32} (kernels_small.hip): validator counts 16..190, n / k in
# {2, 4, 8}, wanted_n < n (last shift partly kept), full / partial / tail tiles
SMALL_ENC = [(100, 34, 64 * 256), (100, 34, 64 * 300 + 5), (150, 50, 64 * 512), (190, 63, 64 * 257 + 1),
             (64, 32, 64 * 256), (60, 20, 32 * 256), (90, 30, 32 * 257 + 3), (40, 14, 16 * 256),
             (16, 8, 4096), (30, 10, 999), (24, 8, 16 * 768), (48, 16, 1), (33, 11, 16 * 256 * 5 + 9),
             # k in {1, 2, 4}: 2 to 21 validators
             (2, 1, 1000), (3, 1, 999), (4, 2, 4096), (7, 3, 5003), (9, 3, 4 * 256 * 3 + 2), (10, 4, 8 * 256 * 3),
             (16, 6, 8 * 300 + 5), (20, 7, 65536 + 3), (13, 5, 12345), (21, 7, 1), (5, 2, 2)]


@pytest.mark.parametrize("nw,kw,plen", SMALL_ENC)
def test_small_encode_shapes(gpu, oracle, nw, kw, plen):
    """Register-only encode kernels for k in {1, 2, 4, 8, 16, 32}, bit-exact
    against the oracle."""
    p = npa.CodeParams.derive_parameters(nw, kw)
    assert p.k() in (1, 2, 4, 8, 16, 32) and p.is_faster8()
    pl = synth.payload(nw + plen, plen)
    got = p.make_encoder(gpu).encode(pl)
    st, want = oracle.encode(pl, p.n(), p.k(), nw)
    assert st == 0
    bad = [v for v in range(nw) if got[v] != want[v]]
    assert not bad, f"{len(bad)} shards differ, first {bad[:5]}"


@pytest.mark.parametrize("nw,kw,plen,erase", [(100, 34, 64 * 256, 66), (100, 34, 64 * 300 + 5, 40),
                                              (100, 34, 64 * 256, -1), (150, 50, 64 * 512, 100),
                                              (190, 63, 64 * 257 + 1, 120), (190, 63, 64 * 256, -1),
                                              (64, 32, 64 * 256, 32), (64, 32, 64 * 99, -1),
                                              (60, 20, 32 * 256, 40), (90, 30, 32 * 257 + 3, 60),
                                              (40, 14, 16 * 256, 26), (40, 14, 16 * 300 + 1, -1),
                                              (16, 8, 4096, 8), (16, 8, 4096, -1), (30, 10, 999, 20),
                                              (24, 8, 16 * 768, 16), (100, 34, 64 * 256, 0),
                                              (2, 1, 1000, 1), (3, 1, 999, 2), (4, 2, 4096, 2), (7, 3, 5003, 5),
                                              (9, 3, 4 * 256 * 3 + 2, 7), (10, 4, 8 * 256 * 3, 6),
                                              (10, 4, 8 * 256 * 3, -1), (16, 6, 8 * 300 + 5, 12),
                                              (20, 7, 65536 + 3, 16), (20, 7, 65536, -1), (13, 5, 12345, 0),
                                              (4, 2, 77, -1)])
def test_small_reconstruct_shapes(gpu, oracle, nw, kw, plen, erase):
    """Register-only reconstruct kernels for k in {8, 16, 32}, n in {2k, 4k,
    8k}: random and worst-case erasure sets (-1: every systematic shard lost),
    bit-exact against the oracle."""
    p = npa.CodeParams.derive_parameters(nw, kw)
    n, k = p.n(), p.k()
    assert k in (1, 2, 4, 8, 16, 32) and n in (2 * k, 4 * k, 8 * k)
    pl = synth.payload(7 * nw + plen, plen)
    shards = p.make_encoder(gpu).encode(pl)
    if erase == -1:
        gone = set(range(k))
    else:
        gone = set(synth.erasure_indices(plen + erase, nw, min(erase, nw - k)).tolist())
    recv = [None if i in gone else s for i, s in enumerate(shards[:nw])]
    assert sum(r is not None for r in recv) >= k
    got = p.make_encoder(gpu).reconstruct(recv)
    st, want = oracle.reconstruct(recv, n, k)
    assert st == 0 and got == want
    assert got[:plen] == pl


@pytest.mark.parametrize("nw,kw,plen,batch", [(1024, 342, 512 * 300, 5), (256, 86, 128 * 256 + 7, 9),
                                              (512, 256, 512 * 256, 3), (2048, 512, 1024 * 40, 2),
                                              (300, 100, 128 * 300, 4), (1200, 400, 512 * 260, 3),
                                              (100, 34, 64 * 300, 4), (60, 20, 32 * 256 + 1, 3)])
def test_device_reconstruct_locator_modes(gpu, oracle, nw, kw, plen, batch):
    """np_reconstruct_batch_dev2 with locators from np_error_locator_dev and with
    d_locators = NULL (computed on the device: fused folded locator on the fast
    path) give the oracle's bytes."""
    import torch

    p = npa.CodeParams.derive_parameters(nw, kw)
    n, k = p.n(), p.k()
    sl = p.make_encoder(gpu).shard_len(plen)
    pls = np.stack([np.frombuffer(synth.payload(900 + b, plen), dtype=np.uint8) for b in range(batch)])
    dp = dev(pls)
    ds = torch.empty((batch, n, sl), dtype=torch.uint8, device="cuda")
    npa.encode_batch_dev(p, dp.data_ptr(), plen, plen, batch, ds.data_ptr(), n * sl, ctx=gpu, stream=stream())
    wn = p.wanted_n  # rows >= wanted_n were never encoded: absent
    pres = np.zeros((batch, n), np.uint8)
    for b in range(batch):
        pres[b, :wn] = synth.present_mask(900 + b, wn, (wn - k) if b % 2 else (wn - k) // 3)
    dpres = dev(pres)
    loc = torch.empty((batch, n), dtype=torch.int16, device="cuda")
    npa.error_locator_dev(n, dpres.data_ptr(), batch, loc.data_ptr(), ctx=gpu, stream=stream())
    olen = (sl // 2) * 2 * k
    outs = []
    for lp in (loc.data_ptr(), 0):
        out = torch.empty((batch, olen), dtype=torch.uint8, device="cuda")
        npa.reconstruct_batch_dev2(p, ds.data_ptr(), sl, n * sl, dpres.data_ptr(), lp, batch, out.data_ptr(), olen,
                                   ctx=gpu, stream=stream())
        outs.append(host(out))
    hs = host(ds)
    for b in range(batch):
        recv = [hs[b, i].tobytes() if pres[b, i] else None for i in range(n)]
        st, want = oracle.reconstruct(recv, n, k)
        assert st == 0
        for o in outs:
            assert o[b].tobytes() == want, b
        assert want[:plen] == pls[b].tobytes()


def _prefix_patterns(n, k, rng):
    """Erasure patterns that steer the fused-locator reconstruct kernel into each
    prefix mode: all systematic rows present (decode = copy), at least k present
    rows in [0, 2k) (2k-row prefix), exactly k there (boundary), fewer (full n)."""
    pats = []
    pres = np.ones(n, np.uint8)
    pres[k + rng.choice(n - k, (n - k) // 2, replace=False)] = 0
    pats.append(pres)
    if n >= 2 * k:
        pres = np.ones(n, np.uint8)
        pres[rng.choice(k, k // 3, replace=False)] = 0
        if n > 2 * k:
            pres[2 * k + rng.choice(n - 2 * k, (n - 2 * k) // 2, replace=False)] = 0
        pats.append(pres)
        pres = np.ones(n, np.uint8)
        pres[rng.choice(2 * k, k, replace=False)] = 0  # exactly k present in the prefix
        pats.append(pres)
    if n > 2 * k:
        pres = np.ones(n, np.uint8)
        pres[rng.choice(2 * k, k + 1, replace=False)] = 0  # k - 1 present in the prefix
        pres[2 * k + rng.choice(n - 2 * k, n - 2 * k - 2, replace=False)] = 0  # k + 1 present overall
        pats.append(pres)
    return pats


@pytest.mark.parametrize("nw,kw,plen", [(1024, 342, 512 * 256), (1024, 342, 512 * 37 + 3), (256, 86, 128 * 256),
                                        (512, 256, 512 * 256), (256, 128, 256 * 99), (128, 34, 64 * 256),
                                        (64, 14, 16 * 300 + 3), (64, 32, 64 * 257)])
def test_reconstruct_prefix_modes(gpu, oracle, nw, kw, plen):
    """Fast reconstruct with the locator computed in the kernel picks the shortest
    row prefix (k, 2k or n rows) that holds k present rows; every mode gives the
    oracle's bytes.  Mixed modes in one batch."""
    import torch

    p = npa.CodeParams.derive_parameters(nw, kw)
    n, k = p.n(), p.k()
    rng = np.random.default_rng(nw * 7 + plen)
    pats = _prefix_patterns(n, k, rng)
    batch = len(pats) * 2
    sl = p.make_encoder(gpu).shard_len(plen)
    pls = np.stack([np.frombuffer(synth.payload(4000 + b, plen), dtype=np.uint8) for b in range(batch)])
    dp = dev(pls)
    ds = torch.empty((batch, n, sl), dtype=torch.uint8, device="cuda")
    npa.encode_batch_dev(p, dp.data_ptr(), plen, plen, batch, ds.data_ptr(), n * sl, ctx=gpu, stream=stream())
    pres = np.stack([pats[b % len(pats)] for b in range(batch)])
    dpres = dev(pres)
    olen = (sl // 2) * 2 * k
    out = torch.empty((batch, olen), dtype=torch.uint8, device="cuda")
    npa.reconstruct_batch_dev2(p, ds.data_ptr(), sl, n * sl, dpres.data_ptr(), 0, batch, out.data_ptr(), olen,
                               ctx=gpu, stream=stream())
    o = host(out)
    hs = host(ds)
    for b in range(batch):
        recv = [hs[b, i].tobytes() if pres[b, i] else None for i in range(n)]
        st, want = oracle.reconstruct(recv, n, k)
        assert st == 0
        assert o[b].tobytes() == want, (b, b % len(pats))
        assert want[:plen] == pls[b].tobytes()


@pytest.mark.parametrize("nw,kw,plen", [(300, 100, 64 * 256), (300, 100, 64 * 37 + 5), (700, 234, 128 * 256 + 3),
                                        (1200, 400, 256 * 257), (512, 64, 64 * 64), (2500, 834, 512 * 100 + 1),
                                        (5000, 1667, 1024 * 64 + 3), (10000, 3334, 2048 * 9 + 1),
                                        (2000, 667, 1024 * 33)])
def test_reconstruct_empty_segments(gpu, oracle, nw, kw, plen):
    """Reconstruct skips the transforms of row blocks without a present row:
    n = 8k fast path, k-row segments (record byte 1, kernels_fast.hip
    segment_occupancy); k >= 512, 256-row sub-segments (kernels_big.hip
    k_big_records occupancy) and whole segments in the fold.  Whole segments
    erased inside wanted_n (alone, several, all but one), single 256-row blocks
    and the blocks past wanted_n, with caller locators and with the fused
    locator, give the oracle's bytes."""
    import torch

    p = npa.CodeParams.derive_parameters(nw, kw)
    n, k, wn = p.n(), p.k(), p.wanted_n
    assert n in (4 * k, 8 * k) or k >= 512
    nseg = (wn + k - 1) // k
    rng = np.random.default_rng(nw + plen)
    blocks = [[(q * k, (q + 1) * k) for q in gone]
              for gone in ([1], [0, 2], [0] + list(range(2, nseg)), list(range(1, nseg)), [nseg - 1], [])]
    if k >= 512:
        blocks += [[(256, 512)], [(0, 256), (k + 512, k + 768)], [(k - 256, k), (2 * k, 2 * k + 256)]]
    pats = []
    for bl in blocks:
        pres = np.zeros(n, np.uint8)
        pres[:wn] = 1
        for r0, r1 in bl:
            pres[r0:r1] = 0
        if pres.sum() > k + 8:  # a few random erasures in what is left
            idx = np.flatnonzero(pres)
            pres[rng.choice(idx, min(len(idx) - k, 5), replace=False)] = 0
        if pres.sum() >= k:
            pats.append(pres)
    batch = len(pats)
    sl = p.make_encoder(gpu).shard_len(plen)
    pls = np.stack([np.frombuffer(synth.payload(5000 + b, plen), dtype=np.uint8) for b in range(batch)])
    dp = dev(pls)
    ds = torch.empty((batch, n, sl), dtype=torch.uint8, device="cuda")
    npa.encode_batch_dev(p, dp.data_ptr(), plen, plen, batch, ds.data_ptr(), n * sl, ctx=gpu, stream=stream())
    pres = np.stack(pats)
    dpres = dev(pres)
    loc = torch.empty((batch, n), dtype=torch.int16, device="cuda")
    npa.error_locator_dev(n, dpres.data_ptr(), batch, loc.data_ptr(), ctx=gpu, stream=stream())
    olen = (sl // 2) * 2 * k
    hs = host(ds)
    for lp in (loc.data_ptr(), 0):
        out = torch.empty((batch, olen), dtype=torch.uint8, device="cuda")
        npa.reconstruct_batch_dev2(p, ds.data_ptr(), sl, n * sl, dpres.data_ptr(), lp, batch, out.data_ptr(), olen,
                                   ctx=gpu, stream=stream())
        o = host(out)
        for b in range(batch):
            recv = [hs[b, i].tobytes() if pres[b, i] else None for i in range(n)]
            st, want = oracle.reconstruct(recv, n, k)
            assert st == 0
            assert o[b].tobytes() == want, (b, bool(lp))
            assert want[:plen] == pls[b].tobytes()


@pytest.mark.parametrize("nw,tpw,batch,stride_pad", [(1024, 2, 8, 0), (1024, 3, 8, 0), (1024, 4, 5, 0),
                                                     (700, 4, 8, 0), (1024, 4, 8, 1), (2048, 3, 3, 0)])
def test_encode_multi_tile_workgroups(gpu, oracle, monkeypatch, nw, tpw, batch, stride_pad):
    """k = 256: one workgroup encodes `tpw` consecutive tiles of a payload and
    the next tile's payload arrives by LDS-DMA during the last shift
    (kernels_fast.hip k_encode_multi; NP_ENC_TPW pins the tile count).  771
    chunks = 3 full tiles and a partial one (loaded without DMA); wanted_n < n
    ends on an earlier shift; an odd payload stride takes the byte path; n = 8k
    runs shifts past the shared top-level products."""
    import torch

    monkeypatch.setenv("NP_ENC_TPW", str(tpw))
    p = npa.CodeParams.derive_parameters(nw, 342)
    n, k = p.n(), p.k()
    assert k == 256
    plen = 512 * (3 * 256 + 3) - 5
    stride = plen + stride_pad
    sl = p.make_encoder(gpu).shard_len(plen)
    pls = np.zeros((batch, stride), np.uint8)
    for b in range(batch):
        pls[b, :plen] = np.frombuffer(synth.payload(9000 + b, plen), dtype=np.uint8)
    dp = dev(pls)
    ds = torch.zeros((batch, n, sl), dtype=torch.uint8, device="cuda")
    npa.encode_batch_dev(p, dp.data_ptr(), plen, stride, batch, ds.data_ptr(), n * sl, ctx=gpu, stream=stream())
    hs = host(ds)
    for b in range(batch):
        st, want = oracle.encode(pls[b, :plen].tobytes(), n, k, nw)
        assert st == 0
        bad = [v for v in range(nw) if hs[b, v].tobytes() != want[v]]
        assert not bad, (b, len(bad), bad[:5])


@pytest.mark.parametrize("nw,kw,tpw,batch", [(256, 86, 2, 5), (256, 86, 4, 3), (300, 100, 3, 4), (512, 128, 2, 6),
                                              (700, 234, 4, 3)])
def test_reconstruct_multi_tile_workgroups_small_k(gpu, oracle, monkeypatch, nw, kw, tpw, batch):
    """k = 64 / 128 (4 and 8 segments) over several tiles per payload with a
    tile-count pin in the environment (one tile per workgroup there: kernels_fast.hip
    kMultiTile; round 4 measured multi-tile workgroups slower at these k).
    771 columns = 3 full tiles and one of 3 columns; random erasures, one
    payload with every systematic row present (copy mode), one with a single
    extra row."""
    import torch

    monkeypatch.setenv("NP_REC_TPW", str(tpw))
    p = npa.CodeParams.derive_parameters(nw, kw)
    n, k = p.n(), p.k()
    assert k in (64, 128)
    plen = 2 * k * (3 * 256 + 3) - 5
    sl = p.make_encoder(gpu).shard_len(plen)
    assert sl // 2 == 771
    pls = np.stack([np.frombuffer(synth.payload(7100 + b, plen), dtype=np.uint8) for b in range(batch)])
    dp = dev(pls)
    ds = torch.empty((batch, n, sl), dtype=torch.uint8, device="cuda")
    npa.encode_batch_dev(p, dp.data_ptr(), plen, plen, batch, ds.data_ptr(), n * sl, ctx=gpu, stream=stream())
    rng = np.random.default_rng(nw * 7 + tpw)
    wn = p.wanted_n  # rows >= wanted_n are never produced: absent
    pres = np.zeros((batch, n), dtype=np.uint8)
    pres[:, :wn] = 1
    for b in range(batch):
        lo = k if b == 1 else 0  # payload 1 keeps every systematic row
        pres[b, lo + rng.choice(wn - lo, wn - k - (1 if b == 2 else 0) - (wn - k) // 3, replace=False)] = 0
    dpres = dev(pres)
    olen = (sl // 2) * 2 * k
    out = torch.empty((batch, olen), dtype=torch.uint8, device="cuda")
    npa.reconstruct_batch_dev2(p, ds.data_ptr(), sl, n * sl, dpres.data_ptr(), 0, batch, out.data_ptr(), olen,
                               ctx=gpu, stream=stream())
    o = host(out)
    hs = host(ds)
    for b in range(batch):
        recv = [hs[b, i].tobytes() if pres[b, i] else None for i in range(n)]
        st, want = oracle.reconstruct(recv, n, k)
        assert st == 0 and o[b].tobytes() == want, b
        assert want[:plen] == pls[b].tobytes()


@pytest.mark.parametrize("tpw,batch", [(2, 8), (3, 8), (4, 5), (8, 8)])
def test_reconstruct_multi_tile_workgroups(gpu, oracle, monkeypatch, tpw, batch):
    """k = 256: one workgroup decodes `tpw` consecutive 256-column tiles of a
    payload (kernels_fast.hip rec_tiles; NP_REC_TPW pins the count the launcher
    derives from the batch size).  771 symbol columns = 3 full tiles and one of
    3 columns, so workgroups end on partial tiles and on tile counts that tpw
    does not divide; every prefix mode, XCD-major and plain workgroup order."""
    import torch

    monkeypatch.setenv("NP_REC_TPW", str(tpw))
    p = npa.CodeParams.derive_parameters(1024, 342)
    n, k = p.n(), p.k()
    plen = 512 * (3 * 256 + 3) - 5
    rng = np.random.default_rng(tpw * 31 + batch)
    pats = _prefix_patterns(n, k, rng)
    sl = p.make_encoder(gpu).shard_len(plen)
    assert sl // 2 == 771
    pls = np.stack([np.frombuffer(synth.payload(7000 + b, plen), dtype=np.uint8) for b in range(batch)])
    dp = dev(pls)
    ds = torch.empty((batch, n, sl), dtype=torch.uint8, device="cuda")
    npa.encode_batch_dev(p, dp.data_ptr(), plen, plen, batch, ds.data_ptr(), n * sl, ctx=gpu, stream=stream())
    pres = np.stack([pats[b % len(pats)] for b in range(batch)])
    dpres = dev(pres)
    olen = (sl // 2) * 2 * k
    out = torch.empty((batch, olen), dtype=torch.uint8, device="cuda")
    npa.reconstruct_batch_dev2(p, ds.data_ptr(), sl, n * sl, dpres.data_ptr(), 0, batch, out.data_ptr(), olen,
                               ctx=gpu, stream=stream())
    o = host(out)
    hs = host(ds)
    for b in range(batch):
        recv = [hs[b, i].tobytes() if pres[b, i] else None for i in range(n)]
        st, want = oracle.reconstruct(recv, n, k)
        assert st == 0
        assert o[b].tobytes() == want, (b, b % len(pats))
        assert want[:plen] == pls[b].tobytes()


@pytest.mark.parametrize("nw,kw,plen,batch", [(1024, 342, 512 * 300 + 7, 3), (16, 8, 4096, 2), (256, 86, 99, 5),
                                              (4096, 1366, 2048 * 70, 2), (2, 1, 3, 4), (300, 100, 64 * 129, 2)])
def test_reconstruct_from_systematic_batch_dev(gpu, oracle, nw, kw, plen, batch):
    """Device batch reconstruct_from_systematic (mod.rs:247-285): the column
    gather of the first k shards equals the oracle's, payload by payload, for
    k below, at and above the 64 x 64 tile."""
    import torch

    p = npa.CodeParams.derive_parameters(nw, kw)
    n, k = p.n(), p.k()
    sl = p.make_encoder(gpu).shard_len(plen)
    pls = np.stack([np.frombuffer(synth.payload(7000 + b, plen), dtype=np.uint8) for b in range(batch)])
    dp = dev(pls)
    ds = torch.empty((batch, n, sl), dtype=torch.uint8, device="cuda")
    npa.encode_batch_dev(p, dp.data_ptr(), plen, plen, batch, ds.data_ptr(), n * sl, ctx=gpu, stream=stream())
    olen = (sl // 2) * 2 * k
    out = torch.empty((batch, olen), dtype=torch.uint8, device="cuda")
    npa.reconstruct_from_systematic_batch_dev(p, ds.data_ptr(), sl, n * sl, batch, out.data_ptr(), olen, ctx=gpu,
                                              stream=stream())
    o, hs = host(out), host(ds)
    for b in range(batch):
        st, want = oracle.reconstruct_from_systematic([hs[b, i].tobytes() for i in range(k)], n, k)
        assert st == 0 and o[b].tobytes() == want
        assert want[:plen] == pls[b].tobytes()


def _host_array(shape, fill, pinned, offset=0):
    """A host array, pageable (numpy) or pinned (torch.pin_memory: mapped into
    the device address space, so np_reconstruct_batch_host gathers its present
    rows with a kernel), starting `offset` bytes into its allocation."""
    if not pinned:
        return np.full(shape, fill, dtype=np.uint8)
    import torch
    size = int(np.prod(shape))
    t = torch.full((size + offset,), fill, dtype=torch.uint8).pin_memory()
    return t.numpy()[offset:].reshape(shape)  # the view's base keeps the pinned tensor alive


@pytest.mark.parametrize("pinned,mode", [pytest.param(False, "pin", marks=pytest.mark.pin_in_place), (False, "stage"),
                                        (True, "stage"), (True, "gather")],
                         ids=["pageable-pin", "pageable", "pinned", "pinned-gather"])
@pytest.mark.parametrize("nw,kw,plen,batch,offset", [(1024, 342, 512 * 256, 9, 0), (256, 86, 128 * 99 + 1, 7, 0),
                                                     (300, 100, 5000, 3, 2), (4096, 1366, 2048 * 40, 2, 0),
                                                     (1024, 342, 512 * 256, 3, 6)])
def test_host_batch_pipeline(gpu, oracle, nw, kw, plen, batch, offset, pinned, mode, monkeypatch):
    """np_encode_batch_host / np_reconstruct_batch_host (host buffers, pipelined
    sub-batches over several streams) give the oracle's shards and payloads;
    strided host layouts, unaligned starts, pinned host memory (present rows
    gathered over PCIe by a kernel) and garbage in the absent rows included.
    Pageable buffers go through host-thread staging (the default) or, with
    NP_PAGEABLE=pin, pinned in place for the call (engine.cpp reads the
    variable per call; those cases run in a child process).  Pinned present
    rows are packed by host threads and DMA'd (the default), or with
    NP_HOST_ROWS=gather read by the k_copy_rows kernel (4-byte aligned rows;
    the unaligned start takes the 2-D DMA)."""
    if mode == "gather":
        monkeypatch.setenv("NP_HOST_ROWS", "gather")
        mode = "stage"
    monkeypatch.setenv("NP_PAGEABLE", mode)
    p = npa.CodeParams.derive_parameters(nw, kw)
    n, k = p.n(), p.k()
    sl = p.make_encoder(gpu).shard_len(plen)
    pstride = plen + 3
    pay = np.zeros((batch, pstride), dtype=np.uint8)
    for b in range(batch):
        pay[b, :plen] = np.frombuffer(synth.payload(9100 + b, plen), dtype=np.uint8)
    wn = p.wanted_n
    bstride = n * sl + 64
    sh = _host_array((batch, bstride), 0xAB, pinned, offset)
    npa.encode_batch_host(p, pay.ctypes.data, plen, pstride, batch, sh.ctypes.data, bstride, ctx=gpu)
    for b in range(batch):
        st, want = oracle.encode(pay[b, :plen].tobytes(), n, k, wn)
        assert st == 0
        got = [sh[b, i * sl:(i + 1) * sl].tobytes() for i in range(wn)]
        assert got == want, b
    assert (sh[:, wn * sl:] == 0xAB).all()  # nothing written past wanted_n rows
    rng = np.random.default_rng(plen)
    pres = np.zeros((batch, n), dtype=np.uint8)
    for b in range(batch):  # erasures among the wanted_n rows that exist
        pres[b, :wn] = 1
        gone = (wn - k) if b % 2 else (wn - k) // 3
        pres[b, rng.choice(wn, gone, replace=False)] = 0
    recvs = [[sh[b, i * sl:(i + 1) * sl].tobytes() if pres[b, i] else None for i in range(n)] for b in range(batch)]
    for b in range(batch):  # the engine must not read absent rows
        for i in np.flatnonzero(pres[b] == 0):
            sh[b, i * sl:(i + 1) * sl] = 0x5C
    olen = (sl // 2) * 2 * k
    ostride = olen + 5
    out = _host_array((batch, ostride), 0, pinned)
    npa.reconstruct_batch_host(p, sh.ctypes.data, sl, bstride, pres.ctypes.data, batch, out.ctypes.data, ostride,
                               ctx=gpu)
    for b in range(batch):
        recv = recvs[b]
        st, want = oracle.reconstruct(recv, n, k)
        assert st == 0 and out[b, :olen].tobytes() == want, b
        assert want[:plen] == pay[b, :plen].tobytes()


# Every systematic row present: the host pipeline ships only the k systematic
# rows when the kernel family it dispatches to has a copy mode (engine.cpp
# rec_path / rows_needed).  k = 4096 (n = 16384) and 8192 (n = 32768) on the
# sub-transform kernels, k = 1024 (n = 4096) and k = 256 (config 3).
_SYS_CASES = [(12289, 4097, 2 * 4096 * 9, 3), (20000, 6667, 2 * 8192 * 5, 2), (4096, 1366, 2048 * 40, 2),
              (1024, 342, 512 * 100, 3)]


@pytest.mark.parametrize("pinned", [False, True], ids=["pageable", "pinned"])
@pytest.mark.parametrize("nw,kw,plen,batch", _SYS_CASES)
def test_host_pipeline_all_systematic(gpu, oracle, nw, kw, plen, batch, pinned):
    import _pipeline_case

    _pipeline_case.run(gpu, oracle, nw, kw, plen, batch, pinned)


@pytest.mark.parametrize("env,nw,kw,plen", [("NP_HUGE=0", 12289, 4097, 2 * 4096 * 9),
                                            ("NP_RES=0", 4096, 1366, 2048 * 40),
                                            ("NP_HUGE=1", 6144, 2049, 2 * 2048 * 300)])
def test_host_pipeline_all_systematic_switched(gpu, env, nw, kw, plen):
    """The same with a kernel-family switch (read once per process, so in a
    child process): NP_HUGE=0 sends k = 4096 to the generic kernels, which have
    no copy mode and read all n rows -- the pipeline must then ship all of them
    (it shipped k rows and the decode read past the slot)."""
    import subprocess
    import sys

    key, val = env.split("=")
    e = dict(os.environ, **{key: val})
    script = os.path.join(os.path.dirname(__file__), "_pipeline_case.py")
    for pinned in (0, 1):
        r = subprocess.run([sys.executable, script, str(nw), str(kw), str(plen), "2", str(pinned)], env=e,
                           capture_output=True, text=True, timeout=100)
        assert r.returncode == 0 and r.stdout.strip().endswith("ok"), (env, pinned, r.stdout[-2000:], r.stderr[-2000:])


# Explicit parameters with n / k >= 16 (CodeParams::derive_parameters accepts
# any k >= 1, mod.rs:43-61; encode(bytes, n) never derives them): the encode
# runs the specialised kernels (k = 256: kernels_fast.hip; k = 512 / 1024:
# kernels_big.hip, their only route there), the reconstruct the generic kernels.
@pytest.mark.parametrize("nw,kw,plen,erase", [(4096, 256, 512 * 40 + 3, 3000), (8192, 512, 1024 * 9 + 1, 7000),
                                              (16384, 512, 1024 * 5, 15000), (16384, 1024, 2048 * 5 + 7, 14000),
                                              (32768, 1024, 2048 * 3, 30000), (8192, 512, 1024 * 4, -1)])
def test_explicit_wide_codes(gpu, oracle, nw, kw, plen, erase):
    p = npa.CodeParams.derive_parameters(nw, kw)
    n, k = p.n(), p.k()
    assert n // k >= 16 and (n, k) == (nw, kw)
    pl = synth.payload(nw + kw + plen, plen)
    shards = p.make_encoder(gpu).encode(pl)
    st, want = oracle.encode(pl, n, k, nw)
    assert st == 0
    bad = [v for v in range(nw) if shards[v] != want[v]]
    assert not bad, f"{len(bad)} shards differ, first {bad[:5]}"
    gone = set(range(k)) if erase == -1 else set(synth.erasure_indices(plen + erase, n, erase).tolist())
    recv = [None if i in gone else s for i, s in enumerate(shards)]
    got = p.make_encoder(gpu).reconstruct(recv)
    st, want = oracle.reconstruct(recv, n, k)
    assert st == 0 and got == want
    assert got[:plen] == pl


@pytest.mark.parametrize("nw,kw,plen,batch", [(1024, 342, 512 * 771 - 5, 6), (1024, 342, 512 * 64, 4),
                                              (512, 256, 512 * 771 - 5, 4), (1200, 400, 512 * 131 + 9, 5),
                                              (2048, 256, 512 * 200, 4)])
def test_reconstruct_res256(gpu, oracle, monkeypatch, nw, kw, plen, batch):
    """k = 256 on the resident kernels (NP_REC_RES256=1, kernels_res.hip
    kResNoHD: a 64-column tile, four workgroups per CU -- the decode A/B of
    DESIGN.md §8) against the oracle: n = 2k, 4k and 8k (wanted_n < n: empty
    segments), every prefix mode, 771 columns = 12 full tiles and one of 3."""
    import torch

    monkeypatch.setenv("NP_REC_RES256", "1")
    p = npa.CodeParams.derive_parameters(nw, kw)
    n, k = p.n(), p.k()
    assert k == 256
    rng = np.random.default_rng(nw + plen)
    sl = p.make_encoder(gpu).shard_len(plen)
    pls = np.stack([np.frombuffer(synth.payload(7300 + b, plen), dtype=np.uint8) for b in range(batch)])
    dp = dev(pls)
    ds = torch.empty((batch, n, sl), dtype=torch.uint8, device="cuda")
    npa.encode_batch_dev(p, dp.data_ptr(), plen, plen, batch, ds.data_ptr(), n * sl, ctx=gpu, stream=stream())
    wn = p.wanted_n
    pats = [pt for pt in _prefix_patterns(n, k, rng) if pt[:wn].sum() >= k]
    for _ in range(2):  # random erasures inside wanted_n
        pt = np.zeros(n, np.uint8)
        pt[rng.choice(wn, k + int(rng.integers(0, wn - k + 1)), replace=False)] = 1
        pats.append(pt)
    pres = np.stack([pats[b % len(pats)] for b in range(batch)])
    pres[:, wn:] = 0  # rows >= wanted_n are never produced
    for b in range(batch):
        if pres[b].sum() < k:
            pres[b, rng.choice(np.flatnonzero(pres[b, :wn] == 0), k - int(pres[b].sum()), replace=False)] = 1
    dpres = dev(pres)
    olen = (sl // 2) * 2 * k
    out = torch.empty((batch, olen), dtype=torch.uint8, device="cuda")
    npa.reconstruct_batch_dev2(p, ds.data_ptr(), sl, n * sl, dpres.data_ptr(), 0, batch, out.data_ptr(), olen,
                               ctx=gpu, stream=stream())
    o = host(out)
    hs = host(ds)
    for b in range(batch):
        recv = [hs[b, i].tobytes() if pres[b, i] else None for i in range(n)]
        st, want = oracle.reconstruct(recv, n, k)
        assert st == 0
        assert o[b].tobytes() == want, b
        assert want[:plen] == pls[b].tobytes()
