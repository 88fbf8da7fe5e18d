"""Multi-device batch entry points (np_*_batch_multi, np_*_batch_host_multi):
the batch split into contiguous ranges, one context and host thread per range.
The test box has one GPU, so the "devices" are several contexts on device 0
(distinct streams, scratch and threads -- the same code path as distinct
GPUs); every payload is checked against the oracle."""
import numpy as np
import pytest

import novelpoly_amd as npa
from novelpoly_amd import synth

pytestmark = pytest.mark.gpu


def _dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("nw,kw,plen,batch,nctx", [(1024, 342, 512 * 300 + 5, 7, 2), (256, 86, 128 * 99, 9, 3),
                                                   (300, 100, 5000, 5, 2)])
def test_device_batch_multi(gpu, oracle, nw, kw, plen, batch, nctx):
    import torch

    ctxs = [npa.Context(0) for _ in range(nctx)]
    p = npa.CodeParams.derive_parameters(nw, kw)
    n, k = p.n(), p.k()
    sl = p.make_encoder(gpu).shard_len(plen)
    olen = (sl // 2) * 2 * k
    pls = np.stack([np.frombuffer(synth.payload(500 + b, plen), np.uint8) for b in range(batch)])
    pres = np.stack([synth.present_mask(500 + b, n, (n - k) // 2) for b in range(batch)])
    rng = np.random.default_rng(batch)
    ranges = [npa.batch_split(batch, nctx, i) for i in range(nctx)]
    d_pay = [_dev(pls[b0:b0 + c]) for b0, c in ranges]
    d_sh = [torch.zeros((c, n, sl), dtype=torch.uint8, device="cuda") for _, c in ranges]
    torch.cuda.synchronize()
    npa.encode_batch_multi(ctxs, p, [t.data_ptr() for t in d_pay], plen, plen, batch, [t.data_ptr() for t in d_sh],
                           n * sl)
    shards = np.concatenate([t.cpu().numpy() for t in d_sh])
    for b in range(batch):
        st, want = oracle.encode(pls[b].tobytes(), n, k, p.wanted_n)
        assert st == 0 and [shards[b, i].tobytes() for i in range(p.wanted_n)] == want, b
    # corrupt a present row of some payloads: the decode must still be the reference's map
    for b in range(0, batch, 2):
        v = int(rng.choice(np.flatnonzero(pres[b])))
        shards[b, v] ^= 0x5C
    d_sh = [_dev(shards[b0:b0 + c]) for b0, c in ranges]
    d_pr = [_dev(pres[b0:b0 + c]) for b0, c in ranges]
    d_out = [torch.zeros((c, olen), dtype=torch.uint8, device="cuda") for _, c in ranges]
    d_st = [torch.full((c, 2), -1, dtype=torch.int32, device="cuda") for _, c in ranges]
    torch.cuda.synchronize()
    npa.reconstruct_batch_multi(ctxs, p, [t.data_ptr() for t in d_sh], sl, n * sl, [t.data_ptr() for t in d_pr],
                                batch, [t.data_ptr() for t in d_out], olen, [t.data_ptr() for t in d_st])
    out = np.concatenate([t.cpu().numpy() for t in d_out])
    stat = np.concatenate([t.cpu().numpy() for t in d_st])
    for b in range(batch):
        st, want = oracle.reconstruct([shards[b, i].tobytes() if pres[b, i] else None for i in range(n)], n, k)
        assert st == 0 and out[b].tobytes() == want, b
        assert tuple(stat[b]) == (0, int(pres[b].sum()))


def test_host_batch_multi(gpu, oracle):
    ctxs = [npa.Context(0), npa.Context(0)]
    p = npa.CodeParams.derive_parameters(1024, 342)
    n, k = p.n(), p.k()
    plen, batch = 512 * 260 + 1, 5
    sl = p.make_encoder(gpu).shard_len(plen)
    pay = np.stack([np.frombuffer(synth.payload(900 + b, plen), np.uint8) for b in range(batch)])
    sh = np.zeros((batch, n * sl), np.uint8)
    npa.encode_batch_host_multi(ctxs, p, pay.ctypes.data, plen, plen, batch, sh.ctypes.data, n * sl)
    pres = np.stack([synth.present_mask(900 + b, n, 342) for b in range(batch)])
    olen = (sl // 2) * 2 * k
    out = np.zeros((batch, olen), np.uint8)
    npa.reconstruct_batch_host_multi(ctxs, p, sh.ctypes.data, sl, n * sl, pres.ctypes.data, batch, out.ctypes.data,
                                     olen)
    for b in range(batch):
        st, want = oracle.encode(pay[b].tobytes(), n, k, n)
        assert st == 0 and sh[b].tobytes() == b"".join(want)
        assert out[b, :plen].tobytes() == pay[b].tobytes()


@pytest.mark.parametrize("mode", [pytest.param("pin", marks=pytest.mark.pin_in_place), "stage"])
@pytest.mark.parametrize("nctx", [2, 3])
def test_host_batch_multi_pageable_unaligned_split(gpu, oracle, monkeypatch, nctx, mode):
    """the ranges of a host multi call are adjacent slices of one
    pageable caller buffer, and with a row stride that is no multiple of the
    page size neighbouring ranges share a page.  Staged (the default), or with
    NP_PAGEABLE=pin the engine pins the whole spans once before the worker
    threads start (engine.cpp np_*_batch_host_multi, PinRegistry), so no
    worker registers or unregisters a page under another's copies.  Guard
    bytes around every buffer; every payload against the oracle."""
    monkeypatch.setenv("NP_PAGEABLE", mode)
    ctxs = [npa.Context(0) for _ in range(nctx)]
    p = npa.CodeParams.derive_parameters(1024, 342)
    n, k = p.n(), p.k()
    plen, batch = 512 * 101 + 3, 7  # shard_len 204
    sl = p.make_encoder(gpu).shard_len(plen)
    bstride, ostride, g = n * sl + 100, (sl // 2) * 2 * k + 37, 4096 + 5
    pay = np.stack([np.frombuffer(synth.payload(950 + b, plen), np.uint8) for b in range(batch)])
    sh_b = np.full(batch * bstride + 2 * g, 0xC3, np.uint8)
    sh = sh_b[g:g + batch * bstride].reshape(batch, bstride)
    sh[...] = 0
    npa.encode_batch_host_multi(ctxs, p, pay.ctypes.data, plen, plen, batch, sh.ctypes.data, bstride)
    pres = np.stack([synth.present_mask(950 + b, n, 342) for b in range(batch)])
    out_b = np.full(batch * ostride + 2 * g, 0xC3, np.uint8)
    out = out_b[g:g + batch * ostride].reshape(batch, ostride)
    npa.reconstruct_batch_host_multi(ctxs, p, sh.ctypes.data, sl, bstride, pres.ctypes.data, batch, out.ctypes.data,
                                     ostride)
    for base in (sh_b, out_b):
        assert (base[:g] == 0xC3).all() and (base[-g:] == 0xC3).all()
    olen = (sl // 2) * 2 * k
    for b in range(batch):
        st, want = oracle.encode(pay[b].tobytes(), n, k, n)
        assert st == 0 and sh[b, :n * sl].tobytes() == b"".join(want), b
        st, rec = oracle.reconstruct([sh[b, i * sl:(i + 1) * sl].tobytes() if pres[b, i] else None for i in range(n)],
                                     n, k)
        assert st == 0 and out[b, :olen].tobytes() == rec, b


def test_multi_reports_need_more_shards(gpu):
    """A host-memory multi call fails like the crate (NeedMoreShards) when one
    range holds a payload with fewer than k present shards."""
    ctxs = [npa.Context(0), npa.Context(0)]
    p = npa.CodeParams.derive_parameters(256, 86)
    n, k = p.n(), p.k()
    sl, batch = 256, 4
    sh = np.zeros((batch, n * sl), np.uint8)
    pres = np.ones((batch, n), np.uint8)
    pres[3, : n - k + 1] = 0  # last payload (second range): k - 1 present
    out = np.zeros((batch, (sl // 2) * 2 * k), np.uint8)
    with pytest.raises(npa.NeedMoreShards) as e:
        npa.reconstruct_batch_host_multi(ctxs, p, sh.ctypes.data, sl, n * sl, pres.ctypes.data, batch,
                                         out.ctypes.data, out.shape[1])
    assert e.value.fields == (k - 1, k, n)


@pytest.mark.parametrize("n,k", [(1000, 300), (1000, 256), (1024, 300), (1024, 1024)])
def test_multi_checks_params_like_single_device(gpu, n, k):
    """Bad parameters fail the multi entries exactly as the single-device entry
    (also with batch == 0, where no per-device call runs): ParamterMustBePowerOf2
    when neither n nor k is a power of two (the crate's rule), an invalid
    argument otherwise."""
    ctxs = [npa.Context(0), npa.Context(0)]
    bad = npa.CodeParams(n, k, n)
    buf = np.zeros(64, np.uint8)
    ptr = buf.ctypes.data
    with pytest.raises(Exception) as single:
        npa.encode_batch_dev(bad, ptr, 16, 16, 0, ptr, 16, ctx=gpu)
    err = type(single.value)
    assert (err is npa.ParamterMustBePowerOf2) == (n == 1000 and k == 300)
    for batch in (0, 2):
        with pytest.raises(err):
            npa.encode_batch_multi(ctxs, bad, [ptr, ptr], 16, 16, batch, [ptr, ptr], 16)
        with pytest.raises(err):
            npa.reconstruct_batch_multi(ctxs, bad, [ptr, ptr], 2, 2 * n, [ptr, ptr], batch, [ptr, ptr], 2 * k)
        with pytest.raises(err):
            npa.encode_batch_host_multi(ctxs, bad, ptr, 16, 16, batch, ptr, 16)
        with pytest.raises(err):
            npa.reconstruct_batch_host_multi(ctxs, bad, ptr, 2, 2 * n, ptr, batch, ptr, 2 * k)


def test_multi_empty_batch_ok(gpu):
    """batch == 0 with valid parameters: nothing to do, as the single-device entry."""
    ctxs = [npa.Context(0), npa.Context(0)]
    p = npa.CodeParams.derive_parameters(1024, 342)
    buf = np.zeros(64, np.uint8)
    ptr = buf.ctypes.data
    bstride = p.n() * p.make_encoder(gpu).shard_len(16)
    npa.encode_batch_dev(p, ptr, 16, 16, 0, ptr, bstride, ctx=gpu)
    npa.encode_batch_multi(ctxs, p, [ptr, ptr], 16, 16, 0, [ptr, ptr], bstride)
    npa.encode_batch_host_multi(ctxs, p, ptr, 16, 16, 0, ptr, bstride)


@pytest.mark.pin_in_place
def test_pin_registry_two_threads_share_pages(gpu, oracle, monkeypatch):
    """two host calls at once, on two contexts from two threads,
    with NP_PAGEABLE=pin, on adjacent slices of one pageable buffer whose
    spans share a page.  Whichever call registers the shared range first, the
    other finds its span inside a registry range (or partly overlapping one)
    and takes a reference (or stages) under the registry's lock
    (engine.cpp PinRegistry::acquire), so no range is unregistered under the
    other call's DMA or gather.  Afterwards no range stays registered and no
    unregistration was refused; every payload against the oracle."""
    import threading

    monkeypatch.setenv("NP_PAGEABLE", "pin")
    ctxs = [npa.Context(0), npa.Context(0)]
    p = npa.CodeParams.derive_parameters(1024, 342)
    n, k = p.n(), p.k()
    plen, per = 128 * 1024 + 5, 3  # shard_len 514: spans of 1.5 MiB per call
    sl = p.make_encoder(gpu).shard_len(plen)
    bstride, olen = n * sl + 100, (sl // 2) * 2 * k
    batch = 2 * per
    pay = np.stack([np.frombuffer(synth.payload(970 + b, plen), np.uint8) for b in range(batch)])
    sh = np.zeros((batch, bstride), np.uint8)
    npa.encode_batch_host(p, pay.ctypes.data, plen, plen, batch, sh.ctypes.data, bstride, ctx=ctxs[0])
    pres = np.stack([synth.present_mask(970 + b, n, 342) for b in range(batch)])
    outs = [np.zeros((per, olen), np.uint8) for _ in range(2)]
    errors = []

    def worker(i):
        try:
            for _ in range(12):
                npa.reconstruct_batch_host(p, sh.ctypes.data + i * per * bstride, sl, bstride,
                                           pres[i * per:].ctypes.data, per, outs[i].ctypes.data, olen, ctx=ctxs[i])
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    assert npa.pin_registry_stats() == {"live_ranges": 0, "failed_unregisters": 0}
    for b in range(batch):
        assert outs[b // per][b % per, :plen].tobytes() == pay[b].tobytes(), b
