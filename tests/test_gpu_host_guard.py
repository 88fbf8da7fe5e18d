"""Regression for round 4's one GPU fault (probe 19): the host
batch calls on pageable buffers whose shard rows are only 2 mod 4 bytes long,
encode then reconstruct on the SAME buffer -- the sequence of
test_host_pipeline_all_systematic[12289-4097-73728-3-pageable], where the
encode pinned and unpinned the numpy buffer and the reconstruct then handed it
to the runtime's pageable 2-D copies.  The engine now never passes a pageable
pointer to a HIP copy (engine.cpp, host-memory pipeline: staged by host
threads, or with NP_PAGEABLE=pin pinned in place through the process-wide
registry; those cases run in a child process, test_gpu_pin_isolated.py).

Every host and device buffer sits between guard bytes, checked after every
call: the engine must neither write outside the caller's ranges nor read
garbage from them (the outputs are checked against the oracle,
mod.rs:162-239, and the payloads must come back)."""
import numpy as np
import pytest

import novelpoly_amd as npa
from novelpoly_amd import synth

pytestmark = pytest.mark.gpu

GUARD = 4096 + 13  # guard bytes on each side (odd: the caller's range starts unaligned)
CANARY = 0xC3


def guarded_host(nbytes, fill=0):
    """(base, view): a pageable numpy buffer of nbytes inside GUARD canary bytes."""
    base = np.full(nbytes + 2 * GUARD, CANARY, np.uint8)
    view = base[GUARD:GUARD + nbytes]
    view[...] = fill
    return base, view


def guards_intact(base):
    return bool((base[:GUARD] == CANARY).all() and (base[-GUARD:] == CANARY).all())


# (validators, k_wanted, payload bytes): shard_len = 18 (huge path, probe 19's
# shape), 202 (config 3's code), 42 (k = 1024, resident path); all 2 mod 4
_CASES = [(12289, 4097, 2 * 4096 * 9), (1024, 342, 512 * 101), (4096, 1366, 2048 * 21)]


def _erasures(p, batch, how, seed):
    n, k, wn = p.n(), p.k(), p.wanted_n
    rng = np.random.default_rng(seed)
    pres = np.zeros((batch, n), np.uint8)
    for b in range(batch):
        pres[b, :wn] = 1
        if how == "parity":  # every systematic row present: the copy mode, k rows cross PCIe
            gone = rng.choice(np.arange(k, wn), min(wn - k, (n - k) // 2), replace=False)
        else:
            gone = rng.choice(wn, wn - k, replace=False)
        pres[b, gone] = 0
    return pres


@pytest.mark.parametrize("mode", [pytest.param("pin", marks=pytest.mark.pin_in_place), "stage"])
@pytest.mark.parametrize("how", ["parity", "any"])
@pytest.mark.parametrize("batch", [3, 5])
@pytest.mark.parametrize("nw,kw,plen", _CASES)
def test_host_encode_then_reconstruct_same_pageable_buffer(gpu, oracle, monkeypatch, nw, kw, plen, batch, how, mode):
    monkeypatch.setenv("NP_PAGEABLE", mode)
    p = npa.CodeParams.derive_parameters(nw, kw)
    n, k, wn = p.n(), p.k(), p.wanted_n
    sl = p.make_encoder(gpu).shard_len(plen)
    assert sl % 4 == 2
    pay_b, pay = guarded_host(batch * plen)
    pay = pay.reshape(batch, plen)
    for b in range(batch):
        pay[b] = np.frombuffer(synth.payload(4100 + b, plen), np.uint8)
    bstride = n * sl
    sh_b, sh = guarded_host(batch * bstride, 0xAB)
    sh = sh.reshape(batch, bstride)
    npa.encode_batch_host(p, pay.ctypes.data, plen, plen, batch, sh.ctypes.data, bstride, ctx=gpu)
    assert guards_intact(pay_b) and guards_intact(sh_b)
    for b in (0, batch - 1):
        st, want = oracle.encode(pay[b].tobytes(), n, k, wn)
        assert st == 0 and [sh[b, i * sl:(i + 1) * sl].tobytes() for i in range(wn)] == want, b
    assert (sh[:, wn * sl:] == 0xAB).all()
    pres_b, pres = guarded_host(batch * n)
    pres = pres.reshape(batch, n)
    pres[...] = _erasures(p, batch, how, plen + batch)
    recvs = [[sh[b, i * sl:(i + 1) * sl].tobytes() if pres[b, i] else None for i in range(n)] for b in range(batch)]
    for b in range(batch):  # garbage in the absent rows: never read
        for i in np.flatnonzero(pres[b] == 0):
            sh[b, i * sl:(i + 1) * sl] = 0x5C
    olen = (sl // 2) * 2 * k
    out_b, out = guarded_host(batch * olen, 0x11)
    out = out.reshape(batch, olen)
    npa.reconstruct_batch_host(p, sh.ctypes.data, sl, bstride, pres.ctypes.data, batch, out.ctypes.data, olen,
                               ctx=gpu)
    assert guards_intact(sh_b) and guards_intact(pres_b) and guards_intact(out_b)
    for b in range(batch):
        st, want = oracle.reconstruct(recvs[b], n, k)
        assert st == 0 and out[b].tobytes() == want, b
        assert want[:plen] == pay[b].tobytes()


@pytest.mark.parametrize("nw,kw,plen", _CASES)
def test_device_buffers_guarded(gpu, oracle, nw, kw, plen):
    """The same shapes through the device batch calls, every device buffer
    between canary bytes (encode_batch_dev, reconstruct_batch_dev2)."""
    import torch

    p = npa.CodeParams.derive_parameters(nw, kw)
    n, k, wn = p.n(), p.k(), p.wanted_n
    sl = p.make_encoder(gpu).shard_len(plen)
    batch = 3
    g = GUARD

    def dbuf(nbytes, fill):
        t = torch.full((nbytes + 2 * g,), CANARY, dtype=torch.uint8, device="cuda")
        t[g:g + nbytes] = fill
        return t

    def intact(t):
        h = t.cpu().numpy()
        return bool((h[:g] == CANARY).all() and (h[-g:] == CANARY).all())

    pls = np.stack([np.frombuffer(synth.payload(4200 + b, plen), np.uint8) for b in range(batch)])
    dp = dbuf(batch * plen, 0)
    dp[g:g + batch * plen] = torch.from_numpy(pls.reshape(-1)).cuda()
    bstride = n * sl
    ds = dbuf(batch * bstride, 0xAB)
    torch.cuda.synchronize()
    npa.encode_batch_dev(p, dp.data_ptr() + g, plen, plen, batch, ds.data_ptr() + g, bstride, ctx=gpu,
                         stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert intact(dp) and intact(ds)
    hs = ds[g:g + batch * bstride].cpu().numpy().reshape(batch, bstride)
    pres = _erasures(p, batch, "any", plen)
    dpres = dbuf(batch * n, 0)
    dpres[g:g + batch * n] = torch.from_numpy(pres.reshape(-1)).cuda()
    olen = (sl // 2) * 2 * k
    dout = dbuf(batch * olen, 0x11)
    torch.cuda.synchronize()
    npa.reconstruct_batch_dev2(p, ds.data_ptr() + g, sl, bstride, dpres.data_ptr() + g, 0, batch,
                               dout.data_ptr() + g, olen, ctx=gpu, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert intact(ds) and intact(dpres) and intact(dout)
    o = dout[g:g + batch * olen].cpu().numpy().reshape(batch, olen)
    for b in range(batch):
        st, want = oracle.reconstruct([hs[b, i * sl:(i + 1) * sl].tobytes() if pres[b, i] else None
                                       for i in range(n)], n, k)
        assert st == 0 and o[b].tobytes() == want, b
        assert want[:plen] == pls[b].tobytes()


def test_device_error_names_its_call(gpu):
    """NP_ERR_DEVICE / NP_ERR_ALLOC carry the HIP call that failed
    (np_last_error_detail {hipError, line, 0} and np_last_error_site).  A
    payload length of 2^50 bytes makes np_rs_encode's device staging allocation
    fail before any byte is read or copied (engine.cpp np_rs_encode)."""
    import ctypes as C

    p = npa.CodeParams.derive_parameters(256, 86)
    huge = 1 << 50
    buf = C.create_string_buffer(16)
    st = npa.lib().np_rs_encode(gpu.handle, C.byref(p._c()), buf.raw, huge, buf, npa.lib().np_shard_len(C.byref(p._c()), huge))
    assert st == 102, st  # NP_ERR_ALLOC
    det = (C.c_size_t * 3)()
    npa.lib().np_last_error_detail(det)
    site = npa.lib().np_last_error_site().decode()
    assert det[0] == 2 and det[1] > 0, tuple(det)  # hipErrorOutOfMemory, the engine line
    assert site.startswith(f"engine.cpp:{det[1]} ") and "d_in.ensure" in site, site
    # the context stays usable
    assert npa.encode(b"x" * 1000, 256, ctx=gpu)
