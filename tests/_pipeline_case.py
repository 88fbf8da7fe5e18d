"""One host-pipeline reconstruct case with every systematic row present
(np_reconstruct_batch_host ships only the k systematic rows then, when the
kernel family it dispatches to has a copy mode: engine.cpp rec_path /
rows_needed).  Imported by tests/test_gpu_parity.py, and run as a script in a
child process so that the NP_HUGE / NP_RES switches, read once per process,
can send k >= 4096 / k in {512, 1024} to other kernel families:

    NP_HUGE=0 python tests/_pipeline_case.py NW KW PLEN BATCH PINNED
"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
for _p in (os.path.join(ROOT, "oracle"), os.path.join(ROOT, "reed-solomon-novelpoly_amd", "python")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import novelpoly_amd as npa  # noqa: E402
from novelpoly_amd import synth  # noqa: E402


_HIP = None


def host_array(shape, fill, pinned):
    """A host array, pageable (numpy) or pinned (hipHostMalloc through the HIP
    runtime, freed with the array; not torch, whose device discovery does not
    run in the child processes of a GPU test)."""
    if not pinned:
        return np.full(shape, fill, dtype=np.uint8)
    import ctypes
    import weakref

    global _HIP
    if _HIP is None:  # the HIP runtime the product library is linked to (dlsym searches its dependencies)
        _HIP = ctypes.CDLL(npa.LIB_PATH)
        _HIP.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
        _HIP.hipHostFree.argtypes = [ctypes.c_void_p]
    size = int(np.prod(shape))
    ptr = ctypes.c_void_p()
    assert _HIP.hipHostMalloc(ctypes.byref(ptr), size, 0) == 0, "hipHostMalloc failed"
    buf = (ctypes.c_uint8 * size).from_address(ptr.value)
    a = np.frombuffer(buf, dtype=np.uint8).reshape(shape)
    a[...] = fill
    weakref.finalize(buf, _HIP.hipHostFree, ptr.value)
    return a


def run(ctx, oracle, nw, kw, plen, batch, pinned, seed=4100):
    """Encode `batch` payloads on the host path, erase only parity rows, put
    garbage in the erased rows, reconstruct on the host path and compare every
    output with the oracle (mod.rs:162-239)."""
    p = npa.CodeParams.derive_parameters(nw, kw)
    n, k = p.n(), p.k()
    sl = p.make_encoder(ctx).shard_len(plen)
    pay = np.stack([np.frombuffer(synth.payload(seed + b, plen), dtype=np.uint8) for b in range(batch)])
    bstride = n * sl
    sh = host_array((batch, bstride), 0, pinned)
    npa.encode_batch_host(p, pay.ctypes.data, plen, plen, batch, sh.ctypes.data, bstride, ctx=ctx)
    rng = np.random.default_rng(seed)
    pres = np.zeros((batch, n), dtype=np.uint8)
    wn = p.wanted_n
    for b in range(batch):
        pres[b, :wn] = 1
        gone = min(wn - k, (n - k) // 2)
        pres[b, k + rng.choice(wn - k, gone, replace=False)] = 0  # systematic rows all present
    recvs = [[sh[b, i * sl:(i + 1) * sl].tobytes() if pres[b, i] else None for i in range(n)] for b in range(batch)]
    for b in range(batch):
        for i in np.flatnonzero(pres[b] == 0):
            sh[b, i * sl:(i + 1) * sl] = 0x5C
    olen = (sl // 2) * 2 * k
    out = host_array((batch, olen), 0, pinned)
    npa.reconstruct_batch_host(p, sh.ctypes.data, sl, bstride, pres.ctypes.data, batch, out.ctypes.data, olen, ctx=ctx)
    for b in range(batch):
        st, want = oracle.reconstruct(recvs[b], n, k)
        assert st == 0 and out[b].tobytes() == want, (nw, b)
        assert want[:plen] == pay[b].tobytes()


if __name__ == "__main__":
    import np_oracle

    nw, kw, plen, batch, pinned = (int(v) for v in sys.argv[1:6])
    run(npa.default_context(0), np_oracle.Oracle(), nw, kw, plen, batch, bool(pinned))
    print("ok", flush=True)
