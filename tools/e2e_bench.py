"""Host-memory end-to-end rate (SURVEY §8(d) "End-to-end", §8(f) 2):
payloads start in pinned host memory and shards / outputs end in pinned host
memory, through the C ABI's host batch calls (np_encode_batch_host,
np_reconstruct_batch_host: sub-batches pipelined over streams, H2D / kernel /
D2H overlapped).  Also reports the PCIe bound for the same bytes.  Never the
bench `value` (that one is device-resident)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-novelpoly_amd", "python"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import novelpoly_amd as npa  # noqa: E402
from novelpoly_amd import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=3)
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--reps", type=int, default=3)
args = ap.parse_args()

cfg = synth.CONFIGS[args.config]
p = npa.CodeParams.derive_parameters(cfg["n_wanted"], cfg["k_wanted"])
n, k, plen, B = p.n(), p.k(), cfg["payload"], args.batch
erase = cfg["erase"] if cfg["erase"] is not None else n - k
ctx = npa.Context(0)
sl = p.make_encoder(ctx).shard_len(plen)
olen = (sl // 2) * 2 * k
h_pay = torch.randint(0, 256, (B, plen), dtype=torch.uint8).pin_memory()
h_sh = torch.empty((B, n, sl), dtype=torch.uint8).pin_memory()
h_out = torch.empty((B, olen), dtype=torch.uint8).pin_memory()
pres = np.ascontiguousarray(np.stack([synth.present_mask(i, n, erase) for i in range(B)]).astype(np.uint8))

# PCIe reference: one pinned H2D and one D2H of 256 MiB
buf_h = torch.empty(256 << 20, dtype=torch.uint8).pin_memory()
buf_d = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
for direction in ("h2d", "d2h"):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        (buf_d.copy_(buf_h, non_blocking=True) if direction == "h2d" else buf_h.copy_(buf_d, non_blocking=True))
    torch.cuda.synchronize()
    globals()["bw_" + direction] = 3 * (256 << 20) / (time.perf_counter() - t0) / 1e9


def timed(fn):
    fn()  # warm
    t0 = time.perf_counter()
    for _ in range(args.reps):
        fn()
    return (time.perf_counter() - t0) / args.reps


t_enc = timed(lambda: npa.encode_batch_host(p, h_pay.data_ptr(), plen, plen, B, h_sh.data_ptr(), n * sl, ctx=ctx))
def rec():
    npa.reconstruct_batch_host(p, h_sh.data_ptr(), sl, n * sl, pres.ctypes.data, B, h_out.data_ptr(), olen, ctx=ctx)


h_out.zero_()
t_rec = timed(rec)
ok = torch.equal(h_out[:, :plen], h_pay)
# pinned buffers, present rows packed by host threads and DMA'd (NP_HOST_ROWS=pack)
# instead of gathered by the k_copy_rows kernel
os.environ["NP_HOST_ROWS"] = "pack"
h_out.zero_()
t_rec_pack = timed(rec)
ok = ok and torch.equal(h_out[:, :plen], h_pay)
os.environ["NP_HOST_ROWS"] = "gather"
h_out.zero_()
t_rec_gather = timed(rec)
ok = ok and torch.equal(h_out[:, :plen], h_pay)
del os.environ["NP_HOST_ROWS"]
# bytes crossing PCIe: encode P in + n*sl out; reconstruct the rows the engine
# reads (engine.cpp rows_needed: the k systematic rows when every payload of the
# batch has them all, else all n rows), of those only the present ones on the
# gather path, (+ flags) in, and 2k*sl/2 out.
# Pageable shards and output (numpy).  Default: host threads copy the present
# rows into pinned staging and the outputs back out of it (engine.cpp,
# host-memory pipeline); NP_PAGEABLE=pin (opt-in): the engine pins them in
# place for the call (PinRegistry) and goes as from pinned memory.
pg_sh = h_sh.numpy().copy()
pg_out = np.zeros((B, olen), dtype=np.uint8)
pg_pay = h_pay.numpy().copy()
pg_enc = np.zeros((B, n * sl), dtype=np.uint8)


def rec_pageable():
    npa.reconstruct_batch_host(p, pg_sh.ctypes.data, sl, n * sl, pres.ctypes.data, B, pg_out.ctypes.data, olen,
                               ctx=ctx)


def enc_pageable():
    npa.encode_batch_host(p, pg_pay.ctypes.data, plen, plen, B, pg_enc.ctypes.data, n * sl, ctx=ctx)


wb = p.wanted_n * sl  # the rows encode writes
os.environ["NP_PAGEABLE"] = "pin"
t_enc_pg = timed(enc_pageable)
ok_pg = bool((pg_enc[:, :wb] == h_sh.numpy().reshape(B, -1)[:, :wb]).all())
t_pg = timed(rec_pageable)
ok_pg = ok_pg and bool((pg_out[:, :plen] == h_pay.numpy()).all())
pg_out[:] = 0
pg_enc[:] = 0
del os.environ["NP_PAGEABLE"]  # the default: staged
t_pg_st = timed(rec_pageable)
t_enc_st = timed(enc_pageable)
ok_pg = ok_pg and bool((pg_out[:, :plen] == h_pay.numpy()).all())
ok_pg = ok_pg and bool((pg_enc[:, :wb] == h_sh.numpy().reshape(B, -1)[:, :wb]).all())
ok = ok and ok_pg


# one payload per call (small calls pay no registration below 1 MiB)
def one_call_ms(fn, reps=20):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return round((time.perf_counter() - t0) / reps * 1e3, 3)


lat = {
    "encode_pinned_ms": one_call_ms(lambda: npa.encode_batch_host(p, h_pay.data_ptr(), plen, plen, 1, h_sh.data_ptr(),
                                                                  n * sl, ctx=ctx)),
    "encode_pageable_ms": one_call_ms(lambda: npa.encode_batch_host(p, pg_pay.ctypes.data, plen, plen, 1,
                                                                    pg_enc.ctypes.data, n * sl, ctx=ctx)),
    "reconstruct_pinned_ms": one_call_ms(lambda: npa.reconstruct_batch_host(p, h_sh.data_ptr(), sl, n * sl,
                                                                            pres.ctypes.data, 1, h_out.data_ptr(),
                                                                            olen, ctx=ctx)),
    "reconstruct_pageable_ms": one_call_ms(lambda: npa.reconstruct_batch_host(p, pg_sh.ctypes.data, sl, n * sl,
                                                                              pres.ctypes.data, 1, pg_out.ctypes.data,
                                                                              olen, ctx=ctx)),
}
rows_dma = k if all(pres[b, :k].all() for b in range(B)) else n
rows = float(pres[:, :rows_dma].sum()) / B
res = {
    "config": args.config, "batch": B, "payload_bytes": plen, "n": n, "k": k,
    "pcie_GB_s": {"h2d": round(bw_h2d, 1), "d2h": round(bw_d2h, 1)},
    "encode": {"GiB_s": round(B * plen / t_enc / 2**30, 2), "ms": round(t_enc * 1e3, 2),
               "pcie_bound_GiB_s": round(B * plen / max(B * plen / (bw_h2d * 1e9), B * n * sl / (bw_d2h * 1e9)) / 2**30, 2)},
    "reconstruct": {"GiB_s": round(B * plen / t_rec / 2**30, 2), "ms": round(t_rec * 1e3, 2), "rows_copied": rows,
                    "pcie_bound_GiB_s": round(B * plen / max(B * rows * sl / (bw_h2d * 1e9), B * olen / (bw_d2h * 1e9)) / 2**30, 2),
                    # the two directions one after the other: kernel reads of host memory and a
                    # concurrent D2H share the link badly (tools/microbench/h2d_gather.hip)
                    "pcie_serial_bound_GiB_s": round(B * plen / (B * rows * sl / (bw_h2d * 1e9) + B * olen / (bw_d2h * 1e9)) / 2**30, 2)},
    "reconstruct_pinned_pack": {"GiB_s": round(B * plen / t_rec_pack / 2**30, 2), "ms": round(t_rec_pack * 1e3, 2)},
    "reconstruct_pinned_gather": {"GiB_s": round(B * plen / t_rec_gather / 2**30, 2),
                                  "ms": round(t_rec_gather * 1e3, 2)},
    "encode_pageable_pinned_in_place": {"GiB_s": round(B * plen / t_enc_pg / 2**30, 2), "ms": round(t_enc_pg * 1e3, 2)},
    "reconstruct_pageable_pinned_in_place": {"GiB_s": round(B * plen / t_pg / 2**30, 2), "ms": round(t_pg * 1e3, 2),
                                             "rows_copied": rows},
    "reconstruct_pageable_staged": {"GiB_s": round(B * plen / t_pg_st / 2**30, 2), "ms": round(t_pg_st * 1e3, 2),
                                    "rows_copied": rows, "host_threads": min(16, os.cpu_count() or 1)},
    "encode_pageable_staged": {"GiB_s": round(B * plen / t_enc_st / 2**30, 2), "ms": round(t_enc_st * 1e3, 2)},
    "one_payload_call": lat,
    "roundtrip_ok": bool(ok),
}
print(json.dumps(res))
