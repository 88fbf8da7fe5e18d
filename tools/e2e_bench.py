"""Host-memory end-to-end rate (SURVEY §8(d) "End-to-end"):
payloads start in pinned host memory, shards/outputs end in pinned host memory.
Measures (1) serial: H2D -> kernel -> D2H on one stream, and (2) pipelined:
the batch split into chunks over two streams so that copies overlap kernels.
Never the bench `value` (that one is device-resident)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-novelpoly_amd", "python"))

import numpy as np
import torch

import novelpoly_amd as npa
from novelpoly_amd import synth

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=3)
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--chunks", type=int, default=8)
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
pres = torch.from_numpy(np.stack([synth.present_mask(i, n, erase) for i in range(B)]))
d_pay = torch.empty((B, plen), dtype=torch.uint8, device="cuda")
d_sh = torch.empty((B, n, sl), dtype=torch.uint8, device="cuda")
d_out = torch.empty((B, olen), dtype=torch.uint8, device="cuda")
d_pres = pres.cuda()
streams = [torch.cuda.Stream(), torch.cuda.Stream()]


def enc_range(lo, hi, s):
    with torch.cuda.stream(s):
        d_pay[lo:hi].copy_(h_pay[lo:hi], non_blocking=True)
        npa.encode_batch_dev(p, d_pay[lo].data_ptr(), plen, plen, hi - lo, d_sh[lo].data_ptr(), n * sl, ctx=ctx,
                             stream=s.cuda_stream)
        h_sh[lo:hi].copy_(d_sh[lo:hi], non_blocking=True)


def rec_range(lo, hi, s):
    # only present shards travel: gather rows on the host side would cost a CPU
    # copy, so we ship the whole shard matrix rows that are present (mask view)
    with torch.cuda.stream(s):
        d_sh[lo:hi].copy_(h_sh[lo:hi], non_blocking=True)
        npa.reconstruct_batch_dev2(p, d_sh[lo].data_ptr(), sl, n * sl, d_pres[lo].data_ptr(), 0, hi - lo,
                                   d_out[lo].data_ptr(), olen, ctx=ctx, stream=s.cuda_stream)
        h_out[lo:hi].copy_(d_out[lo:hi], non_blocking=True)


def run(fn, chunks):
    step = (B + chunks - 1) // chunks
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for r in range(args.reps):
        for i, lo in enumerate(range(0, B, step)):
            fn(lo, min(B, lo + step), streams[i % 2] if chunks > 1 else streams[0])
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / args.reps


res = {"config": args.config, "batch": B, "payload_bytes": plen, "n": n, "k": k}
for name, fn in (("encode", enc_range), ("reconstruct", rec_range)):
    run(fn, 1)  # warm
    t1 = run(fn, 1)
    tp = run(fn, args.chunks)
    res[name] = {"serial_GiB_s": B * plen / t1 / 2**30, "pipelined_GiB_s": B * plen / tp / 2**30,
                 "serial_ms": t1 * 1e3, "pipelined_ms": tp * 1e3, "chunks": args.chunks}
ok = torch.equal(h_out[:, :plen], h_pay)
res["roundtrip_ok"] = bool(ok)
print(json.dumps(res))
