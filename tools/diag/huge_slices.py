"""Diagnostic (not a test): 65,536 validators, 1 MiB payloads, large batches.
Which step goes wrong for which payloads: the batched encode against per-payload
encodes, then the batched decode against the payloads."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-novelpoly_amd", "python"))
import novelpoly_amd as npa  # noqa: E402

batch = int(sys.argv[1]) if len(sys.argv) > 1 else 1801
ctx = npa.Context(0)
torch.cuda.set_stream(torch.cuda.Stream())  # not torch's null stream: a NULL stream is the context's own
p = npa.CodeParams.derive_parameters(65536, 21846)
n, k = p.n(), p.k()
plen = 1 << 20
sl = p.make_encoder(ctx).shard_len(plen)
s = torch.cuda.current_stream().cuda_stream
g = torch.Generator(device="cuda")
g.manual_seed(batch)
pays = torch.randint(0, 256, (batch, plen), dtype=torch.uint8, device="cuda", generator=g)
shards = torch.empty((batch, n, sl), dtype=torch.uint8, device="cuda")
npa.encode_batch_dev(p, pays.data_ptr(), plen, plen, batch, shards.data_ptr(), n * sl, ctx=ctx, stream=s)
torch.cuda.synchronize()
# systematic rows must equal the payload bytes (chunk c of 2k bytes -> column c)
sysrows = shards[:, :k, :].permute(0, 2, 1).reshape(batch, sl // 2, 2, k).permute(0, 1, 3, 2).reshape(batch, plen)
bad_sys = torch.nonzero((sysrows != pays).any(dim=1)).flatten().cpu().numpy()
print("systematic rows wrong:", bad_sys.size, bad_sys[:10], flush=True)
# parity rows: per-payload encodes of a sample
one = torch.empty((1, n, sl), dtype=torch.uint8, device="cuda")
sample = sorted(set([0, 1, 100, 145, 146, 147, 150, 200, 255, 256, 300, 1000, batch - 1]) & set(range(batch)))
bad_par = []
for b in sample:
    npa.encode_batch_dev(p, pays[b].data_ptr(), plen, plen, 1, one.data_ptr(), n * sl, ctx=ctx, stream=s)
    torch.cuda.synchronize()
    if not torch.equal(one[0], shards[b]):
        rows = torch.nonzero((one[0] != shards[b]).any(dim=1)).flatten().cpu().numpy()
        bad_par.append((b, rows.size, rows[:4].tolist()))
print("encode sample mismatches (payload, rows, first rows):", bad_par, flush=True)
keep = torch.rand((batch, n), device="cuda", generator=g) >= 1 / 3
pres = keep.to(torch.uint8)
out = torch.full((batch, plen), 0xA5, dtype=torch.uint8, device="cuda")
npa.reconstruct_batch_dev2(p, shards.data_ptr(), sl, n * sl, pres.data_ptr(), 0, batch, out.data_ptr(), plen,
                           ctx=ctx, stream=s)
torch.cuda.synchronize()
bad = torch.nonzero((out != pays).any(dim=1)).flatten().cpu().numpy()
print("decode wrong:", bad.size, bad[:10], bad[-5:] if bad.size else [], flush=True)
