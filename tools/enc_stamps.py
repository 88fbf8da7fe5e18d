"""Experiment: per-wave phase timing of the multi-tile encode (config 3) from an
NP_EXP=192 build (fast_common.hpp `stamp`: lane 0 of every wave writes
s_memtime at each phase boundary of kernels_fast.hip encode_tile_multi /
encode_shift, into the batch-stride padding past each payload's shard rows).
For every phase: mean duration over waves and tiles, the slowest wave's, and
the spread of arrival times.  GPU box:
NP_LIB_PATH=$PWD/tools/exp/lib_st192.so python tools/enc_stamps.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-novelpoly_amd", "python"))
import novelpoly_amd as npa  # noqa: E402

p = npa.CodeParams.derive_parameters(1024, 342)
n, k, plen, b = p.n(), p.k(), 1 << 20, int(os.environ.get("BATCH", "1024"))
ctx = npa.Context(0)
torch.cuda.set_stream(torch.cuda.Stream())
s = torch.cuda.current_stream().cuda_stream
sl = p.make_encoder(ctx).shard_len(plen)
tiles = (plen // (2 * k) + 255) // 256
bstride = n * sl + 4096 * tiles
pay = torch.randint(0, 256, (b, plen), dtype=torch.uint8, device="cuda")
sh = torch.zeros((b, bstride), dtype=torch.uint8, device="cuda")
for it in range(3):
    sh[:, n * sl:].zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    npa.encode_batch_dev(p, pay.data_ptr(), plen, plen, b, sh.data_ptr(), bstride, ctx=ctx, stream=s)
    e1.record()
    torch.cuda.synchronize()
print(f"encode {e0.elapsed_time(e1):.3f} ms (stamped build)")
st = sh[:, n * sl:].cpu().numpy().view(np.uint64).reshape(b * tiles, 16, 32).astype(np.int64)
st = st[(st[:, :, 0] != 0).all(axis=1)]
names = {0: "tile start", 1: "DMA wait + tables + barrier", 2: "cq_read + systematic row stores",
         3: "convert + IFFT cq levels", 4: "barrier + cq_write_q", 5: "barrier + hi_read_q", 6: "IFFT hi levels"}
for sh_ in range(3):
    b0 = 7 + 4 * sh_
    names.update({b0: f"shift {sh_ + 1} hi levels", b0 + 1: f"shift {sh_ + 1} barriers + exchange (+DMA)",
                  b0 + 2: f"shift {sh_ + 1} cq levels + convert", b0 + 3: f"shift {sh_ + 1} row stores"})
used = [i for i in range(32) if (st[:, :, i] != 0).all()]
tot = (st[:, :, used[-1]].max(axis=1) - st[:, :, 0].min(axis=1)).mean()
print(f"tiles with stamps: {len(st)}; per tile {tot:.0f} ticks (first wave's start to last wave's end)")
print(f"{'phase end':>40} {'mean dur':>9} {'share':>6} {'max-wave dur':>12} {'arrival spread':>14}")
for a, c in zip(used, used[1:]):
    dur = st[:, :, c] - st[:, :, a]
    spread = st[:, :, c].max(axis=1) - st[:, :, c].min(axis=1)
    print(f"{names.get(c, c):>40} {dur.mean():9.0f} {100 * dur.mean() / tot:5.1f}% {dur.max(axis=1).mean():12.0f} "
          f"{spread.mean():14.0f}")
# tile-to-tile: start of the next tile of the same workgroup vs this tile's end
# per-wave mean durations (wave w runs on SIMD w % 4; a SIMD favours its
# older waves, so waves 12-15 run last on each SIMD: their barrier phases are
# the SIMD's idle time)
print("per-wave mean duration (ticks), waves 0..15")
for a, c in zip(used, used[1:]):
    dur = (st[:, :, c] - st[:, :, a]).mean(axis=0)
    print(f"{names.get(c, c):>40} " + " ".join(f"{v:6.0f}" for v in dur))
