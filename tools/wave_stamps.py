"""Experiment: per-wave phase timing of the fast reconstruct kernel (config 3)
from an NP_EXP=192 build (fast_common.hpp `stamp`: lane 0 of every wave
writes s_memtime at each phase boundary).  For every stamp point: the mean
spread between the first and the last wave of a workgroup to reach it, and
each phase's mean duration over waves; barrier-ended phases show how long the
early waves wait.  GPU box:
NP_LIB_PATH=$PWD/tools/exp/lib_192.so python tools/wave_stamps.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-novelpoly_amd", "python"))
import novelpoly_amd as npa  # noqa: E402
from novelpoly_amd import synth  # noqa: E402

cfg = synth.CONFIGS[3]
p = npa.CodeParams.derive_parameters(cfg["n_wanted"], cfg["k_wanted"])
n, k, plen, b = p.n(), p.k(), cfg["payload"], int(os.environ.get("BATCH", "1024"))
ctx = npa.Context(0)
torch.cuda.set_stream(torch.cuda.Stream())
s = torch.cuda.current_stream().cuda_stream
sl = p.make_encoder(ctx).shard_len(plen)
pay = torch.randint(0, 256, (b, plen), dtype=torch.uint8, device="cuda")
# the stamped encode (NP_EXP bit 6) writes its own stamps past each payload's
# rows (kernels_fast.hip encode_tile_multi: n shard_len + 4 KiB per tile)
enc_tiles = (plen // (2 * k) + 255) // 256 + 1
bstride = n * sl + 4096 * enc_tiles
sh = torch.zeros((b, bstride), dtype=torch.uint8, device="cuda")
pres = torch.from_numpy(np.stack([synth.present_mask(i, n, cfg["erase"]) for i in range(b)])).cuda()
out_len = (sl // 2) * 2 * k
tiles = (sl // 2 + 255) // 256
stride = out_len + 4096 * tiles
out = torch.zeros((b, stride), dtype=torch.uint8, device="cuda")
npa.encode_batch_dev(p, pay.data_ptr(), plen, plen, b, sh.data_ptr(), bstride, ctx=ctx, stream=s)
for it in range(3):
    out.zero_()
    npa.reconstruct_batch_dev2(p, sh.data_ptr(), sl, bstride, pres.data_ptr(), 0, b, out.data_ptr(), stride,
                               ctx=ctx, stream=s)
    torch.cuda.synchronize()
st = out[:, out_len:].cpu().numpy().view(np.uint64).reshape(b * tiles, 16, 32).astype(np.int64)
st = st[(st[:, :, 0] != 0).all(axis=1)]
print(f"tiles with stamps: {len(st)}")
names = {0: "start", 1: "tables", 26: "segments done", 27: "FFT hi", 28: "hi_write+syncs",
         29: "cq_read+FFT cq", 30: "merge", 31: "copy-out"}
for s_ in range(4):
    names.update({2 + 6 * s_: f"s{s_} rows/top", 3 + 6 * s_: f"s{s_} premul", 4 + 6 * s_: f"s{s_} cq levels",
                  5 + 6 * s_: f"s{s_} sync+cq_write+sync", 6 + 6 * s_: f"s{s_} hi levels"})
used = [i for i in range(32) if (st[:, :, i] != 0).all()]
tot = (st[:, :, 31].max(axis=1) - st[:, :, 0].min(axis=1)).mean()
print(f"per tile {tot:.0f} ticks (first wave's start to last wave's end)")
print(f"{'phase end':>26} {'mean dur':>9} {'max-wave dur':>12} {'arrival spread':>14}")
for a, c in zip(used, used[1:]):
    dur = st[:, :, c] - st[:, :, a]
    spread = st[:, :, c].max(axis=1) - st[:, :, c].min(axis=1)
    print(f"{names.get(c, c):>26} {dur.mean():9.0f} {dur.max(axis=1).mean():12.0f} {spread.mean():14.0f}")
# per-wave mean durations of the phases that end without a barrier (work
# imbalance between the waves of a workgroup; wave w runs on SIMD w % 4)
print("per-wave mean duration (ticks), waves 0..15")
for a, c in zip(used, used[1:]):
    if "sync" in names.get(c, "") or "write" in names.get(c, ""):
        continue
    dur = (st[:, :, c] - st[:, :, a]).mean(axis=0)
    print(f"{names.get(c, c):>26} " + " ".join(f"{v:6.0f}" for v in dur))
