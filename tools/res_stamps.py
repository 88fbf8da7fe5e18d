"""Experiment: per-wave phase timing of the resident k = 1024 reconstruct
(config 4, kernels_res.hip k_reconstruct_res<1024, 4>) from an NP_EXP=192
build (kernels_res.hip `rstamp`: lane 0 of every wave writes s_memtime at each
phase boundary into the output-stride padding).  For every phase: mean
duration over waves and tiles, the slowest wave's, and its share of the tile.
GPU box: NP_LIB_PATH=$PWD/tools/exp/lib_st192.so python tools/res_stamps.py
CFG=3 with NP_REC_RES256=1: the k = 256 decode on the resident kernels
(k_reconstruct_res<256, 4>, 4 waves per tile; no HD levels, so the HD
phases read 0 and the last step's fold holds D(x0)'s two exchanges)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-novelpoly_amd", "python"))
import novelpoly_amd as npa  # noqa: E402
from novelpoly_amd import synth  # noqa: E402

cfg = synth.CONFIGS[int(os.environ.get("CFG", "4"))]
p = npa.CodeParams.derive_parameters(cfg["n_wanted"], cfg["k_wanted"])
n, k, plen, b = p.n(), p.k(), cfg["payload"], int(os.environ.get("BATCH", "256"))
nw = k // 64  # waves per tile
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
tiles = (sl // 2 + 63) // 64
stride = out_len + 8192 * tiles
out = torch.zeros((b, stride), dtype=torch.uint8, device="cuda")
npa.encode_batch_dev(p, pay.data_ptr(), plen, plen, b, sh.data_ptr(), bstride, ctx=ctx, stream=s)
for it in range(3):
    out.zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    npa.reconstruct_batch_dev2(p, sh.data_ptr(), sl, bstride, pres.data_ptr(), 0, b, out.data_ptr(), stride,
                               ctx=ctx, stream=s)
    e1.record()
    torch.cuda.synchronize()
print(f"reconstruct {e0.elapsed_time(e1):.3f} ms (stamped build)")
st = out[:, out_len:].cpu().numpy().view(np.uint64).reshape(b * tiles, 16, 64)[:, :nw].astype(np.int64)
st = st[(st[:, :, 0] != 0).all(axis=1)]
names = {0: "start", 1: "stage CQ delta + HA/HD tables", 40: "FFT hd levels", 41: "sync+HD write+sync+HA read",
         42: "FFT ha levels", 43: "sync+HA write+sync+CQ read", 44: "FFT cq levels",
         45: "merge rows + sync + stage row tables + sync", 46: "merge postmultiply", 47: "copy-out"}
for s_ in range(4):
    b0 = 2 + 8 * s_
    names.update({b0: f"s{s_} rows + sync + stage row tables + sync", b0 + 1: f"s{s_} premultiply",
                  b0 + 2: f"s{s_} cq levels", b0 + 3: f"s{s_} sync+CQ write+sync+HA read", b0 + 4: f"s{s_} ha levels",
                  b0 + 5: f"s{s_} sync+HA write+sync+HD read", b0 + 6: f"s{s_} hd levels", b0 + 7: f"s{s_} fold"})
used = [i for i in range(64) if (st[:, :, i] != 0).all()]
tot = (st[:, :, used[-1]].max(axis=1) - st[:, :, 0].min(axis=1)).mean()
print(f"tiles with stamps: {len(st)}; per tile {tot:.0f} ticks (first wave's start to last wave's end)")
print(f"{'phase end':>46} {'mean dur':>9} {'share':>6} {'max-wave dur':>12}")
groups = {}
for a, c in zip(used, used[1:]):
    dur = st[:, :, c] - st[:, :, a]
    nm = names.get(c, str(c))
    print(f"{nm:>46} {dur.mean():9.0f} {100 * dur.mean() / tot:5.1f}% {dur.max(axis=1).mean():12.0f}")
    key = nm.split(" ", 1)[1] if nm[0] == "s" and nm[1].isdigit() else nm
    groups[key] = groups.get(key, 0.0) + dur.mean()
print("by phase kind (sum over the segment steps):")
for key, v in sorted(groups.items(), key=lambda kv: -kv[1]):
    print(f"{key:>46} {v:9.0f} {100 * v / tot:5.1f}%")
