"""Experiment: per-phase durations of the fast reconstruct kernel from the
s_memtime stamps of an NP_EXP=64 build (fast_common.hpp `stamp`).  GPU box:
NP_LIB_PATH=tools/exp/lib_64.so python tools/phase_stamps.py"""
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
stride = out_len + 4096
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
ms = e0.elapsed_time(e1)
st = out[:, out_len:out_len + 8 * 256].cpu().numpy().view(np.uint64).reshape(b, 8, 32).astype(np.int64)
st = st.reshape(-1, 32)
st = st[st[:, 0] != 0]
span = st[:, 31].max() - st[:, 0].min()
print(f"kernel {ms:.3f} ms, stamp span {span} ticks -> {span / (ms * 1e3):.1f} ticks/us; tiles {len(st)}")
names = {0: "start", 1: "E+vpools staged", 26: "segments done", 27: "FFT hi", 28: "hi_write+syncs",
         29: "cq_read+FFT cq", 30: "merge", 31: "copy-out"}
for s_ in range(4):
    names.update({2 + 6 * s_: f"s{s_} top", 3 + 6 * s_: f"s{s_} premul", 4 + 6 * s_: f"s{s_} cq levels",
                  5 + 6 * s_: f"s{s_} sync+cq_write+sync", 6 + 6 * s_: f"s{s_} hi levels"})
used = [i for i in range(32) if (st[:, i] != 0).all()]
tot = (st[:, 31] - st[:, 0]).mean()
print(f"per tile {tot:.0f} ticks")
for a, c in zip(used, used[1:]):
    d = (st[:, c] - st[:, a]).mean()
    print(f"  {names.get(c, c):>24}: {d:9.0f} ticks {100 * d / tot:5.1f}%")
