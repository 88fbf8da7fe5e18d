"""Host-pipeline probe (not product code): the host reconstruct
of a BASELINE config from pinned buffers (k_copy_rows gather, or packed rows
by host threads + DMA) and from pageable ones (staged), at several sub-batch
sizes, with the engine's NP_PIPE_STATS time split on stderr.
python tools/pipe_probe.py --config 3 --batch 256"""
import argparse
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
ap.add_argument("--grid", default="3:6,3:12,4:6,4:8,6:4,6:6", help="slots:payloads-per-sub-batch pairs")
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
npa.encode_batch_host(p, h_pay.data_ptr(), plen, plen, B, h_sh.data_ptr(), n * sl, ctx=ctx)
pg_sh = h_sh.numpy().copy()
pg_out = np.zeros((B, olen), dtype=np.uint8)


def run(label, src, dst, env):
    for kk in ("NP_HOST_ROWS", "NP_PIPE_STATS", "NP_PIPE_SLOTS", "NP_PIPE_SB"):
        os.environ.pop(kk, None)
    os.environ.update(env)
    f = lambda: npa.reconstruct_batch_host(p, src, sl, n * sl, pres.ctypes.data, B, dst, olen, ctx=ctx)  # noqa: E731
    f()
    os.environ["NP_PIPE_STATS"] = "1"
    t0 = time.perf_counter()
    for _ in range(args.reps):
        f()
    dt = (time.perf_counter() - t0) / args.reps
    print(f"{label:40s} {B * plen / dt / 2**30:7.2f} GiB/s  {dt * 1e3:7.2f} ms", flush=True)


run("pinned gather (default sizes)", h_sh.data_ptr(), h_out.data_ptr(), {"NP_HOST_ROWS": "gather"})
run("pinned pack (default sizes)", h_sh.data_ptr(), h_out.data_ptr(), {"NP_HOST_ROWS": "pack"})
run("pageable staged (default sizes)", pg_sh.ctypes.data, pg_out.ctypes.data, {})
for g in args.grid.split(","):
    slots, sb = g.split(":")
    env = {"NP_PIPE_SLOTS": slots, "NP_PIPE_SB": sb}
    run(f"pinned pack {slots} slots x {sb}", h_sh.data_ptr(), h_out.data_ptr(), dict(env, NP_HOST_ROWS="pack"))
    run(f"pageable staged {slots} slots x {sb}", pg_sh.ctypes.data, pg_out.ctypes.data, env)
ok = bool((pg_out[:, :plen] == h_pay.numpy()).all()) and torch.equal(h_out[:, :plen], h_pay)
print("roundtrip_ok", ok)
