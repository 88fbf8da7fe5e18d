"""Profiling driver: run only the batched encode (config 3 shape) a few times."""
import os, sys, argparse
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "reed-solomon-novelpoly_amd", "python")]
import torch
import novelpoly_amd as npa
from novelpoly_amd import synth

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=3)
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--iters", type=int, default=3)
ap.add_argument("--what", default="encode")
args = ap.parse_args()
cfg = synth.CONFIGS[args.config]
p = npa.CodeParams.derive_parameters(cfg["n_wanted"], cfg["k_wanted"])
n, k, plen, b = p.n(), p.k(), cfg["payload"], args.batch
ctx = npa.Context(0)
torch.cuda.set_stream(torch.cuda.Stream())
s = torch.cuda.current_stream().cuda_stream
sl = p.make_encoder(ctx).shard_len(plen)
pay = torch.randint(0, 256, (b, plen), dtype=torch.uint8, device="cuda")
sh = torch.empty((b, n, sl), dtype=torch.uint8, device="cuda")
erase = cfg["erase"] if cfg["erase"] is not None else n - k
pres = torch.from_numpy(__import__("numpy").stack([synth.present_mask(i, n, erase) for i in range(b)])).cuda()
loc = torch.empty((b, n), dtype=torch.int16, device="cuda")
out = torch.empty((b, (sl // 2) * 2 * k), dtype=torch.uint8, device="cuda")
for _ in range(args.iters):
    if args.what in ("encode", "all"):
        npa.encode_batch_dev(p, pay.data_ptr(), plen, plen, b, sh.data_ptr(), n * sl, ctx=ctx, stream=s)
    if args.what in ("reconstruct", "all"):
        npa.error_locator_dev(n, pres.data_ptr(), b, loc.data_ptr(), ctx=ctx, stream=s)
        npa.reconstruct_batch_dev2(p, sh.data_ptr(), sl, n * sl, pres.data_ptr(), loc.data_ptr(), b, out.data_ptr(),
                                   out.shape[1], ctx=ctx, stream=s)
torch.cuda.synchronize()
print("done", args)
