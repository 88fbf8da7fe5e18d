"""GPU box: reconstruct one 64-column tile at n = 2048 or 4096, k = 1024
with an experiment build (NP_EXP bit 8192: the kernel writes the accumulated
d = D(x0) ^ sum kappa_q x_q, in tower coordinates, instead of decoding) and
compares it with a numpy model of that algebra (kernels_res.hip)."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "reed-solomon-novelpoly_amd", "python")]
import np_oracle  # noqa: E402

o = np_oracle.Oracle()
LOG = o.log_table().astype(np.int64)
EXP = o.exp_table().astype(np.int64)
TOWER_A = [0, 207, 171, 33, 138, 157, 39, 31]


def mul_add(x, c):
    r = EXP[(LOG[x] + LOG[c]) % 65535]
    return np.where((x == 0) | (c == 0), 0, r)


def to_tower(x):
    lo = x & 0xFF
    for i in range(8):
        lo = lo ^ np.where((x >> (8 + i)) & 1, TOWER_A[i], 0)
    return (x & 0xFF00) | lo


def transform(v, index, inverse):
    v = v.copy()
    size = v.shape[0]
    levels = range(int(np.log2(size)))
    for b in (levels if inverse else reversed(levels)):
        d = 1 << b
        for g in range(size // (2 * d)):
            c = 2 * g + (index >> b)
            x = v[2 * d * g:2 * d * g + d]
            y = v[2 * d * g + d:2 * d * (g + 1)]
            if inverse:
                y ^= x
                x ^= mul_add(y, np.full_like(y, c))
            else:
                x ^= mul_add(y, np.full_like(y, c))
                y ^= x
    return v


def transform_levels(v, index, levels):  # inverse levels only
    v = v.copy()
    for b in sorted(levels):
        d = 1 << b
        for g in range(v.shape[0] // (2 * d)):
            c = 2 * g + (index >> b)
            x = v[2 * d * g:2 * d * g + d]
            y = v[2 * d * g + d:2 * d * (g + 1)]
            y ^= x
            x ^= mul_add(y, np.full_like(y, c))
    return v


def deriv(v):
    size = v.shape[0]
    out = v.copy()
    for b in range(int(np.log2(size))):
        l = 1 << b
        for j in range(size):
            if not j & l:
                out[j] ^= v[j | l]
    return out


n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
mode = sys.argv[2] if len(sys.argv) > 2 else "d"  # d: accumulated d; pm: first step premultiplied; cq: + CQ levels
k, NQ = 1024, n // 1024
rng = np.random.default_rng(7)
sl = 128  # 64 symbols per shard: one tile
shards = rng.integers(0, 256, (n, sl), dtype=np.uint8)
pres = np.ones(n, np.uint8)
pres[rng.choice(n, n - k - 5, replace=False)] = 0
pres[:k][rng.integers(0, k)] = 0  # at least one systematic row missing: a decode
np.save("/tmp/sh.npy", shards)
np.save("/tmp/pr.npy", pres)
code = f"""
import sys, numpy as np, torch
sys.path.insert(0, {os.path.join(ROOT, 'reed-solomon-novelpoly_amd', 'python')!r})
import novelpoly_amd as npa
p = npa.CodeParams.derive_parameters({n}, {n // 3 + 1 if n == 4096 else 1024})
sh = torch.from_numpy(np.load('/tmp/sh.npy')).cuda()
pr = torch.from_numpy(np.load('/tmp/pr.npy')).cuda()
out = torch.zeros(({sl} // 2) * 2 * 1024, dtype=torch.uint8, device='cuda')
npa.reconstruct_batch_dev2(p, sh.data_ptr(), {sl}, {n} * {sl}, pr.data_ptr(), 0, 1, out.data_ptr(), out.numel())
torch.cuda.synchronize()
np.save('/tmp/out.npy', out.cpu().numpy())
"""
env = dict(os.environ, NP_LIB_PATH=os.path.join(ROOT, "dbg", f"lib_dump{mode}.so"))
subprocess.run([sys.executable, "-c", code], check=True, env=env, timeout=300)
got = np.load("/tmp/out.npy").view(">u2").astype(np.int64).reshape(64, 1024).T  # [pos, col]

loc = o.eval_error_polynomial((pres == 0).astype(np.uint8)).astype(np.int64)
recv = shards.view(">u2").astype(np.int64)  # [row, col]
E = EXP[loc[:n] % 65535]
pm = np.where(pres[:, None] != 0, mul_add(recv, E[:, None] * np.ones_like(recv)), 0)
q0 = 1 if NQ == 2 else 2  # the first step's segment
if mode == "pm":
    want = to_tower(pm[1024 * q0:1024 * (q0 + 1)])
elif mode == "cq":
    want = to_tower(transform_levels(pm[1024 * q0:1024 * (q0 + 1)], 1024 * q0, [0, 1, 2, 3]))
xs = [transform(pm[1024 * q:1024 * (q + 1)], 1024 * q, True) for q in range(NQ)]
if mode != "d":
    pass
elif NQ == 2:
    d = deriv(xs[0]) ^ xs[0] ^ xs[1]
else:
    b = 2
    d = deriv(xs[0]) ^ xs[1] ^ xs[2] ^ mul_add(xs[2] ^ xs[3], np.full_like(xs[2], b))
if mode == "d":
    want = to_tower(d)
bad = got != want
print("n", n, "mismatch", int(bad.sum()), "of", bad.size)
if bad.any():
    ps = np.flatnonzero(bad.any(axis=1))
    print("positions (first 32):", ps[:32].tolist())
    print("by p&3:", [int(bad[p::4].sum()) for p in range(4)], "by (p>>2)&15:", [int(bad[[q for q in range(1024) if (q >> 2) & 15 == i]].sum()) for i in range(16)])
    print("by p>>6:", [int(bad[64 * i:64 * (i + 1)].sum()) for i in range(16)])
    # also test the model pieces without the derivative
    for name, alt in (("no D", (xs[0] ^ xs[1]) if NQ == 2 else None),):
        if alt is not None:
            print(name, "mismatch", int((got != to_tower(alt)).sum()))
