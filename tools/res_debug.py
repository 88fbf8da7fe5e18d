"""GPU box: encode one 64-column tile at n = 4096, k = 1024 with experiment
builds that skip level sets of kernels_res.hip (NP_EXP bits 8-10), against a
numpy model of the transforms restricted to the same levels (field level:
the tower coordinates cancel).  Reports which row blocks differ."""
import ctypes as C
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


def mul_add(x, c):
    r = EXP[(LOG[x] + LOG[c]) % 65535]
    return np.where((x == 0) | (c == 0), 0, r)


def transform(v, index, levels, inverse):
    v = v.copy()  # [positions, columns]
    size = v.shape[0]
    order = sorted(levels) if inverse else sorted(levels, reverse=True)
    for b in order:
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


def model(payload, levels, flevels=None):
    cols = np.frombuffer(payload, dtype=">u2").astype(np.int64).reshape(64, 1024).T  # [pos, col]
    m = transform(cols, 0, levels, True)
    rows = [cols]
    for s in range(1, 4):
        rows.append(transform(m, 1024 * s, levels if flevels is None else flevels, False))
    return np.concatenate(rows)  # [4096, 64]


def run(libpath, payload):
    env = dict(os.environ, NP_LIB_PATH=libpath)
    code = f"""
import sys, numpy as np
sys.path.insert(0, {os.path.join(ROOT, 'reed-solomon-novelpoly_amd', 'python')!r})
import novelpoly_amd as npa
p = npa.CodeParams.derive_parameters(4096, 1366)
sh = npa.encode(open(sys.argv[1], 'rb').read(), 4096)
np.save(sys.argv[2], np.stack([np.frombuffer(x, dtype='>u2') for x in sh]).astype(np.int64))
"""
    open("/tmp/pl.bin", "wb").write(payload)
    subprocess.run([sys.executable, "-c", code, "/tmp/pl.bin", "/tmp/rows.npy"], check=True, env=env, timeout=300)
    return np.load("/tmp/rows.npy")  # [4096 rows, 64 symbols]


payload = np.random.default_rng(5).integers(0, 256, 2048 * 64, dtype=np.uint8).tobytes()
variants = {"base": (list(range(10)), "reed-solomon-novelpoly_amd/lib/libnovelpoly_hip.so")}
for name, skip in (("cq", 256 | 512 | 1024), ("ha", 256 | 1024), ("hd", 256 | 512), ("all", 1)):
    pass
for name, levels in (("onlycq", [0, 1, 2, 3]), ("cqinv", ([0, 1, 2, 3], [])), ("cqfwd", ([], [0, 1, 2, 3]))):
    variants[name] = (levels, f"dbg/lib_{name}.so")
for name, (levels, lib) in variants.items():
    got = run(os.path.join(ROOT, lib), payload)
    want = model(payload, *levels) if isinstance(levels, tuple) else model(payload, levels)
    for blk in range(1, 4):
        d = got[1024 * blk:1024 * (blk + 1)] != want[1024 * blk:1024 * (blk + 1)]
        print("  block", blk, "mismatch by u:", [int(d[[p for p in range(1024) if (p >> 4) & 3 == u]].sum()) for u in range(4)],
              "by p&15:", [int(d[[p for p in range(1024) if p & 15 == i]].sum()) for i in range(16)])
    bad = [(blk, int((got[1024 * blk:1024 * (blk + 1)] != want[1024 * blk:1024 * (blk + 1)]).sum()))
           for blk in range(4)]
    print(name, "mismatching symbols per row block:", bad, flush=True)
