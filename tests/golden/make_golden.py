#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the reference itself.

The reference crate is Rust and cannot run in this image (no cargo/rustc,
SURVEY F1), but it ships the same algorithm as C: cxx/RSErasureCode.c.
oracle/Makefile compiles that file unmodified, by path, into
oracle/_ref/librsec_ref.so.  This script drives it (oracle.np_oracle.RefC)
to produce input/output vectors.  The crate's Rust-only glue (byte packing,
shard transpose, column gather; mod.rs:117-239, inc_encode.rs:165-208,
inc_reconstruct.rs:1-55) is restated below in numpy (`py_encode`,
`py_reconstruct`) on top of the reference C core.

Known-answer values that the reference's own tests hold are recorded in
kat.json with their file:line.

Run (in the container that has /root/reference):
    make -C oracle && python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-novelpoly_amd", "python"))

from np_oracle import RefC  # noqa: E402
from novelpoly_amd import synth  # noqa: E402


def sha(a) -> str:
    if isinstance(a, np.ndarray):
        a = np.ascontiguousarray(a).tobytes()
    return hashlib.sha256(a).hexdigest()


def next_pow2(x):
    p = 1
    while p < x:
        p *= 2
    return p


def prev_pow2(x):
    p = 1
    while p * 2 <= x:
        p *= 2
    return p


def params(n_wanted, k_wanted=None):
    kw = (n_wanted - 1) // 3 + 1 if k_wanted is None else k_wanted
    return next_pow2(n_wanted), prev_pow2(kw)


def pack_chunks(payload: bytes, k: int) -> np.ndarray:
    """Chunk payload into 2k-byte pieces of big-endian symbols (inc_encode.rs:190-197)."""
    nch = (len(payload) + 2 * k - 1) // (2 * k)
    buf = np.zeros(nch * 2 * k, dtype=np.uint8)
    buf[: len(payload)] = np.frombuffer(payload, dtype=np.uint8)
    return buf.view(">u2").astype(np.uint16).reshape(nch, k)


def py_encode(ref: RefC, payload: bytes, n_wanted: int, k_wanted=None):
    n, k = params(n_wanted, k_wanted)
    syms = pack_chunks(payload, k)
    nch = syms.shape[0]
    shards = np.zeros((n_wanted, nch), dtype=np.uint16)
    for c in range(nch):
        cw = ref.encode_low(syms[c], k, n)
        shards[:, c] = cw[:n_wanted]
    return [shards[v].astype(">u2").tobytes() for v in range(n_wanted)]


def py_reconstruct(ref: RefC, received, n_wanted: int, k_wanted=None) -> bytes:
    n, k = params(n_wanted, k_wanted)
    recv = list(received[:n]) + [None] * max(0, n - len(received))
    erased = np.array([s is None for s in recv], dtype=np.uint8)
    first = next(s for s in recv if s is not None)
    nsym = len(first) // 2
    cols = np.zeros((n, nsym), dtype=np.uint16)
    for v, s in enumerate(recv):
        if s is not None:
            cols[v] = np.frombuffer(s, dtype=">u2")
    loc = ref.eval_error_polynomial(erased)
    out = np.zeros((nsym, k), dtype=np.uint16)
    for s in range(nsym):
        col = cols[:, s].copy()
        dec = ref.decode_main(col, k, erased, loc)
        out[s] = np.where(erased[:k] == 1, dec[:k], col[:k])
    return out.astype(">u2").tobytes()


def main():
    ref = RefC()
    rng = np.random.default_rng(0x60_1DE4)

    # ---- tables --------------------------------------------------------------
    tabs = {}
    for name, size in (("LOG_TABLE", 65536), ("EXP_TABLE", 65536), ("skewVec", 65535), ("log_walsh", 65536)):
        t = ref.table(name, size)
        tabs[name] = {"sha256": sha(t.astype("<u2")), "head": t[:16].tolist(), "size": size}
    with open(os.path.join(HERE, "tables.json"), "w") as f:
        json.dump(tabs, f, indent=1)

    # ---- transforms ------------------------------------------------------------
    arrs = {}
    cases = []
    for size in (2, 4, 8, 16, 32, 64, 128, 256, 1024, 4096):
        for index in sorted({0, size, 3 * size, 1 << 12, 65536 - size}):
            if index % size or index + size > 65536:
                continue
            x = rng.integers(0, 65536, size, dtype=np.uint16)
            key = f"s{size}_i{index}"
            arrs[key + "_in"] = x
            arrs[key + "_afft"] = ref.afft(x, size, index)
            arrs[key + "_ifft"] = ref.inverse_afft(x, size, index)
            cases.append([size, index])
    for size in (2, 16, 256, 4096):
        x = rng.integers(0, 65536, size, dtype=np.uint16)
        arrs[f"walsh{size}_in"] = x
        arrs[f"walsh{size}_out"] = ref.walsh(x)
        arrs[f"deriv{size}_in"] = x
        arrs[f"deriv{size}_out"] = ref.formal_derivative(x)
    a = rng.integers(0, 65536, 4096, dtype=np.uint16)
    m = rng.integers(0, 65536, 4096, dtype=np.uint16)
    m[:8] = 65535
    a[8:16] = 0
    arrs["mul_a"], arrs["mul_m"] = a, m
    arrs["mul_out"] = np.array([ref.mul(int(x), int(y)) for x, y in zip(a, m)], dtype=np.uint16)
    arrs["transform_cases"] = np.array(cases, dtype=np.int64)

    # ---- codec (encode_low / error locator / decode_main) ------------------------
    codec = []
    for (n, k) in ((2, 1), (4, 2), (16, 8), (32, 4), (256, 64), (256, 8), (1024, 256), (4096, 1024)):
        d = rng.integers(0, 65536, k, dtype=np.uint16)
        cw = ref.encode_low(d, k, n)
        pres = np.ones(n, dtype=np.uint8)
        pres[rng.choice(n, n - k, replace=False)] = 0
        er = 1 - pres
        loc = ref.eval_error_polynomial(er)
        c = cw.copy()
        c[er == 1] = 0
        dec = ref.decode_main(c, k, er, loc)
        key = f"n{n}_k{k}"
        arrs[key + "_data"] = d
        arrs[key + "_codeword"] = cw
        arrs[key + "_present"] = pres
        arrs[key + "_locator"] = loc[:n]
        arrs[key + "_locator_sha"] = np.frombuffer(bytes.fromhex(sha(loc.astype("<u2"))), dtype=np.uint8)
        arrs[key + "_decoded"] = dec
        codec.append([n, k])
    arrs["codec_cases"] = np.array(codec, dtype=np.int64)
    np.savez_compressed(os.path.join(HERE, "vectors.npz"), **arrs)

    # ---- API-level small cases (RefC core + restated glue) ------------------------
    api = []
    for (n_wanted, plen, seed) in ((2, 1, 1), (3, 10, 2), (4, 2, 3), (4, 100, 4), (10, 16, 5), (16, 4096, 6),
                                   (100, 1, 7), (123, 1337, 8), (2003, 17, 9), (128, 64, 10), (5, 99, 11),
                                   (770, 5120, 12)):
        pl = synth.payload(1000 + seed, plen)
        shards = py_encode(ref, pl, n_wanted)
        n, k = params(n_wanted)
        r = np.random.default_rng(seed)
        keep = sorted(r.choice(n_wanted, size=min(n_wanted, k + (n_wanted - k) // 2), replace=False).tolist())
        received = [shards[i] if i in set(keep) else None for i in range(n_wanted)]
        rec = py_reconstruct(ref, received, n_wanted)
        api.append({"n_wanted": n_wanted, "payload": pl.hex(), "shards": [s.hex() for s in shards],
                    "kept": keep, "reconstructed": rec.hex()})
    with open(os.path.join(HERE, "api_cases.json"), "w") as f:
        json.dump(api, f)

    # ---- BASELINE config digests (payload index 0) ----------------------------------
    digests = {}
    for cid in (1, 2, 3, 4):
        cfg = synth.CONFIGS[cid]
        nw, kw, plen = cfg["n_wanted"], cfg["k_wanted"], cfg["payload"]
        n, k = params(nw, kw)
        assert (n, k) == (cfg["n"], cfg["k"])
        pl = synth.payload(0, plen)
        shards = py_encode(ref, pl, nw, kw)
        ent = {"n": n, "k": k, "n_wanted": nw, "k_wanted": kw, "payload_len": plen, "payload_sha256": sha(pl),
               "shard_len": len(shards[0]), "encode_sha256": sha(b"".join(shards))}
        erase = cfg["erase"] if cfg["erase"] is not None else nw - k
        pres = synth.present_mask(0, n, erase)
        received = [shards[v] if (v < nw and pres[v]) else None for v in range(nw)]
        rec = py_reconstruct(ref, received, nw, kw)
        ent.update({"erase": erase, "present_sha256": sha(pres), "reconstruct_sha256": sha(rec),
                    "reconstruct_len": len(rec), "roundtrip_ok": rec[:plen] == pl})
        digests[f"cfg{cid}"] = ent
        print(cid, ent)
    with open(os.path.join(HERE, "digests.json"), "w") as f:
        json.dump(digests, f, indent=1)
    print("wrote fixtures to", HERE)


if __name__ == "__main__":
    main()
