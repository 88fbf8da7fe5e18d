"""Debug helper: compare the GPU encode against the oracle on several shapes."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "reed-solomon-novelpoly_amd", "python")]
import numpy as np
import novelpoly_amd as npa
import np_oracle
from novelpoly_amd import synth

o = np_oracle.Oracle()
ctx = npa.default_context(0)
cases = [(256, 86, 128 * 256), (256, 86, 128 * 300), (256, 86, 128 * 10), (512, 100, 128 * 256),
         (1024, 342, 512 * 256), (1024, 342, 512 * 10), (1024, 342, 512 * 512), (300, 100, 77777),
         (512, 128, 256 * 256), (1024, 256, 512 * 256)]
for nw, kw, plen in cases:
    p = npa.CodeParams.derive_parameters(nw, kw)
    rs = p.make_encoder(ctx)
    pl = synth.payload(nw + plen, plen)
    got = rs.encode(pl)
    st, want = o.encode(pl, p.n(), p.k(), nw)
    bad = [v for v in range(nw) if got[v] != want[v]]
    msg = "OK" if not bad else f"BAD rows {len(bad)} first {bad[:8]}"
    if bad:
        v = bad[0]
        g = np.frombuffer(got[v], ">u2"); w = np.frombuffer(want[v], ">u2")
        cols = np.nonzero(g != w)[0]
        msg += f" row {v}: {len(cols)} cols differ, first {cols[:8].tolist()}"
    print(f"n_wanted={nw} k_wanted={kw} (n={p.n()} k={p.k()}) len={plen} fast={p.is_faster8()}: {msg}", flush=True)
