"""CPU tests: the oracle (C restatement) against the reference's own C build,
the golden fixtures generated from it, and the known-answer tests of the
reference test-suite (paths relative to /root/reference/reed-solomon-novelpoly)."""
import hashlib

import numpy as np
import pytest

from novelpoly_amd import synth


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


# ---------------------------------------------------------------- tables ----
def test_tables_match_golden(oracle, golden_json):
    tabs = golden_json("tables.json")
    assert sha(oracle.log_table().astype("<u2")) == tabs["LOG_TABLE"]["sha256"]
    assert sha(oracle.exp_table().astype("<u2")) == tabs["EXP_TABLE"]["sha256"]
    assert sha(oracle.skews().astype("<u2")) == tabs["skewVec"]["sha256"]
    assert sha(oracle.log_walsh().astype("<u2")) == tabs["log_walsh"]["sha256"]


def test_table_sentinels(oracle):
    # LOG[0]=65535, EXP[0]=EXP[65535]=1, 16 skip sentinels at 2^m-1
    log, exp, sk = oracle.log_table(), oracle.exp_table(), oracle.skews()
    assert log[0] == 65535 and exp[0] == 1 and exp[65535] == 1
    assert sorted(np.nonzero(sk == 65535)[0].tolist()) == [(1 << m) - 1 for m in range(16)]


def test_skews_are_cantor_points(oracle):
    # Structural fact used by the kernels: additive skew of group t at level d
    # (index 0) is the field element with Cantor coordinates 2t.
    sk, exp = oracle.skews(), oracle.exp_table()
    add = np.where(sk == 65535, 0, exp[sk]).astype(np.int64)
    for m in range(15):
        d = 1 << m
        t = np.arange((65535 // d + 1) // 2)
        idx = (2 * t + 1) * d - 1
        idx = idx[idx < 65535]
        assert np.array_equal(add[idx], 2 * t[: idx.size])


def test_cantor_basis():
    # inc_log_mul.rs:236-246: BASE[i] == BASE[i+1]^2 + BASE[i+1] over GF(2)[x]/(x^16+x^5+x^3+x^2+1)
    base = [1, 44234, 15374, 5694, 50562, 60718, 37196, 16402, 27800, 4312, 27250, 47360, 64952, 64308, 65336,
            39198]

    def mulpoly(a, b):
        r = 0
        for i in range(16):
            if (b >> i) & 1:
                r ^= a << i
        for i in range(30, 15, -1):
            if r & (1 << i):
                r ^= 0x1002D << (i - 16)
        return r

    for a, b in zip(base, base[1:]):
        assert a == mulpoly(b, b) ^ b


# ----------------------------------------------------------- field / KAT ----
def test_mul_kat(oracle):
    # faster8/f2e16.rs:394-402 single_operation_works
    xor = [0x798b, 0x9284, 0x43ae, 0x0489, 0x4037, 0x8943, 0x9527, 0x3c5f]
    val = [0x104a, 0x371e, 0x2213, 0x4006, 0x0000, 0x2b5a, 0x10ec, 0xac45]
    exp = [0xe41e, 0xfdbb, 0xca9c, 0x5e82, 0x4037, 0xa969, 0x08c6, 0x2081]
    assert [x ^ oracle.mul(v, 0x0808) for x, v in zip(xor, val)] == exp
    # faster8/f2e16.rs:405-420 regression pairs: plain mul reference values
    for a, m in [(0x0003, 20182), (0xFA1C, 63493), (0, 1), (1, 0), (0x16e7, 18124), (0x3d3d, 15677)]:
        assert oracle.mul(a, m) == (0 if a == 0 else oracle.exp_table()[(int(oracle.log_table()[a]) + m) % 65535])


def test_mul_golden(oracle, golden_vectors):
    g = golden_vectors
    got = np.array([oracle.mul(int(a), int(m)) for a, m in zip(g["mul_a"], g["mul_m"])], dtype=np.uint16)
    assert np.array_equal(got, g["mul_out"])


def test_mul_is_linear(oracle):
    # multiplication by a fixed multiplier is GF(2)-linear
    rng = np.random.default_rng(6)
    for _ in range(2000):
        a, b, m = (int(x) for x in rng.integers(0, 65536, 3))
        assert oracle.mul(a ^ b, m) == oracle.mul(a, m) ^ oracle.mul(b, m)


# -------------------------------------------------------------- transforms ----
def test_transforms_golden(oracle, golden_vectors):
    g = golden_vectors
    for size, index in g["transform_cases"]:
        key = f"s{size}_i{index}"
        x = g[key + "_in"]
        assert np.array_equal(oracle.afft(x, size, index), g[key + "_afft"]), key
        assert np.array_equal(oracle.inverse_afft(x, size, index), g[key + "_ifft"]), key


def test_walsh_and_derivative_golden(oracle, golden_vectors):
    g = golden_vectors
    for size in (2, 16, 256, 4096):
        assert np.array_equal(oracle.walsh(g[f"walsh{size}_in"]), g[f"walsh{size}_out"])
        assert np.array_equal(oracle.formal_derivative(g[f"deriv{size}_in"]), g[f"deriv{size}_out"])


def test_flt_roundtrip_small(oracle):
    # tests.rs:309-327 and RSErasureCode.c:349-370
    exp = np.array([1, 2, 3, 5, 8, 13, 21, 44, 65, 0, 0xFFFF, 2, 3, 5, 7, 11], dtype=np.uint16)
    y = oracle.afft(exp, 16, 4)
    assert not np.array_equal(y, exp)
    assert np.array_equal(oracle.inverse_afft(y, 16, 4), exp)


def test_flt_back_and_forth(oracle):
    # tests.rs:66-81 (N=128, index N/4)
    rng = np.random.default_rng(66)
    x = rng.integers(0, 65536, 128, dtype=np.uint16)
    y = oracle.afft(x, 128, 32)
    assert (y != x).any()
    assert np.array_equal(oracle.inverse_afft(y, 128, 32), x)


def test_oracle_vs_reference_c_random(oracle, refc):
    rng = np.random.default_rng(123)
    for size in (2, 8, 64, 512, 2048):
        for index in (0, size, 5 * size):
            x = rng.integers(0, 65536, size, dtype=np.uint16)
            assert np.array_equal(oracle.afft(x, size, index), refc.afft(x, size, index))
            assert np.array_equal(oracle.inverse_afft(x, size, index), refc.inverse_afft(x, size, index))
    for n, k in ((16, 4), (64, 16), (512, 128)):
        d = rng.integers(0, 65536, k, dtype=np.uint16)
        assert np.array_equal(oracle.encode_low(d, k, n), refc.encode_low(d, k, n))
        er = (rng.random(n) < 0.5).astype(np.uint8)
        assert np.array_equal(oracle.eval_error_polynomial(er), refc.eval_error_polynomial(er))


# ------------------------------------------------------------------- codec ----
def test_codec_golden(oracle, golden_vectors):
    g = golden_vectors
    for n, k in g["codec_cases"]:
        key = f"n{n}_k{k}"
        d = g[key + "_data"]
        cw = oracle.encode_low(d, k, n)
        assert np.array_equal(cw, g[key + "_codeword"]), key
        er = 1 - g[key + "_present"]
        loc = oracle.eval_error_polynomial(er)
        assert np.array_equal(loc[:n], g[key + "_locator"]), key
        assert hashlib.sha256(loc.astype("<u2").tobytes()).digest() == g[key + "_locator_sha"].tobytes()
        c = cw.copy()
        c[er == 1] = 0
        dec = oracle.decode_main(c, k, er, loc)
        assert np.array_equal(dec, g[key + "_decoded"]), key
        rec = np.where(er[:k] == 1, dec[:k], c[:k])
        assert np.array_equal(rec, d), key


def test_ported_c_test(oracle):
    # tests.rs:329-419: N=256, K=8, data[i]=i*i%65535, first N-K erased
    n, k = 256, 8
    data = np.array([i * i % 65535 for i in range(k)], dtype=np.uint16)
    cw = oracle.encode_low(data, k, n)
    er = np.zeros(n, dtype=np.uint8)
    er[: n - k] = 1
    cw[er == 1] = 0
    loc = oracle.eval_error_polynomial(er)
    dec = oracle.decode_main(cw, k, er, loc)
    assert np.array_equal(dec[:k], data)


def test_sub_encode_decode(oracle):
    # tests.rs:83-113: N=32, K=4, erase {0,1,2,29,30,31}
    n, k = 32, 4
    data = bytes(range(7, 7 + 2 * k))
    cw = oracle.encode_sub(data, n, k)
    er = np.zeros(n, dtype=np.uint8)
    er[[0, 1, 2, n - 3, n - 2, n - 1]] = 1
    c = cw.copy()
    c[er == 1] = 0
    dec = oracle.decode_main(c, k, er, oracle.eval_error_polynomial(er))
    rec = np.where(er[:k] == 1, dec[:k], c[:k]).astype(">u2").tobytes()
    assert rec == data


def test_systematic_for_sure(oracle):
    # lib.rs:47-56
    cw = oracle.encode_sub(bytes([1, 2, 3, 4]), 8, 4)
    assert cw[:2].astype(">u2").tobytes() == bytes([1, 2, 3, 4])


# ------------------------------------------------------------------- glue ----
def test_api_cases_oracle(oracle, golden_json):
    for case in golden_json("api_cases.json"):
        nw = case["n_wanted"]
        st, (n, k, wn) = oracle.derive_parameters(nw, oracle.recoverability_subset_size(nw))
        assert st == 0
        pl = bytes.fromhex(case["payload"])
        st, shards = oracle.encode(pl, n, k, wn)
        assert st == 0
        assert [s.hex() for s in shards] == case["shards"]
        keep = set(case["kept"])
        recv = [shards[i] if i in keep else None for i in range(nw)]
        st, rec = oracle.reconstruct(recv, n, k)
        assert st == 0
        assert rec.hex() == case["reconstructed"]
        assert rec[: len(pl)] == pl


@pytest.mark.parametrize("cid", [1, 2])
def test_config_digests_oracle(oracle, golden_json, cid):
    d = golden_json("digests.json")[f"cfg{cid}"]
    n, k, nw = d["n"], d["k"], d["n_wanted"]
    pl = synth.payload(0, d["payload_len"])
    assert hashlib.sha256(pl).hexdigest() == d["payload_sha256"]
    st, shards = oracle.encode(pl, n, k, nw)
    assert st == 0 and hashlib.sha256(b"".join(shards)).hexdigest() == d["encode_sha256"]
    pres = synth.present_mask(0, n, d["erase"])
    assert hashlib.sha256(pres.tobytes()).hexdigest() == d["present_sha256"]
    st, rec = oracle.reconstruct([shards[v] if pres[v] else None for v in range(nw)], n, k)
    assert st == 0 and hashlib.sha256(rec).hexdigest() == d["reconstruct_sha256"]


def test_glue_errors(oracle):
    # mod.rs:118-120, 178-180, 195-197, 200-211; errors.rs:4-28 numbering
    assert oracle.encode(b"", 16, 4, 16)[0] == 4  # PayloadSizeIsZero
    st, shards = oracle.encode(bytes(range(40)), 16, 4, 16)
    recv = [shards[0], None, None] + [None] * 13
    assert oracle.reconstruct(recv, 16, 4) == (5, (1, 4, 16))  # NeedMoreShards{have,min,all}
    recv = [b""] * 4 + [None] * 12
    assert oracle.reconstruct(recv, 16, 4)[0] == 8  # EmptyShard
    recv = list(shards[:3]) + [shards[3][:-2]] + [None] * 12
    assert oracle.reconstruct(recv, 16, 4) == (7, (shards[0].__len__() // 2, len(shards[3]) // 2 - 1, 0))
    assert oracle.reconstruct_from_systematic([], 16, 4)[0] == 5
    assert oracle.reconstruct_from_systematic(shards[:3], 16, 4) == (5, (3, 4, 16))


@pytest.mark.parametrize("n", [16, 256, 1024, 4096])
def test_locator_fold_identity(oracle, n):
    """SURVEY F8, used by the fused locator of the fast reconstruct kernel: for an
    erasure set inside [0, n) the 65536-point Walsh pair of eval_error_polynomial
    equals two n-point Walsh transforms around the folded LOG_WALSH, mod 65535."""
    lw = oracle.log_walsh().astype(np.int64)
    fold = lw.reshape(-1, n).sum(axis=0) % 65535

    def wht(v):
        v = v.copy()
        h = 1
        while h < len(v):
            v = v.reshape(-1, 2, h)
            a, b = v[:, 0, :].copy(), v[:, 1, :].copy()
            v[:, 0, :], v[:, 1, :] = a + b, a - b
            v = v.reshape(-1)
            h *= 2
        return v

    rng = np.random.default_rng(n)
    for trial in range(6):
        erased = rng.random(n) < (0.05, 0.33, 0.67, 0.0, 0.9, 0.5)[trial]
        want = oracle.eval_error_polynomial(erased.tolist())[:n].astype(np.int64)
        loc = wht((wht(erased.astype(np.int64)) % 65535) * fold % 65535) % 65535
        loc = np.where(erased, (65535 - loc) % 65535, loc)
        assert np.array_equal(loc % 65535, want % 65535), trial


def test_corrupted_row_beyond_prefix_changes_reference(oracle):
    """Pins that tests/test_gpu_noncodeword.py's corrupted-row case is
    meaningful: at config 3 the reference's reconstruct output depends on a
    present row >= 2k even when [0, 2k) holds k present rows, so a decoder that
    reads only the first 2k rows cannot match it on non-codeword input."""
    import numpy as np
    from novelpoly_amd import synth

    n, k, sl = 1024, 256, 64
    rng = np.random.default_rng(3)
    rows = rng.integers(0, 256, (n, sl), dtype=np.uint8)
    pres = synth.present_mask(0, n, 341)
    assert pres[: 2 * k].sum() >= k
    recv = lambda: [rows[i].tobytes() if pres[i] else None for i in range(n)]  # noqa: E731
    st, a = oracle.reconstruct(recv(), n, k)
    v = [i for i in range(2 * k, n) if pres[i]][0]
    rows[v] ^= 0xFF
    st2, b = oracle.reconstruct(recv(), n, k)
    assert st == st2 == 0 and a != b


def test_rec8_kappa(oracle):
    """The n = 8k decode folds the top inverse levels and the derivative's
    single-bit terms into one coefficient per segment (kernels_fast.hip
    rec8_kappa): d = D_K(x0) ^ sum_q kappa_q x_q equals the first K entries of
    formal_derivative(inverse_afft(a, n, 0)) (inc_reconstruct.rs:76-78) for
    random inputs; and the constants in the kernel source are these."""
    import os
    import re

    import numpy as np

    src = open(os.path.join(os.path.dirname(__file__), "..", "reed-solomon-novelpoly_amd", "csrc",
                            "kernels_fast.hip")).read()
    kappa = [int(v) for v in re.search(r"constexpr uint32_t k\[8\] = \{([^}]*)\}", src).group(1).split(",")]
    rng = np.random.default_rng(8)
    for K in (8, 16):
        n = 8 * K
        for _ in range(5):
            a = rng.integers(0, 65536, n, dtype=np.uint16)
            want = oracle.formal_derivative(oracle.inverse_afft(a.copy(), n, 0))[:K]
            xs = [oracle.inverse_afft(a[q * K:(q + 1) * K].copy(), K, q * K) for q in range(8)]
            d = oracle.formal_derivative(xs[0].copy()).astype(np.uint16)
            for q in range(8):
                m = oracle.log_table()[kappa[q]]  # mul by the element kappa_q: log form
                d ^= np.array([oracle.mul(int(x), int(m)) for x in xs[q]], dtype=np.uint16)
            assert np.array_equal(d, want)
