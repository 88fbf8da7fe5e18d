"""ctypes bindings for the CPU parity checkers.

TEST INFRASTRUCTURE ONLY: only tests/, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of bench.py may import this module.  The product path
(``libnovelpoly_hip.so`` and its Python mirror) never touches it.

Two checkers are exposed:

* :class:`Oracle` -- our scalar C restatement (``oracle/libnp_oracle.so``),
  whose functions cite the reference file:line they restate (np_oracle.h).
* :class:`RefC` -- the reference's own C implementation
  (``cxx/RSErasureCode.c``) compiled from /root/reference into
  ``oracle/_ref/librsec_ref.so`` by ``oracle/Makefile``.  It is used to pin
  the restatement; it only exists where the reference tree was present at
  build time.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libnp_oracle.so")
REF_PATH = os.path.join(HERE, "_ref", "librsec_ref.so")

FIELD_SIZE = 65536
ONEMASK = 65535

_u16p = np.ctypeslib.ndpointer(dtype=np.uint16, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_sz = C.c_size_t


def build() -> None:
    """Compile the checkers (make -C oracle)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


class Oracle:
    def __init__(self, path: str = LIB_PATH):
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        self.L = L
        L.npo_init.restype = None
        for name in ("npo_log_table", "npo_exp_table", "npo_skews", "npo_log_walsh"):
            getattr(L, name).restype = C.POINTER(C.c_uint16)
        L.npo_mul.argtypes = [C.c_uint16, C.c_uint16]
        L.npo_mul.restype = C.c_uint16
        L.npo_walsh.argtypes = [_u16p, _sz]
        L.npo_afft.argtypes = [_u16p, _sz, _sz]
        L.npo_inverse_afft.argtypes = [_u16p, _sz, _sz]
        L.npo_formal_derivative.argtypes = [_u16p, _sz]
        L.npo_encode_low.argtypes = [_u16p, _sz, _u16p, _sz]
        L.npo_encode_sub.argtypes = [C.c_char_p, _sz, _sz, _sz, _u16p]
        L.npo_encode_sub.restype = C.c_int
        L.npo_eval_error_polynomial.argtypes = [_u8p, _sz, _u16p]
        L.npo_decode_main.argtypes = [_u16p, _sz, _u8p, _u16p, _sz]
        L.npo_recoverability_subset_size.argtypes = [_sz]
        L.npo_recoverability_subset_size.restype = _sz
        L.npo_derive_parameters.argtypes = [_sz, _sz, C.POINTER(_sz), C.POINTER(_sz), C.POINTER(_sz)]
        L.npo_derive_parameters.restype = C.c_int
        L.npo_shard_len.argtypes = [_sz, _sz]
        L.npo_shard_len.restype = _sz
        L.npo_encode.argtypes = [C.c_char_p, _sz, _sz, _sz, _sz, _u8p, _sz]
        L.npo_encode.restype = C.c_int
        L.npo_encode_batch.argtypes = [C.c_void_p, _sz, _sz, _sz, _sz, C.c_void_p]
        L.npo_encode_batch.restype = C.c_int
        for name in ("npo_reconstruct", "npo_reconstruct_from_systematic"):
            f = getattr(L, name)
            f.argtypes = [C.POINTER(C.c_void_p), C.POINTER(_sz), _sz, _sz, _sz, _u8p, _sz, C.POINTER(_sz),
                          C.POINTER(_sz)]
            f.restype = C.c_int
        L.npo_init()

    # tables -----------------------------------------------------------------
    def _tab(self, name: str, size: int) -> np.ndarray:
        p = getattr(self.L, name)()
        return np.ctypeslib.as_array(p, shape=(size,)).copy()

    def log_table(self) -> np.ndarray:
        return self._tab("npo_log_table", FIELD_SIZE)

    def exp_table(self) -> np.ndarray:
        return self._tab("npo_exp_table", FIELD_SIZE)

    def skews(self) -> np.ndarray:
        return self._tab("npo_skews", ONEMASK)

    def log_walsh(self) -> np.ndarray:
        return self._tab("npo_log_walsh", FIELD_SIZE)

    # field / transforms -------------------------------------------------------
    def mul(self, a: int, m: int) -> int:
        return int(self.L.npo_mul(a, m))

    def walsh(self, v: np.ndarray) -> np.ndarray:
        v = np.ascontiguousarray(v, dtype=np.uint16).copy()
        self.L.npo_walsh(v, v.size)
        return v

    def afft(self, v: np.ndarray, size: int, index: int) -> np.ndarray:
        v = np.ascontiguousarray(v, dtype=np.uint16).copy()
        self.L.npo_afft(v, size, index)
        return v

    def inverse_afft(self, v: np.ndarray, size: int, index: int) -> np.ndarray:
        v = np.ascontiguousarray(v, dtype=np.uint16).copy()
        self.L.npo_inverse_afft(v, size, index)
        return v

    def formal_derivative(self, v: np.ndarray) -> np.ndarray:
        v = np.ascontiguousarray(v, dtype=np.uint16).copy()
        self.L.npo_formal_derivative(v, v.size)
        return v

    def encode_low(self, data: np.ndarray, k: int, n: int) -> np.ndarray:
        d = np.zeros(n, dtype=np.uint16)
        d[: len(data)] = data
        cw = np.zeros(n, dtype=np.uint16)
        self.L.npo_encode_low(d, k, cw, n)
        return cw

    def encode_sub(self, data: bytes, n: int, k: int) -> np.ndarray:
        cw = np.zeros(n, dtype=np.uint16)
        st = self.L.npo_encode_sub(bytes(data), len(data), n, k, cw)
        if st:
            raise ValueError(f"encode_sub status {st}")
        return cw

    def eval_error_polynomial(self, erasures) -> np.ndarray:
        er = np.ascontiguousarray(np.asarray(erasures, dtype=np.uint8))
        out = np.zeros(FIELD_SIZE, dtype=np.uint16)
        self.L.npo_eval_error_polynomial(er, er.size, out)
        return out

    def decode_main(self, codeword: np.ndarray, k: int, erasures, locator: np.ndarray) -> np.ndarray:
        cw = np.ascontiguousarray(codeword, dtype=np.uint16).copy()
        er = np.ascontiguousarray(np.asarray(erasures, dtype=np.uint8))
        self.L.npo_decode_main(cw, k, er, np.ascontiguousarray(locator, dtype=np.uint16), cw.size)
        return cw

    # API glue -----------------------------------------------------------------
    def recoverability_subset_size(self, n: int) -> int:
        return int(self.L.npo_recoverability_subset_size(n))

    def derive_parameters(self, n: int, k: int):
        a, b, c = _sz(), _sz(), _sz()
        st = self.L.npo_derive_parameters(n, k, C.byref(a), C.byref(b), C.byref(c))
        return st, (a.value, b.value, c.value)

    def shard_len(self, k: int, payload_len: int) -> int:
        return int(self.L.npo_shard_len(k, payload_len))

    def encode(self, payload: bytes, n: int, k: int, wanted_n: int):
        sl = self.shard_len(k, len(payload)) if payload else 0
        out = np.zeros(max(1, wanted_n * sl), dtype=np.uint8)
        st = self.L.npo_encode(bytes(payload), len(payload), n, k, wanted_n, out, sl)
        if st:
            return st, None
        return 0, [out[v * sl:(v + 1) * sl].tobytes() for v in range(wanted_n)]

    def encode_batch(self, payloads: np.ndarray, n: int, k: int) -> np.ndarray:
        """payloads: (batch, len) uint8 -> (batch, n, shard_len) uint8 (single thread)."""
        payloads = np.ascontiguousarray(payloads, dtype=np.uint8)
        b, ln = payloads.shape
        sl = self.shard_len(k, ln)
        out = np.empty((b, n, sl), dtype=np.uint8)
        st = self.L.npo_encode_batch(payloads.ctypes.data, ln, b, n, k, out.ctypes.data)
        if st:
            raise ValueError(f"encode_batch status {st}")
        return out

    def _shard_call(self, fn, shards, n: int, k: int):
        m = len(shards)
        ptrs = (C.c_void_p * max(1, m))()
        lens = (_sz * max(1, m))()
        keep = []
        maxsyms = 0
        for i, s in enumerate(shards):
            if s is None:
                ptrs[i] = None
                lens[i] = 0
            else:
                b = C.create_string_buffer(bytes(s), max(1, len(s)))
                keep.append(b)
                ptrs[i] = C.cast(b, C.c_void_p)
                lens[i] = len(s)
                maxsyms = max(maxsyms, (len(s) + 1) // 2)
        cap = max(1, maxsyms * 2 * k)
        out = np.zeros(cap, dtype=np.uint8)
        olen = _sz()
        det = (_sz * 3)()
        st = fn(ptrs, lens, m, n, k, out, cap, C.byref(olen), det)
        if st:
            return st, tuple(det)
        return 0, out[: olen.value].tobytes()

    def reconstruct(self, shards, n: int, k: int):
        return self._shard_call(self.L.npo_reconstruct, shards, n, k)

    def reconstruct_from_systematic(self, shards, n: int, k: int):
        return self._shard_call(self.L.npo_reconstruct_from_systematic, shards, n, k)


class RefC:
    """The reference's cxx/RSErasureCode.c, compiled unmodified (oracle/Makefile)."""

    def __init__(self, path: str = REF_PATH):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        L = C.CDLL(path)
        self.L = L
        L.setup.restype = None
        L.setup()
        L.mulE.argtypes = [C.c_uint16, C.c_uint16]
        L.mulE.restype = C.c_uint16
        L.walsh.argtypes = [_u16p, C.c_int]
        L.FLT.argtypes = [_u16p, C.c_int, C.c_int]
        L.IFLT.argtypes = [_u16p, C.c_int, C.c_int]
        L.formal_derivative.argtypes = [_u16p, C.c_int]
        L.encodeL.argtypes = [_u16p, C.c_int, _u16p, C.c_int]
        L.decode_init.argtypes = [_i32p, _u16p, C.c_int]
        L.decode_main.argtypes = [_u16p, C.c_int, _i32p, _u16p, C.c_int]

    def table(self, name: str, size: int) -> np.ndarray:
        arr = (C.c_uint16 * size).in_dll(self.L, name)
        return np.ctypeslib.as_array(arr).copy()

    def mul(self, a: int, m: int) -> int:
        return int(self.L.mulE(a, m))

    def walsh(self, v):
        v = np.ascontiguousarray(v, dtype=np.uint16).copy()
        self.L.walsh(v, v.size)
        return v

    def afft(self, v, size, index):
        v = np.ascontiguousarray(v, dtype=np.uint16).copy()
        self.L.FLT(v, size, index)
        return v

    def inverse_afft(self, v, size, index):
        v = np.ascontiguousarray(v, dtype=np.uint16).copy()
        self.L.IFLT(v, size, index)
        return v

    def formal_derivative(self, v):
        v = np.ascontiguousarray(v, dtype=np.uint16).copy()
        self.L.formal_derivative(v, v.size)
        return v

    def encode_low(self, data, k, n):
        d = np.zeros(n, dtype=np.uint16)
        d[: len(data)] = data
        cw = np.zeros(n, dtype=np.uint16)
        self.L.encodeL(d, k, cw, n)
        return cw

    def eval_error_polynomial(self, erasures):
        er = np.zeros(FIELD_SIZE, dtype=np.int32)
        e = np.asarray(erasures, dtype=np.int32)
        er[: e.size] = e
        out = np.zeros(FIELD_SIZE, dtype=np.uint16)
        self.L.decode_init(er, out, FIELD_SIZE)
        return out

    def decode_main(self, codeword, k, erasures, locator):
        cw = np.ascontiguousarray(codeword, dtype=np.uint16).copy()
        er = np.zeros(FIELD_SIZE, dtype=np.int32)
        e = np.asarray(erasures, dtype=np.int32)
        er[: e.size] = e
        self.L.decode_main(cw, k, er, np.ascontiguousarray(locator, dtype=np.uint16), cw.size)
        return cw


def ref_available() -> bool:
    return os.path.exists(REF_PATH)
