"""Python mirror of the reed-solomon-novelpoly crate surface over the C ABI.

This is plumbing for tests and the bench: every call goes through
``libnovelpoly_hip.so`` (include/novelpoly.h), whose work runs in HIP kernels
on a gfx950 GPU.  There is no CPU fallback: if the library is missing or no
MI355X is visible, calls raise.

Names follow the crate (paths relative to /root/reference/reed-solomon-novelpoly):

* :func:`encode` / :func:`reconstruct`        -- src/novel_poly_basis/{encode,reconstruct}.rs
* :class:`CodeParams`, :class:`ReedSolomon`    -- src/novel_poly_basis/mod.rs:24-285
* :class:`WrappedShard`                        -- src/wrapped_shard.rs
* :class:`Error` and its variants              -- src/errors.rs:4-28
* :func:`recoverablity_subset_size` etc.       -- src/util.rs
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from typing import List, Optional, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.abspath(os.path.join(_HERE, "..", ".."))
# NP_LIB_PATH: an experiment build of the same library (tools/exp_variants.sh)
LIB_PATH = os.environ.get("NP_LIB_PATH") or os.path.join(PKG_ROOT, "lib", "libnovelpoly_hip.so")
FIELD_SIZE = 65536

_sz = C.c_size_t
_lib = None
_lib_lock = threading.Lock()


class _Params(C.Structure):
    _fields_ = [("n", _sz), ("k", _sz), ("wanted_n", _sz)]


def lib() -> C.CDLL:
    """Load libnovelpoly_hip.so (fails loudly if it was not built)."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built; run `make -C {PKG_ROOT}` (hipcc, gfx950)")
        L = C.CDLL(LIB_PATH)
        P = C.POINTER(_Params)
        vp = C.c_void_p
        sig = {
            "np_last_error_detail": (None, [C.POINTER(_sz)]),
            "np_last_error_site": (C.c_char_p, []),
            "np_status_message": (C.c_char_p, [C.c_int]),
            "np_version": (C.c_char_p, []),
            "np_recoverability_subset_size": (_sz, [_sz]),
            "np_derive_parameters": (C.c_int, [_sz, _sz, P]),
            "np_params_new": (C.c_int, [_sz, _sz, _sz, P]),
            "np_shard_len": (_sz, [P, _sz]),
            "np_is_fast_path": (C.c_int, [P]),
            "np_ctx_create": (C.c_int, [C.c_int, C.POINTER(vp)]),
            "np_ctx_destroy": (None, [vp]),
            "np_ctx_stream": (vp, [vp]),
            "np_ctx_device": (C.c_int, [vp]),
            "np_ctx_synchronize": (C.c_int, [vp]),
            "np_encode": (C.c_int, [vp, C.c_char_p, _sz, _sz, vp, _sz]),
            "np_rs_encode": (C.c_int, [vp, P, C.c_char_p, _sz, vp, _sz]),
            "np_reconstruct": (C.c_int, [vp, C.POINTER(vp), C.POINTER(_sz), _sz, _sz, vp, _sz, C.POINTER(_sz)]),
            "np_rs_reconstruct": (C.c_int, [vp, P, C.POINTER(vp), C.POINTER(_sz), _sz, vp, _sz, C.POINTER(_sz)]),
            "np_rs_reconstruct_from_systematic": (
                C.c_int, [vp, P, C.POINTER(vp), C.POINTER(_sz), _sz, vp, _sz, C.POINTER(_sz)]),
            "np_encode_batch_dev": (C.c_int, [vp, P, vp, _sz, _sz, _sz, vp, _sz, vp]),
            "np_reconstruct_batch_dev": (C.c_int, [vp, P, vp, _sz, _sz, vp, _sz, vp, _sz, vp]),
            "np_reconstruct_batch_dev3": (C.c_int, [vp, P, vp, _sz, _sz, vp, vp, _sz, vp, _sz, vp, vp]),
            "np_reconstruct_batch_dev2": (C.c_int, [vp, P, vp, _sz, _sz, vp, vp, _sz, vp, _sz, vp]),
            "np_reconstruct_codewords_batch_dev": (C.c_int, [vp, P, vp, _sz, _sz, vp, _sz, vp, _sz, vp, vp]),
            "np_error_locator_dev": (C.c_int, [vp, _sz, vp, _sz, vp, vp]),
            "np_reconstruct_from_systematic_batch_dev": (C.c_int, [vp, P, vp, _sz, _sz, _sz, vp, _sz, vp]),
            "np_encode_batch_host": (C.c_int, [vp, P, vp, _sz, _sz, _sz, vp, _sz]),
            "np_reconstruct_batch_host": (C.c_int, [vp, P, vp, _sz, _sz, vp, _sz, vp, _sz]),
            "np_batch_split": (None, [_sz, _sz, _sz, C.POINTER(_sz), C.POINTER(_sz)]),
            "np_encode_batch_multi": (C.c_int, [C.POINTER(vp), _sz, P, C.POINTER(vp), _sz, _sz, _sz, C.POINTER(vp), _sz]),
            "np_reconstruct_batch_multi": (C.c_int, [C.POINTER(vp), _sz, P, C.POINTER(vp), _sz, _sz, C.POINTER(vp), _sz,
                                                     C.POINTER(vp), _sz, C.POINTER(vp)]),
            "np_encode_batch_host_multi": (C.c_int, [C.POINTER(vp), _sz, P, vp, _sz, _sz, _sz, vp, _sz]),
            "np_reconstruct_batch_host_multi": (C.c_int, [C.POINTER(vp), _sz, P, vp, _sz, _sz, vp, _sz, vp, _sz]),
            "np_afft_dev": (C.c_int, [vp, vp, _sz, _sz, _sz, vp]),
            "np_inverse_afft_dev": (C.c_int, [vp, vp, _sz, _sz, _sz, vp]),
            "np_walsh_dev": (C.c_int, [vp, vp, _sz, vp]),
            "np_mul_dev": (C.c_int, [vp, vp, vp, vp, _sz, vp]),
            "np_encode_low_dev": (C.c_int, [vp, vp, _sz, vp, _sz, _sz, vp]),
            "np_decode_main_dev": (C.c_int, [vp, vp, _sz, vp, vp, _sz, _sz, vp]),
            "np_debug_bounds_check": (C.c_int, [vp, C.POINTER(C.c_uint32)]),
            "np_pin_registry_stats": (None, [C.POINTER(_sz)]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
        return L


# ----------------------------------------------------------------- errors ----
class Error(Exception):
    """errors.rs:4 `Error`."""

    code = -1

    def __init__(self, *fields):
        self.fields = fields
        super().__init__(self._msg())

    def _msg(self) -> str:
        return f"{type(self).__name__}{self.fields}"

    def __eq__(self, other):
        return type(self) is type(other) and self.fields == other.fields

    def __hash__(self):
        return hash((type(self), self.fields))


class WantedShardCountTooHigh(Error):
    code = 1


class WantedShardCountTooLow(Error):
    code = 2


class WantedPayloadShardCountTooLow(Error):
    code = 3


class PayloadSizeIsZero(Error):
    code = 4


class NeedMoreShards(Error):
    code = 5

    @property
    def have(self):
        return self.fields[0]

    @property
    def min(self):
        return self.fields[1]

    @property
    def all(self):
        return self.fields[2]


class ParamterMustBePowerOf2(Error):
    code = 6


class InconsistentShardLengths(Error):
    code = 7


class EmptyShard(Error):
    code = 8


class InvalidArgument(Error):
    """A case the crate `assert!`s on (the C ABI reports it instead of panicking)."""

    code = 100


class DeviceError(Error):
    code = 101


_BY_CODE = {cls.code: cls for cls in (WantedShardCountTooHigh, WantedShardCountTooLow,
                                      WantedPayloadShardCountTooLow, PayloadSizeIsZero, NeedMoreShards,
                                      ParamterMustBePowerOf2, InconsistentShardLengths, EmptyShard,
                                      InvalidArgument)}
_ARITY = {1: 1, 2: 1, 3: 1, 4: 0, 5: 3, 6: 2, 7: 2, 8: 0}


def _raise(st: int):
    if st == 0:
        return
    det = (_sz * 3)()
    lib().np_last_error_detail(det)
    cls = _BY_CODE.get(st)
    if cls is None:
        msg = lib().np_status_message(st).decode()
        if st in (DeviceError.code, 102):  # NP_ERR_DEVICE / NP_ERR_ALLOC: the failing HIP call
            msg += f" [{lib().np_last_error_site().decode()}]"
        raise DeviceError(st, msg)
    raise cls(*tuple(det)[: _ARITY.get(st, 3)])


# ------------------------------------------------------------------ util ----
def recoverablity_subset_size(n_wanted_shards: int) -> int:
    """util.rs:40 (the crate's spelling)."""
    return int(lib().np_recoverability_subset_size(n_wanted_shards))


recoverability_subset_size = recoverablity_subset_size


def is_power_of_2(x: int) -> bool:
    return x > 0 and (x & (x - 1)) == 0


def next_higher_power_of_2(k: int) -> int:
    return k if is_power_of_2(k) else 1 << k.bit_length()


def next_lower_power_of_2(k: int) -> int:
    return k if is_power_of_2(k) else 1 << (k.bit_length() - 1)


# --------------------------------------------------------------- context ----
class Context:
    """One HIP device + stream + uploaded field tables (np_ctx)."""

    def __init__(self, device: int = -1):
        h = C.c_void_p()
        _raise(lib().np_ctx_create(device, C.byref(h)))
        self.handle = h

    @property
    def stream(self) -> int:
        return lib().np_ctx_stream(self.handle) or 0

    @property
    def device(self) -> int:
        return lib().np_ctx_device(self.handle)

    def synchronize(self):
        _raise(lib().np_ctx_synchronize(self.handle))

    def close(self):
        if self.handle:
            lib().np_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default_ctx: dict = {}


def default_context(device: int = -1) -> Context:
    if device not in _default_ctx:
        _default_ctx[device] = Context(device)
    return _default_ctx[device]


# ---------------------------------------------------------------- shards ----
class WrappedShard:
    """wrapped_shard.rs:2-78: a byte vector padded to an even length."""

    __slots__ = ("inner",)

    def __init__(self, data: bytes):
        data = bytes(data)
        if len(data) & 1:
            data += b"\x00"
        self.inner = data

    def into_inner(self) -> bytes:
        return self.inner

    def __bytes__(self):
        return self.inner

    def __len__(self):
        return len(self.inner)

    def __eq__(self, other):
        return isinstance(other, WrappedShard) and other.inner == self.inner

    def __repr__(self):
        return f"WrappedShard({self.inner!r})"


def _as_bytes(s) -> bytes:
    if isinstance(s, WrappedShard):
        return s.inner
    return bytes(s)


def _shard_arrays(shards):
    m = len(shards)
    ptrs = (C.c_void_p * max(1, m))()
    lens = (_sz * max(1, m))()
    keep = []
    for i, s in enumerate(shards):
        if s is None:
            ptrs[i] = None
            lens[i] = 0
        else:
            b = _as_bytes(s)
            buf = C.create_string_buffer(b, max(1, len(b)))
            keep.append(buf)
            ptrs[i] = C.cast(buf, C.c_void_p)
            lens[i] = len(b)
    return ptrs, lens, keep


# ---------------------------------------------------------- code params ----
class CodeParams:
    """mod.rs:24-88."""

    __slots__ = ("_n", "_k", "wanted_n")

    def __init__(self, n: int, k: int, wanted_n: int):
        self._n, self._k, self.wanted_n = n, k, wanted_n

    @staticmethod
    def derive_parameters(n: int, k: int) -> "CodeParams":
        p = _Params()
        _raise(lib().np_derive_parameters(n, k, C.byref(p)))
        return CodeParams(p.n, p.k, p.wanted_n)

    def n(self) -> int:
        return self._n

    def k(self) -> int:
        return self._k

    def is_faster8(self) -> bool:
        """True when a specialised gfx950 kernel serves (n, k)."""
        return bool(lib().np_is_fast_path(C.byref(self._c())))

    def make_encoder(self, ctx: Optional[Context] = None) -> "ReedSolomon":
        return ReedSolomon(self._n, self._k, self.wanted_n, ctx=ctx)

    def _c(self) -> _Params:
        return _Params(self._n, self._k, self.wanted_n)

    def __eq__(self, other):
        return isinstance(other, CodeParams) and (self._n, self._k, self.wanted_n) == (
            other._n, other._k, other.wanted_n)

    def __repr__(self):
        return f"CodeParams(n={self._n}, k={self._k}, wanted_n={self.wanted_n})"


class ReedSolomon:
    """mod.rs:91-285."""

    def __init__(self, n: int, k: int, wanted_n: int, ctx: Optional[Context] = None):
        p = _Params()
        _raise(lib().np_params_new(n, k, wanted_n, C.byref(p)))
        self.n, self.k, self.wanted_n = n, k, wanted_n
        self._p = p
        self.ctx = ctx or default_context()

    def params(self) -> CodeParams:
        return CodeParams(self.n, self.k, self.wanted_n)

    def shard_len(self, payload_size: int) -> int:
        return int(lib().np_shard_len(C.byref(self._p), payload_size))

    def encode(self, data: bytes, shard_type=bytes) -> List:
        data = bytes(data)
        if not data:
            _raise(PayloadSizeIsZero.code)
        sl = self.shard_len(len(data))
        out = C.create_string_buffer(max(1, self.wanted_n * sl))
        _raise(lib().np_rs_encode(self.ctx.handle, C.byref(self._p), data, len(data), out, sl))
        raw = out.raw
        return [shard_type(raw[v * sl:(v + 1) * sl]) for v in range(self.wanted_n)]

    def reconstruct(self, received: Sequence[Optional[bytes]]) -> bytes:
        ptrs, lens, keep = _shard_arrays(received)
        maxsyms = max([(len(_as_bytes(s)) + 1) // 2 for s in received if s is not None] or [0])
        cap = max(1, maxsyms * 2 * self.k)
        out = C.create_string_buffer(cap)
        olen = _sz()
        _raise(lib().np_rs_reconstruct(self.ctx.handle, C.byref(self._p), ptrs, lens, len(received), out, cap,
                                       C.byref(olen)))
        return out.raw[: olen.value]

    def reconstruct_from_systematic(self, chunks: Sequence[bytes]) -> bytes:
        ptrs, lens, keep = _shard_arrays(chunks)
        maxsyms = max([(len(_as_bytes(s)) + 1) // 2 for s in chunks] or [0])
        cap = max(1, maxsyms * 2 * self.k)
        out = C.create_string_buffer(cap)
        olen = _sz()
        _raise(lib().np_rs_reconstruct_from_systematic(self.ctx.handle, C.byref(self._p), ptrs, lens, len(chunks),
                                                       out, cap, C.byref(olen)))
        return out.raw[: olen.value]


def encode(data: bytes, n_min: int, shard_type=bytes, ctx: Optional[Context] = None) -> List:
    """encode.rs:6-11."""
    params = CodeParams.derive_parameters(n_min, recoverablity_subset_size(n_min))
    return params.make_encoder(ctx).encode(data, shard_type=shard_type)


def reconstruct(received: Sequence[Optional[bytes]], validator_count: int, ctx: Optional[Context] = None) -> bytes:
    """reconstruct.rs:4-9."""
    params = CodeParams.derive_parameters(validator_count, recoverablity_subset_size(validator_count))
    return params.make_encoder(ctx).reconstruct(received)


# -------------------------------------------------- device-resident batch ----
def encode_batch_dev(params: CodeParams, d_payloads: int, payload_len: int, payload_stride: int, batch: int,
                     d_shards: int, batch_stride: int, ctx: Optional[Context] = None, stream: int = 0) -> None:
    ctx = ctx or default_context()
    _raise(lib().np_encode_batch_dev(ctx.handle, C.byref(params._c()), d_payloads, payload_len, payload_stride,
                                     batch, d_shards, batch_stride, stream or None))


def error_locator_dev(n: int, d_present: int, batch: int, d_locators: int, ctx: Optional[Context] = None,
                      stream: int = 0) -> None:
    ctx = ctx or default_context()
    _raise(lib().np_error_locator_dev(ctx.handle, n, d_present, batch, d_locators, stream or None))


def reconstruct_batch_dev2(params: CodeParams, d_shards: int, shard_len: int, batch_stride: int, d_present: int,
                           d_locators: int, batch: int, d_out: int, out_stride: int,
                           ctx: Optional[Context] = None, stream: int = 0, d_status: int = 0) -> None:
    """Device batch reconstruct, bit-exact with the crate for any received bytes.

    d_status: device address of ``batch`` np_payload_status entries (int32 status,
    uint32 have; see :func:`payload_errors`) or 0."""
    ctx = ctx or default_context()
    _raise(lib().np_reconstruct_batch_dev3(ctx.handle, C.byref(params._c()), d_shards, shard_len, batch_stride,
                                           d_present, d_locators or None, batch, d_out, out_stride,
                                           d_status or None, stream or None))


def reconstruct_codewords_batch_dev(params: CodeParams, d_shards: int, shard_len: int, batch_stride: int,
                                    d_present: int, batch: int, d_out: int, out_stride: int,
                                    ctx: Optional[Context] = None, stream: int = 0, d_status: int = 0) -> None:
    """OPT-IN prefix decode for shards known to form a codeword (include/novelpoly.h);
    not crate-equivalent for other bytes."""
    ctx = ctx or default_context()
    _raise(lib().np_reconstruct_codewords_batch_dev(ctx.handle, C.byref(params._c()), d_shards, shard_len,
                                                    batch_stride, d_present, batch, d_out, out_stride,
                                                    d_status or None, stream or None))


def payload_errors(params: CodeParams, status_pairs) -> List[Optional[Error]]:
    """np_payload_status entries (a sequence of (status, have) pairs, e.g. a
    ``batch x 2`` int array copied to the host) as the crate's per-call result:
    None for a decoded payload, ``NeedMoreShards(have, k, n)`` (mod.rs:178-180)
    otherwise."""
    out: List[Optional[Error]] = []
    for st, have in status_pairs:
        st = int(st)
        if st == 0:
            out.append(None)
        elif st == NeedMoreShards.code:
            out.append(NeedMoreShards(int(have), params.k(), params.n()))
        else:
            out.append(DeviceError(st, "unexpected payload status"))
    return out


def encode_batch_host(params: CodeParams, payloads: int, payload_len: int, payload_stride: int, batch: int,
                      shards: int, batch_stride: int, ctx: Optional[Context] = None) -> None:
    """Host-memory batch encode (addresses of host buffers, e.g. numpy / pinned torch)."""
    ctx = ctx or default_context()
    _raise(lib().np_encode_batch_host(ctx.handle, C.byref(params._c()), payloads, payload_len, payload_stride, batch,
                                      shards, batch_stride))


def reconstruct_batch_host(params: CodeParams, shards: int, shard_len: int, batch_stride: int, present: int,
                           batch: int, out: int, out_stride: int, ctx: Optional[Context] = None) -> None:
    """Host-memory batch reconstruct; present: address of batch*n host flags."""
    ctx = ctx or default_context()
    _raise(lib().np_reconstruct_batch_host(ctx.handle, C.byref(params._c()), shards, shard_len, batch_stride, present,
                                           batch, out, out_stride))


def reconstruct_from_systematic_batch_dev(params: CodeParams, d_shards: int, shard_len: int, batch_stride: int,
                                          batch: int, d_out: int, out_stride: int, ctx: Optional[Context] = None,
                                          stream: int = 0) -> None:
    """mod.rs:247-285 for a device batch whose first k shards are present."""
    ctx = ctx or default_context()
    _raise(lib().np_reconstruct_from_systematic_batch_dev(ctx.handle, C.byref(params._c()), d_shards, shard_len,
                                                          batch_stride, batch, d_out, out_stride, stream or None))


def reconstruct_batch_dev(params: CodeParams, d_shards: int, shard_len: int, batch_stride: int, present,
                          batch: int, d_out: int, out_stride: int, ctx: Optional[Context] = None,
                          stream: int = 0) -> None:
    """present: host bytes-like of batch*n flags."""
    ctx = ctx or default_context()
    pres = bytes(present)
    _raise(lib().np_reconstruct_batch_dev(ctx.handle, C.byref(params._c()), d_shards, shard_len, batch_stride,
                                          pres, batch, d_out, out_stride, stream or None))


# ------------------------------------------------------------ multi-GPU ----
def batch_split(batch: int, ndev: int, i: int):
    """np_batch_split: (begin, count) of device i's contiguous payload range."""
    b, c = _sz(), _sz()
    lib().np_batch_split(batch, ndev, i, C.byref(b), C.byref(c))
    return b.value, c.value


def _ptr_array(vals):
    arr = (C.c_void_p * max(1, len(vals)))()
    for i, v in enumerate(vals):
        arr[i] = v or None
    return arr


def _ctx_array(ctxs):
    return _ptr_array([c.handle.value for c in ctxs])


def encode_batch_multi(ctxs, params: CodeParams, d_payloads, payload_len: int, payload_stride: int, batch: int,
                       d_shards, batch_stride: int) -> None:
    """Device-resident batch over several contexts (one per GPU); d_payloads[i] /
    d_shards[i]: device i's buffers for its range (:func:`batch_split`)."""
    _raise(lib().np_encode_batch_multi(_ctx_array(ctxs), len(ctxs), C.byref(params._c()), _ptr_array(d_payloads),
                                       payload_len, payload_stride, batch, _ptr_array(d_shards), batch_stride))


def reconstruct_batch_multi(ctxs, params: CodeParams, d_shards, shard_len: int, batch_stride: int, d_present,
                            batch: int, d_out, out_stride: int, d_status=None) -> None:
    st = _ptr_array(d_status) if d_status else None
    _raise(lib().np_reconstruct_batch_multi(_ctx_array(ctxs), len(ctxs), C.byref(params._c()), _ptr_array(d_shards),
                                            shard_len, batch_stride, _ptr_array(d_present), batch, _ptr_array(d_out),
                                            out_stride, st))


def encode_batch_host_multi(ctxs, params: CodeParams, payloads: int, payload_len: int, payload_stride: int,
                            batch: int, shards: int, batch_stride: int) -> None:
    _raise(lib().np_encode_batch_host_multi(_ctx_array(ctxs), len(ctxs), C.byref(params._c()), payloads, payload_len,
                                            payload_stride, batch, shards, batch_stride))


def reconstruct_batch_host_multi(ctxs, params: CodeParams, shards: int, shard_len: int, batch_stride: int,
                                 present: int, batch: int, out: int, out_stride: int) -> None:
    _raise(lib().np_reconstruct_batch_host_multi(_ctx_array(ctxs), len(ctxs), C.byref(params._c()), shards, shard_len,
                                                 batch_stride, present, batch, out, out_stride))


# ---------------------------------------------------- low-level hooks ----
def afft_dev(d_data: int, size: int, index: int, cols: int, inverse: bool = False,
             ctx: Optional[Context] = None, stream: int = 0) -> None:
    ctx = ctx or default_context()
    f = lib().np_inverse_afft_dev if inverse else lib().np_afft_dev
    _raise(f(ctx.handle, d_data, size, index, cols, stream or None))


def walsh_dev(d_data: int, size: int, ctx: Optional[Context] = None, stream: int = 0) -> None:
    ctx = ctx or default_context()
    _raise(lib().np_walsh_dev(ctx.handle, d_data, size, stream or None))


def mul_dev(d_a: int, d_m: int, d_out: int, count: int, ctx: Optional[Context] = None, stream: int = 0) -> None:
    ctx = ctx or default_context()
    _raise(lib().np_mul_dev(ctx.handle, d_a, d_m, d_out, count, stream or None))


def encode_low_dev(d_data: int, k: int, d_codeword: int, n: int, cols: int, ctx: Optional[Context] = None,
                   stream: int = 0) -> None:
    ctx = ctx or default_context()
    _raise(lib().np_encode_low_dev(ctx.handle, d_data, k, d_codeword, n, cols, stream or None))


def decode_main_dev(d_codeword: int, recover_up_to: int, d_present: int, d_locator: int, n: int, cols: int,
                    ctx: Optional[Context] = None, stream: int = 0) -> None:
    ctx = ctx or default_context()
    _raise(lib().np_decode_main_dev(ctx.handle, d_codeword, recover_up_to, d_present, d_locator, n, cols,
                                    stream or None))


def version() -> str:
    return lib().np_version().decode()


# ----------------------------------------------------------- diagnostics ----
BOUNDS_KINDS = ("shards", "present", "locators", "records", "out", "status", "zeros", "payloads")


def debug_bounds_check(ctx: Optional[Context] = None) -> Optional[dict]:
    """Checked builds (lib/libnovelpoly_hip_chk.so through NP_LIB_PATH): the
    out-of-extent global accesses of the instrumented kernels since the last
    call, {count, kind, line, workgroup, thread, offset, bytes} (count 0: none);
    None with the product library."""
    ctx = ctx or default_context()
    r = (C.c_uint32 * 8)()
    if lib().np_debug_bounds_check(ctx.handle, r) != 0:
        return None
    kind = BOUNDS_KINDS[r[1]] if r[0] and r[1] < len(BOUNDS_KINDS) else r[1]
    return {"count": r[0], "kind": kind, "line": r[2], "workgroup": r[3], "thread": r[4],
            "offset": r[5] | (r[6] << 32), "bytes": r[7]}


def pin_registry_stats() -> dict:
    """The engine's in-place pin registry: ranges registered now, and
    hipHostUnregister calls the runtime refused (include/novelpoly.h)."""
    o = (_sz * 2)()
    lib().np_pin_registry_stats(o)
    return {"live_ranges": o[0], "failed_unregisters": o[1]}
