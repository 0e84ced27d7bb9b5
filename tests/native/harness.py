"""TEST INFRASTRUCTURE ONLY: ctypes wrapper of tests/native/libcoreharness.so."""
import ctypes
import os
import subprocess

import numpy as np

from nex_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libcoreharness.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        subprocess.check_call(["make", "-s", "-C", HERE, "libcoreharness.so"])
        L = ctypes.CDLL(LIB)
        P, U32, U64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
        L.harness_parse.restype = ctypes.c_int
        L.harness_parse.argtypes = [P, U64, P, P, U32, U64, U32, U32, U32, ctypes.c_int, P]
        L.harness_sparse.restype = ctypes.c_int
        L.harness_sparse.argtypes = [P, U64, U32, U32, P, P, P]
        L.harness_sparse_decode.restype = ctypes.c_int
        L.harness_sparse_decode.argtypes = [P, P, U64, U32, U32, P, P]
        L.harness_slice.restype = ctypes.c_int
        L.harness_slice.argtypes = [P, U64, P, P, U32, U64, U32, U32, U32, P]
        L.harness_tile_map.restype = None
        L.harness_tile_map.argtypes = [U32, U32, P]
        L.harness_span_groups.restype = ctypes.c_int
        L.harness_span_groups.argtypes = [P, U64, P, U64, U32, U32, P]
        L.harness_span_declined.restype = None
        L.harness_span_declined.argtypes = [P]
        _lib = L
    return _lib


def parse_packed(data, offsets=None, lengths=None, stride=0, flags=0, ip_offset=0, window=128,
                 use_fast=False, poison=0xA5):
    """poison: the byte pattern the harness puts past each frame's length
    where the kernels would hold the next frame's bytes (they must not matter)."""
    lib().harness_set_poison(poison)
    data = np.ascontiguousarray(data, dtype=np.uint8)
    count = (len(lengths) if lengths is not None else
             (len(offsets) - 1 if offsets is not None else len(data) // stride))
    offs = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
    lens = None if lengths is None else np.ascontiguousarray(lengths, dtype=np.uint32)
    recs = np.zeros(count, dtype=abi.RECORD_DTYPE)
    rc = lib().harness_parse(data.ctypes.data, data.nbytes,
                             None if offs is None else offs.ctypes.data,
                             None if lens is None else lens.ctypes.data, stride, count, flags,
                             ip_offset, window, int(use_fast), recs.ctypes.data)
    assert rc == 0, f"harness_parse: {rc} (-2: canonical80_code differs from sparse_encode)"
    return recs


def slice_packed(data, offsets=None, lengths=None, stride=0, flags=0, ip_offset=0, window=128):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    count = (len(lengths) if lengths is not None else
             (len(offsets) - 1 if offsets is not None else len(data) // stride))
    offs = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
    lens = None if lengths is None else np.ascontiguousarray(lengths, dtype=np.uint32)
    out = np.zeros(count, dtype=abi.SLICE_DTYPE)
    lib().harness_slice(data.ctypes.data, data.nbytes,
                        None if offs is None else offs.ctypes.data,
                        None if lens is None else lens.ctypes.data, stride, count, flags,
                        ip_offset, window, out.ctypes.data)
    return out


def sparse(recs, flags=0, ip_offset=0):
    """(codes, device-decoder descs, header-decoder descs) of the kernels'
    NEXG_OUT_SPARSE encoder run on the host over `recs`."""
    import numpy as np
    from nex_amd import abi
    recs = np.ascontiguousarray(recs)
    n = len(recs)
    codes = np.zeros(max(n, 1), np.uint8)
    dd = np.zeros(max(n, 1), abi.DESC_DTYPE)
    hd = np.zeros(max(n, 1), abi.DESC_DTYPE)
    assert lib().harness_sparse(recs.ctypes.data, n, flags, ip_offset, codes.ctypes.data, dd.ctypes.data,
                                hd.ctypes.data) == 0
    return codes[:n], dd[:n], hd[:n]


def sparse_decode(codes, lens, flags=0, ip_offset=0):
    """(kernels' decoder, C header decoder) descriptors of (code, length) pairs."""
    import numpy as np
    from nex_amd import abi
    codes = np.ascontiguousarray(codes, np.uint8)
    lens = np.ascontiguousarray(lens, np.uint32)
    n = len(codes)
    dd = np.zeros(max(n, 1), abi.DESC_DTYPE)
    hd = np.zeros(max(n, 1), abi.DESC_DTYPE)
    assert lib().harness_sparse_decode(codes.ctypes.data, lens.ctypes.data, n, flags, ip_offset,
                                       dd.ctypes.data, hd.ctypes.data) == 0
    return dd[:n], hd[:n]


def span_groups(data, offsets, flags=0, ip_offset=0, declined=None):
    """k_parse_span's fast path (with the lanes' slots for IPv4 options) +
    generic section (slots, bucketed items) emulated group by group over a
    packed batch. `declined` (uint8[count], optional) receives 1 for every
    frame the fast path declined to the generic core."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offs = np.ascontiguousarray(offsets, dtype=np.uint64)
    count = len(offs) - 1
    recs = np.zeros(count, dtype=abi.RECORD_DTYPE)
    if declined is not None:
        assert declined.dtype == np.uint8 and declined.flags.c_contiguous and len(declined) >= count
        declined[:count] = 0
    lib().harness_span_declined(ctypes.c_void_p(declined.ctypes.data if declined is not None else None))
    try:
        rc = lib().harness_span_groups(data.ctypes.data, data.nbytes, offs.ctypes.data, count, flags, ip_offset,
                                       recs.ctypes.data)
    finally:
        lib().harness_span_declined(ctypes.c_void_p(None))
    assert rc == 0, f"harness_span_groups: {rc}"
    return recs


def tile_map(nb, order):
    """tile_of(b, nb, order) for b in [0, nb): the kernels' workgroup -> tile map."""
    out = np.zeros(nb, np.uint64)
    lib().harness_tile_map(nb, order, out.ctypes.data)
    return out
