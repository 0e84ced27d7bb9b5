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
        L.harness_slice.restype = ctypes.c_int
        L.harness_slice.argtypes = [P, U64, P, P, U32, U64, U32, U32, U32, P]
        _lib = L
    return _lib


def parse_packed(data, offsets=None, lengths=None, stride=0, flags=0, ip_offset=0, window=128,
                 use_fast=False):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    count = (len(lengths) if lengths is not None else
             (len(offsets) - 1 if offsets is not None else len(data) // stride))
    offs = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
    lens = None if lengths is None else np.ascontiguousarray(lengths, dtype=np.uint32)
    recs = np.zeros(count, dtype=abi.RECORD_DTYPE)
    lib().harness_parse(data.ctypes.data, data.nbytes,
                        None if offs is None else offs.ctypes.data,
                        None if lens is None else lens.ctypes.data, stride, count, flags,
                        ip_offset, window, int(use_fast), recs.ctypes.data)
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
