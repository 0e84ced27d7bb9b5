"""nex_amd — MI355X-native batched packet dissect + checksum engine.

Drop-in for shellrow/nex nex-packet's per-frame hot path (Frame parse and the
IPv4 / TCP / UDP / ICMP / ICMPv6 checksums, plus the udp_ping frame builder):
hand-written gfx950 HIP kernels behind the C ABI in include/nexg.h, compiled
into nex_amd/libnexg.so. This package is the Python host binding.
"""
from . import abi
from .frame import (Frame, ParseError, ParseMode, ParseOption, frame_from_record,
                    frame_view_payload)

__all__ = ["abi", "Frame", "ParseError", "ParseMode", "ParseOption", "frame_from_record",
           "frame_view_payload", "Engine", "FrameBatch", "NexgError"]


def __getattr__(name):
    # The engine needs libnexg.so (and torch); import it lazily so the pure
    # host mirror stays importable for CPU-only tooling.
    if name in ("Engine", "FrameBatch", "NexgError"):
        from . import engine
        return getattr(engine, name)
    raise AttributeError(name)
