"""Loader for the in-tree HIP library nex_amd/libnexg.so.

The library is the product: there is no CPU fallback. If it is missing the
import of the engine fails loudly with instructions to build it.
"""
import ctypes
import os

from . import abi

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libnexg.so")

_lib = None


class NexgLibraryMissing(RuntimeError):
    pass


def load():
    """Load libnexg.so (after torch, so both share torch's HIP runtime)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NexgLibraryMissing(
            f"{LIB_PATH} not found: build it with `make -C nex_amd/csrc` "
            "(or __graft_entry__.build()); nex_amd has no CPU fallback")
    try:
        import torch  # noqa: F401  (load torch's libamdhip64 first: one HIP runtime)
    except ImportError:
        pass
    lib = ctypes.CDLL(LIB_PATH)
    P, I, U32, U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint64
    sig = {
        "nexg_abi_version": (I, []),
        "nexg_strerror": (ctypes.c_char_p, [I]),
        "nexg_ctx_create": (I, [I, ctypes.POINTER(P)]),
        "nexg_ctx_destroy": (I, [P]),
        "nexg_ctx_last_error": (ctypes.c_char_p, [P]),
        "nexg_ctx_cu_count": (I, [P]),
        "nexg_parse_batch": (I, [P, ctypes.POINTER(abi.Frames), ctypes.POINTER(abi.ParseOptionC), I, P, P]),
        "nexg_checksum_batch": (I, [P, ctypes.POINTER(abi.Frames), U32, P, P]),
        "nexg_sparse_expand": (I, [P, ctypes.POINTER(abi.Frames), ctypes.POINTER(abi.ParseOptionC), P, P, P]),
        "nexg_grouped_expand": (I, [P, ctypes.POINTER(abi.Frames), ctypes.POINTER(abi.ParseOptionC), P, P, P]),
        "nexg_recompute_checksums_batch": (I, [P, ctypes.POINTER(abi.Frames), ctypes.POINTER(abi.ParseOptionC),
                                               U32, P, P]),
        "nexg_probe_stream": (I, [P, P, U64, U32, P, P]),
        "nexg_probe_span_clock": (I, [P, ctypes.POINTER(abi.Frames), ctypes.POINTER(abi.ParseOptionC), P, P, P]),
        "nexg_probe_latency": (I, [P, P, U64, U32, U32, U32, P, P]),
        "nexg_decode_options": (I, [P, ctypes.POINTER(abi.Frames), P, P, P]),
        "nexg_build_udp4_batch": (I, [P, ctypes.POINTER(abi.Udp4Build), P, U32, P]),
        "nexg_build_udp4_tuples": (I, [P, ctypes.POINTER(abi.Udp4Build), P, P, U32, P]),
        "nexg_build_udp6_batch": (I, [P, ctypes.POINTER(abi.Udp6Build), P, U32, P]),
        "nexg_build_tcp_batch": (I, [P, ctypes.POINTER(abi.TcpBuild), P, U32, P]),
        "nexg_build_icmp_echo_batch": (I, [P, ctypes.POINTER(abi.IcmpEchoBuild), P, U32, P]),
        "nexg_build_arp_batch": (I, [P, ctypes.POINTER(abi.ArpBuild), P, U32, P]),
        "nexg_build_ndp_ns_batch": (I, [P, ctypes.POINTER(abi.NdpNsBuild), P, U32, P]),
        "nexg_pcap_open": (I, [ctypes.c_char_p, ctypes.POINTER(P)]),
        "nexg_pcap_linktype": (I, [P]),
        "nexg_pcap_last_error": (ctypes.c_char_p, [P]),
        "nexg_pcap_read_batch": (I, [P, P, U64, P, U64, P, ctypes.POINTER(U64)]),
        "nexg_pcap_read_raw": (I, [P, P, U64, P, P, U64, P, ctypes.POINTER(U64), ctypes.POINTER(U64)]),
        "nexg_pcap_map": (I, [P, ctypes.POINTER(P), ctypes.POINTER(U64), ctypes.POINTER(U64)]),
        "nexg_pcap_walk_mapped": (I, [P, U64, U64, P, P, U64, P, ctypes.POINTER(U64), ctypes.POINTER(U64)]),
        "nexg_pcap_set_read_threads": (I, [P, U32]),
        "nexg_pcap_close": (I, [P]),
        "nexg_rx_config_default": (None, [P]),
        "nexg_rx_open": (I, [ctypes.c_char_p, P, ctypes.POINTER(P)]),
        "nexg_rx_next_batch": (I, [P, P, U64, P, U64, P, ctypes.POINTER(U64)]),
        "nexg_rx_stats": (I, [P, ctypes.POINTER(U64), ctypes.POINTER(U64)]),
        "nexg_rx_close": (I, [P]),
        "nexg_tpacket3_walk": (I, [P, U64, U32, U32, U32, P, U64, ctypes.POINTER(U64), P, U64, P,
                                   ctypes.POINTER(U64), ctypes.POINTER(U32)]),
        "nexg_tx_open": (I, [ctypes.c_char_p, ctypes.POINTER(P)]),
        "nexg_tx_send_batch": (I, [P, P, P, P, U32, U64, ctypes.POINTER(U64)]),
        "nexg_tx_close": (I, [P]),
        "nexg_gen_lengths": (I, [P, I, U64, U64, U64, P, P]),
        "nexg_gen_frames": (I, [P, I, U64, U64, U64, P, P, U32, P]),
        "nexg_gen_udp4_params": (I, [P, U64, U64, U64, P, P, P, P, P, P]),
    }
    # NEXG_AB_LIB_LENIENT=1 (measurement tools loading an older build for an
    # in-process A/B): entry points that build lacks are left unbound
    lenient = os.environ.get("NEXG_AB_LIB_LENIENT") == "1"
    for name, (res, args) in sig.items():
        if lenient and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.nexg_abi_version() != abi.ABI_VERSION:
        raise RuntimeError("libnexg.so ABI version mismatch; rebuild nex_amd/csrc")
    _lib = lib
    return lib
