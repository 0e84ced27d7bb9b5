"""Live datalink batch rx / tx (nexg_rx_* / nexg_tx_* in include/nexg.h).

Mirrors nex-datalink's Linux channel: `channel(interface, Config)`
(nex-datalink/src/lib.rs:324-330, linux.rs:102-218) with the same Config
knobs (read_buffer_size, read_timeout, promiscuous, linux_fanout) — but the
receiver hands over whole batches (TPACKET_V3 ring or recvmmsg) instead of
one frame per `RawReceiver::next`, and the sender takes a batch per
sendmmsg instead of one `sendto` per `RawSender::send`. `device_batches`
moves each received batch to the GPU as a packed FrameBatch.
"""
import ctypes
from dataclasses import dataclass
from typing import Iterator, Optional, Tuple

import numpy as np

from . import abi
from ._lib import load

RX_RING, RX_MMSG = 0, 1
RX_SKIP_OUTGOING = 0x1
# FanoutType (nex-datalink/src/lib.rs:70-90)
FANOUT_HASH, FANOUT_LB, FANOUT_CPU, FANOUT_ROLLOVER, FANOUT_RND, FANOUT_QM = range(6)
FANOUT_FLAG_ROLLOVER, FANOUT_FLAG_DEFRAG = 0x1000, 0x8000


class DatalinkError(OSError):
    pass


class RxConfig(ctypes.Structure):
    """struct nexg_rx_config"""
    _fields_ = [(n, ctypes.c_int32 if n == "read_timeout_ms" else ctypes.c_uint32) for n in (
        "read_buffer_size", "read_timeout_ms", "promiscuous", "fanout", "fanout_type", "fanout_group",
        "mode", "ring_block_size", "ring_blocks", "ring_block_tov_ms", "flags", "reserved")]


@dataclass
class FanoutOption:  # lib.rs:119-131
    group_id: int
    fanout_type: int = FANOUT_HASH
    defrag: bool = False
    rollover: bool = False


@dataclass
class Config:  # lib.rs:159-307 (the Linux subset) + the batch ring knobs
    read_buffer_size: int = 4096
    read_timeout_ms: Optional[int] = None
    promiscuous: bool = True
    linux_fanout: Optional[FanoutOption] = None
    mode: int = RX_RING
    ring_block_size: int = 1 << 20
    ring_blocks: int = 64
    ring_block_tov_ms: int = 2
    skip_outgoing: bool = False

    def to_c(self) -> RxConfig:
        c = RxConfig()
        load().nexg_rx_config_default(ctypes.byref(c))
        c.read_buffer_size = self.read_buffer_size
        c.read_timeout_ms = -1 if self.read_timeout_ms is None else int(self.read_timeout_ms)
        c.promiscuous = int(self.promiscuous)
        if self.linux_fanout is not None:
            f = self.linux_fanout
            c.fanout = 1
            c.fanout_group = f.group_id
            c.fanout_type = f.fanout_type | (FANOUT_FLAG_DEFRAG if f.defrag else 0) | \
                (FANOUT_FLAG_ROLLOVER if f.rollover else 0)
        c.mode = self.mode
        c.ring_block_size, c.ring_blocks, c.ring_block_tov_ms = \
            self.ring_block_size, self.ring_blocks, self.ring_block_tov_ms
        c.flags = RX_SKIP_OUTGOING if self.skip_outgoing else 0
        return c


def _check(rc, what):
    if rc == abi.EPERM:
        raise PermissionError(f"{what}: AF_PACKET needs CAP_NET_RAW")
    if rc != abi.OK:
        raise DatalinkError(f"{what}: status {rc}")


class RawReceiver:
    """Batch receiver on one interface (the RawReceiver of linux.rs:350-398)."""

    def __init__(self, ifname: str, config: Config = Config()):
        self.lib = load()
        h = ctypes.c_void_p()
        c = config.to_c()
        _check(self.lib.nexg_rx_open(ifname.encode(), ctypes.byref(c), ctypes.byref(h)), f"rx on {ifname}")
        self.h = h

    def next_batch_into(self, data: np.ndarray, offsets: np.ndarray, ts_ns: Optional[np.ndarray] = None) -> int:
        n = ctypes.c_uint64()
        _check(self.lib.nexg_rx_next_batch(self.h, data.ctypes.data, data.nbytes, offsets.ctypes.data,
                                           len(offsets) - 1, None if ts_ns is None else ts_ns.ctypes.data,
                                           ctypes.byref(n)), "rx batch")
        return n.value

    def next_batch(self, max_frames: int = 1 << 14, data_cap: int = 1 << 24) -> Tuple[np.ndarray, np.ndarray]:
        data = np.empty(data_cap, np.uint8)
        offs = np.empty(max_frames + 1, np.uint64)
        n = self.next_batch_into(data, offs)
        return data[: int(offs[n])] if n else data[:0], offs[: n + 1]

    def stats(self) -> Tuple[int, int]:
        p, d = ctypes.c_uint64(), ctypes.c_uint64()
        _check(self.lib.nexg_rx_stats(self.h, ctypes.byref(p), ctypes.byref(d)), "rx stats")
        return p.value, d.value

    def close(self):
        if getattr(self, "h", None):
            self.lib.nexg_rx_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class RawSender:
    """Batch sender on one interface (the RawSender of linux.rs:220-347)."""

    def __init__(self, ifname: str):
        self.lib = load()
        h = ctypes.c_void_p()
        _check(self.lib.nexg_tx_open(ifname.encode(), ctypes.byref(h)), f"tx on {ifname}")
        self.h = h

    def send_batch(self, data: np.ndarray, offsets: Optional[np.ndarray] = None,
                   lengths: Optional[np.ndarray] = None, stride: int = 0, count: Optional[int] = None) -> int:
        """Frames from host memory in the nexg_frames layout; returns the count sent."""
        data = np.ascontiguousarray(data, np.uint8)
        if count is None:
            count = (len(offsets) - (0 if lengths is not None else 1)) if offsets is not None else len(data) // stride
        offs = None if offsets is None else np.ascontiguousarray(offsets, np.uint64)
        lens = None if lengths is None else np.ascontiguousarray(lengths, np.uint32)
        n = ctypes.c_uint64()
        _check(self.lib.nexg_tx_send_batch(self.h, data.ctypes.data, None if offs is None else offs.ctypes.data,
                                           None if lens is None else lens.ctypes.data, stride, count,
                                           ctypes.byref(n)), "tx batch")
        return n.value

    def send(self, packet: bytes) -> int:  # RawSender::send (lib.rs:333-359), one frame
        b = np.frombuffer(bytes(packet), np.uint8)
        return self.send_batch(b, np.array([0, len(b)], np.uint64))

    def close(self):
        if getattr(self, "h", None):
            self.lib.nexg_tx_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def channel(ifname: str, config: Config = Config()) -> Tuple[RawSender, RawReceiver]:
    """datalink::channel (lib.rs:324-330) for the Linux Ethernet channel."""
    return RawSender(ifname), RawReceiver(ifname, config)


def walk_block(block: bytes, snap: int = 4096, flags: int = 0, first: int = 0,
               max_frames: int = 1 << 16, data_cap: int = 1 << 24):
    """nexg_tpacket3_walk on one TPACKET_V3 block (host bytes): (frames, next packet)."""
    lib = load()
    b = np.frombuffer(bytes(block), np.uint8)
    data = np.empty(data_cap, np.uint8)
    offs = np.empty(max_frames + 1, np.uint64)
    pos, n, nxt = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint32(0)
    _check(lib.nexg_tpacket3_walk(b.ctypes.data, len(b), first, snap, flags, data.ctypes.data, data_cap,
                                  ctypes.byref(pos), offs.ctypes.data, max_frames, None, ctypes.byref(n),
                                  ctypes.byref(nxt)), "tpacket3 walk")
    offs[n.value] = pos.value
    return [bytes(data[int(offs[k]):int(offs[k + 1])]) for k in range(n.value)], nxt.value


def device_batches(rx: RawReceiver, max_frames: int = 1 << 18, data_cap: int = 1 << 26, device="cuda",
                   stream=None, batches: Optional[int] = None) -> Iterator[object]:
    """Received batches moved H2D as packed FrameBatch objects (pinned staging)."""
    import torch
    from .engine import FrameBatch
    data = torch.empty(data_cap, dtype=torch.uint8, pin_memory=True)
    offs = torch.empty(max_frames + 1, dtype=torch.int64, pin_memory=True)
    dnp, onp = data.numpy(), offs.numpy().view(np.uint64)
    k = 0
    while batches is None or k < batches:
        n = rx.next_batch_into(dnp, onp)
        if n == 0:
            return
        nbytes = int(onp[n])
        s = stream or torch.cuda.current_stream()
        with torch.cuda.stream(s):
            d = data[:max(nbytes, 1)].to(device, non_blocking=True)
            o = offs[: n + 1].to(device, non_blocking=True)
        s.synchronize()
        k += 1
        yield FrameBatch(data=d[:nbytes], count=n, offsets=o)
