"""Capture-file batch ingest (nexg_pcap_* in include/nexg.h).

The host half of the end-to-end path: nex-datalink hands frames over one at a
time (`RawReceiver::next`, nex-datalink/src/lib.rs:363-366; the file channel
is pcap::from_file, pcap.rs:95-109). Here a native reader (libnexg.so,
nex_amd/csrc/nexg_pcap.cpp) fills a packed batch — bytes back to back plus an
offset table — in (optionally pinned) host memory, and `device_batches`
moves each batch to the GPU as a FrameBatch for nexg_parse_batch.
"""
import ctypes
from typing import Iterator, Optional, Tuple

import numpy as np

from . import abi
from ._lib import load

LINKTYPE_ETHERNET = 1
LINKTYPE_RAW = 101


class PcapError(RuntimeError):
    pass


class PcapReader:
    """Classic pcap (µs/ns, either byte order) or pcapng reader."""

    def __init__(self, path: str):
        self.lib = load()
        h = ctypes.c_void_p()
        rc = self.lib.nexg_pcap_open(str(path).encode(), ctypes.byref(h))
        if rc != abi.OK:
            raise PcapError(f"cannot open {path} as pcap/pcapng (status {rc})")
        self.h = h

    @property
    def linktype(self) -> int:
        return self.lib.nexg_pcap_linktype(self.h)

    def read_into(self, data: np.ndarray, offsets: np.ndarray,
                  ts_ns: Optional[np.ndarray] = None) -> int:
        """Fill caller arrays (data uint8, offsets uint64 with room for
        max_frames + 1 entries); returns the frame count (0 at end of file)."""
        n = ctypes.c_uint64()
        max_frames = len(offsets) - 1
        rc = self.lib.nexg_pcap_read_batch(
            self.h, data.ctypes.data, data.nbytes, offsets.ctypes.data, max_frames,
            None if ts_ns is None else ts_ns.ctypes.data, ctypes.byref(n))
        if rc != abi.OK:
            raise PcapError(self.lib.nexg_pcap_last_error(self.h).decode() or f"status {rc}")
        return n.value

    def read_raw_into(self, buf: np.ndarray, offsets: np.ndarray, lengths: np.ndarray,
                      ts_ns: Optional[np.ndarray] = None) -> Tuple[int, int]:
        """In-place shape: file bytes read straight into buf, records described
        by offsets/lengths into it. Returns (frames, bytes used); (0, 0) at
        end of file."""
        n, used = ctypes.c_uint64(), ctypes.c_uint64()
        rc = self.lib.nexg_pcap_read_raw(
            self.h, buf.ctypes.data, buf.nbytes, offsets.ctypes.data, lengths.ctypes.data,
            len(offsets), None if ts_ns is None else ts_ns.ctypes.data, ctypes.byref(n),
            ctypes.byref(used))
        if rc != abi.OK:
            raise PcapError(self.lib.nexg_pcap_last_error(self.h).decode() or f"status {rc}")
        return n.value, used.value

    def read_batch(self, max_frames: int = 1 << 16, data_cap: int = 1 << 26
                   ) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """Next batch as (data, offsets[n+1], ts_ns[n]) numpy arrays."""
        data = np.empty(data_cap, np.uint8)
        offs = np.empty(max_frames + 1, np.uint64)
        ts = np.empty(max_frames, np.uint64)
        n = self.read_into(data, offs, ts)
        return data[: int(offs[n])] if n else data[:0], offs[: n + 1], ts[:n]

    def frames(self, **kw) -> Iterator[bytes]:
        while True:
            data, offs, _ = self.read_batch(**kw)
            if len(offs) <= 1:
                return
            for a, b in zip(offs[:-1], offs[1:]):
                yield bytes(data[int(a):int(b)])

    def map(self) -> Tuple[np.ndarray, int]:
        """Zero-copy shape (nexg_pcap_map): (read-only uint8 array over the
        file's page-cache mapping, offset of the first record). The array is
        valid until close()."""
        data, size, first = ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_uint64()
        rc = self.lib.nexg_pcap_map(self.h, ctypes.byref(data), ctypes.byref(size), ctypes.byref(first))
        if rc != abi.OK:
            raise PcapError(self.lib.nexg_pcap_last_error(self.h).decode() or f"status {rc}")
        if size.value == 0:
            return np.zeros(0, np.uint8), first.value
        arr = np.ctypeslib.as_array((ctypes.c_uint8 * size.value).from_address(data.value))
        arr.flags.writeable = False  # PROT_READ
        return arr, first.value

    def walk_mapped(self, start: int, max_bytes: int, offsets: np.ndarray, lengths: np.ndarray,
                    ts_ns: Optional[np.ndarray] = None) -> Tuple[int, int]:
        """Records in the mapping window [start, start + max_bytes)
        (nexg_pcap_walk_mapped): (frames, next start); offsets relative to
        start."""
        n, nxt = ctypes.c_uint64(), ctypes.c_uint64()
        rc = self.lib.nexg_pcap_walk_mapped(
            self.h, start, max_bytes, offsets.ctypes.data, lengths.ctypes.data, len(offsets),
            None if ts_ns is None else ts_ns.ctypes.data, ctypes.byref(n), ctypes.byref(nxt))
        if rc != abi.OK:
            raise PcapError(self.lib.nexg_pcap_last_error(self.h).decode() or f"status {rc}")
        return n.value, nxt.value

    def set_read_threads(self, threads: int):
        """Split read_raw's file reads over `threads` parallel preads (and the
        classic-pcap record walk of read_raw / walk_mapped over as many threads)."""
        rc = self.lib.nexg_pcap_set_read_threads(self.h, threads)
        if rc != abi.OK:
            raise PcapError(f"invalid thread count {threads}")

    def close(self):
        if getattr(self, "h", None):
            self.lib.nexg_pcap_close(self.h)
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


def raw_frames(reader: PcapReader, cap: int = 1 << 22, max_frames: int = 1 << 14) -> Iterator[bytes]:
    """All frames via the in-place shape (test / inspection helper)."""
    buf = np.empty(cap, np.uint8)
    offs = np.empty(max_frames, np.uint64)
    lens = np.empty(max_frames, np.uint32)
    while True:
        n, used = reader.read_raw_into(buf, offs, lens)
        if n == 0 and used == 0:
            return
        for k in range(n):
            yield bytes(buf[int(offs[k]):int(offs[k]) + int(lens[k])])


def device_batches(reader: PcapReader, max_frames: int = 1 << 20, data_cap: int = 1 << 28,
                   device="cuda", stream=None):
    """Yield FrameBatch objects on `device`: each batch is read into pinned
    host memory by the native reader and copied H2D on `stream` (the packed
    offsets-only layout, parsed by the SpanTile kernel)."""
    import torch
    from .engine import FrameBatch
    data = torch.empty(data_cap, dtype=torch.uint8, pin_memory=True)
    offs = torch.empty(max_frames + 1, dtype=torch.int64, pin_memory=True)
    dnp, onp = data.numpy(), offs.numpy().view(np.uint64)
    while True:
        n = reader.read_into(dnp, onp)
        if n == 0:
            return
        nbytes = int(onp[n])
        s = stream or torch.cuda.current_stream()
        with torch.cuda.stream(s):
            d = data[:max(nbytes, 1)].to(device, non_blocking=True)
            o = offs[: n + 1].to(device, non_blocking=True)
        s.synchronize()  # the pinned staging buffers are reused by the next read
        yield FrameBatch(data=d[:nbytes], count=n, offsets=o)


def device_raw_batches(reader: PcapReader, max_frames: int = 1 << 20, cap: int = 1 << 28,
                       device="cuda", stream=None):
    """Yield FrameBatch objects in the in-place shape (nexg_pcap_read_raw):
    the file bytes themselves go H2D, frames are described by offsets +
    lengths with the record headers left in place. The batch carries
    NEXG_FRAMES_MONOTONE (records are in file order), so the parse streams each
    256-frame group as one span through the gaps instead of the two-pass
    explicit-length kernels (include/nexg.h)."""
    import torch
    from .engine import FrameBatch
    buf = torch.empty(cap, dtype=torch.uint8, pin_memory=True)
    offs = torch.empty(max_frames, dtype=torch.int64, pin_memory=True)
    lens = torch.empty(max_frames, dtype=torch.int32, pin_memory=True)
    bnp, onp, lnp = buf.numpy(), offs.numpy().view(np.uint64), lens.numpy().view(np.uint32)
    while True:
        n, used = reader.read_raw_into(bnp, onp, lnp)
        if n == 0 and used == 0:
            return
        s = stream or torch.cuda.current_stream()
        with torch.cuda.stream(s):
            d = buf[:max(used, 1)].to(device, non_blocking=True)
            o = offs[:max(n, 1)].to(device, non_blocking=True)
            ln = lens[:max(n, 1)].to(device, non_blocking=True)
        s.synchronize()  # the pinned staging buffers are reused by the next read
        yield FrameBatch(data=d[:used], count=n, offsets=o[:n], lengths=ln[:n], hints=abi.FRAMES_MONOTONE)


def mapped_frames(reader: PcapReader, window: int = 1 << 22, max_frames: int = 1 << 14) -> Iterator[bytes]:
    """All frames via the zero-copy shape (test / inspection helper)."""
    arr, pos = reader.map()
    offs = np.empty(max_frames, np.uint64)
    lens = np.empty(max_frames, np.uint32)
    while pos < len(arr):
        n, nxt = reader.walk_mapped(pos, window, offs, lens)
        for k in range(n):
            a = pos + int(offs[k])
            yield bytes(arr[a:a + int(lens[k])])
        pos = nxt


def device_mapped_batches(reader: PcapReader, max_frames: int = 1 << 20, window: int = 1 << 28,
                          device="cuda", stream=None):
    """Yield FrameBatch objects in the zero-copy shape (nexg_pcap_map /
    nexg_pcap_walk_mapped): the file's page-cache mapping is registered for
    DMA (hipHostRegister, one window-sized chunk at a time as the walk
    reaches it) and each window of complete records goes H2D as is,
    record headers in place, described by offsets + lengths with
    NEXG_FRAMES_MONOTONE — no host copy of the frame bytes, so the rate is
    the PCIe rate. Parse each batch on `stream` before asking for the next
    (the device window and the offset staging are reused)."""
    import torch
    from .engine import FrameBatch
    arr, pos = reader.map()
    size = len(arr)
    if pos >= size:
        return
    hip = ctypes.CDLL("libamdhip64.so")  # torch's HIP runtime (already loaded)
    base = arr.ctypes.data
    chunk = window  # registered for DMA chunk by chunk as the walk reaches it
    registered = []  # chunk indices currently page-locked (at most the two the window touches)
    nxt_chunk = [0]

    def register_upto(end):
        for c in range(nxt_chunk[0], (min(end, size) + chunk - 1) // chunk):
            a, b = c * chunk, min(size, (c + 1) * chunk)
            if hip.hipHostRegister(ctypes.c_void_p(base + a), ctypes.c_size_t(b - a), ctypes.c_uint(0)) != 0:
                raise PcapError("hipHostRegister of the capture mapping failed")
            registered.append(c)
            nxt_chunk[0] = c + 1

    def unregister_below(p):  # chunks wholly behind the walk: their copies have completed
        while registered and (registered[0] + 1) * chunk <= p:
            hip.hipHostUnregister(ctypes.c_void_p(base + registered.pop(0) * chunk))
    s = stream or torch.cuda.current_stream()
    try:
        buf = torch.empty(window, dtype=torch.uint8, device=device)
        offs = torch.empty(max_frames, dtype=torch.int64, pin_memory=True)
        lens = torch.empty(max_frames, dtype=torch.int32, pin_memory=True)
        onp, lnp = offs.numpy().view(np.uint64), lens.numpy().view(np.uint32)
        while pos < size:
            s.synchronize()  # the previous batch's copies and parse are done with the staging
            unregister_below(pos)  # a capture may be far larger than host memory: pin only the window
            register_upto(pos + window)
            n, nxt = reader.walk_mapped(pos, window, onp, lnp)
            if n == 0:  # pcapng blocks without packets
                pos = nxt
                continue
            nbytes = nxt - pos
            a = pos
            while a < nxt:  # one copy per registered chunk the window touches
                b = min(nxt, (a // chunk + 1) * chunk)
                if hip.hipMemcpyAsync(ctypes.c_void_p(buf.data_ptr() + a - pos), ctypes.c_void_p(base + a),
                                      ctypes.c_size_t(b - a), ctypes.c_int(1), ctypes.c_void_p(s.cuda_stream)) != 0:
                    raise PcapError("H2D copy from the capture mapping failed")
                a = b
            with torch.cuda.stream(s):
                o = offs[:n].to(device, non_blocking=True)
                ln = lens[:n].to(device, non_blocking=True)
            yield FrameBatch(data=buf[:nbytes], count=n, offsets=o, lengths=ln, hints=abi.FRAMES_MONOTONE)
            pos = nxt
    finally:
        s.synchronize()
        for c in registered:
            hip.hipHostUnregister(ctypes.c_void_p(base + c * chunk))
