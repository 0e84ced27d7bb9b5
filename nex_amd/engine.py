"""Batched device engine over the C ABI (include/nexg.h).

torch is used only as device-memory / stream plumbing: frames, offsets and
outputs are torch CUDA(HIP) tensors whose data pointers go straight to
libnexg.so, and work is enqueued on torch's current stream.
"""
import ctypes
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from . import abi
from ._lib import load
from .frame import ParseMode, ParseOption


class NexgError(RuntimeError):
    def __init__(self, status, message=""):
        super().__init__(f"nexg error {status}: {message}")
        self.status = status


def _torch():
    import torch
    return torch


def u32_tensor(values, device="cuda"):
    """Device tensor holding u32 values (stored as int32 bit patterns)."""
    a = np.asarray(values, dtype=np.uint64).astype(np.uint32).view(np.int32)
    return _torch().from_numpy(np.ascontiguousarray(a)).to(device)


def u16_tensor(values, device="cuda"):
    """Device tensor holding u16 values (stored as int16 bit patterns)."""
    a = np.asarray(values, dtype=np.uint64).astype(np.uint16).view(np.int16)
    return _torch().from_numpy(np.ascontiguousarray(a)).to(device)


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


@dataclass
class FrameBatch:
    """A device-resident batch of raw frames (nexg_frames).

    data     uint8 tensor on the device
    offsets  int64 tensor (count or count+1 entries), or a uint8 tensor
             holding a NEXG_FRAMES_OFFSETS32 table (abi.offsets32_table;
             hints must carry abi.FRAMES_OFFSETS32), or None (fixed stride)
    lengths  int32 tensor or None
    """
    data: "object"
    count: int
    stride: int = 0
    offsets: Optional[object] = None
    lengths: Optional[object] = None
    hints: int = 0  # abi.FRAMES_* (nexg_frames.hints)

    def to_c(self):
        return abi.Frames(
            data=self.data.data_ptr() if self.count else None,
            data_bytes=self.data.numel(),
            offsets=None if self.offsets is None else self.offsets.data_ptr(),
            lengths=None if self.lengths is None else self.lengths.data_ptr(),
            stride=self.stride, hints=self.hints, count=self.count)

    def host_offsets(self):
        """Host int64 array of the table's offsets (count + 1 entries for a
        packed batch), decoding a NEXG_FRAMES_OFFSETS32 table."""
        if self.hints & abi.FRAMES_OFFSETS32:
            return abi.offsets32_decode(self.offsets.cpu().numpy(), self.count,
                                        self.data.numel()).astype(np.int64)
        return self.offsets.cpu().numpy().astype(np.int64)

    def frame_lengths(self):
        """Host int64 array of every frame's length (the nexg_frames rules)."""
        if self.lengths is not None:
            return self.lengths[: self.count].cpu().numpy().astype(np.int64)
        if self.offsets is not None:
            return np.diff(self.host_offsets()[: self.count + 1])
        return np.full(self.count, self.stride, np.int64)

    @property
    def total_bytes(self):
        if self.lengths is not None:
            return int(self.lengths.sum().item())
        if self.offsets is not None and self.hints & abi.FRAMES_OFFSETS32:
            o = self.host_offsets()
            return int(o[self.count] - o[0])
        if self.offsets is not None:
            return int((self.offsets[self.count] - self.offsets[0]).item())
        return self.count * self.stride

    def with_offsets32(self):
        """The same frames described by a NEXG_FRAMES_OFFSETS32 table (4 B per
        frame instead of 8, plus one 8-B base per 256 frames over 4 GiB)."""
        torch = _torch()
        assert self.offsets is not None and not self.hints & abi.FRAMES_OFFSETS32
        n = self.count + (0 if self.lengths is not None else 1)
        o = self.offsets[:n].cpu().numpy().astype(np.uint64)
        if self.lengths is not None:  # count entries: the table still has count + 1 slots
            o = np.concatenate([o, o[-1:] if len(o) else np.zeros(1, np.uint64)])
        t = torch.from_numpy(abi.offsets32_table(o, self.data.numel())).to(self.data.device)
        return FrameBatch(data=self.data, count=self.count, stride=self.stride, offsets=t, lengths=self.lengths,
                          hints=self.hints | abi.FRAMES_OFFSETS32)

    @classmethod
    def from_frames(cls, frames: Sequence[bytes], device="cuda", pad_to=4):
        """Pack host frames back to back (each start aligned to `pad_to`)."""
        torch = _torch()
        offs = np.zeros(len(frames) + 1, dtype=np.int64)
        lens = np.array([len(f) for f in frames], dtype=np.int32)
        pos = 0
        for i, f in enumerate(frames):
            offs[i] = pos
            pos += (len(f) + pad_to - 1) // pad_to * pad_to
        offs[len(frames)] = pos
        buf = np.zeros(max(pos, 16), dtype=np.uint8)
        for i, f in enumerate(frames):
            buf[offs[i]:offs[i] + len(f)] = np.frombuffer(bytes(f), dtype=np.uint8)
        return cls(data=torch.from_numpy(buf).to(device), count=len(frames),
                   offsets=torch.from_numpy(offs).to(device),
                   lengths=torch.from_numpy(lens).to(device))

    @classmethod
    def from_packed(cls, frames: Sequence[bytes], device="cuda", pad_to=1, shift=0):
        """Offset table only (lengths implied by consecutive offsets): frames
        zero-padded to `pad_to`, back to back, starting `shift` bytes into an
        allocation (the packed layout nexg_parse_batch streams by spans)."""
        torch = _torch()
        padded = [bytes(f) + bytes((-len(f)) % pad_to) for f in frames]
        offs = np.zeros(len(padded) + 1, dtype=np.int64)
        offs[1:] = np.cumsum([len(f) for f in padded])
        buf = np.zeros(shift + int(offs[-1]) + 16, dtype=np.uint8)
        buf[shift:shift + int(offs[-1])] = np.frombuffer(b"".join(padded), dtype=np.uint8)
        dev = torch.from_numpy(buf).to(device)
        return cls(data=dev[shift:shift + int(offs[-1])], count=len(padded),
                   offsets=torch.from_numpy(offs).to(device))

    @classmethod
    def from_strided(cls, array: np.ndarray, device="cuda", lengths=None):
        """count x stride uint8 host array -> fixed-stride device batch."""
        torch = _torch()
        count, stride = array.shape
        data = torch.from_numpy(np.ascontiguousarray(array).reshape(-1)).to(device)
        lt = None if lengths is None else torch.from_numpy(np.asarray(lengths, np.int32)).to(device)
        return cls(data=data, count=count, stride=stride, lengths=lt)


class Engine:
    """One nexg context bound to one gfx950 device (nexg_ctx_create)."""

    def __init__(self, device: int = 0):
        self.lib = load()
        torch = _torch()
        self.device = device
        self.torch_device = torch.device("cuda", device)
        h = ctypes.c_void_p()
        rc = self.lib.nexg_ctx_create(device, ctypes.byref(h))
        if rc != abi.OK:
            raise NexgError(rc, self.lib.nexg_strerror(rc).decode())
        self.ctx = h

    def close(self):
        if self.ctx:
            self.lib.nexg_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def cu_count(self):
        return self.lib.nexg_ctx_cu_count(self.ctx)

    def _stream(self, stream):
        torch = _torch()
        s = stream if stream is not None else torch.cuda.current_stream(self.torch_device)
        return ctypes.c_void_p(s.cuda_stream)

    def _check(self, rc):
        if rc != abi.OK:
            raise NexgError(rc, self.lib.nexg_ctx_last_error(self.ctx).decode())

    # --- hot path -------------------------------------------------------
    def parse(self, batch: FrameBatch, option: ParseOption = ParseOption(),
              mode: ParseMode = ParseMode.Lenient, out_kind: int = abi.OUT_DESC,
              out=None, stream=None):
        """Frame::try_from_buf_with_mode on every frame (frame.rs:309), or
        FrameSlice::try_from_buf (frame.rs:86) with out_kind=OUT_SLICE.

        Returns a uint8 device tensor holding nexg_desc[count] (8 B each),
        nexg_record[count] (64 B), nexg_slice[count] (16 B) or, with
        out_kind=OUT_FLAGS, the nexg_desc.flags word alone (4 B), or with
        OUT_VERDICT its lossless 2-B form (abi.verdict_to_flags)."""
        torch = _torch()
        nbytes = self.out_bytes(out_kind, batch.count)
        if out is None:
            out = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=self.torch_device)
        elif out.numel() * out.element_size() < nbytes or out.device != self.torch_device:
            raise ValueError(f"out holds {out.numel() * out.element_size()} B on {out.device}; "
                             f"{nbytes} B on {self.torch_device} needed")
        fr = batch.to_c()
        opt = abi.ParseOptionC(option.flags(mode), option.offset)
        self._check(self.lib.nexg_parse_batch(self.ctx, ctypes.byref(fr), ctypes.byref(opt), out_kind,
                                              _ptr(out), self._stream(stream)))
        return out

    @staticmethod
    def out_bytes(out_kind, count):
        """Bytes of a nexg_parse_batch output of `out_kind` for `count` frames."""
        if out_kind == abi.OUT_SPARSE:
            return abi.sparse_bytes(count)
        if out_kind == abi.OUT_GROUPED:
            return abi.grouped_offsets(count)[3]
        return count * {abi.OUT_DESC: 8, abi.OUT_RECORD: 64, abi.OUT_SLICE: 16, abi.OUT_FLAGS: 4,
                        abi.OUT_VERDICT: 2}[out_kind]

    def parse_to_numpy(self, batch, option=ParseOption(), mode=ParseMode.Lenient,
                       out_kind=abi.OUT_RECORD):
        """Host copy of the parse output; OUT_SPARSE / OUT_GROUPED come back
        decoded on the host into nexg_desc (abi.sparse_to_desc / grouped_to_desc)."""
        out = self.parse(batch, option, mode, out_kind)
        _torch().cuda.synchronize(self.torch_device)
        if out_kind in (abi.OUT_SPARSE, abi.OUT_GROUPED):
            dec = abi.sparse_to_desc if out_kind == abi.OUT_SPARSE else abi.grouped_to_desc
            return dec(out.cpu().numpy(), batch.count, batch.frame_lengths(), option.flags(mode), option.offset)
        dt = {abi.OUT_DESC: abi.DESC_DTYPE, abi.OUT_RECORD: abi.RECORD_DTYPE,
              abi.OUT_SLICE: abi.SLICE_DTYPE, abi.OUT_FLAGS: abi.FLAGS_DTYPE,
              abi.OUT_VERDICT: abi.VERDICT_DTYPE}[out_kind]
        return out.cpu().numpy()[: batch.count * dt.itemsize].view(dt)

    def sparse_expand(self, batch: FrameBatch, sparse, option: ParseOption = ParseOption(),
                      mode: ParseMode = ParseMode.Lenient, out=None, stream=None, grouped=False):
        """nexg_desc[count] (uint8 device tensor) from a NEXG_OUT_SPARSE output
        (grouped=True: NEXG_OUT_GROUPED) of the same batch and option
        (nexg_sparse_expand / nexg_grouped_expand)."""
        torch = _torch()
        if out is None:
            out = torch.empty(max(batch.count, 1) * 8, dtype=torch.uint8, device=self.torch_device)
        fr = batch.to_c()
        opt = abi.ParseOptionC(option.flags(mode), option.offset)
        fn = self.lib.nexg_grouped_expand if grouped else self.lib.nexg_sparse_expand
        self._check(fn(self.ctx, ctypes.byref(fr), ctypes.byref(opt), _ptr(sparse), _ptr(out), self._stream(stream)))
        return out

    def recompute_checksums(self, batch: FrameBatch, which: int = abi.FIX_IP | abi.FIX_L4,
                            option: ParseOption = ParseOption(), report=True, stream=None):
        """In-place checksum fix-up of batch.data with the mutable views'
        raw-buffer semantics (nexg_recompute_checksums_batch; ipv4.rs:669-679,
        udp.rs:338-369, tcp.rs:1009-1040, icmp.rs:372-377, icmpv6.rs:450-470).
        Returns the nexg_fixup[count] report (uint8 device tensor) or None."""
        torch = _torch()
        out = torch.empty(max(batch.count, 1) * 8, dtype=torch.uint8, device=self.torch_device) if report else None
        fr = batch.to_c()
        opt = abi.ParseOptionC(option.flags(ParseMode.Lenient), option.offset)
        self._check(self.lib.nexg_recompute_checksums_batch(self.ctx, ctypes.byref(fr), ctypes.byref(opt), which,
                                                            _ptr(out), self._stream(stream)))
        return out

    def decode_options(self, batch: FrameBatch, records, stream=None):
        """Ipv4Header.options / TcpHeader.options of every frame as positions
        (nexg_decode_options; ipv4.rs:442-508, tcp.rs:767-818). `records` is
        the uint8 device tensor a NEXG_OUT_RECORD parse of `batch` returned."""
        torch = _torch()
        out = torch.empty(max(batch.count, 1) * 96, dtype=torch.uint8, device=self.torch_device)
        fr = batch.to_c()
        self._check(self.lib.nexg_decode_options(self.ctx, ctypes.byref(fr), _ptr(records), _ptr(out),
                                                 self._stream(stream)))
        return out

    def probe_stream(self, data, write8, out=None, stream=None):
        """Calibration stream over a uint8 device tensor (nexg_probe_stream):
        the parse kernels' load shape, read-only or with the 8-B-per-64-B
        descriptor store stream (write8 = 9: that stream at the fixed-stride
        parse kernel's 6 workgroups per CU). Not a reference entry point."""
        torch = _torch()
        nbytes = data.numel() // 16384 * 16384
        if out is None:
            n = nbytes // 64 * 8 if write8 else nbytes // 16384 * 4
            out = torch.empty(max(n, 8), dtype=torch.uint8, device=self.torch_device)
        self._check(self.lib.nexg_probe_stream(self.ctx, _ptr(data), nbytes, 9 if write8 == 9 else 8 if write8 else 0,
                                               _ptr(out), self._stream(stream)))
        return out

    def probe_write(self, out, stream=None):
        """Write-only calibration stream (nexg_probe_stream, out_per_64 = 64):
        the builders' copy-out shape over a uint8 device tensor (whole 16-KiB
        tiles). Not a reference entry point."""
        nbytes = out.numel() // 16384 * 16384
        self._check(self.lib.nexg_probe_stream(self.ctx, None, nbytes, 64, _ptr(out), self._stream(stream)))
        return out

    def probe_span_clock(self, batch: FrameBatch, option: ParseOption = ParseOption(),
                         mode: ParseMode = ParseMode.Lenient, out=None, stream=None):
        """One stamped launch of the span kernel over `batch`
        (nexg_probe_span_clock; calibration, not a reference entry point):
        returns (grouped output, stamps) device tensors, stamps int64
        (workgroups, 8) as include/nexg.h lays them out; span_clock_summary
        reduces them on the host."""
        torch = _torch()
        nbytes = self.out_bytes(abi.OUT_GROUPED, batch.count)
        if out is None:
            out = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=self.torch_device)
        nwg = max(1, (batch.count + 255) // 256)
        stamps = torch.zeros((nwg, 8), dtype=torch.int64, device=self.torch_device)
        fr = batch.to_c()
        opt = abi.ParseOptionC(option.flags(mode), option.offset)
        self._check(self.lib.nexg_probe_span_clock(self.ctx, ctypes.byref(fr), ctypes.byref(opt), _ptr(out),
                                                   _ptr(stamps), self._stream(stream)))
        return out, stamps

    def probe_latency(self, buf, steps: int = 2000, start: int = 0, loaded: bool = False, stream=None):
        """Dependent HBM load latency (nexg_probe_latency; calibration, not a
        reference entry point) over a uint8 device scratch tensor (>= 4 MiB):
        returns (ns per step, shader-clock cycles per step)."""
        torch = _torch()
        out = torch.zeros(4, dtype=torch.int64, device=self.torch_device)
        nbytes = buf.numel() // 64 * 64
        self._check(self.lib.nexg_probe_latency(self.ctx, _ptr(buf), nbytes, int(steps), int(start) & 0xFFFFFFFF,
                                                1 if loaded else 0, _ptr(out), self._stream(stream)))
        torch.cuda.synchronize(self.torch_device)
        cyc, ticks = (int(v) for v in out[:2].cpu())
        return ticks * 10.0 / steps, cyc / steps

    def checksum(self, batch: FrameBatch, skipword: int, stream=None):
        """util::checksum(buf, skipword) per buffer (util.rs:65)."""
        torch = _torch()
        out = torch.empty(max(batch.count, 1), dtype=torch.int16, device=self.torch_device)
        fr = batch.to_c()
        skip = min(int(skipword), 0xFFFFFFFF)
        self._check(self.lib.nexg_checksum_batch(self.ctx, ctypes.byref(fr), skip, _ptr(out),
                                                 self._stream(stream)))
        return out[: batch.count]

    # --- serialize path ---------------------------------------------------
    @staticmethod
    def _check_rows(count, row_bytes, shared_ok=False, **arrays):
        """Per-frame parameter arrays hold `count` rows of `row_bytes` each
        (or exactly one row where the builder takes one value for the batch,
        `shared_ok`): the kernels read row i for frame i, so a short array
        would be read past on the device."""
        for name, t in arrays.items():
            if t is None:
                continue
            nb = t.numel() * t.element_size()
            if shared_ok and nb == row_bytes:
                continue
            if nb < count * row_bytes:
                raise ValueError(f"{name} holds {nb} B; {count} frames need {count * row_bytes} B"
                                 + (f" (or one {row_bytes}-B value for the batch)" if shared_ok else ""))

    @staticmethod
    def _check_out(out, count, stride):
        if out is not None and out.numel() * out.element_size() < count * stride:
            raise ValueError(f"out holds {out.numel() * out.element_size()} B; {count} frames of stride "
                             f"{stride} need {count * stride} B")

    def build_udp4(self, src_ip, dst_ip, src_port=None, dst_port=None, ip_id=None,
                   def_src_port=0, def_dst_port=0, def_ip_id=0,
                   src_mac=b"\0" * 6, dst_mac=b"\0" * 6, ttl=64, ip_flags=0, dscp_ecn=0,
                   payload=None, out_stride=None, out=None, stream=None, def_src_ip=0):
        """UdpPacketBuilder -> Ipv4PacketBuilder -> EthernetPacketBuilder
        (udp_ping.rs:68-109) on every tuple. Tensors are int32/int16 device
        tensors holding the u32/u16 values; src_ip=None takes def_src_ip (a
        u32 value) for every frame — with no other array, the udp_ping probe
        batch: one source, one port pair, a destination per frame."""
        torch = _torch()
        count = dst_ip.numel()
        plen = 0 if payload is None else payload.numel()
        stride = out_stride or (42 + plen)
        self._check_rows(count, 4, src_ip=src_ip)
        self._check_rows(count, 2, src_port=src_port, dst_port=dst_port, ip_id=ip_id)
        self._check_out(out, count, stride)
        if out is None:
            out = torch.empty(max(count, 1) * stride, dtype=torch.uint8, device=self.torch_device)
        p = abi.Udp4Build()
        p.src_ip = None if src_ip is None else src_ip.data_ptr()
        p.dst_ip = dst_ip.data_ptr()
        p.def_src_ip = def_src_ip & 0xFFFFFFFF
        p.src_port = None if src_port is None else src_port.data_ptr()
        p.dst_port = None if dst_port is None else dst_port.data_ptr()
        p.ip_id = None if ip_id is None else ip_id.data_ptr()
        p.src_mac = p.dst_mac = None
        p.payload = None if payload is None else payload.data_ptr()
        p.payload_len = plen
        p.def_src_port, p.def_dst_port, p.def_ip_id = def_src_port, def_dst_port, def_ip_id
        p.def_src_mac[:] = list(src_mac)
        p.def_dst_mac[:] = list(dst_mac)
        p.ttl, p.ip_flags, p.dscp_ecn, p.count = ttl, ip_flags, dscp_ecn, count
        self._check(self.lib.nexg_build_udp4_batch(self.ctx, ctypes.byref(p), _ptr(out), stride,
                                                   self._stream(stream)))
        return out

    @staticmethod
    def pack_udp4_tuples(src_ip, dst_ip, src_port, dst_port, ip_id):
        """The five per-frame tuple arrays of build_udp4 (int32 / int16 device
        tensors) as one (count, 4) int32 tensor of 16-B nexg_udp4_tuple records."""
        torch = _torch()
        lo16 = lambda t: t.to(torch.int32) & 0xFFFF
        return torch.stack([src_ip.to(torch.int32), dst_ip.to(torch.int32),
                            lo16(src_port) | (lo16(dst_port) << 16), lo16(ip_id)], dim=1).contiguous()

    def build_udp4_tuples(self, tuples, src_mac=b"\0" * 6, dst_mac=b"\0" * 6, ttl=64, ip_flags=0, dscp_ecn=0,
                          payload=None, out_stride=None, out=None, stream=None):
        """build_udp4 with each frame's tuple as one 16-B record
        (nexg_build_udp4_tuples; `tuples` from pack_udp4_tuples)."""
        torch = _torch()
        count = tuples.shape[0]
        plen = 0 if payload is None else payload.numel()
        stride = out_stride or (42 + plen)
        self._check_rows(count, 16, tuples=tuples)
        self._check_out(out, count, stride)
        if out is None:
            out = torch.empty(max(count, 1) * stride, dtype=torch.uint8, device=self.torch_device)
        p = abi.Udp4Build()
        p.payload = None if payload is None else payload.data_ptr()
        p.payload_len = plen
        p.def_src_mac[:] = list(src_mac)
        p.def_dst_mac[:] = list(dst_mac)
        p.ttl, p.ip_flags, p.dscp_ecn, p.count = ttl, ip_flags, dscp_ecn, count
        self._check(self.lib.nexg_build_udp4_tuples(self.ctx, ctypes.byref(p), _ptr(tuples), _ptr(out), stride,
                                                    self._stream(stream)))
        return out

    def build_udp6(self, src_ip, dst_ip, src_port=None, dst_port=None, def_src_port=0,
                   def_dst_port=0, src_mac=b"\0" * 6, dst_mac=b"\0" * 6, hop_limit=64,
                   traffic_class=0, flow_label=0, payload=None, out_stride=None, out=None,
                   stream=None):
        """udp_ping's IPv6 branch (udp_ping.rs:83-89): UdpPacketBuilder ->
        Ipv6PacketBuilder -> EthernetPacketBuilder on every tuple. src_ip /
        dst_ip are (count, 16) uint8 device tensors in network order; src_ip
        may be one address (every frame's source: the probe batch)."""
        torch = _torch()
        count = dst_ip.shape[0] if dst_ip.dim() > 1 else dst_ip.numel() // 16
        plen = 0 if payload is None else payload.numel()
        stride = out_stride or (62 + plen)
        self._check_rows(count, 16, shared_ok=True, src_ip=src_ip)
        self._check_rows(count, 2, src_port=src_port, dst_port=dst_port)
        self._check_out(out, count, stride)
        if out is None:
            out = torch.empty(max(count, 1) * stride, dtype=torch.uint8, device=self.torch_device)
        p = abi.Udp6Build()
        p.src_ip, p.dst_ip = src_ip.data_ptr(), dst_ip.data_ptr()
        p.src_shared = 1 if src_ip.numel() == 16 and count != 1 else 0
        p.src_port = None if src_port is None else src_port.data_ptr()
        p.dst_port = None if dst_port is None else dst_port.data_ptr()
        p.src_mac = p.dst_mac = None
        p.payload = None if payload is None else payload.data_ptr()
        p.payload_len = plen
        p.flow_label = flow_label
        p.def_src_port, p.def_dst_port = def_src_port, def_dst_port
        p.def_src_mac[:] = list(src_mac)
        p.def_dst_mac[:] = list(dst_mac)
        p.hop_limit, p.traffic_class, p.count = hop_limit, traffic_class, count
        self._check(self.lib.nexg_build_udp6_batch(self.ctx, ctypes.byref(p), _ptr(out), stride,
                                                   self._stream(stream)))
        return out

    @staticmethod
    def _ip_build(family, src_ip, dst_ip, ip_id, def_ip_id, src_mac, dst_mac, ttl, ip_flags, tos,
                  flow_label):
        """src_ip: (count, 4|16) per frame, or ONE address ((4|16,) or (1, 4|16)):
        the probe batches' single source (nexg_ip_build.src_shared)."""
        ip = abi.IpBuild()
        ip.src_ip, ip.dst_ip = src_ip.data_ptr(), dst_ip.data_ptr()
        w = 4 if family == 4 else 16
        ip.src_shared = 1 if src_ip.numel() == w and dst_ip.numel() != w else 0
        ip.ip_id = None if ip_id is None else ip_id.data_ptr()
        ip.src_mac = ip.dst_mac = None
        ip.family, ip.flow_label, ip.def_ip_id = family, flow_label, def_ip_id
        ip.def_src_mac[:] = list(src_mac)
        ip.def_dst_mac[:] = list(dst_mac)
        ip.ttl, ip.ip_flags, ip.tos = ttl, ip_flags, tos
        return ip

    def build_tcp(self, family, src_ip, dst_ip, src_port=None, dst_port=None, seq=None, ack=None,
                  def_src_port=0, def_dst_port=0, def_seq=0, def_ack=0, flags=0, window=0xFFFF,
                  urgent_ptr=0, options=b"", payload=None, ip_id=None, def_ip_id=0,
                  src_mac=b"\0" * 6, dst_mac=b"\0" * 6, ttl=64, ip_flags=0, tos=0, flow_label=0,
                  out_stride=None, out=None, stream=None):
        """tcp_ping (examples/tcp_ping.rs:111-163): TcpPacketBuilder -> IPv4/IPv6
        builder -> EthernetPacketBuilder on every tuple. Addresses are
        (count, 4|16) uint8 device tensors (src_ip may be one address: every
        frame's source); ports/ids int16, seq/ack int32. One source, a
        destination per frame and no other array is tcp_ping's probe batch."""
        torch = _torch()
        count = dst_ip.shape[0]
        plen = 0 if payload is None else payload.numel()
        padded = (len(options) + 3) // 4 * 4
        flen = 14 + (20 if family == 4 else 40) + 20 + padded + plen
        stride = out_stride or flen
        w = 4 if family == 4 else 16
        self._check_rows(count, w, shared_ok=True, src_ip=src_ip)
        self._check_rows(count, 2, src_port=src_port, dst_port=dst_port, ip_id=ip_id)
        self._check_rows(count, 4, seq=seq, ack=ack)
        self._check_out(out, count, stride)
        if out is None:
            out = torch.empty(max(count, 1) * stride, dtype=torch.uint8, device=self.torch_device)
        p = abi.TcpBuild()
        p.ip = self._ip_build(family, src_ip, dst_ip, ip_id, def_ip_id, src_mac, dst_mac, ttl,
                              ip_flags, tos, flow_label)
        p.src_port = None if src_port is None else src_port.data_ptr()
        p.dst_port = None if dst_port is None else dst_port.data_ptr()
        p.seq = None if seq is None else seq.data_ptr()
        p.ack = None if ack is None else ack.data_ptr()
        p.payload = None if payload is None else payload.data_ptr()
        p.payload_len = plen
        p.def_seq, p.def_ack, p.def_src_port, p.def_dst_port = def_seq, def_ack, def_src_port, def_dst_port
        p.window, p.urgent_ptr, p.flags = window, urgent_ptr, flags
        p.options_len = min(len(options), 255)
        p.options[:min(len(options), 40)] = list(options[:40])
        p.count = count
        self._check(self.lib.nexg_build_tcp_batch(self.ctx, ctypes.byref(p), _ptr(out), stride,
                                                  self._stream(stream)))
        return out

    def build_icmp_echo(self, family, src_ip, dst_ip, identifier=None, sequence=None,
                        def_identifier=0, def_sequence=0, icmp_type=None, icmp_code=0, payload=None,
                        ip_id=None, def_ip_id=0, src_mac=b"\0" * 6, dst_mac=b"\0" * 6, ttl=64,
                        ip_flags=0, tos=0, flow_label=0, out_stride=None, out=None, stream=None):
        """icmp_ping (examples/icmp_ping.rs:67-102): Icmp(v6)PacketBuilder with
        echo_fields -> IPv4/IPv6 builder -> EthernetPacketBuilder. src_ip may
        be one address (every frame's source: icmp_ping's probe batch)."""
        torch = _torch()
        count = dst_ip.shape[0]
        plen = 0 if payload is None else payload.numel()
        flen = 14 + (20 if family == 4 else 40) + 8 + plen
        stride = out_stride or flen
        w = 4 if family == 4 else 16
        self._check_rows(count, w, shared_ok=True, src_ip=src_ip)
        self._check_rows(count, 2, identifier=identifier, sequence=sequence, ip_id=ip_id)
        self._check_out(out, count, stride)
        if out is None:
            out = torch.empty(max(count, 1) * stride, dtype=torch.uint8, device=self.torch_device)
        p = abi.IcmpEchoBuild()
        p.ip = self._ip_build(family, src_ip, dst_ip, ip_id, def_ip_id, src_mac, dst_mac, ttl,
                              ip_flags, tos, flow_label)
        p.identifier = None if identifier is None else identifier.data_ptr()
        p.sequence = None if sequence is None else sequence.data_ptr()
        p.payload = None if payload is None else payload.data_ptr()
        p.payload_len = plen
        p.def_identifier, p.def_sequence = def_identifier, def_sequence
        p.icmp_type = (8 if family == 4 else 128) if icmp_type is None else icmp_type
        p.icmp_code = icmp_code
        p.count = count
        self._check(self.lib.nexg_build_icmp_echo_batch(self.ctx, ctypes.byref(p), _ptr(out), stride,
                                                        self._stream(stream)))
        return out

    # --- synthetic workloads ----------------------------------------------
    def build_arp(self, target_ip, sender_ip=None, def_sender_ip=b"\0" * 4, sender_mac=None,
                  def_sender_mac=b"\0" * 6, target_mac=None, def_target_mac=b"\0" * 6, eth_dst=None,
                  def_eth_dst=b"\xff" * 6, hardware_type=1, protocol_type=0x0800, operation=1,
                  hw_addr_len=6, proto_addr_len=4, out_stride=42, out=None, stream=None):
        """examples/arp.rs:59-67: ArpPacketBuilder::new(sender_mac, sender_ip,
        target_ip) (builder/arp.rs) behind EthernetPacketBuilder (broadcast
        destination) on every target. Addresses are (count, 4) / (count, 6)
        uint8 device tensors or None for the defaults."""
        torch = _torch()
        count = target_ip.shape[0]
        if out is None:
            out = torch.empty(max(count, 1) * out_stride, dtype=torch.uint8, device=self.torch_device)
        p = abi.ArpBuild()
        p.target_ip = target_ip.data_ptr()
        p.sender_ip = None if sender_ip is None else sender_ip.data_ptr()
        p.sender_mac = None if sender_mac is None else sender_mac.data_ptr()
        p.target_mac = None if target_mac is None else target_mac.data_ptr()
        p.eth_dst = None if eth_dst is None else eth_dst.data_ptr()
        p.def_sender_ip[:] = list(def_sender_ip)
        p.def_sender_mac[:] = list(def_sender_mac)
        p.def_target_mac[:] = list(def_target_mac)
        p.def_eth_dst[:] = list(def_eth_dst)
        p.hardware_type, p.protocol_type, p.operation = hardware_type, protocol_type, operation
        p.hw_addr_len, p.proto_addr_len = hw_addr_len, proto_addr_len
        p.count = count
        self._check(self.lib.nexg_build_arp_batch(self.ctx, ctypes.byref(p), _ptr(out), out_stride,
                                                  self._stream(stream)))
        return out

    def build_ndp_ns(self, src_ip, target_ip, src_mac=b"\0" * 6, dst_mac=None, hop_limit=255, tos=0,
                     flow_label=0, out_stride=86, out=None, stream=None):
        """examples/ndp.rs:82-108: NdpPacketBuilder::new(src_mac, src_ip,
        target) (builder/ndp.rs) -> Ipv6PacketBuilder (next header 58, hop
        limit 255) -> EthernetPacketBuilder with destination 33:33 + the
        target's last four bytes (ipv6_multicast_mac), or `dst_mac` when
        given. Addresses are (count, 16) uint8 device tensors."""
        torch = _torch()
        count = target_ip.shape[0]
        if out is None:
            out = torch.empty(max(count, 1) * out_stride, dtype=torch.uint8, device=self.torch_device)
        p = abi.NdpNsBuild()
        p.ip = self._ip_build(6, src_ip, target_ip, None, 0, src_mac, dst_mac or b"\0" * 6, hop_limit, 0, tos,
                              flow_label)
        p.eth_dst_multicast = 1 if dst_mac is None else 0
        p.count = count
        self._check(self.lib.nexg_build_ndp_ns_batch(self.ctx, ctypes.byref(p), _ptr(out), out_stride,
                                                     self._stream(stream)))
        return out

    def gen_batch(self, workload: int, count: int, seed: int = abi.DEFAULT_SEED,
                  first_index: int = 0, stream=None, record_gap: int = 0) -> FrameBatch:
        """Device-generated SURVEY.md App. C workload (UDP64: fixed 64-B
        stride; IMIX: packed with an int64 offset table of count+1 entries).
        record_gap > 0 (IMIX): each frame preceded by that many zero bytes and
        described by offsets + lengths + the monotone hint, the shape
        nexg_pcap_read_raw hands over (16 = classic pcap record headers)."""
        torch = _torch()
        dev = self.torch_device
        s = self._stream(stream)
        if workload == abi.WL_UDP64:
            data = torch.empty(max(count, 1) * 64, dtype=torch.uint8, device=dev)
            self._check(self.lib.nexg_gen_frames(self.ctx, workload, seed, first_index, count,
                                                 _ptr(data), None, 64, s))
            return FrameBatch(data=data, count=count, stride=64)
        lengths = torch.empty(max(count, 1), dtype=torch.int32, device=dev)
        self._check(self.lib.nexg_gen_lengths(self.ctx, workload, seed, first_index, count,
                                              _ptr(lengths), s))
        offsets = torch.zeros(count + 1, dtype=torch.int64, device=dev)
        if count:
            torch.cumsum(lengths[:count].to(torch.int64) + record_gap, 0, out=offsets[1:])
        total = int(offsets[count].item()) if count else 0
        if record_gap:
            offsets = offsets + record_gap  # frame i starts after its record header
            data = torch.zeros(max(total, 16) + 16, dtype=torch.uint8, device=dev)
        else:
            data = torch.empty(max(total, 16) + 16, dtype=torch.uint8, device=dev)
        self._check(self.lib.nexg_gen_frames(self.ctx, workload, seed, first_index, count,
                                             _ptr(data), _ptr(offsets), 0, s))
        if record_gap:
            return FrameBatch(data=data[:max(total, 16)], count=count, offsets=offsets,
                              lengths=lengths, hints=abi.FRAMES_MONOTONE)
        return FrameBatch(data=data, count=count, offsets=offsets)

    def gen_udp4_params(self, count, seed=abi.DEFAULT_SEED, first_index=0, stream=None):
        torch = _torch()
        dev = self.torch_device
        t32 = [torch.empty(max(count, 1), dtype=torch.int32, device=dev) for _ in range(2)]
        t16 = [torch.empty(max(count, 1), dtype=torch.int16, device=dev) for _ in range(3)]
        self._check(self.lib.nexg_gen_udp4_params(self.ctx, seed, first_index, count,
                                                  *[_ptr(t) for t in t32 + t16], self._stream(stream)))
        return [t[:count] for t in t32 + t16]
