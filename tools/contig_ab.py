#!/usr/bin/env python3
"""Does a physically contiguous allocation remove the placement spread of a
packed batch? The real-traffic (or mix / IMIX) batch is copied into N
allocations made by hipExtMallocWithFlags with the default flags and N made
with hipDeviceMallocContiguous, interleaved and all kept alive, and every copy
is timed twice with HIP events (grouped output, the bench's kernel).
usage: python tools/contig_ab.py [--workload real|mix|imix] [--copies 4]"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HIP_DEVICE_MALLOC_DEFAULT = 0x0
HIP_DEVICE_MALLOC_CONTIGUOUS = 0x4  # hip_runtime_api.h: hipDeviceMallocContiguous
HIP_MEMCPY_D2D = 3


class RawBuf:
    """A device allocation made outside torch, shaped like the tensor
    FrameBatch reads (data_ptr / numel)."""

    def __init__(self, hip, nbytes, flags):
        p = ctypes.c_void_p()
        rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(nbytes), ctypes.c_uint(flags))
        if rc != 0:
            raise RuntimeError(f"hipExtMallocWithFlags({nbytes}, {flags:#x}) = {rc}")
        self.hip, self.ptr, self.nbytes = hip, p.value, nbytes

    def data_ptr(self):
        return self.ptr

    def numel(self):
        return self.nbytes

    def free(self):
        self.hip.hipFree(ctypes.c_void_p(self.ptr))


class _Loc(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("id", ctypes.c_int)]


class _AllocFlags(ctypes.Structure):
    _fields_ = [("compressionType", ctypes.c_ubyte), ("gpuDirectRDMACapable", ctypes.c_ubyte),
                ("usage", ctypes.c_ushort)]


class _AllocProp(ctypes.Structure):  # hipMemAllocationProp
    _fields_ = [("type", ctypes.c_int), ("requestedHandleType", ctypes.c_int), ("location", _Loc),
                ("win32HandleMetaData", ctypes.c_void_p), ("allocFlags", _AllocFlags)]


class _AccessDesc(ctypes.Structure):  # hipMemAccessDesc
    _fields_ = [("location", _Loc), ("flags", ctypes.c_int)]


class VmmBuf:
    """A device allocation through the virtual memory API: one physical
    handle (hipMemCreate) mapped into a reserved range aligned to `align`."""

    def __init__(self, hip, nbytes, align=1 << 30, device=0):
        prop = _AllocProp(type=1, requestedHandleType=0, location=_Loc(1, device))
        g = ctypes.c_size_t()
        rc = hip.hipMemGetAllocationGranularity(ctypes.byref(g), ctypes.byref(prop), ctypes.c_int(1))
        if rc != 0:
            raise RuntimeError(f"hipMemGetAllocationGranularity = {rc}")
        self.gran = g.value
        size = (nbytes + self.gran - 1) // self.gran * self.gran
        p, h = ctypes.c_void_p(), ctypes.c_void_p()
        for call, args in (("hipMemAddressReserve", (ctypes.byref(p), ctypes.c_size_t(size), ctypes.c_size_t(align),
                                                      None, ctypes.c_ulonglong(0))),
                           ("hipMemCreate", (ctypes.byref(h), ctypes.c_size_t(size), ctypes.byref(prop),
                                             ctypes.c_ulonglong(0)))):
            rc = getattr(hip, call)(*args)
            if rc != 0:
                raise RuntimeError(f"{call} = {rc}")
        rc = hip.hipMemMap(p, ctypes.c_size_t(size), ctypes.c_size_t(0), h, ctypes.c_ulonglong(0))
        if rc != 0:
            raise RuntimeError(f"hipMemMap = {rc}")
        desc = _AccessDesc(location=_Loc(1, device), flags=3)
        rc = hip.hipMemSetAccess(p, ctypes.c_size_t(size), ctypes.byref(desc), ctypes.c_size_t(1))
        if rc != 0:
            raise RuntimeError(f"hipMemSetAccess = {rc}")
        self.hip, self.ptr, self.h, self.size, self.nbytes = hip, p.value, h, size, nbytes

    def data_ptr(self):
        return self.ptr

    def numel(self):
        return self.nbytes

    def free(self):
        self.hip.hipMemUnmap(ctypes.c_void_p(self.ptr), ctypes.c_size_t(self.size))
        self.hip.hipMemRelease(self.h)
        self.hip.hipMemAddressFree(ctypes.c_void_p(self.ptr), ctypes.c_size_t(self.size))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="real")
    ap.add_argument("--copies", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--outs", default="", help="map mode: extra output kinds (flags,desc,sparse,fresh_grouped) per allocation")
    ap.add_argument("--clock", action="store_true", help="map mode: span kernel clock stamps on each allocation")
    ap.add_argument("--latency", action="store_true", help="map mode: k_chase latency on each allocation")
    ap.add_argument("--libs", default="", help="map mode: extra library builds timed on each allocation")
    ap.add_argument("--vmm", type=int, default=0,
                    help="N default and N virtual-memory-API allocations, interleaved, each timed twice")
    ap.add_argument("--map", type=int, default=0,
                    help="N default allocations timed in order; then the first half freed and refilled")
    args = ap.parse_args()
    import torch
    from nex_amd import abi, workloads
    from nex_amd.engine import Engine, FrameBatch
    from nex_amd import _lib
    extra = []
    for path in filter(None, args.libs.split(",")):
        _lib._lib, _lib.LIB_PATH = None, os.path.abspath(path)
        extra.append((os.path.basename(path), Engine(0)))
    _lib._lib, _lib.LIB_PATH = None, os.path.join(ROOT, "nex_amd", "libnexg.so")
    eng = Engine(0)
    hip = ctypes.CDLL("libamdhip64.so")
    if args.workload == "imix":
        b = eng.gen_batch(abi.WL_IMIX, 16 << 20)
    else:
        mk = workloads.malformed_mix if args.workload == "mix" else workloads.real_traffic
        m, _ = mk(eng, 1 << 20, seed=abi.DEFAULT_SEED + (0 if args.workload == "mix" else 7))
        b = workloads.tiled(m, 16)
    out = torch.empty(Engine.out_bytes(abi.OUT_GROUPED, b.count), dtype=torch.uint8, device="cuda")
    kinds = {"flags": abi.OUT_FLAGS, "desc": abi.OUT_DESC, "sparse": abi.OUT_SPARSE}
    outs_by_kind = {k: torch.empty(Engine.out_bytes(v, b.count), dtype=torch.uint8, device="cuda")
                    for k, v in kinds.items() if k in args.outs.split(",")}
    s = torch.cuda.current_stream()
    torch.cuda.synchronize()

    def time_batch(c, e=None, kind=abi.OUT_GROUPED, o=None):
        e, o = e or eng, out if o is None else o
        for _ in range(10):
            e.parse(c, out_kind=kind, out=o, stream=s)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(s)
        for _ in range(args.steps):
            e.parse(c, out_kind=kind, out=o, stream=s)
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.steps

    nbytes = b.data.numel()
    rs = ctypes.CDLL(os.path.join(ROOT, "tools", "libreadstream.so"))  # make -C tools libreadstream.so
    rs.readstream_launch.restype = ctypes.c_uint64
    rs.readstream_launch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    rs.readspan_launch.restype = ctypes.c_uint64
    rs.readspan_launch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                   ctypes.c_void_p, ctypes.c_void_p]
    scratch = torch.empty(4096, dtype=torch.uint8, device="cuda")
    per_wg = (b.total_bytes // b.count * 256) & ~15  # the span kernel's bytes per workgroup

    def time_read(ptr, span=False, skew=0):
        """Bare read stream (or the span kernel's read structure) over the same
        allocation: its fraction of 8 TB/s."""
        def go():
            if span:
                n = rs.readspan_launch(ctypes.c_void_p(ptr), nbytes, per_wg, skew,
                                       ctypes.c_void_p(scratch.data_ptr()), ctypes.c_void_p(s.cuda_stream))
            else:
                n = rs.readstream_launch(ctypes.c_void_p(ptr), nbytes, ctypes.c_void_p(scratch.data_ptr()),
                                         ctypes.c_void_p(s.cuda_stream))
            if n == 0:
                raise RuntimeError("readstream_launch failed")
            return n
        for _ in range(5):
            go()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(s)
        for _ in range(args.steps):
            n = go()
        e1.record(s)
        torch.cuda.synchronize()
        return round(n / (e0.elapsed_time(e1) / args.steps * 1e-3) / 8e12, 4)

    if args.vmm:  # does the virtual memory API's mapping take the slow class?
        bufs = []
        for k in range(args.vmm):
            for name in ("default", "vmm"):
                buf = RawBuf(hip, nbytes, HIP_DEVICE_MALLOC_DEFAULT) if name == "default" else VmmBuf(hip, nbytes)
                rc = hip.hipMemcpy(ctypes.c_void_p(buf.ptr), ctypes.c_void_p(b.data.data_ptr()),
                                   ctypes.c_size_t(nbytes), ctypes.c_int(HIP_MEMCPY_D2D))
                if rc != 0:
                    raise RuntimeError(f"hipMemcpy = {rc}")
                bufs.append((k, name, buf))
        torch.cuda.synchronize()
        print(json.dumps({"vmm_granularity": [x for x in bufs if x[1] == "vmm"][0][2].gran}), flush=True)
        for r in range(2):
            for k, name, buf in bufs:
                ms = time_batch(FrameBatch(data=buf, count=b.count, offsets=b.offsets))
                print(json.dumps({"round": r, "copy": k, "alloc": name, "ptr": hex(buf.ptr),
                                  "frac": round(b.total_bytes / (ms * 1e-3) / 8e12, 4)}), flush=True)
        for _, _, buf in bufs:
            buf.free()
        return
    if args.map:  # which allocations of a process are slow, and does freed memory stay slow?
        def one(tag, k):
            buf = RawBuf(hip, nbytes, HIP_DEVICE_MALLOC_DEFAULT)
            hip.hipMemcpy(ctypes.c_void_p(buf.ptr), ctypes.c_void_p(b.data.data_ptr()),
                          ctypes.c_size_t(nbytes), ctypes.c_int(HIP_MEMCPY_D2D))
            torch.cuda.synchronize()
            ms = time_batch(FrameBatch(data=buf, count=b.count, offsets=b.offsets))
            frac = round(b.total_bytes / (ms * 1e-3) / 8e12, 4)
            rd = time_read(buf.ptr)
            row = {"phase": tag, "k": k, "ptr": hex(buf.ptr), "frac": frac, "read_frac": rd,
                   "parse_over_read": round(frac / rd, 4), "span_read": time_read(buf.ptr, True, 0),
                   "span_read_skew": time_read(buf.ptr, True, 48)}
            c = FrameBatch(data=buf, count=b.count, offsets=b.offsets)
            for name, e in extra:
                row[name] = round(b.total_bytes / (time_batch(c, e) * 1e-3) / 8e12, 4)
            for name in filter(None, args.outs.split(",")):
                if name == "fresh_grouped":  # a new output allocation next to this batch
                    o = torch.empty(Engine.out_bytes(abi.OUT_GROUPED, b.count), dtype=torch.uint8, device="cuda")
                    ms2 = time_batch(c, None, abi.OUT_GROUPED, o)
                    del o
                    torch.cuda.empty_cache()
                else:
                    ms2 = time_batch(c, None, kinds[name], outs_by_kind[name])
                row["out_" + name] = round(b.total_bytes / (ms2 * 1e-3) / 8e12, 4)
            if args.clock:  # the span kernel's own stamps on this allocation, right after its timed launches
                from nex_amd import clocks
                _, st = eng.probe_span_clock(c)
                sm = clocks.span_summary(st.cpu().numpy())
                row["clock_ghz"] = sm.get("shader_clock_ghz", {}).get("median")
                row["wg_cycles"] = sm.get("workgroup_cycles", {}).get("mean")
                row["wg_us"] = sm.get("workgroup_us", {}).get("mean")
                row["phase_cycles"] = sm.get("phase_cycles")
            if args.latency:  # dependent-load latency over this allocation (overwrites the copy)
                row["lat_idle_ns"] = round(eng.probe_latency(buf, 2000, 12345)[0], 1)
                row["lat_loaded_ns"] = round(eng.probe_latency(buf, 2000, 12345, loaded=True)[0], 1)
            print(json.dumps(row), flush=True)
            return buf
        live = [one("fill", k) for k in range(args.map)]
        for buf in live[: args.map // 2]:
            buf.free()
        live = live[args.map // 2:] + [one("refill", k) for k in range(args.map // 2)]
        for buf in live:
            buf.free()
        return
    bufs = []
    for k in range(args.copies):
        for name, flags in (("default", HIP_DEVICE_MALLOC_DEFAULT), ("contiguous", HIP_DEVICE_MALLOC_CONTIGUOUS)):
            try:
                buf = RawBuf(hip, nbytes, flags)
            except RuntimeError as e:
                print(json.dumps({"copy": k, "alloc": name, "error": str(e)}), flush=True)
                continue
            rc = hip.hipMemcpy(ctypes.c_void_p(buf.ptr), ctypes.c_void_p(b.data.data_ptr()),
                               ctypes.c_size_t(nbytes), ctypes.c_int(HIP_MEMCPY_D2D))
            if rc != 0:
                raise RuntimeError(f"hipMemcpy = {rc}")
            bufs.append((k, name, buf))
    torch.cuda.synchronize()
    rows = []
    for r in range(2):
        for k, name, buf in bufs:
            c = FrameBatch(data=buf, count=b.count, offsets=b.offsets)
            ms = time_batch(c)
            rows.append({"round": r, "copy": k, "alloc": name, "ptr": hex(buf.ptr), "kernel_ms": round(ms, 4),
                         "frac": round(b.total_bytes / (ms * 1e-3) / 8e12, 4)})
            print(json.dumps(rows[-1]), flush=True)
    for _, _, buf in bufs:
        buf.free()
    for name in ("default", "contiguous"):
        f = [x["frac"] for x in rows if x["alloc"] == name]
        if f:
            print(json.dumps({"alloc": name, "n": len(f), "min": min(f), "max": max(f)}), flush=True)
    print(json.dumps({"workload": args.workload, "bytes": b.total_bytes, "rows": rows}), flush=True)


if __name__ == "__main__":
    main()
