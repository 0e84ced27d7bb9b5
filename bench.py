#!/usr/bin/env python3
"""Headline benchmark: device-resident batched Frame parse + checksum verify.

BASELINE.json metric "Mpkt/s + GiB/s device-resident parse+cksum, 64B & IMIX,
1/2/4/8 MI355X". A step is one pass of the hot path (one nexg_parse_batch
launch) over one batch of synthetic frames already resident in HBM. Default
workload = BASELINE configs[1]: 16M x 64-B Eth/IPv4/UDP frames per GPU.

Multi-GPU (torchrun, one process per GPU): each rank regenerates its own
16M-frame shard from the global index range [rank*F, (rank+1)*F) — weak
scaling, no data-path collective; only a barrier and a MAX over ranks of the
elapsed time. value = frames processed by all ranks / max elapsed.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from nex_amd import clocks  # noqa: E402  (imports no torch)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
IMIX_WARMUP = 40  # untimed launches before the 6-GB packed batches are timed (see imix_line)
# every timed line also warms up for at least this long: the kernel-trace of a
# fresh 16M UDP64 batch runs its first ~10 launches at 150-155 us, the next ~40
# at 163-170 us and settles near 160 us only after ~80 (profiles/r03/warmup/);
# W untimed launches alone (the driver passes --warmup 5) time that transient
WARMUP_SECONDS = 0.25
#: --out name -> nexg out_kind (include/nexg.h NEXG_OUT_*)
OUT_KINDS = {"desc": 1, "record": 2, "flags": 4, "verdict": 5, "sparse": 6, "grouped": 7}
OUT_NOTE = {
    "sparse": "lossless sparse descriptors (NEXG_OUT_SPARSE: 1-B shape code/frame + 8-B exceptions)",
    "grouped": "lossless grouped descriptors (NEXG_OUT_GROUPED: 64-frame groups as head + 2 verdict "
               "bits/frame, else 1-B codes + 8-B exceptions)",
    "desc": "8-B nexg_desc per frame", "record": "64-B nexg_record per frame",
    "flags": "4-B flags word per frame (no payload location)",
    "verdict": "2-B lossless flags per frame (no payload location)"}
METRIC = "Mpkt/s + GiB/s device-resident parse+cksum, 64B & IMIX, 1/2/4/8 MI355X"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_threads():
    """CPU share to use for the threaded baseline: the box grants 16 CPUs per
    GPU (os.cpu_count() shows the whole machine there), this container 8."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return max(1, min(16, n))


def cpu_baseline(batch, workload, count, seconds, nthreads=1):
    """Oracle (C restatement of nex-packet's Frame path + reference-semantic
    checksums) on the host over the first `count` frames of the same
    workload, repeated until ~`seconds` of CPU work; `nthreads` static
    index-range shards of the sample."""
    import numpy as np
    from nex_amd import abi
    from oracle import oracle
    n = min(count, batch.count)
    if batch.offsets is None:
        data = batch.data[: n * batch.stride].cpu().numpy()
        offs, lens, stride = None, None, batch.stride
        nbytes = n * batch.stride
    elif batch.lengths is not None:  # offsets + lengths (capture-record shape)
        offs = batch.host_offsets()[:n].astype(np.uint64)
        lens = batch.lengths[:n].cpu().numpy().astype(np.uint32)
        data = batch.data[: int(offs[-1]) + int(lens[-1])].cpu().numpy()
        stride = 0
        nbytes = int(lens.sum())
    else:
        offs = batch.host_offsets()[: n + 1].astype(np.uint64)
        data = batch.data[: int(offs[n])].cpu().numpy()
        lens, stride = None, 0
        nbytes = int(offs[n] - offs[0])
    reps, t = 0, 0.0
    while t < seconds and reps < 1000:
        t0 = time.perf_counter()
        oracle.parse_packed(data, offs, lens, stride=stride, nthreads=nthreads)
        t += time.perf_counter() - t0
        reps += 1
    mpps = n * reps / t / 1e6
    return {"value": round(mpps, 3), "unit": "Mpkt/s", "cores": nthreads, "kind": "port",
            "gib_s": round(nbytes * reps / t / 2**30, 3),
            "sample": f"{nthreads} thr, first {n} frames of {workload}, {reps} passes, {t:.1f} s",
            "desc": "oracle/nex_oracle.c (literal restatement of Frame::try_from_buf + ipv4/udp/tcp/icmp "
                    "checksum; Rust reference not buildable here)"}


SER_MACS = (b"\x02\0\0\0\0\1", b"\x02\0\0\0\0\2")  # udp_ping's interface MACs (synthetic)
SER_SRC_IP = 0xC0A80164  # udp_ping's interface address (synthetic: 192.168.1.100)
SER_PORTS = (53443, 33435)  # udp_ping.rs:30-31 SRC_PORT / DST_PORT


def ser_probe_params(p):
    """The udp_ping probe batch's tuples as the oracle takes them: the batch's
    destinations, udp_ping's one source address and port pair, id 0 (the
    Ipv4PacketBuilder default, builder/ipv4.rs:34)."""
    import torch
    n = p[1].numel()
    full = lambda v, dt: torch.full((n,), v, dtype=dt)
    return (full(SER_SRC_IP - (1 << 32), torch.int32), p[1], full(SER_PORTS[0] - (1 << 16), torch.int16),
            full(SER_PORTS[1] - (1 << 16), torch.int16), full(0, torch.int16))


def ser_step(eng, p, out, stream, shape):
    """One serialize launch: `probe` = the udp_ping probe batch (a destination
    per frame, src_ip NULL -> one source, ports / id from the batch defaults:
    4 B of parameters read per frame); `tuples` = a full per-frame 5-tuple +
    IPv4 id (14 B read per frame)."""
    if shape == "tuples_aos":  # p[5]: the same tuples packed as 16-B records
        return lambda: eng.build_udp4_tuples(p[5], src_mac=SER_MACS[0], dst_mac=SER_MACS[1], ip_flags=2, out=out,
                                             stream=stream)
    if shape == "probe":
        return lambda: eng.build_udp4(None, p[1], def_src_ip=SER_SRC_IP, def_src_port=SER_PORTS[0],
                                      def_dst_port=SER_PORTS[1], src_mac=SER_MACS[0], dst_mac=SER_MACS[1],
                                      ip_flags=2, out=out, stream=stream)
    return lambda: eng.build_udp4(p[0], p[1], p[2], p[3], p[4], src_mac=SER_MACS[0], dst_mac=SER_MACS[1],
                                  ip_flags=2, out=out, stream=stream)


SER_SHAPE_NOTE = {
    "probe": "udp_ping probe batch: a destination IPv4 per frame (4 B read), udp_ping's one source "
             "address, SRC_PORT/DST_PORT and id 0 from the batch defaults",
    "tuples": "a full per-frame tuple (src/dst IPv4, ports, IPv4 id: 14 B read from five arrays)",
    "tuples_aos": "a full per-frame tuple as one 16-B record (nexg_build_udp4_tuples: 16 B read, one "
                  "dwordx4 load per frame)"}
SER_READ = {"probe": 4, "tuples": 14, "tuples_aos": 16}
#: tools/pmc.sh records the builds as <key>.desc (the build has no output kind)
SER_TRAFFIC_KEY = {"probe": "ser_probe", "tuples": "ser", "tuples_aos": "ser_aos"}


def ser_params(eng, F, first, shape):
    """The serialize batch's parameters: the five SoA tuple arrays, plus the
    same tuples packed as 16-B records for the AoS shape."""
    p = eng.gen_udp4_params(F, first_index=first)
    return tuple(p) + ((eng.pack_udp4_tuples(*p),) if shape == "tuples_aos" else ())


def cpu_baseline_ser(params, count, seconds, nthreads=1):
    """Oracle udp_ping builds (nexo_build_udp4_batch: the restatement of
    UdpPacketBuilder -> Ipv4PacketBuilder -> EthernetPacketBuilder, one tuple
    at a time) over the first `count` tuples of the same parameter batch."""
    import numpy as np
    from oracle import oracle
    n = min(count, params[0].numel())
    host = [t[:n].cpu().numpy().view(np.uint32 if t.element_size() == 4 else np.uint16) for t in params]
    out = np.empty((n, 42), np.uint8)
    reps, t = 0, 0.0
    while t < seconds and reps < 1000:
        t0 = time.perf_counter()
        oracle.build_udp4_batch(SER_MACS[0], SER_MACS[1], *host, 64, 2, nthreads=nthreads, out=out)
        t += time.perf_counter() - t0
        reps += 1
    return {"value": round(n * reps / t / 1e6, 3), "unit": "Mpkt/s", "cores": nthreads, "kind": "port",
            "gib_s": round(42 * n * reps / t / 2**30, 3),
            "sample": f"{nthreads} thr, first {n} tuples, {reps} passes, {t:.1f} s",
            "desc": "oracle/nex_oracle.c nexo_build_udp4 (literal restatement of the udp_ping.rs:68-109 "
                    "builder chain; Rust reference not buildable here)"}


def write_ceiling(eng, out, args, stream, device):
    """Write-only HBM stream on the serialize path's own output buffer
    (nexg_probe_stream out_per_64 = 64: the builders' 16-B non-temporal
    copy-out shape), same steps / warmup / HIP-event timing."""
    nbytes = out.numel() // 16384 * 16384
    _, ks = timed(lambda: eng.probe_write(out, stream=stream), args.steps, args.warmup, stream, device)
    return {"write_only_gbs": round(nbytes / ks / 1e9, 1),
            "source": "nexg_probe_stream(out_per_64=64) over the build output buffer, same steps/warmup: "
                      "16 KiB of 16-B non-temporal stores per workgroup at the builder's tile order and 5 "
                      "workgroups per CU; a reference stream, not a bound (the builder's 10.75-KiB tiles "
                      "run faster, DESIGN.md §6 round 4)"}


def ser_line(eng, args, F, first, stream, device, rank, world):
    """configs[3] beside the default run: build+checksum F udp_ping frames
    (42 B) per GPU — the probe batch (a destination per frame, as udp_ping.rs
    builds them) with the full-tuple form nested under "tuples" — with the
    write-only stream ceiling of the same buffer and the oracle builder on
    the host."""
    import torch
    from nex_amd import dist
    p = ser_params(eng, F, first, "tuples")
    out = torch.empty(F * 42, dtype=torch.uint8, device=device)
    torch.cuda.synchronize(device)
    alg = F * 42
    ceil = write_ceiling(eng, out, args, stream, device)
    res = {}
    # ser.tuples_aos (nexg_build_udp4_tuples) is an entry-point check, slower than
    # the five arrays: --workload ser --ser-shape tuples_aos
    for shape in ("probe", "tuples"):
        elapsed, kernel_s = timed(ser_step(eng, p, out, stream, shape), args.steps, args.warmup, stream, device)
        tp = dist.throughput(F, alg, args.steps, elapsed, device)
        if rank != 0:
            continue
        ach = alg / kernel_s / 1e9
        r = {"workload": f"configs[3] udp_ping {shape}",
             "desc": f"configs[3]: build+checksum {F} udp_ping Eth/IPv4/UDP frames (42 B) per GPU, "
                     + SER_SHAPE_NOTE[shape],
             "value": tp["value"], "unit": "Mpkt/s", "steps": args.steps, "ms_per_step": tp["ms_per_step"],
             "gib_s": tp["gib_s"], "bytes_per_gpu": alg,
             "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": round(ach / HBM_PEAK_GBS, 4),
                          "traffic": load_traffic(SER_TRAFFIC_KEY[shape], "desc"),
                          "kernel_ms": round(kernel_s * 1e3, 4), "algorithmic_bytes_per_launch": alg,
                          "basis": f"bytes written (SURVEY.md 8(d) SER); parameter reads ({SER_READ[shape]} "
                                   "B/frame) not counted",
                          "stream_ceilings": dict(ceil, frac_of_write_only=round(ach / ceil["write_only_gbs"], 4))}}
        if world == 1 and not args.no_cpu_baseline:
            try:
                hp = ser_probe_params(p) if shape == "probe" else p[:5]
                r["cpu_baseline"] = cpu_baseline_ser(hp, 1 << 20, args.cpu_seconds / 4, host_threads())
            except Exception as e:
                r["cpu_baseline"] = {"value": None, "error": repr(e)}
        res[shape] = r
    del out, p
    for shape in PROBE_SHAPES:
        r = probe_object(eng, args, F, first, shape, stream, device, rank, world)
        if r is not None:
            res[shape] = r
    if rank != 0:
        return None
    return dict(res["probe"], tuples=res["tuples"], **{k: res[k] for k in PROBE_SHAPES})


#: the other ping callers' probe batches in the serialize line
PROBE_SHAPES = ("tcp_ping", "icmp_ping", "udp6")


def cpu_baseline_probe(shape, dst_host, seconds, nthreads):
    """Oracle builds of a probe batch (oracle/nex_oracle.c nexo_build_probe_batch:
    the single-frame restatements of the example's builder chain, one per
    destination) over a bounded sample of the same destinations."""
    from nex_amd import probes
    from oracle import oracle
    from tests import helpers
    n = dst_host.shape[0]
    out = np.empty((n, probes.frame_len(shape)), np.uint8)
    reps, t = 0, 0.0
    while t < seconds and reps < 1000:
        t0 = time.perf_counter()
        helpers.probe_oracle_build(oracle, shape, dst_host, nthreads=nthreads, out=out)
        t += time.perf_counter() - t0
        reps += 1
    L = probes.frame_len(shape)
    return {"value": round(n * reps / t / 1e6, 3), "unit": "Mpkt/s", "cores": nthreads, "kind": "port",
            "gib_s": round(L * n * reps / t / 2**30, 3),
            "sample": f"{nthreads} thr, first {n} destinations, {reps} passes, {t:.1f} s",
            "desc": "oracle/nex_oracle.c nexo_build_probe_batch (literal restatement of the example's builder "
                    "chain per frame; Rust reference not buildable here)"}


def probe_object(eng, args, F, first, shape, stream, device, rank, world):
    """One probe batch of nex_amd/probes.py (tcp_ping / icmp_ping / udp_ping's
    IPv6 branch): F frames per GPU, a destination per frame (4 / 16 B read),
    roofline on the bytes written, the oracle builder on the host."""
    import torch
    from nex_amd import dist, probes
    L = probes.frame_len(shape)
    g = torch.Generator(device=device).manual_seed(0x6E6578 + first)
    dst = torch.randint(0, 256, (F, probes.dst_bytes(shape)), dtype=torch.uint8, device=device, generator=g)
    src = probes.source(shape, device)
    pay = torch.tensor(list(probes.ICMP_PAYLOAD), dtype=torch.uint8, device=device)
    out = torch.empty(F * L, dtype=torch.uint8, device=device)
    torch.cuda.synchronize(device)
    alg = F * L
    step = lambda: probes.build(eng, shape, dst, src=src, out=out, stream=stream, payload_t=pay)
    elapsed, kernel_s = timed(step, args.steps, args.warmup, stream, device)
    tp = dist.throughput(F, alg, args.steps, elapsed, device)
    if rank != 0:
        return None
    ach = alg / kernel_s / 1e9
    rd = probes.dst_bytes(shape)
    r = {"workload": f"8(f)3 {shape} probe batch",
         "desc": f"SURVEY 8(f)3 probe batch: build+checksum {F} frames per GPU, " + probes.NOTE[shape]
                 + f"; one source, a destination per frame ({rd} B read), the rest the example's constants",
         "value": tp["value"], "unit": "Mpkt/s", "steps": args.steps, "ms_per_step": tp["ms_per_step"],
         "gib_s": tp["gib_s"], "bytes_per_gpu": alg,
         "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": load_traffic(f"ser_{shape}", "desc"),
                      "kernel_ms": round(kernel_s * 1e3, 4), "algorithmic_bytes_per_launch": alg,
                      "frac_counting_reads": round((alg + F * rd) / kernel_s / 1e9 / HBM_PEAK_GBS, 4),
                      "basis": f"bytes written ({L} B/frame); the destination reads ({rd} B/frame) not counted"}}
    if world == 1 and not args.no_cpu_baseline:
        try:
            n = min(F, 1 << 20)
            r["cpu_baseline"] = cpu_baseline_probe(shape, dst[:n].cpu().numpy(), args.cpu_seconds / 4,
                                                   host_threads())
        except Exception as e:
            r["cpu_baseline"] = {"value": None, "error": repr(e)}
    return r


def load_traffic(workload, out_kind):
    """HBM bytes per launch from the committed rocprofv3 PMC pass (FETCH_SIZE
    doubled per the gfx950 correction + WRITE_SIZE), if one exists."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            t = json.load(f)
        e = t.get(f"{workload}:{out_kind}")
        return None if e is None else e["hbm_bytes_per_launch"]
    except (OSError, ValueError):
        return None


def timed(step, steps, warmup, stream, device, host_clock=False, with_local=False, stats=None):
    """W untimed steps (continued until WARMUP_SECONDS have passed), then
    exactly K steps bracketed by barrier + sync on both sides
    (nex_amd.dist.timed_steps). Returns (max-over-ranks elapsed seconds,
    per-launch kernel seconds from HIP events on the launch stream); `stats`
    receives the warmup actually run."""
    import torch
    from nex_amd import dist
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    elapsed, local = dist.timed_steps(step, steps, warmup, sync=lambda: torch.cuda.synchronize(device),
                                      device=device, before=lambda: ev0.record(stream),
                                      after=lambda: ev1.record(stream), warmup_seconds=WARMUP_SECONDS,
                                      stats=stats)
    kernel_s = ev0.elapsed_time(ev1) / 1e3 / steps
    if host_clock:  # copies + kernels on side streams: the host clock is the measure
        kernel_s = local / steps
    return (elapsed, kernel_s, local) if with_local else (elapsed, kernel_s)


def stream_ceilings(eng, batch, args, stream, device):
    """HBM stream ceilings on the same buffer, box and timing discipline
    (nexg_probe_stream, the parse kernels' load shape): read only, and
    64 B read / 8 B written (the descriptor stream's shape)."""
    import torch
    from nex_amd.engine import Engine
    need = max(Engine.out_bytes(k, batch.count) for k in (1, 4, 5, 6, 7))
    out = torch.empty(max(batch.data.numel() // 8, need + 16), dtype=torch.uint8, device=device)
    nbytes = batch.data.numel() // 16384 * 16384
    r = {}
    for key, w8 in (("read_only_gbs", False), ("read64_write8_gbs", True), ("read64_write8_6cu_gbs", 9)):
        _, ks = timed(lambda: eng.probe_stream(batch.data, w8, out=out, stream=stream),
                      args.steps, args.warmup, stream, device)
        r[key] = round(nbytes / ks / 1e9, 1)
    r["source"] = ("nexg_probe_stream on this batch, same steps/warmup, HIP events on the launch stream: "
                   "a bare 16-B non-temporal read stream in the parse kernel's tile order at 8 workgroups per "
                   "CU; a reference stream, not a bound (the parse kernel at 6 per CU runs faster; the best "
                   "bare read stream found, 3 per CU, is 0.89 / 0.93 of 8 TB/s at 1 / 3.25 GiB: "
                   "profiles/r04/occupancy/)")
    if args.out in ("sparse", "desc", "grouped"):  # the same parse with the other output kinds
        from nex_amd import abi
        for key, kind in (("desc_output", abi.OUT_DESC), ("flags_output", abi.OUT_FLAGS),
                          ("verdict_output", abi.OUT_VERDICT), ("sparse_output", abi.OUT_SPARSE),
                          ("grouped_output", abi.OUT_GROUPED)):
            if OUT_KINDS[args.out] == kind:
                continue
            _, ks = timed(lambda: eng.parse(batch, out_kind=kind, out=out, stream=stream),
                          args.steps, args.warmup, stream, device)
            r[key] = output_rate(batch, kind, ks)
    return r


OUT_WIDTH = {1: 8, 4: 4, 5: 2}  # nexg_desc / flags / verdict bytes per frame


def output_rate(batch, kind, ks):
    """An output kind's kernel time on a batch: fraction of 8 TB/s on the read
    bytes (the roofline's basis) and counting the bytes it writes per frame."""
    ach = batch.total_bytes / ks / 1e9
    r = {"kernel_ms": round(ks * 1e3, 4), "achieved": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4)}
    if kind in OUT_WIDTH:
        moved = batch.total_bytes + OUT_WIDTH[kind] * batch.count
        r["frac_counting_writes"] = round(moved / ks / 1e9 / HBM_PEAK_GBS, 4)
    return r


def object_clocks(eng, batch, sampler, stream, device):
    """The clocks a timed object ran at: the sysfs DPM levels / power sampled
    during its warmup + timed launches, and for the span kernel's batches one
    stamped launch right after them (nexg_probe_span_clock: the shader clock
    the workgroups held and their cycles per phase)."""
    import torch
    r = {"sysfs": sampler.summary()}
    if batch.offsets is not None:  # packed / monotone batches: the span kernel
        try:
            _, st = eng.probe_span_clock(batch, stream=stream)
            torch.cuda.synchronize(device)
            r["span"] = clocks.span_summary(st.cpu().numpy())
            r["hbm_latency"] = hbm_latency(eng, device)
        except Exception as e:  # reported, never fatal to the measurement
            r["span"] = {"error": repr(e)}
    return r


_LAT_BUF = {}


def hbm_latency(eng, device, steps=2000):
    """Dependent HBM load latency on this box (nexg_probe_latency over a
    1-GiB scratch ring, a ~1-MiB stride per step): alone and while 4
    workgroups per CU stream-read the ring — the condition the span kernel's
    generic section waits in."""
    import random

    import torch
    buf = _LAT_BUF.get(device.index)
    if buf is None:
        buf = _LAT_BUF[device.index] = torch.empty(1 << 30, dtype=torch.uint8, device=device)
    start = random.randrange(1 << 24)  # another chain each call: no line left in the caches by the last
    idle_ns, idle_cyc = eng.probe_latency(buf, steps=steps, start=start)
    loaded_ns, loaded_cyc = eng.probe_latency(buf, steps=steps, start=start + 7919, loaded=True)
    return {"idle_ns": round(idle_ns, 1), "idle_cycles": round(idle_cyc, 1), "loaded_ns": round(loaded_ns, 1),
            "loaded_cycles": round(loaded_cyc, 1), "steps": steps}


def parse_object(eng, args, batch, out_kind, stream, device, rank, world, workload, traffic_key,
                 warmup, steps, cpu_label=None, extra=None, also=(), desc=None):
    """One parse workload beside the default run, same output kind and timing
    discipline: W untimed launches (+ the warmup floor), K timed, max over
    ranks. Returns the object rank 0 adds to the JSON line (None elsewhere)."""
    import torch
    from nex_amd import dist
    from nex_amd.engine import Engine
    n = batch.count
    out = torch.empty(Engine.out_bytes(out_kind, n), dtype=torch.uint8, device=device)
    torch.cuda.synchronize(device)
    alg = batch.total_bytes
    wstats = {}
    with clocks.Sampler(device.index) as smp:
        elapsed, kernel_s = timed(lambda: eng.parse(batch, out_kind=out_kind, out=out, stream=stream),
                                  steps, warmup, stream, device, stats=wstats)
    tp = dist.throughput(n, alg, steps, elapsed, device)
    per_rank = dist.all_ranks(round(kernel_s * 1e3, 4), device)
    clk = object_clocks(eng, batch, smp, stream, device)
    per_rank_clock = dist.all_ranks(clk.get("span", {}).get("shader_clock_ghz", {}).get("median", 0.0), device)
    other = {}
    for key, kind in also:  # the same batch with other output kinds (same timing discipline)
        o2 = torch.empty(Engine.out_bytes(kind, n), dtype=torch.uint8, device=device)
        _, ks = timed(lambda: eng.parse(batch, out_kind=kind, out=o2, stream=stream), steps, warmup, stream, device)
        other[key] = output_rate(batch, kind, ks)
        del o2
    share = None
    if extra is not None and extra.pop("shape_share", False):  # share of frames with a shape code
        from nex_amd import abi
        torch.cuda.synchronize(device)
        if out_kind == abi.OUT_SPARSE:
            share = round(float((out[:n] != 0).float().mean().item()), 4)
        elif out_kind == abi.OUT_GROUPED:
            share = round(float((abi.grouped_codes(out.cpu().numpy(), n) != 0).mean()), 4)
    if rank != 0:
        return None
    ach = alg / kernel_s / 1e9
    r = {"workload": workload, "desc": desc, "value": tp["value"], "unit": "Mpkt/s", "steps": steps,
         "ms_per_step": tp["ms_per_step"], "gib_s": tp["gib_s"], "frames_per_gpu": n, "bytes_per_gpu": alg,
         "warmup_run": wstats,
         "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": load_traffic(traffic_key, args.out),
                      "kernel_ms": round(kernel_s * 1e3, 4), "algorithmic_bytes_per_launch": alg}}
    if share is not None:
        r["sparse_shape_share"] = share
    if extra:
        r.update(extra)
    r["clocks"] = clk
    if other:
        r["other_outputs"] = other
    if world > 1:
        r["per_rank_kernel_ms"] = per_rank
        if "span" in clk:
            r["per_rank_shader_clock_ghz"] = per_rank_clock
    if cpu_label and world == 1 and not args.no_cpu_baseline:
        try:
            r["cpu_baseline"] = cpu_baseline(batch, cpu_label, 1 << 20, args.cpu_seconds / 2, host_threads())
        except Exception as e:
            r["cpu_baseline"] = {"value": None, "error": repr(e)}
    return r


IMIX_DESC = ("(64/576/1500 at 7:4:1, {IPv4,IPv6}x{TCP,UDP,ICMP}), packed with a u32 offset table "
             "(NEXG_FRAMES_OFFSETS32 + a u64 base per 256 frames: the batch is over 4 GiB); ")


def imix_batch(eng, F, first):
    """configs[2]'s batch: F IMIX frames packed back to back, described by
    the u32 offset table (half the u64 table's bytes: HBM traffic 1.023x the
    frame bytes against 1.033x, profiles/r06/pmc/imix_offsets32_pmc.json)."""
    from nex_amd import abi
    return eng.gen_batch(abi.WL_IMIX, F, first_index=first).with_offsets32()


def imix_line(eng, args, F, first, out_kind, width, stream, device, rank, world):
    """configs[2] beside the default configs[1] run (the metric names both
    64B and IMIX): 16M IMIX frames per GPU, same output kind, same timing
    discipline. The first ~30 launches of a 6-GB batch (about 30 ms of
    back-to-back load) run 5-25 % slow before the chip settles
    (profiles/r01_staging/imix_ramp.txt, profiles/r03_final/imix_ramp.txt),
    so the IMIX objects warm up for IMIX_WARMUP untimed launches."""
    batch = imix_batch(eng, F, first)
    return parse_object(eng, args, batch, out_kind, stream, device, rank, world, f"configs[2] IMIX {args.out}",
                        "imix", max(IMIX_WARMUP, args.warmup), max(1, args.steps // 2), cpu_label="imix",
                        desc=f"configs[2]: {F} IMIX frames per GPU " + IMIX_DESC + OUT_NOTE[args.out])


def malformed_line(eng, args, F, first, out_kind, stream, device, rank, world):
    """The SURVEY.md App. C malformed mix (nex_amd/workloads.py: half of the
    IMIX frames carry one structural mutation) at the configs[2] size, same
    output kind and timing: the cost of the frames that leave the canonical
    fast paths for the generic parse core. 1M distinct frames tiled to F."""
    from nex_amd import abi, workloads
    distinct = min(F, 1 << 20)
    mix, counts = workloads.malformed_mix(eng, distinct, seed=abi.DEFAULT_SEED + first)
    batch = workloads.tiled(mix, max(1, F // distinct))
    return parse_object(eng, args, batch, out_kind, stream, device, rank, world, f"App. C malformed mix {args.out}",
                        "malformed", max(IMIX_WARMUP, args.warmup), max(1, args.steps // 2), cpu_label="malformed",
                        extra={"shape_share": True},
                        desc=f"SURVEY App. C malformed mix: {batch.count} frames per GPU ({distinct} distinct, "
                             f"tiled), IMIX with half the frames mutated {counts}; " + OUT_NOTE[args.out])


def real_traffic_batch(eng, F, first):
    from nex_amd import abi, workloads
    distinct = min(F, 1 << 20)
    mix, counts = workloads.real_traffic(eng, distinct, seed=abi.DEFAULT_SEED + 7 + first)
    batch = workloads.tiled(mix, max(1, F // distinct))
    desc = (f"real-traffic TCP shapes: {batch.count} IMIX frames per GPU ({distinct} distinct, tiled) whose TCP "
            f"segments carry option lists ({int(workloads.REAL_TRAFFIC_SHARE * 100)} %: NOP NOP timestamps, "
            f"NOP NOP SACK 1-4 blocks, MSS alone; tcp.rs:731-836) {counts}, checksums made valid by "
            "nexg_recompute_checksums_batch; ")
    return batch, desc


def real_traffic_line(eng, args, F, first, out_kind, stream, device, rank, world):
    """IMIX with the TCP option lists real segments carry (VERDICT r03
    missing 3), same output kind and timing as the IMIX object."""
    batch, desc = real_traffic_batch(eng, F, first)
    from nex_amd import abi
    # the per-frame descriptors a parse_frame / dump caller reads (examples/dump.rs:96-224)
    # on the shape where the grouped output degenerates to per-frame codes
    return parse_object(eng, args, batch, out_kind, stream, device, rank, world, f"real-traffic IMIX {args.out}",
                        "real_traffic", max(IMIX_WARMUP, args.warmup), max(1, args.steps // 2),
                        cpu_label="real_traffic", extra={"shape_share": True},
                        also=(("desc_output", abi.OUT_DESC),) if out_kind != abi.OUT_DESC else (),
                        desc=desc + OUT_NOTE[args.out])


LARGE_FRAMES = 52 << 20  # 3.25 GiB of 64-B frames: 13x the 256-MiB Infinity Cache


def large_line(eng, args, first, out_kind, stream, device, rank, world):
    """The UDP64 headline at 52M frames (3.25 GiB, 13x the 256-MiB MALL): a
    batch no cache can hold between launches, so its rate is HBM's."""
    from nex_amd import abi
    batch = eng.gen_batch(abi.WL_UDP64, LARGE_FRAMES, first_index=rank * LARGE_FRAMES)  # this rank's index range
    return parse_object(eng, args, batch, out_kind, stream, device, rank, world, f"configs[1] UDP64 52M {args.out}",
                        "udp64_large", args.warmup, args.steps,
                        desc=f"configs[1] at {LARGE_FRAMES} x 64-B Eth/IPv4/UDP frames per GPU (3.25 GiB, 13x the "
                             "256-MiB Infinity Cache: no cross-launch cache reuse possible); " + OUT_NOTE[args.out])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=25,
                    help="untimed steps; a freshly generated batch runs its first launches "
                         "slow (clock ramp), profiles/r01_staging/imix_ramp.txt")
    ap.add_argument("--workload", choices=["udp64", "imix", "imix_pcap", "malformed", "real_traffic", "ser"], default="udp64")
    ap.add_argument("--frames", type=int, default=16 << 20, help="frames per GPU")
    ap.add_argument("--out", choices=list(OUT_KINDS), default="grouped",
                    help="output kind (default: lossless grouped descriptors, NEXG_OUT_GROUPED)")
    ap.add_argument("--no-imix", action="store_true",
                    help="skip the configs[2] IMIX line reported beside the default UDP64 run")
    ap.add_argument("--no-malformed", action="store_true",
                    help="skip the malformed-mix line (fallback cost) reported beside the default run")
    ap.add_argument("--no-real", action="store_true",
                    help="skip the real-traffic TCP-options line reported beside the default run")
    ap.add_argument("--no-large", action="store_true",
                    help="skip the 52M-frame (3.25 GiB) UDP64 line reported beside the default run")
    ap.add_argument("--no-ser", action="store_true",
                    help="skip the configs[3] serialize line reported beside the default run")
    ap.add_argument("--ser-shape", choices=["probe", "tuples", "tuples_aos"], default="probe",
                    help="--workload ser: udp_ping probe batch (a destination per frame) or full tuples")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--e2e", action="store_true",
                    help="frames start and end in pinned host memory: chunked H2D -> parse -> "
                         "D2H pipeline on two streams (PCIe-inclusive rate, DESIGN.md §6)")
    ap.add_argument("--e2e-chunk", type=int, default=1 << 20, help="frames per pipelined chunk")
    ap.add_argument("--lib", default=None,
                    help="another build of libnexg.so (A/B tools: nex_amd/libnexg_knobs.so reads the "
                         "measurement overrides NEXG_TILE_ORDER etc. from the environment)")
    args = ap.parse_args()
    if args.lib:
        from nex_amd import _lib
        _lib.LIB_PATH = os.path.abspath(args.lib)

    # --gpus N > 1 outside torchrun: start N ranks as a child process and relay
    # rank 0's line (this process makes no GPU call); exits unless this
    # process is the bench itself (--gpus 1, or a rank whose WORLD_SIZE == N)
    from nex_amd import launch
    launch.main_or_spawn(sys.argv[1:], args.gpus, os.path.abspath(__file__))

    import torch
    from nex_amd import abi, dist
    from nex_amd.engine import Engine

    rank, world, local = dist.env_rank_world()
    local = dist.device_index(local)  # 1:1 on a full node; folded for a shared-GPU rehearsal
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    dist.init()  # RCCL when this process has a GPU, gloo otherwise (NEXG_DIST_BACKEND overrides)
    eng = Engine(local)
    F = args.frames
    first = rank * F
    stream = torch.cuda.current_stream(device)
    out_kind = OUT_KINDS[args.out]
    width = {"desc": 8, "record": 64, "flags": 4, "verdict": 2, "sparse": 1, "grouped": 1}[args.out]

    if args.workload in ("udp64", "imix", "imix_pcap", "malformed", "real_traffic"):
        wl = abi.WL_UDP64 if args.workload == "udp64" else abi.WL_IMIX
        if args.workload == "malformed":  # the malformed object's batch as the main workload (PMC / rocprof)
            from nex_amd import workloads
            distinct = min(F, 1 << 20)
            mix, mcounts = workloads.malformed_mix(eng, distinct, seed=abi.DEFAULT_SEED + first)
            batch = workloads.tiled(mix, max(1, F // distinct))
            F = batch.count
        elif args.workload == "real_traffic":  # the real_traffic object's batch (PMC / rocprof)
            batch, rdesc = real_traffic_batch(eng, F, first)
            F = batch.count
        elif args.workload == "imix" and not args.e2e:
            batch = imix_batch(eng, F, first)
        else:
            batch = eng.gen_batch(wl, F, first_index=first, record_gap=16 if args.workload == "imix_pcap" else 0)
        torch.cuda.synchronize(device)
        alg_bytes = batch.total_bytes  # Σ frame_len: every byte is read (L4 checksum)
        out = torch.empty(Engine.out_bytes(out_kind, F), dtype=torch.uint8, device=device)

        def step():
            eng.parse(batch, out_kind=out_kind, out=out, stream=stream)
        if args.workload == "udp64":
            cfg = {"workload": "configs[1]: 16M x 64-B Eth/IPv4/UDP frames per GPU, fixed 64-B "
                               "stride, device-resident; Frame parse (L2/L3/L4) + IPv4 header and "
                               "UDP checksum verify -> " + OUT_NOTE[args.out] if F == 16 << 20
                               else f"{F} x 64-B Eth/IPv4/UDP frames per GPU; " + OUT_NOTE[args.out]}
        elif args.workload == "malformed":
            cfg = {"workload": f"SURVEY App. C malformed mix: {F} frames per GPU ({distinct} distinct, tiled), "
                               f"IMIX with half the frames mutated {mcounts}; " + OUT_NOTE[args.out]}
        elif args.workload == "real_traffic":
            cfg = {"workload": rdesc + OUT_NOTE[args.out]}
        elif args.workload == "imix":
            cfg = {"workload": f"configs[2]: {F} IMIX frames per GPU " + IMIX_DESC + OUT_NOTE[args.out]}
        else:
            cfg = {"workload": f"configs[4] ingest shape: {F} IMIX frames per GPU, each after a 16-B "
                               "capture record header (nexg_pcap_read_raw layout: offsets + lengths + "
                               "monotone hint, headers read through, not counted); " + OUT_NOTE[args.out]}
    else:
        p = ser_params(eng, F, first, args.ser_shape)
        out = torch.empty(F * 42, dtype=torch.uint8, device=device)
        alg_bytes = F * 42
        batch = None

        step = ser_step(eng, p, out, stream, args.ser_shape)
        cfg = {"workload": f"configs[3]: build+checksum {F} udp_ping Eth/IPv4/UDP frames (42 B) per GPU, "
                           + SER_SHAPE_NOTE[args.ser_shape]}

    cfg.update({"frames_per_gpu": F, "bytes_per_gpu": alg_bytes, "output": args.out,
                "parallelism": f"{world} ranks x index-range shards, no collective",
                "seed": hex(abi.DEFAULT_SEED)})

    if args.e2e:
        assert args.workload in ("udp64", "imix"), "--e2e covers the packed parse path"
        # host-resident copy of the same frames (pinned), chunked pipeline:
        # copy stream: H2D chunk i; compute stream: parse chunk i; D2H descs
        host = torch.empty(batch.data.numel(), dtype=torch.uint8, pin_memory=True)
        host.copy_(batch.data)
        cs, ps = torch.cuda.Stream(device), torch.cuda.Stream(device)
        C = args.e2e_chunk
        from nex_amd.engine import FrameBatch
        offs_host = None if batch.offsets is None else batch.offsets.cpu()
        chunks, o0 = [], 0
        for c0 in range(0, F, C):
            c1 = min(F, c0 + C)
            if batch.offsets is None:
                b0, b1 = c0 * batch.stride, c1 * batch.stride
                sub = FrameBatch(data=batch.data[b0:b1], count=c1 - c0, stride=batch.stride)
            else:
                b0, b1 = int(offs_host[c0]), int(offs_host[c1])
                sub = FrameBatch(data=batch.data[b0:b1], count=c1 - c0,
                                 offsets=batch.offsets[c0:c1 + 1] - b0)
            # each chunk's whole output (sparse: codes + exception slots) goes back
            ob = (Engine.out_bytes(out_kind, c1 - c0) + 255) // 256 * 256
            chunks.append((b0, b1, o0, o0 + ob, sub))
            o0 += ob
        out = torch.empty(o0, dtype=torch.uint8, device=device)
        host_out = torch.empty(o0, dtype=torch.uint8, pin_memory=True)

        def step():
            for (b0, b1, p0, p1, sub) in chunks:
                with torch.cuda.stream(cs):
                    batch.data[b0:b1].copy_(host[b0:b1], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(cs)
                ps.wait_event(ev)
                eng.parse(sub, out_kind=out_kind, out=out[p0:p1], stream=ps)
                with torch.cuda.stream(ps):
                    host_out[p0:p1].copy_(out[p0:p1], non_blocking=True)
            ps.synchronize()
        cfg["workload"] += "; END-TO-END: frames in pinned host memory, chunked H2D/parse/D2H"
        cfg["e2e_chunk_frames"] = C

    warm = max(args.warmup, IMIX_WARMUP) if args.workload in ("imix", "imix_pcap", "malformed", "real_traffic") and not args.e2e else args.warmup  # see imix_line
    wstats = {}
    with clocks.Sampler(device.index) as smp:
        elapsed, kernel_s, local_s = timed(step, args.steps, warm, stream, device, host_clock=args.e2e,
                                           with_local=True, stats=wstats)
    head_clocks = object_clocks(eng, batch, smp, stream, device) if batch is not None and not args.e2e \
        else {"sysfs": smp.summary()}
    tp = dist.throughput(F, alg_bytes, args.steps, elapsed, device)
    # each rank's kernel time and its own timed-region wall time (balance across GPUs)
    per_rank = {"kernel_ms": dist.all_ranks(round(kernel_s * 1e3, 4), device),
                "elapsed_ms_per_step": dist.all_ranks(round(local_s / args.steps * 1e3, 4), device)}
    ceilings = None
    if args.workload == "udp64" and not args.e2e and not args.no_imix:
        ceilings = stream_ceilings(eng, batch, args, stream, device)
    elif args.workload == "ser":
        ceilings = write_ceiling(eng, out, args, stream, device)
    imix = None
    if args.workload == "udp64" and not args.e2e and not args.no_imix and F == 16 << 20:
        imix = imix_line(eng, args, F, first, out_kind, width, stream, device, rank, world)
    malformed = None
    if args.workload == "udp64" and not args.e2e and not args.no_malformed and F == 16 << 20:
        malformed = malformed_line(eng, args, F, first, out_kind, stream, device, rank, world)
    real = None
    if args.workload == "udp64" and not args.e2e and not args.no_real and F == 16 << 20:
        real = real_traffic_line(eng, args, F, first, out_kind, stream, device, rank, world)
    ser = None
    if args.workload == "udp64" and not args.e2e and not args.no_ser and F == 16 << 20:
        ser = ser_line(eng, args, F, first, stream, device, rank, world)
    large = None
    if args.workload == "udp64" and not args.e2e and not args.no_large and F == 16 << 20:
        large = large_line(eng, args, first, out_kind, stream, device, rank, world)

    if rank != 0:
        return
    achieved = alg_bytes / kernel_s / 1e9
    traffic = load_traffic("udp64_large" if args.workload == "udp64" and F == LARGE_FRAMES else args.workload,
                           args.out)
    res = {
        "metric": METRIC if args.workload != "ser" else "Mpkt/s build+checksum udp_ping-shape frames",
        "value": tp["value"],
        "unit": "Mpkt/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": tp["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: SURVEY.md App. C generator (splitmix64, seed 0x6E6578), generated on device",
        "config": cfg,
        "gib_s": tp["gib_s"],
        # untimed launches actually run before the K timed ones: W, continued
        # in batches of 32 until WARMUP_SECONDS have passed
        "warmup_run": dict(wstats, floor_s=WARMUP_SECONDS),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic,
                     "kernel_ms": round(kernel_s * 1e3, 4),
                     "algorithmic_bytes_per_launch": alg_bytes},
    }
    if args.workload == "ser":
        res["roofline"]["basis"] = (f"bytes written (SURVEY.md 8(d) SER); parameter reads "
                                    f"({SER_READ[args.ser_shape]} B/frame) not counted")
        # the build has no output kind; tools/pmc.sh records it as ser.desc / ser_probe.desc
        res["roofline"]["traffic"] = load_traffic(SER_TRAFFIC_KEY[args.ser_shape], "desc")
        if world == 1 and not args.no_cpu_baseline:
            try:
                hp = ser_probe_params(p) if args.ser_shape == "probe" else p[:5]
                res["cpu_baseline"] = cpu_baseline_ser(hp, 1 << 20, args.cpu_seconds / 2, host_threads())
                res["cpu_baseline"]["single_thread"] = cpu_baseline_ser(hp, 1 << 20, args.cpu_seconds / 2, 1)
            except Exception as e:
                res["cpu_baseline"] = {"value": None, "error": repr(e)}
    if world == 1 and not args.no_cpu_baseline and batch is not None:
        try:
            res["cpu_baseline"] = cpu_baseline(batch, args.workload, 1 << 20, args.cpu_seconds / 2,
                                               host_threads())
            res["cpu_baseline"]["single_thread"] = cpu_baseline(batch, args.workload, 1 << 20,
                                                                args.cpu_seconds / 2, 1)
        except Exception as e:  # reported, never fatal to the GPU measurement
            res["cpu_baseline"] = {"value": None, "error": repr(e)}
    if ceilings is not None and args.workload == "ser":
        res["roofline"]["stream_ceilings"] = dict(
            ceilings, frac_of_write_only=round(achieved / ceilings["write_only_gbs"], 4))
    elif ceilings is not None:
        res["roofline"]["stream_ceilings"] = dict(
            ceilings, frac_of_read_only=round(achieved / ceilings["read_only_gbs"], 4),
            frac_of_read64_write8=round(achieved / ceilings["read64_write8_gbs"], 4))
    res["clocks"] = head_clocks
    if world > 1:
        res["per_rank"] = per_rank
    # the driver keeps the last ~8 KB of stdout: the configs[2] IMIX object and
    # the packed-batch mixes go last, after the serialize and 52M objects
    for key, obj in (("ser", ser), ("large", large), ("imix", imix), ("malformed", malformed),
                     ("real_traffic", real)):
        if obj is not None:
            res[key] = obj
    log("bench detail: " + json.dumps(res))  # every field, prose and full clock histograms (stderr)
    print(json.dumps(shrink(res), separators=(",", ":")), flush=True)


#: prose fields kept only in the stderr detail line (DESIGN.md §6 "Bench line keys")
DETAIL_ONLY = ("desc", "source", "basis", "note")


def shrink(o, depth=0, parent=None):
    """The stdout form of the bench line (<= 7 KB): prose fields dropped,
    `clocks` objects compacted (nex_amd/clocks.py compact), the CPU
    baseline's single-thread leg reduced to its value. Below the top level
    (the contract's fields stay whole there): `bytes_per_gpu` (= the
    roofline's algorithmic bytes) is dropped, `algorithmic_bytes_per_launch`
    is spelled `alg_bytes`, a roofline omits the top level's bound / peak /
    unit (hbm, 8000, GB/s) and a CPU baseline its unit / kind (Mpkt/s,
    port). DESIGN.md §6 lists the keys."""
    if isinstance(o, dict):
        r = {}
        for k, v in o.items():
            if k in DETAIL_ONLY:
                continue
            if depth > 0 and parent != "config" and k == "bytes_per_gpu":
                continue
            if depth > 1 and parent == "roofline" and k in ("bound", "peak", "unit") and \
                    v in ("hbm", HBM_PEAK_GBS, "GB/s"):
                continue
            if depth > 1 and parent == "cpu_baseline" and (k, v) in (("unit", "Mpkt/s"), ("kind", "port")):
                continue
            if k == "clocks" and isinstance(v, dict):
                r[k] = clocks.compact(v)
            elif k == "single_thread" and isinstance(v, dict):
                r[k] = v.get("value")
            elif k == "algorithmic_bytes_per_launch" and depth > 1:
                r["alg_bytes"] = v
            else:
                r[k] = shrink(v, depth + 1, k)
        return r
    if isinstance(o, list):
        return [shrink(v, depth + 1, parent) for v in o]
    return o


if __name__ == "__main__":
    main()
