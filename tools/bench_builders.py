#!/usr/bin/env python3
"""Kernel time of the udp_ping-family builders other than the IPv4 probe batch
(SURVEY.md 8(f) row 3): udp_ping's IPv6 branch (62 B), tcp_ping SYN without
and with its option list (54 / 66 B), icmp_ping echo (IPv4 42 B, IPv6 62 B),
16M frames each, per-frame addresses / ports / ids from random device arrays,
HIP events around the launches. Prints one JSON object: per shape kernel ms
and the fraction of 8 TB/s written. Run once per NEXG_BUILD_LDS_PAD setting
to compare occupancies (the pad is read once per process).
usage: [NEXG_BUILD_LDS_PAD=0] [NEXG_L4_ORDER=linear|xcd|xcdK] python tools/bench_builders.py [--frames N]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

TCP_PING_OPTS = bytes.fromhex("020405b4" "0402" "01" "01" "030307")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16 << 20)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--probe", action="store_true", help="time the probe batches (nex_amd/probes.py) instead")
    ap.add_argument("--lib", default=os.path.join(ROOT, "nex_amd", "libnexg_knobs.so"),
                    help="build of libnexg.so (default: the -DNEXG_AB_KNOBS build, which reads the NEXG_* overrides)")
    args = ap.parse_args()
    import torch
    from nex_amd import _lib
    from nex_amd.engine import Engine
    if args.lib:
        _lib._lib, _lib.LIB_PATH = None, os.path.abspath(args.lib)
    eng = Engine(0)
    n = args.frames
    g = torch.Generator(device="cuda").manual_seed(7)
    rb = lambda *shape: torch.randint(0, 256, shape, dtype=torch.uint8, device="cuda", generator=g)
    r16 = lambda: torch.randint(-32768, 32767, (n,), dtype=torch.int16, device="cuda", generator=g)
    r32 = lambda: torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device="cuda", generator=g)
    a4s, a4d, a6s, a6d = rb(n, 4), rb(n, 4), rb(n, 16), rb(n, 16)
    sp, dp, ipid, seq = r16(), r16(), r16(), r32()
    shapes = {
        "udp6_62B": (62, lambda out: eng.build_udp6(a6s, a6d, sp, dp, out=out)),
        "tcp4_syn_54B": (54, lambda out: eng.build_tcp(4, a4s, a4d, sp, dp, seq, None, flags=0x02, window=64240,
                                                       ip_id=ipid, out=out)),
        "tcp4_ping_66B": (66, lambda out: eng.build_tcp(4, a4s, a4d, sp, dp, seq, None, flags=0x02, window=64240,
                                                        options=TCP_PING_OPTS, ip_id=ipid, out=out)),
        "icmp4_echo_42B": (42, lambda out: eng.build_icmp_echo(4, a4s, a4d, sp, dp, ip_id=ipid, out=out)),
        "icmp6_echo_62B": (62, lambda out: eng.build_icmp_echo(6, a6s, a6d, sp, dp, out=out)),
    }
    if args.probe:  # the probe batches of nex_amd/probes.py (one source, a destination per frame)
        from nex_amd import probes
        shapes = {}
        for name in probes.SHAPES:
            d = rb(n, probes.dst_bytes(name))
            shapes[f"probe_{name}_{probes.frame_len(name)}B"] = (
                probes.frame_len(name), lambda out, name=name, d=d: probes.build(eng, name, d, out=out))
        # udp_ping's IPv4 probe batch (bench.py's ser object): a BE u32 destination value per frame
        d4 = r32()
        shapes["probe_udp_ping_42B"] = (42, lambda out: eng.build_udp4(
            None, d4, def_src_ip=0xC0A80164, def_src_port=53443, def_dst_port=33435, src_mac=b"\x02\0\0\0\0\1",
            dst_mac=b"\x02\0\0\0\0\2", ip_flags=2, out=out))
    res = {"frames": n, "lib": args.lib or "default", "lds_pad": os.environ.get("NEXG_BUILD_LDS_PAD", "default"),
           "probe_wgs": os.environ.get("NEXG_PROBE_WGS", "default"), "probe_waves": os.environ.get("NEXG_PROBE_WAVES", "default"),
           "order": os.environ.get("NEXG_L4_ORDER", "default"),
           "build_order": os.environ.get("NEXG_BUILD_ORDER", "default"),
           "probe_icmp": os.environ.get("NEXG_PROBE_ICMP", "default"),
           "probe_lane_tcp": os.environ.get("NEXG_PROBE_LANE_TCP", "default"),
           "probe_udp4": os.environ.get("NEXG_PROBE_UDP4", "default"),
           "lane_wgs": os.environ.get("NEXG_LANE_WGS", "default")}
    for name, (flen, fn) in shapes.items():
        out = torch.empty(n * flen, dtype=torch.uint8, device="cuda")
        for _ in range(10):
            fn(out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = None
        for _ in range(3):
            e0.record()
            for _ in range(args.steps):
                fn(out)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.steps
            best = ms if best is None else min(best, ms)
        res[name] = {"kernel_ms": round(best, 4), "frac_written": round(n * flen / (best * 1e-3) / 8e12, 4)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
