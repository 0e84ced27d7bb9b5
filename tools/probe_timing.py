#!/usr/bin/env python3
"""Where a builder workgroup's time goes, per probe shape: one launch of each
probe batch (16M frames, nex_amd/probes.py shapes and udp_ping's IPv4 probe
batch) through a measurement build of the library (-DNEXG_PROBE_TIMING=1:
thread 0 of every workgroup stamps s_memtime at its phase boundaries, see
nexg_build.hip), then per shape: the kernel time, the shader clock
(s_memtime ticks / 100-MHz ticks), each phase's mean cycles, and how many
workgroups were alive on average (sum of workgroup lifetimes / kernel time).
Phases: [0-1] prologue (destination load issued, template / pattern, first
barrier), [1-2] fill, [2-3] patch (waits for the destination), [3-4]
copy-out issue, [4-5] store completion. The per-lane kernels stamp [1] after
their frame is written (phases fill / patch are 0 for them).
usage: python tools/probe_timing.py --lib abvar/libnexg_ptime.so"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = ("prologue", "fill", "patch", "store_issue", "store_drain")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--frames", type=int, default=16 << 20)
    args = ap.parse_args()
    import numpy as np
    import torch
    from nex_amd import _lib, probes
    from nex_amd.engine import Engine
    _lib._lib, _lib.LIB_PATH = None, os.path.abspath(args.lib)
    eng = Engine(0)
    raw = ctypes.CDLL(os.path.abspath(args.lib))
    raw.nexg_debug_build_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int]
    n = args.frames
    g = torch.Generator(device="cuda").manual_seed(7)
    shapes = {}
    for name in probes.SHAPES:
        d = torch.randint(0, 256, (n, probes.dst_bytes(name)), dtype=torch.uint8, device="cuda", generator=g)
        shapes[name] = (probes.frame_len(name), lambda out, name=name, d=d: probes.build(eng, name, d, out=out))
    d4 = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device="cuda", generator=g)
    macs = (b"\x02\0\0\0\0\1", b"\x02\0\0\0\0\2")
    shapes["udp4"] = (42, lambda out: eng.build_udp4(None, d4, def_src_ip=0xC0A80164, def_src_port=53443,
                                                     def_dst_port=33435, src_mac=macs[0], dst_mac=macs[1],
                                                     ip_flags=2, out=out))
    res = {"lib": args.lib, "frames": n, "env": {k: v for k, v in os.environ.items() if k.startswith("NEXG_")}}
    cap = 8 * (1 << 18)
    host = np.zeros(cap, np.uint64)
    for name, (flen, fn) in shapes.items():
        out = torch.empty(n * flen, dtype=torch.uint8, device="cuda")
        for _ in range(5):
            fn(out)
        torch.cuda.synchronize()
        raw.nexg_debug_build_stamps(host.ctypes.data, cap, 1)  # reset
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn(out)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        assert raw.nexg_debug_build_stamps(host.ctypes.data, cap, 0) == 0
        s = host.reshape(-1, 8).astype(np.int64)
        s = s[(s[:, 0] > 0) & (s[:, 7] > 0)]
        t, rt = s[:, :6], s[:, 6:8]
        d = np.diff(t, axis=1)
        ok = (d >= 0).all(axis=1) & (rt[:, 1] > rt[:, 0])
        s, t, rt, d = s[ok], t[ok], rt[ok], d[ok]
        if len(s) == 0:  # a kernel without stamps
            res[name] = {"kernel_ms": round(ms, 4), "frac_written": round(n * flen / (ms * 1e-3) / 8e12, 4),
                         "workgroups": 0}
            print(name, json.dumps(res[name]), flush=True)
            continue
        ticks = rt[:, 1] - rt[:, 0]
        cyc = t[:, 5] - t[:, 0]
        span_ticks = rt[:, 1].max() - rt[:, 0].min()
        res[name] = {
            "kernel_ms": round(ms, 4), "frac_written": round(n * flen / (ms * 1e-3) / 8e12, 4),
            "workgroups": int(len(s)),
            "shader_clock_ghz": round(float(np.median(cyc / (ticks * 10.0))), 3),
            "wg_us": round(float(ticks.mean()) / 100.0, 3),
            "wg_cycles": round(float(cyc.mean()), 1),
            "phase_cycles": {k: round(float(v), 1) for k, v in zip(PHASES, d.mean(axis=0))},
            "alive_wgs": round(float(ticks.sum()) / float(span_ticks), 1),
        }
        print(name, json.dumps(res[name]), flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
