#!/usr/bin/env python3
"""Where a span-kernel workgroup's time goes: runs 16M IMIX (and the App. C
mix) through a -DNEXG_SPAN_TIMING build of libnexg (tools/build_variant.sh
abvar/libnexg_timing.so -DNEXG_SPAN_TIMING) and summarises the per-workgroup
s_memtime stamps: start (entry -> span check), sub-tile loop, fast path,
generic section, stores (s_memtime of the workgroup's own XCD; stamps of
different XCDs are not comparable).
usage: python tools/span_timing.py abvar/libnexg_timing.so"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from nex_amd import _lib, abi
    from nex_amd.engine import Engine
    path = os.path.abspath(sys.argv[1])
    _lib._lib, _lib.LIB_PATH = None, path
    eng = Engine(0)
    lib = ctypes.CDLL(path)
    lib.nexg_debug_span_times.restype = ctypes.c_int
    lib.nexg_debug_span_times.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    res = {}
    batches = {"imix": eng.gen_batch(abi.WL_IMIX, 16 << 20)}
    from nex_amd import workloads
    mix, _ = workloads.malformed_mix(eng, 1 << 20)
    batches["malformed"] = workloads.tiled(mix, 16)
    for name, b in batches.items():
        if b is None:
            continue
        nwg = (b.count + 255) // 256
        out = torch.empty(Engine.out_bytes(abi.OUT_GROUPED, b.count), dtype=torch.uint8, device="cuda")
        for _ in range(20):
            eng.parse(b, out_kind=abi.OUT_GROUPED, out=out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        eng.parse(b, out_kind=abi.OUT_GROUPED, out=out)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        host = np.zeros((nwg, 8), np.uint64)
        assert lib.nexg_debug_span_times(host.ctypes.data, nwg) == 0
        t = host[:, :6].astype(np.int64)
        d = np.diff(t, axis=1)  # start, loop, fast, generic, stores (one workgroup's own clock)
        total = t[:, 5] - t[:, 0]
        names = ["start", "subtile_loop", "fast_path", "generic", "stores"]
        r = {"kernel_ms_event": round(ms, 4), "workgroups": int(nwg),
             "mean_cycles": {k: round(float(v), 1) for k, v in zip(names + ["total"], list(d.mean(axis=0)) + [total.mean()])},
             "share": {k: round(float(v / total.mean()), 3) for k, v in zip(names, d.mean(axis=0))},
             "p90_cycles_total": int(np.percentile(total, 90)),
             "distinct_cu_ids": int(len(np.unique(host[:, 6])))}
        res[name] = r
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
