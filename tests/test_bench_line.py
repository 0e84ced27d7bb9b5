"""CPU: the bench line's stdout form and the product library's surface.

- bench.shrink keeps the driver's record readable: the round-5 driver-command
  line (18.8 KB, profiles/r05/s7/driver_cmd.log) shrinks below 7 KB with
  every object's roofline fraction, the contract's top-level fields whole,
  and the configs[2] IMIX / App. C mix / real-traffic objects printed last;
- the product library reads no environment variable (the measurement
  overrides live only in nex_amd/libnexg_knobs.so);
- the builders refuse per-frame arrays and outputs shorter than the batch
  before anything reaches the device (Engine._check_rows / _check_out)."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _r05_line():
    with open(os.path.join(ROOT, "profiles", "r05", "s7", "driver_cmd.log")) as f:
        for ln in f:
            if ln.startswith("{"):
                return json.loads(ln)
    raise AssertionError("no line")


def test_shrink_keeps_every_frac_under_7kb():
    import bench
    full = _r05_line()
    # the long prose fields round 6 moved to "desc": emulate their new short form

    def short(o, top):
        if isinstance(o, dict):
            for k, v in list(o.items()):
                if k == "config":
                    continue
                if k == "workload" and not top:
                    o["desc"], o["workload"] = v, v[:30]
                elif k == "sample":
                    o[k] = v[:60]
                else:
                    short(v, False)
    short(full, True)
    order = ["ser", "large", "imix", "malformed", "real_traffic"]
    full = {**{k: v for k, v in full.items() if k not in order}, **{k: full[k] for k in order}}
    s = json.dumps(bench.shrink(full), separators=(",", ":"))
    assert len(s) < 7000, len(s)
    d = json.loads(s)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert d[k] == full[k], k
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert d["roofline"][k] == full["roofline"][k], k
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in d["cpu_baseline"], k
    assert list(d)[-3:] == ["imix", "malformed", "real_traffic"]
    for k in ("imix", "malformed", "real_traffic", "large"):
        assert d[k]["roofline"]["frac"] == full[k]["roofline"]["frac"], k
        assert d[k]["roofline"]["alg_bytes"] == full[k]["roofline"]["algorithmic_bytes_per_launch"]
    for k in ("tuples", "tcp_ping", "icmp_ping", "udp6"):
        assert d["ser"][k]["roofline"]["frac"] == full["ser"][k]["roofline"]["frac"], k
    # the driver keeps the last 8,081 characters: the three packed-batch objects are all inside
    tail = s[-8000:]
    for k in ("imix", "malformed", "real_traffic"):
        assert f'"{k}":' in tail
    c = d["imix"]["clocks"]
    assert set(c) >= {"sclk_mhz", "mclk_mhz", "span_ghz", "span_share", "lat_ns"}
    assert len(c["span_share"]) == 5 and abs(sum(c["span_share"]) - 1) < 0.02


def test_product_library_reads_no_environment():
    lib = os.path.join(ROOT, "nex_amd", "libnexg.so")
    if not os.path.exists(lib):
        pytest.skip("libnexg.so not built")
    out = subprocess.run(["strings", lib], capture_output=True, text=True, check=True).stdout
    names = sorted({w for w in out.split() if w.startswith("NEXG_") and w.upper() == w})
    assert names == [], names
    knobs = os.path.join(ROOT, "nex_amd", "libnexg_knobs.so")
    if os.path.exists(knobs):
        out = subprocess.run(["strings", knobs], capture_output=True, text=True, check=True).stdout
        assert "NEXG_TILE_ORDER" in out


def test_builder_argument_rows():
    import torch
    from nex_amd.engine import Engine
    dst = torch.zeros((100, 4), dtype=torch.uint8)
    Engine._check_rows(100, 4, shared_ok=True, src_ip=torch.zeros(4, dtype=torch.uint8))
    Engine._check_rows(100, 4, shared_ok=True, src_ip=dst)
    with pytest.raises(ValueError):
        Engine._check_rows(100, 4, shared_ok=True, src_ip=torch.zeros((2, 4), dtype=torch.uint8))
    with pytest.raises(ValueError):
        Engine._check_rows(100, 2, src_port=torch.zeros(99, dtype=torch.int16))
    Engine._check_rows(100, 2, src_port=torch.zeros(100, dtype=torch.int16), dst_port=None)
    Engine._check_out(torch.zeros(100 * 42, dtype=torch.uint8), 100, 42)
    with pytest.raises(ValueError):
        Engine._check_out(torch.zeros(100 * 42 - 1, dtype=torch.uint8), 100, 42)
