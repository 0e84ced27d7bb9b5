"""GPU: the calibration probes behind bench.py's `clocks` field.
nexg_probe_span_clock runs the span kernel the parse runs (same grouped
output as nexg_parse_batch) and stamps every workgroup consistently;
nexg_probe_latency's dependent-load chain reports a plausible HBM latency,
alone and under a read stream."""
import numpy as np
import pytest

from nex_amd import abi, clocks
from nex_amd.engine import Engine

pytestmark = pytest.mark.gpu


def test_span_clock_output_equals_parse(engine):
    import torch
    b = engine.gen_batch(abi.WL_IMIX, 100_000)
    want = engine.parse(b, out_kind=abi.OUT_DESC)
    got, st = engine.probe_span_clock(b)
    ex = engine.sparse_expand(b, got, grouped=True)  # grouped -> 8-B descriptors (exception order aside)
    torch.cuda.synchronize()
    n = Engine.out_bytes(abi.OUT_DESC, b.count)
    assert torch.equal(ex[:n], want[:n])
    s = st.cpu().numpy()
    assert s.shape == ((b.count + 255) // 256, 8)
    r = clocks.span_summary(s)
    assert r["valid"] == r["workgroups"]
    assert 0.5 < r["shader_clock_ghz"]["median"] < 3.5
    assert (np.diff(s[:, :6], axis=1) >= 0).all()


def test_probe_latency_plausible(engine):
    import torch
    buf = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
    idle_ns, idle_cyc = engine.probe_latency(buf, steps=500, start=12345)
    loaded_ns, loaded_cyc = engine.probe_latency(buf, steps=500, start=777, loaded=True)
    assert 100 < idle_ns < 20_000, idle_ns
    assert 100 < loaded_ns < 100_000, loaded_ns
    assert idle_cyc > 0 and loaded_cyc > 0
    # the ring: line i -> (i + 16411) mod n
    n = buf.numel() // 64
    ring = buf.view(torch.int32)[:: 16][:1000].cpu().numpy()
    assert (ring == (np.arange(1000) + 16411) % n).all()
