"""GPU parity of the probe batches of udp_ping's IPv6 branch, tcp_ping and
icmp_ping (nex_amd/probes.py; examples/udp_ping.rs:68-89, tcp_ping.rs:108-163,
icmp_ping.rs:67-102): one source, a destination per frame, everything else
the example's constant. The kernels' probe form (nexg_ip_build.src_shared /
nexg_udp6_build.src_shared with no other per-frame array: only the
destination is read per frame) against the oracle's builders
(oracle.build_probe_batch over the single-frame restatements), byte for
byte: at ragged counts every frame, at the bench's 16M frames a sample plus
the first and last tiles; the probe form equals the general form fed the
same source per frame; every frame verifies through the GPU parse path."""
import numpy as np
import pytest

from nex_amd import abi, probes
from nex_amd.engine import FrameBatch
from tests import helpers

pytestmark = pytest.mark.gpu

SHAPES = list(probes.SHAPES)


def _dst(n, shape, seed):
    import torch
    g = torch.Generator(device="cuda").manual_seed(seed)
    return torch.randint(0, 256, (n, probes.dst_bytes(shape)), dtype=torch.uint8, device="cuda", generator=g)


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("n", [1, 255, 257, 5000])
def test_probe_batch_matches_oracle(engine, oracle, shape, n):
    import torch
    dst = _dst(n, shape, 17 + n)
    L = probes.frame_len(shape)
    out = probes.build(engine, shape, dst)
    torch.cuda.synchronize()
    got = out.cpu().numpy()[: n * L].reshape(n, L)
    want = helpers.probe_oracle_build(oracle, shape, dst.cpu().numpy())
    assert want.shape == (n, L)
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert bad.size == 0, (shape, n, bad[:8])


@pytest.mark.parametrize("shape", SHAPES)
def test_probe_form_equals_general_form(engine, shape):
    """The same frames through the general kernel: the source repeated per
    frame (src_shared 0) and, for the L4 shapes, a per-frame array of the
    constant value (not the probe form any more)."""
    import torch
    n = 3000
    dst = _dst(n, shape, 5)
    probe = probes.build(engine, shape, dst)
    src = probes.source(shape, "cuda").repeat(n, 1).contiguous()
    general = probes.build(engine, shape, dst, src=src)
    torch.cuda.synchronize()
    L = probes.frame_len(shape)
    assert torch.equal(probe[: n * L], general[: n * L])
    fam, kind, _ = probes.SHAPES[shape]
    if kind == "udp6":
        sp = torch.full((n,), 53443 - 65536, dtype=torch.int16, device="cuda")
        mixed = engine.build_udp6(probes.source(shape, "cuda"), dst, src_port=sp, def_dst_port=33435,
                                  src_mac=probes.SRC_MAC, dst_mac=probes.DST_MAC)
    elif kind == "tcp":
        sq = torch.zeros(n, dtype=torch.int32, device="cuda")
        mixed = engine.build_tcp(fam, probes.source(shape, "cuda"), dst, seq=sq, def_src_port=53443,
                                 def_dst_port=probes.TCP_PING_DPORT, flags=0x02, window=64240,
                                 options=probes.TCP_PING_OPTS, src_mac=probes.SRC_MAC, dst_mac=probes.DST_MAC,
                                 ip_flags=2 if fam == 4 else 0)
    else:
        ident = torch.full((n,), 0x1234, dtype=torch.int16, device="cuda")
        pay = torch.tensor(list(probes.ICMP_PAYLOAD), dtype=torch.uint8, device="cuda")
        mixed = engine.build_icmp_echo(fam, probes.source(shape, "cuda"), dst, identifier=ident, def_sequence=1,
                                       payload=pay, src_mac=probes.SRC_MAC, dst_mac=probes.DST_MAC,
                                       ip_flags=2 if fam == 4 else 0)
    torch.cuda.synchronize()
    assert torch.equal(probe[: n * L], mixed[: n * L]), shape


@pytest.mark.parametrize("shape", ["udp6", "tcp_ping", "icmp_ping"])
def test_probe_batch_16m(engine, oracle, shape):
    """The bench's batch (16M frames): a 65,536-frame random sample plus the
    first and last 4096 frames against the oracle, and every frame's
    checksums verify through the GPU parse path (the parse's verdicts)."""
    import torch
    n = 16 << 20
    L = probes.frame_len(shape)
    dst = _dst(n, shape, 99)
    out = probes.build(engine, shape, dst)
    torch.cuda.synchronize()
    rng = np.random.default_rng(3)
    sel = np.unique(np.concatenate([np.arange(4096), np.arange(n - 4096, n),
                                    rng.choice(n, 65536, replace=False)]))
    idx = torch.from_numpy(sel).cuda()
    frames = out[: n * L].view(n, L)[idx].cpu().numpy()
    want = helpers.probe_oracle_build(oracle, shape, dst[idx].cpu().numpy(), nthreads=8)
    bad = np.nonzero((frames != want).any(axis=1))[0]
    assert bad.size == 0, (shape, sel[bad[:8]])
    batch = FrameBatch(data=out, count=n, stride=L)
    v = engine.parse(batch, out_kind=abi.OUT_FLAGS)
    torch.cuda.synchronize()
    flags = v[: n * 4].view(torch.int32)
    need = abi.C_L4_OK | (abi.C_IP_OK if probes.SHAPES[shape][0] == 4 else 0)
    assert int(((flags & need) != need).sum().item()) == 0
