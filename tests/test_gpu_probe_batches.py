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


@pytest.mark.parametrize("plen,stride", [(0, 42), (5, 47), (5, 64), (13, 63), (64, 128), (65, 107), (0, 129)])
def test_udp4_probe_payload_stride(engine, oracle, plen, stride):
    """udp_ping's IPv4 probe batch with a payload and a frame stride past the
    frame (zero padding) or odd: the per-lane kernel's staged (stride <= 128)
    and direct forms give the oracle's bytes."""
    import torch
    n = 1000
    L = 42 + plen
    dst = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device="cuda",
                        generator=torch.Generator(device="cuda").manual_seed(plen + stride))
    pay = bytes(range(7, 7 + plen))
    pt = torch.tensor(list(pay), dtype=torch.uint8, device="cuda") if plen else None
    smac, dmac = bytes([2, 0, 0, 0, 0, 1]), bytes([2, 0, 0, 0, 0, 2])
    out = engine.build_udp4(None, dst, def_src_ip=0xC0A80164, def_src_port=53443, def_dst_port=33435, def_ip_id=9,
                            src_mac=smac, dst_mac=dmac, ttl=61, ip_flags=2, dscp_ecn=0x2e, payload=pt, out_stride=stride)
    torch.cuda.synchronize()
    data = out.cpu().numpy()[: n * stride].reshape(n, stride)
    hd = dst.cpu().numpy().view(np.uint32)
    for i in list(range(0, n, 13)) + [n - 1]:
        want = oracle.build_udp4(smac, dmac, 0xC0A80164, int(hd[i]), 53443, 33435, 9, 61, 2, 0x2e, pay)
        assert bytes(data[i, :L]) == want, (plen, stride, i)
        if stride <= 128:  # the LDS-staged kernels zero the gap (the direct one leaves it)
            assert not data[i, L:].any(), (plen, stride, i)


@pytest.mark.parametrize("family", [4, 6])
@pytest.mark.parametrize("plen,stride", [(5, None), (0, 71), (33, None), (64, 128)])
def test_l4_probe_payload_stride(engine, oracle, family, plen, stride):
    """tcp / icmp probe batches with other payloads and strides (odd, padded,
    the 64-B payload limit of the template kernel, which builds the tcp
    shapes) against the oracle."""
    import torch
    n = 777
    w = 4 if family == 4 else 16
    g = torch.Generator(device="cuda").manual_seed(family * 100 + plen)
    dst = torch.randint(0, 256, (n, w), dtype=torch.uint8, device="cuda", generator=g)
    src = torch.randint(0, 256, (w,), dtype=torch.uint8, device="cuda", generator=g)
    pay = bytes((3 * k + 1) & 0xFF for k in range(plen))
    pt = torch.tensor(list(pay), dtype=torch.uint8, device="cuda") if plen else None
    smac, dmac = bytes([2, 0, 0, 0, 0, 3]), bytes([2, 0, 0, 0, 0, 4])
    hs, hd = bytes(src.cpu().numpy()), dst.cpu().numpy()
    Lt = 14 + (20 if family == 4 else 40) + 20 + 12 + plen
    St = stride or Lt
    if St >= Lt:
        out = engine.build_tcp(family, src, dst, def_src_port=1234, def_dst_port=443, def_seq=0x01020304,
                               def_ack=0x0a0b0c0d, flags=0x12, window=501, urgent_ptr=7, options=probes.TCP_PING_OPTS,
                               payload=pt, def_ip_id=0x55, src_mac=smac, dst_mac=dmac, ttl=33, ip_flags=2, tos=0x10,
                               flow_label=0x12345, out_stride=St)
        torch.cuda.synchronize()
        data = out.cpu().numpy()[: n * St].reshape(n, St)
        for i in list(range(0, n, 11)) + [n - 1]:
            spec = oracle.ip_spec(family, hs, bytes(hd[i]), smac, dmac, 0x55, 33, 2, 0x10, 0x12345)
            want = oracle.build_tcp(spec, 1234, 443, 0x01020304, 0x0a0b0c0d, 0x12, 501, 7, probes.TCP_PING_OPTS, pay)
            assert bytes(data[i, :Lt]) == want, ("tcp", family, plen, St, i)
    Li = 14 + (20 if family == 4 else 40) + 8 + plen
    Si = stride or Li
    if Si >= Li:
        out = engine.build_icmp_echo(family, src, dst, def_identifier=0x77, def_sequence=0x88, payload=pt,
                                     def_ip_id=0x99, src_mac=smac, dst_mac=dmac, ttl=12, ip_flags=2,
                                     flow_label=0x54321, out_stride=Si)
        torch.cuda.synchronize()
        data = out.cpu().numpy()[: n * Si].reshape(n, Si)
        typ = 8 if family == 4 else 128
        for i in list(range(0, n, 11)) + [n - 1]:
            spec = oracle.ip_spec(family, hs, bytes(hd[i]), smac, dmac, 0x99, 12, 2, 0, 0x54321)
            want = oracle.build_icmp_echo(spec, typ, 0, 0x77, 0x88, pay)
            assert bytes(data[i, :Li]) == want, ("icmp", family, plen, Si, i)


@pytest.mark.parametrize("shift,stride,plen", [(1, None, 0), (1, None, 2), (0, 130, 0), (0, 200, 9), (3, 129, 5)])
def test_udp6_probe_per_lane_forms(engine, oracle, shift, stride, plen):
    """udp_ping's IPv6 probe batch where the template kernel does not take it
    (an output not 16-B aligned, a frame period past 128 B): the per-lane
    kernel's src_shared branch, staged and direct, against the oracle."""
    import torch
    n = 1031
    L = 62 + plen
    S = stride or L
    dst = _dst(n, "udp6", 40 + shift + S)
    src = probes.source("udp6", "cuda")
    pay = bytes((5 * k + 3) & 0xFF for k in range(plen))
    pt = torch.tensor(list(pay), dtype=torch.uint8, device="cuda") if plen else None
    buf = torch.zeros(n * S + 16, dtype=torch.uint8, device="cuda")
    out = buf[shift: shift + n * S]
    engine.build_udp6(src, dst, def_src_port=53443, def_dst_port=33435, src_mac=probes.SRC_MAC,
                      dst_mac=probes.DST_MAC, hop_limit=64, payload=pt, out_stride=S, out=out)
    torch.cuda.synchronize()
    data = out.cpu().numpy().reshape(n, S)
    hs, hd = bytes(src.cpu().numpy()), dst.cpu().numpy()
    for i in list(range(0, n, 7)) + [n - 1]:
        want = oracle.build_udp6(probes.SRC_MAC, probes.DST_MAC, hs, bytes(hd[i]), 53443, 33435, 64, 0, 0, pay)
        assert bytes(data[i, :L]) == want, (shift, S, plen, i)


KNOBS_CHILD = r'''
import sys
import torch
from nex_amd import _lib, probes
_lib.LIB_PATH = sys.argv[1]  # the -DNEXG_AB_KNOBS build: NEXG_PROBE_FAIL=1 fails the template launch
from nex_amd.engine import Engine, NexgError
e = Engine(0)
res = {}
for shape in ("tcp_ping", "udp6"):
    d = torch.zeros((300, probes.dst_bytes(shape)), dtype=torch.uint8, device="cuda")
    try:
        probes.build(e, shape, d)
        torch.cuda.synchronize()
        res[shape] = "ok"
    except NexgError as x:
        res[shape] = "error: " + str(x)[:60]
print(res)
'''


def test_template_launch_failure_reaches_caller():
    """A failed launch of the template kernel (fault injection in the
    measurement build) comes back as an error from nexg_build_tcp_batch /
    nexg_build_udp6_batch, not NEXG_OK with the output unwritten."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "nex_amd", "libnexg_knobs.so")
    for fail in ("1", "0"):
        r = subprocess.run([sys.executable, "-c", KNOBS_CHILD, lib], cwd=root, capture_output=True, text=True,
                           timeout=240, env=dict(os.environ, NEXG_PROBE_FAIL=fail))
        assert r.returncode == 0, r.stderr[-2000:]
        res = eval(r.stdout.strip().splitlines()[-1])
        for shape in ("tcp_ping", "udp6"):
            assert res[shape].startswith("error") == (fail == "1"), (fail, res)
