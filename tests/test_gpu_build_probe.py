"""GPU: the arp / ndp probe builders (examples/arp.rs, examples/ndp.rs) —
nexg_build_arp_batch (ArpPacketBuilder behind Ethernet) and
nexg_build_ndp_ns_batch (NdpPacketBuilder inside IPv6 + Ethernet) — byte-exact
against the oracle's restatement at every stride the builders stage, and
the frames they build parse back on the GPU to the fields they were built
from, with every NS checksum verifying (a full-size 16M build included)."""
import numpy as np
import pytest

from nex_amd import abi
from nex_amd.engine import NexgError
from tests import helpers

pytestmark = pytest.mark.gpu


def _t(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.fixture(scope="module")
def arp_inputs():
    rng = np.random.default_rng(606)
    n = 20000 + 77
    return (rng.integers(0, 256, (n, 4), dtype=np.uint8), rng.integers(0, 256, (n, 4), dtype=np.uint8),
            rng.integers(0, 256, (n, 6), dtype=np.uint8), rng.integers(0, 256, (n, 6), dtype=np.uint8))


@pytest.mark.parametrize("stride", [42, 64, 97, 200])
def test_arp_build_matches_oracle(engine, oracle, arp_inputs, stride):
    tip, sip, smac, tmac = arp_inputs
    n = len(tip)
    out = engine.build_arp(_t(tip), sender_ip=_t(sip), sender_mac=_t(smac), out_stride=stride).cpu().numpy()
    out = out[: n * stride].reshape(n, stride)
    for i in range(0, n, 7):
        want = oracle.build_arp(b"\xff" * 6, bytes(smac[i]), bytes(sip[i]), bytes(6), bytes(tip[i]))
        assert out[i, :42].tobytes() == want, i
    if stride <= 128:  # staged tiles zero the gap after each frame; wider strides leave it as is
        assert not out[:, 42:].any()
    # per-frame target MACs and Ethernet destinations, other header words
    out = engine.build_arp(_t(tip), def_sender_ip=bytes([10, 0, 0, 1]), def_sender_mac=bytes(range(6)),
                           target_mac=_t(tmac), eth_dst=_t(smac[::-1].copy()), operation=2).cpu().numpy()
    out = out[: n * 42].reshape(n, 42)
    for i in range(0, n, 13):
        want = oracle.build_arp(bytes(smac[::-1][i]), bytes(range(6)), bytes([10, 0, 0, 1]), bytes(tmac[i]),
                                bytes(tip[i]), operation=2)
        assert out[i].tobytes() == want, i


def test_arp_frames_parse_back(engine, arp_inputs):
    """The built requests parse (GPU) to ARP frames carrying the inputs
    (arp.rs:340-371 through Frame), sender / target addresses in place."""
    from nex_amd.engine import FrameBatch
    tip, sip, smac, _ = arp_inputs
    n = len(tip)
    out = engine.build_arp(_t(tip), sender_ip=_t(sip), sender_mac=_t(smac))
    recs = engine.parse_to_numpy(FrameBatch(data=out, count=n, stride=42), out_kind=abi.OUT_RECORD)
    assert ((recs["flags"] & 0x3FF) == (abi.L_ETHERNET | abi.L_ARP)).all()
    assert (recs["ethertype"] == 0x0806).all()
    host = out.cpu().numpy().reshape(n, 42)
    assert (host[:, 22:28] == smac).all() and (host[:, 28:32] == sip).all() and (host[:, 38:42] == tip).all()


def test_arp_invalid_field_length(engine, arp_inputs):
    """builder/arp.rs:101-118 (arp_builder_rejects_non_ethernet_address_length)."""
    tip = _t(arp_inputs[0][:4])
    with pytest.raises(NexgError, match="ARP hardware address"):
        engine.build_arp(tip, hw_addr_len=5)
    with pytest.raises(NexgError, match="ARP protocol address"):
        engine.build_arp(tip, proto_addr_len=16)


@pytest.fixture(scope="module")
def ns_inputs():
    rng = np.random.default_rng(607)
    n = 12000 + 33
    src = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    dst = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    dst[:50] = 0
    dst[:50, 15] = 1          # ::1 targets
    dst[50:60, 0:2] = [0xfe, 0x80]  # link-local
    return src, dst


@pytest.mark.parametrize("stride,multicast", [(86, True), (128, True), (87, False), (200, False)])
def test_ndp_ns_build_matches_oracle(engine, oracle, ns_inputs, stride, multicast):
    src, dst = ns_inputs
    n = len(src)
    smac = bytes([0x02, 0x11, 0x22, 0x33, 0x44, 0x55])
    dmac = None if multicast else bytes([0x0a, 0x0b, 0x0c, 0x0d, 0x0e, 0x0f])
    out = engine.build_ndp_ns(_t(src), _t(dst), src_mac=smac, dst_mac=dmac, out_stride=stride).cpu().numpy()
    out = out[: n * stride].reshape(n, stride)
    for i in range(0, n, 5):
        em = bytes([0x33, 0x33]) + bytes(dst[i, 12:16]) if multicast else dmac  # ndp.rs:25-35
        sp = oracle.ip_spec(6, bytes(src[i]), bytes(dst[i]), src_mac=smac, dst_mac=em, ttl=255)
        assert out[i, :86].tobytes() == oracle.build_ndp_ns(sp), i
    if stride <= 128:
        assert not out[:, 86:].any()


def test_ndp_ns_independent_checksum_and_reference_shape(engine, oracle, ns_inputs):
    """The NS checksum is an independent RFC 1071 sum over the IPv6
    pseudo-header + message; the message is the 32-B NeighborSolicit whose
    Icmpv6Packet payload is 28 B (builder/ndp.rs:90-101,
    ndp_builder_produces_aligned_source_link_layer_option); it decodes with
    the NDP views to the target and the source link-layer option."""
    import ipaddress

    from nex_amd import views
    src, dst = ns_inputs
    n = 64
    smac = bytes([0x02, 0, 0, 0, 0, 0x99])
    out = engine.build_ndp_ns(_t(src[:n]), _t(dst[:n]), src_mac=smac).cpu().numpy()[: n * 86].reshape(n, 86)
    for i in range(n):
        f = out[i].tobytes()
        msg = f[54:]
        assert len(msg) == 32 and len(msg) - 4 == 28
        pseudo = bytes(src[i]) + bytes(dst[i]) + (32).to_bytes(4, "big") + bytes([0, 0, 0, 58])
        assert int.from_bytes(msg[2:4], "big") == helpers.rfc1071(pseudo + msg[:2] + b"\0\0" + msg[4:]), i
        ns = views.NeighborSolicitPacket.from_bytes(msg)
        assert ns.target_addr == ipaddress.IPv6Address(bytes(dst[i])) and ns.payload == b""
        assert [(o.option_type, o.length, o.payload) for o in ns.options] == [(1, 1, smac)]


def test_ndp_ns_full_size_verifies(engine):
    """16M NS frames (86-B stride) built and parsed on the GPU: every frame is
    Eth/IPv6/ICMPv6 type 135 and its checksum verifies (size-independent
    property at the configs[3] scale)."""
    import torch

    from nex_amd.engine import FrameBatch
    n = 16 << 20
    g = torch.Generator(device="cuda").manual_seed(5)
    src = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device="cuda", generator=g)
    dst = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device="cuda", generator=g)
    out = engine.build_ndp_ns(src, dst, src_mac=bytes([2, 0, 0, 0, 0, 1]))
    fl = engine.parse(FrameBatch(data=out, count=n, stride=86), out_kind=abi.OUT_FLAGS)
    torch.cuda.synchronize()
    f = fl[: n * 4].view(torch.int32)
    want = abi.L_ETHERNET | abi.L_IP | abi.L_IPV6 | abi.L_ICMPV6 | abi.C_L4_CHECKED | abi.C_L4_OK
    assert bool(((f & want) == want).all().item())
    host = out[: 86 * 1024].cpu().numpy().reshape(1024, 86)
    assert (host[:, 54] == 135).all() and (host[:, 20] == 58).all() and (host[:, 21] == 255).all()


def test_ndp_ns_rejects_ipv4(engine, ns_inputs):
    import torch
    src = torch.zeros((4, 16), dtype=torch.uint8, device="cuda")
    p = abi.NdpNsBuild()
    p.ip = engine._ip_build(4, src, src, None, 0, bytes(6), bytes(6), 255, 0, 0, 0)
    p.count = 4
    out = torch.empty(4 * 86, dtype=torch.uint8, device="cuda")
    import ctypes
    rc = engine.lib.nexg_build_ndp_ns_batch(engine.ctx, ctypes.byref(p), ctypes.c_void_p(out.data_ptr()), 86, None)
    assert rc == abi.EINVAL


def test_udp6_rejects_null_src_ip(engine):
    """nexg_build_udp6_batch has no def_src_ip (only the IPv4 probe batch
    does): a NULL per-frame source array is NEXG_EINVAL, not a device fault."""
    import ctypes

    import torch
    dst = torch.zeros((4, 16), dtype=torch.uint8, device="cuda")
    out = torch.empty(4 * 62, dtype=torch.uint8, device="cuda")
    p = abi.Udp6Build()
    p.src_ip, p.dst_ip = None, dst.data_ptr()
    p.src_port = p.dst_port = p.src_mac = p.dst_mac = p.payload = None
    p.payload_len, p.count, p.hop_limit = 0, 4, 64
    rc = engine.lib.nexg_build_udp6_batch(engine.ctx, ctypes.byref(p), ctypes.c_void_p(out.data_ptr()), 62, None)
    assert rc == abi.EINVAL
    # the same call with the source array builds
    p.src_ip = dst.data_ptr()
    rc = engine.lib.nexg_build_udp6_batch(engine.ctx, ctypes.byref(p), ctypes.c_void_p(out.data_ptr()), 62, None)
    assert rc == 0
    torch.cuda.synchronize()
