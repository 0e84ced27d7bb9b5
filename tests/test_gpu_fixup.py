"""GPU: nexg_recompute_checksums_batch (mutable-view checksum fix-up, in
place) against the oracle, and the reference's own checksum-consistency
relations as fixed-point tests: a packet whose checksum field is rewritten by
recompute_checksum (raw-buffer semantics) verifies under the packet API that
parse uses (ipv4.rs:1073-1174, udp.rs:579-628, tcp.rs:1385-1428,
icmp.rs:817-855, icmpv6.rs:527-600). Plus the 16M udp_ping SER batch checked
in full through the parse path (configs[3] at its full size)."""
import numpy as np
import pytest

from nex_amd import abi
from nex_amd.engine import FrameBatch
from nex_amd.frame import ParseMode, ParseOption
from tests import helpers

pytestmark = pytest.mark.gpu

BOTH = abi.FIX_IP | abi.FIX_L4


def eth(p, et=0x0800):
    return bytes([2, 0, 0, 0, 0, 2, 2, 0, 0, 0, 0, 1]) + et.to_bytes(2, "big") + p


def ipv4(payload, proto, src, dst, ttl=64, ident=0):
    tot = 20 + len(payload)
    return bytes([0x45, 0, tot >> 8, tot & 255, ident >> 8, ident & 255, 0x40, 0, ttl, proto, 0, 0]) + \
        bytes(src) + bytes(dst) + payload


def ipv6(payload, nh, src, dst):
    return bytes([0x60, 0, 0, 0]) + len(payload).to_bytes(2, "big") + bytes([nh, 64]) + bytes(src) + \
        bytes(dst) + payload


LOOP6 = bytes(15) + b"\x01"  # Ipv6Addr::LOCALHOST


def fix_on_gpu(engine, frames, which=BOTH, option=ParseOption()):
    import torch
    b = FrameBatch.from_frames(frames, pad_to=4)
    rep = engine.recompute_checksums(b, which, option)
    torch.cuda.synchronize()
    data = b.data.cpu().numpy()
    offs = b.offsets.cpu().numpy()
    out = [bytes(data[offs[i]:offs[i] + len(f)]) for i, f in enumerate(frames)]
    return out, rep.cpu().numpy()[: len(frames) * 8].view(abi.FIXUP_DTYPE)


def parse(engine, frames, option=ParseOption()):
    return engine.parse_to_numpy(FrameBatch.from_frames(frames, pad_to=4), option, ParseMode.Lenient,
                                 abi.OUT_RECORD)


def check_fixed_point(engine, oracle, frames, which=BOTH, option=ParseOption()):
    """recompute on the GPU == oracle bytes; the value written equals the
    packet-API checksum of the same packet; the fixed packet verifies."""
    flags = option.flags(ParseMode.Lenient)
    fixed, rep = fix_on_gpu(engine, frames, which, option)
    before = parse(engine, frames, option)
    for i, f in enumerate(frames):
        want, wrep = oracle.recompute_frame(f, which, flags, option.offset)
        assert fixed[i] == want, (i, f.hex())
        assert rep[i].tobytes() == wrep.tobytes(), i
    after = parse(engine, fixed, option)
    for i in range(len(frames)):
        if which & abi.FIX_IP and rep[i]["done"] & abi.FIX_IP:
            assert rep[i]["ip_csum"] == before[i]["ip_csum_calc"], i  # raw == ipv4::checksum(&pkt)
            assert after[i]["flags"] & abi.C_IP_OK, i
        if rep[i]["done"] & abi.FIX_L4:
            assert rep[i]["l4_csum"] == before[i]["l4_csum_calc"], i  # raw == packet API
            assert after[i]["flags"] & abi.C_L4_OK, i
    return fixed, rep, after


def test_ipv4_checksum_roundtrip(engine, oracle):
    """ipv4.rs:1073-1095: checksum(&p) written back; the bytes equal raw with
    bytes 10..11 = computed, and the reparsed header verifies."""
    raw = bytes([0x45, 0x00, 0x00, 0x14, 0x00, 0x00, 0x40, 0x00, 0x40, 0x06, 0x00, 0x00,
                 0x0a, 0x00, 0x00, 0x01, 0x0a, 0x00, 0x00, 0x02])
    opt = ParseOption(True, 0)
    fixed, rep, after = check_fixed_point(engine, oracle, [raw], abi.FIX_IP, opt)
    computed = int(rep[0]["ip_csum"])
    raw_copy = raw[:10] + computed.to_bytes(2, "big") + raw[12:]
    assert fixed[0] == raw_copy
    assert int(after[0]["ip_csum"]) == computed == helpers.rfc1071(raw)


def test_ipv4_auto_and_manual_checksum(engine, oracle):
    """ipv4.rs:1120-1174: recompute == checksum(&frozen) before and after
    set_ttl(0x41) / set_identification(0x1c47), and the two differ."""
    raw = bytes([0x45, 0x00, 0x00, 0x1c, 0x1c, 0x46, 0x40, 0x00, 0x40, 0x06, 0x00, 0x00, 0xc0, 0xa8,
                 0x00, 0x01, 0xc0, 0xa8, 0x00, 0xc7, 0xde, 0xad, 0xbe, 0xef, 0xca, 0xfe, 0xba, 0xbe])
    ttl = raw[:8] + b"\x41" + raw[9:]
    manual = raw[:4] + b"\x1c\x47" + raw[6:10] + b"\xb1\xe6" + raw[12:]
    opt = ParseOption(True, 0)
    _, rep, _ = check_fixed_point(engine, oracle, [raw, ttl, manual], abi.FIX_IP, opt)
    assert rep[0]["ip_csum"] != rep[1]["ip_csum"]


def test_udp_checksum_with_context(engine, oracle):
    """udp.rs:579-628: auto (192.168.0.1 -> .2, then set_destination(0xabce))
    and manual (10.0.0.1 -> 10.0.0.2, set_source(0x2222)) contexts."""
    u = bytes([0x12, 0x34, 0xab, 0xcd, 0x00, 0x0c, 0x00, 0x00]) + b"data"
    u2 = u[:2] + b"\xab\xce" + u[4:]
    m = b"\x22\x22" + u[2:]
    frames = [eth(ipv4(u, 17, [192, 168, 0, 1], [192, 168, 0, 2])),
              eth(ipv4(u2, 17, [192, 168, 0, 1], [192, 168, 0, 2])),
              eth(ipv4(m, 17, [10, 0, 0, 1], [10, 0, 0, 2]))]
    _, rep, _ = check_fixed_point(engine, oracle, frames)
    assert (rep["done"] == BOTH).all() and rep[0]["l4_csum"] != rep[1]["l4_csum"]


def test_tcp_checksum_with_context(engine, oracle):
    """tcp.rs:1385-1428: IPv4 context 192.0.2.1 -> 198.51.100.2 before/after
    set_window(0x2000); IPv6 ::1 -> ::1 with set_flags(0x12)."""
    t = bytes([0x00, 0x50, 0x01, 0xbb, 0x00, 0x00, 0x00, 0x01, 0x00, 0x00, 0x00, 0x00, 0x50, 0x18,
               0x40, 0x00, 0x00, 0x00, 0x00, 0x00]) + b"hello"
    tw = t[:14] + b"\x20\x00" + t[16:]
    t6 = bytes([0x12, 0x34, 0xab, 0xcd, 0, 0, 0, 0, 0, 0, 0, 0, 0x50, 0x12, 0x10, 0x00, 0, 0, 0, 0])
    frames = [eth(ipv4(t, 6, [192, 0, 2, 1], [198, 51, 100, 2])),
              eth(ipv4(tw, 6, [192, 0, 2, 1], [198, 51, 100, 2])),
              eth(ipv6(t6, 6, LOOP6, LOOP6), 0x86DD)]
    _, rep, _ = check_fixed_point(engine, oracle, frames)
    assert (rep["done"] & abi.FIX_L4).all() and rep[0]["l4_csum"] != rep[1]["l4_csum"]


def test_icmp_and_icmpv6_recompute(engine, oracle):
    """icmp.rs:817-855 (EchoReply type, then code 1) and icmpv6.rs:527-600
    (::1 context, EchoReply 129, then code 1)."""
    ic = bytes([0, 0, 0, 0, 0, 1, 0, 1]) + b"pi"
    ic1 = bytes([0, 1, 0, 0, 0, 1, 0, 1]) + b"pi"
    i6 = bytes([129, 0, 0, 0, 0, 1, 0, 1]) + b"pi"
    i61 = bytes([129, 1, 0, 0, 0, 1, 0, 1]) + b"pi"
    frames = [eth(ipv4(ic, 1, [10, 0, 0, 1], [10, 0, 0, 2])), eth(ipv4(ic1, 1, [10, 0, 0, 1], [10, 0, 0, 2])),
              eth(ipv6(i6, 58, LOOP6, LOOP6), 0x86DD), eth(ipv6(i61, 58, LOOP6, LOOP6), 0x86DD)]
    _, rep, after = check_fixed_point(engine, oracle, frames)
    assert (rep["done"] & abi.FIX_L4).all()
    assert rep[0]["l4_csum"] != rep[1]["l4_csum"] and rep[2]["l4_csum"] != rep[3]["l4_csum"]
    assert (after["flags"][:2] & abi.L_ICMP).all() and (after["flags"][2:] & abi.L_ICMPV6).all()


@pytest.mark.parametrize("which", [BOTH, abi.FIX_IP, abi.FIX_L4])
@pytest.mark.parametrize("option", [ParseOption(), ParseOption(True, 14)], ids=["eth", "from_ip"])
def test_mutated_corpus_matches_oracle(engine, oracle, which, option):
    """Every frame of a malformed/mutated mix: the in-place bytes and the
    report equal the oracle's; canonical frames (the synthetic IMIX shapes
    with corrupted checksums) verify after the fix-up."""
    rng = np.random.default_rng(31 + which)
    canon = [oracle.gen_frame(abi.WL_IMIX, i) for i in range(3000)]
    # corrupt both checksum fields of the canonical frames
    bad = []
    for f in canon:
        b = bytearray(f)
        b[24] ^= 0x5A  # IPv4: checksum byte; IPv6: a source-address byte (pseudo-header)
        b[-1] ^= 0x01  # a payload byte: the L4 checksum no longer matches
        bad.append(bytes(b))
    base = ([bytes.fromhex(v["frame"]) for v in helpers.golden()["frames"]] + helpers.crafted_frames() +
            helpers.vlan_frames() + canon[:200])
    frames = bad + base + helpers.mutate_frames(rng, base, 20000)
    flags = option.flags(ParseMode.Lenient)
    fixed, rep = fix_on_gpu(engine, frames, which, option)
    for i, f in enumerate(frames):
        want, wrep = oracle.recompute_frame(f, which, flags, option.offset)
        assert fixed[i] == want, (i, f.hex())
        assert rep[i].tobytes() == wrep.tobytes(), (i, rep[i], wrep)
    if option.from_ip_packet:
        return
    after = parse(engine, fixed[:len(bad)])
    need = (abi.C_IP_OK if which & abi.FIX_IP else 0) | (abi.C_L4_OK if which & abi.FIX_L4 else 0)
    v4 = (after["flags"] & abi.L_IPV4) != 0
    assert ((after["flags"][v4] & need) == need).all()
    if which & abi.FIX_L4:
        assert (after["flags"] & abi.C_L4_OK).all()


def test_fixup_full_size_imix(engine, oracle):
    """configs[2] shape at full size: the generator corrupts 1/16 of the
    checksums; fixing the whole batch in place makes every frame verify."""
    import torch
    n = 16 << 20
    b = engine.gen_batch(abi.WL_IMIX, n)
    d0 = engine.parse(b, out_kind=abi.OUT_DESC)
    engine.recompute_checksums(b, BOTH, report=False)
    d1 = engine.parse(b, out_kind=abi.OUT_DESC)
    torch.cuda.synchronize()
    f0 = d0.cpu().numpy().view(abi.DESC_DTYPE)["flags"]
    f1 = d1.cpu().numpy().view(abi.DESC_DTYPE)["flags"]
    bad0 = ((f0 & abi.C_L4_OK) == 0) | (((f0 & abi.C_IP_CHECKED) != 0) & ((f0 & abi.C_IP_OK) == 0))
    assert abs(bad0.mean() - 1 / 16) < 0.002  # the generator's corrupted share
    assert (f1 & abi.C_L4_OK).all()
    v4 = (f1 & abi.C_IP_CHECKED) != 0
    assert (f1[v4] & abi.C_IP_OK).all()
    # payload locations unchanged by the fix-up
    assert (d0.cpu().numpy().view(abi.DESC_DTYPE)["payload_off"] ==
            d1.cpu().numpy().view(abi.DESC_DTYPE)["payload_off"]).all()


@pytest.mark.parametrize("shape", ["tuples", "probe"])
def test_ser_full_size_verifies(engine, oracle, shape):
    """configs[3] at its full size (16M udp_ping frames), in both bench forms
    (a full tuple per frame; the udp_ping probe batch: a destination per
    frame, one source and port pair): every built frame verifies through the
    GPU parse path, and a 65536-frame random sample is byte-identical to the
    oracle's builder."""
    import torch
    n = 16 << 20
    p = engine.gen_udp4_params(n)
    smac, dmac = b"\x02\0\0\0\0\1", b"\x02\0\0\0\0\2"
    if shape == "probe":
        src, sport, dport = 0xC0A80164, 53443, 33435
        out = engine.build_udp4(None, p[1], def_src_ip=src, def_src_port=sport, def_dst_port=dport,
                                src_mac=smac, dst_mac=dmac, ip_flags=2)
        p = [torch.full((n,), src - (1 << 32), dtype=torch.int32), p[1],
             torch.full((n,), sport - (1 << 16), dtype=torch.int16),
             torch.full((n,), dport - (1 << 16), dtype=torch.int16), torch.zeros(n, dtype=torch.int16)]
    else:
        out = engine.build_udp4(p[0], p[1], p[2], p[3], p[4], src_mac=smac, dst_mac=dmac, ip_flags=2)
    sp = engine.parse(FrameBatch(data=out, count=n, stride=42), out_kind=abi.OUT_SPARSE)
    torch.cuda.synchronize()
    codes = sp[:n].cpu().numpy()
    ok = abi.SPARSE_IP_OK | abi.SPARSE_L4_OK
    assert ((codes & 0xF) == 1).all() and ((codes & ok) == ok).all()  # IPv4/UDP, both checksums verify
    rng = np.random.default_rng(3)
    idx = np.sort(rng.choice(n, 65536, replace=False))
    data = out.cpu().numpy()[: n * 42].reshape(n, 42)[idx]
    host = [t.cpu().numpy()[idx] for t in p]
    for k in range(len(idx)):
        want = oracle.build_udp4(smac, dmac, int(host[0][k]) & 0xFFFFFFFF, int(host[1][k]) & 0xFFFFFFFF,
                                 int(host[2][k]) & 0xFFFF, int(host[3][k]) & 0xFFFF, int(host[4][k]) & 0xFFFF,
                                 64, 2, 0, b"")
        assert bytes(data[k]) == want, int(idx[k])
