"""GPU parity of the tcp_ping / icmp_ping builders against
the oracle restatement (oracle/nex_oracle.c nexo_build_tcp /
nexo_build_icmp_echo), byte for byte, IPv4 and IPv6, in the LDS-staged
(even / odd stride) and direct (stride > 128) kernels; every built frame also
verifies through the GPU parse path."""
import numpy as np
import pytest

from nex_amd import abi
from nex_amd.engine import FrameBatch
from tests import helpers

pytestmark = pytest.mark.gpu

TCP_PING_OPTS = bytes.fromhex("020405b4" "0402" "01" "01" "030307")


def _addrs(rng, n, family):
    w = 4 if family == 4 else 16
    return (rng.integers(0, 256, (n, w), dtype=np.uint8), rng.integers(0, 256, (n, w), dtype=np.uint8))


def _u16(rng, n):
    return rng.integers(0, 65536, n).astype(np.uint16)


@pytest.mark.parametrize("family", [4, 6])
@pytest.mark.parametrize("opts,payload_len,stride", [(TCP_PING_OPTS, 0, None), (b"", 3, None),
                                                     (TCP_PING_OPTS, 0, 129), (bytes([1] * 40), 7, None),
                                                     (b"\x02\x04\x05\xb4", 1, 97)])
def test_build_tcp_matches_oracle(engine, oracle, family, opts, payload_len, stride):
    import torch
    n = 3000
    rng = np.random.default_rng(family * 100 + payload_len + len(opts))
    src, dst = _addrs(rng, n, family)
    sp, dp = _u16(rng, n), _u16(rng, n)
    seq = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    ack = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    ipid = _u16(rng, n)
    payload = bytes(rng.integers(0, 256, payload_len, dtype=np.uint8))
    pt = torch.tensor(list(payload), dtype=torch.uint8, device="cuda") if payload_len else None
    smac, dmac = bytes([2, 0, 0, 0, 0, 1]), bytes([2, 0, 0, 0, 0, 2])
    L = 14 + (20 if family == 4 else 40) + 20 + (len(opts) + 3) // 4 * 4 + payload_len
    S = stride or L
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    out = engine.build_tcp(family, cu(src), cu(dst), cu(sp.view(np.int16)), cu(dp.view(np.int16)),
                           cu(seq.view(np.int32)), cu(ack.view(np.int32)), flags=0x12, window=64240,
                           urgent_ptr=3, options=opts, payload=pt, ip_id=cu(ipid.view(np.int16)),
                           src_mac=smac, dst_mac=dmac, ttl=61, ip_flags=2, tos=0x28, flow_label=0x54321,
                           out_stride=S)
    torch.cuda.synchronize()
    data = out.cpu().numpy()[: n * S].reshape(n, S)
    for i in range(0, n, 7):
        spec = oracle.ip_spec(family, bytes(src[i]), bytes(dst[i]), smac, dmac, int(ipid[i]), 61, 2,
                              0x28, 0x54321)
        want = oracle.build_tcp(spec, int(sp[i]), int(dp[i]), int(seq[i]), int(ack[i]), 0x12, 64240, 3,
                                opts, payload)
        assert bytes(data[i, :L]) == want, i
        if L < S <= 128:
            assert not data[i, L:].any(), i
    recs = engine.parse_to_numpy(FrameBatch.from_strided(np.ascontiguousarray(data[:, :L])),
                                 out_kind=abi.OUT_DESC)
    assert (recs["flags"] & abi.C_L4_OK).all()
    if family == 4:
        assert (recs["flags"] & abi.C_IP_OK).all()


@pytest.mark.parametrize("family", [4, 6])
@pytest.mark.parametrize("payload_len,stride", [(5, None), (0, 64), (1, 63), (300, None), (5, 200)])
def test_build_icmp_echo_matches_oracle(engine, oracle, family, payload_len, stride):
    import torch
    n = 3000
    rng = np.random.default_rng(family * 1000 + payload_len)
    src, dst = _addrs(rng, n, family)
    ident, seqno = _u16(rng, n), _u16(rng, n)
    payload = bytes(rng.integers(0, 256, payload_len, dtype=np.uint8))
    pt = torch.tensor(list(payload), dtype=torch.uint8, device="cuda") if payload_len else None
    L = 14 + (20 if family == 4 else 40) + 8 + payload_len
    S = stride or L
    if S < L:
        pytest.skip("stride shorter than the frame")
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    typ = 8 if family == 4 else 128
    out = engine.build_icmp_echo(family, cu(src), cu(dst), cu(ident.view(np.int16)),
                                 cu(seqno.view(np.int16)), payload=pt, def_ip_id=0x4242, ttl=64,
                                 ip_flags=2, out_stride=S)
    torch.cuda.synchronize()
    data = out.cpu().numpy()[: n * S].reshape(n, S)
    for i in range(0, n, 7):
        spec = oracle.ip_spec(family, bytes(src[i]), bytes(dst[i]), ip_id=0x4242, ttl=64, ip_flags=2)
        want = oracle.build_icmp_echo(spec, typ, 0, int(ident[i]), int(seqno[i]), payload)
        assert bytes(data[i, :L]) == want, i
    recs = engine.parse_to_numpy(FrameBatch.from_strided(np.ascontiguousarray(data[:, :L])),
                                 out_kind=abi.OUT_DESC)
    assert (recs["flags"] & abi.C_L4_OK).all()


def test_builder_errors(engine):
    import torch
    from nex_amd.engine import NexgError
    a = torch.zeros((4, 4), dtype=torch.uint8, device="cuda")
    with pytest.raises(NexgError) as e:  # builder/tcp.rs:211-228 (5 x timestamp option = 50 B)
        engine.build_tcp(4, a, a, options=(bytes([8, 10]) + bytes(8)) * 5)
    assert e.value.status == abi.ERANGE
    big = torch.zeros(65535, dtype=torch.uint8, device="cuda")
    with pytest.raises(NexgError) as e:  # builder/icmp.rs:104-117
        engine.build_icmp_echo(4, a, a, payload=big)
    assert e.value.status == abi.ERANGE
