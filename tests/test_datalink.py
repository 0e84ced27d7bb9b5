"""Live datalink batch rx / tx (nexg_rx_* / nexg_tx_*, nex_amd/datalink.py),
on the CPU: the TPACKET_V3 ring walker on synthetic kernel-layout blocks must
produce the same packed batch as the capture-file path for the same frames;
where this process may open AF_PACKET sockets (CAP_NET_RAW), frames sent in a
batch over loopback come back in a batch through the ring and through
recvmmsg, split without loss or duplication across a PACKET_FANOUT group, and
truncated to read_buffer_size as the reference's recvfrom truncates them."""
import os
import struct
import subprocess
import time

import numpy as np
import pytest

from nex_amd import abi
from tests import helpers, pcapfile

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "nex_amd", "libnexg.so")
pytestmark = pytest.mark.skipif(not os.path.exists(LIB), reason="libnexg.so not built")

MAC_SRC = bytes([2, 0x6E, 0x65, 0x78, 0, 1])


@pytest.fixture(scope="module")
def layout(tmp_path_factory):
    """Offsets of the kernel's TPACKET_V3 structs, from the C compiler."""
    d = tmp_path_factory.mktemp("tp")
    src = d / "p.c"
    src.write_text("""#include <stdio.h>
#include <stddef.h>
#include <linux/if_packet.h>
int main(void){printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\\n",
 sizeof(struct tpacket_block_desc), offsetof(struct tpacket_block_desc, hdr.bh1.block_status),
 offsetof(struct tpacket_block_desc, hdr.bh1.num_pkts), offsetof(struct tpacket_block_desc, hdr.bh1.offset_to_first_pkt),
 sizeof(struct tpacket3_hdr), offsetof(struct tpacket3_hdr, tp_next_offset), offsetof(struct tpacket3_hdr, tp_sec),
 offsetof(struct tpacket3_hdr, tp_nsec), offsetof(struct tpacket3_hdr, tp_snaplen), offsetof(struct tpacket3_hdr, tp_len),
 offsetof(struct tpacket3_hdr, tp_mac), TPACKET_ALIGN(sizeof(struct tpacket3_hdr)),
 offsetof(struct sockaddr_ll, sll_pkttype)); return 0;}""")
    exe = d / "p"
    subprocess.check_call(["gcc", "-o", str(exe), str(src)])
    keys = ("bd_size", "status", "num", "first", "h_size", "next", "sec", "nsec", "snap", "len", "mac",
            "sll", "pkttype")
    return dict(zip(keys, map(int, subprocess.check_output([str(exe)], text=True).split())))


def make_block(L, frames, outgoing=(), block_size=1 << 16, ts0=1_700_000_000):
    """A retired TPACKET_V3 block holding `frames`, laid out as the kernel does."""
    b = bytearray(block_size)
    off = (L["bd_size"] + 15) // 16 * 16
    struct.pack_into("<I", b, L["status"], 1)  # TP_STATUS_USER
    struct.pack_into("<I", b, L["num"], len(frames))
    struct.pack_into("<I", b, L["first"], off)
    for i, f in enumerate(frames):
        mac = (L["sll"] + 20 + 15) // 16 * 16
        size = (mac + len(f) + 15) // 16 * 16
        nxt = size if i + 1 < len(frames) else 0
        struct.pack_into("<IIIII", b, off + L["next"], nxt, ts0 + i, 1000 * i, len(f), len(f) + 7)
        struct.pack_into("<H", b, off + L["mac"], mac)
        b[off + L["sll"] + L["pkttype"]] = 4 if i in outgoing else 0  # PACKET_OUTGOING / PACKET_HOST
        b[off + mac:off + mac + len(f)] = f
        off += size
    return bytes(b)


@pytest.fixture(scope="module")
def frames(oracle):
    return [oracle.gen_frame(abi.WL_IMIX, i) for i in range(60)] + [f for f in helpers.crafted_frames() if f]


def test_ring_walker_matches_pcap_path(tmp_path, layout, frames):
    """configs[4] ingest: a synthetic block walks to exactly the packed batch
    the capture-file reader produces for the same frames."""
    from nex_amd.datalink import walk_block
    from nex_amd.ingest import PcapReader
    fr = [f for f in frames if len(f) <= 1500][:40]
    got, nxt = walk_block(make_block(layout, fr))
    assert nxt == len(fr) and got == fr
    path = tmp_path / "x.pcap"
    path.write_bytes(pcapfile.classic(fr))
    with PcapReader(str(path)) as r:
        data, offs, _ = r.read_batch(max_frames=1000)
    packed = [bytes(data[int(a):int(b)]) for a, b in zip(offs[:-1], offs[1:])]
    assert got == packed


def test_ring_walker_snap_skip_and_resume(layout, frames):
    from nex_amd.datalink import RX_SKIP_OUTGOING, walk_block
    fr = frames[:30]
    blk = make_block(layout, fr, outgoing={1, 5, 7})
    got, _ = walk_block(blk, snap=100)  # read_buffer_size truncation (lib.rs:229-240)
    assert got == [f[:100] for f in fr]
    got, _ = walk_block(blk, flags=RX_SKIP_OUTGOING)
    assert got == [f for i, f in enumerate(fr) if i not in (1, 5, 7)]
    first, nxt = walk_block(blk, max_frames=11)
    assert nxt == 11 and first == fr[:11]
    rest, nxt = walk_block(blk, first=11)
    assert nxt == len(fr) and first + rest == fr
    bad = bytearray(blk)
    struct.pack_into("<I", bad, layout["num"], 1000)  # more packets than the chain holds
    with pytest.raises(OSError):
        walk_block(bytes(bad))


def _sockets_allowed():
    import socket
    try:
        s = socket.socket(socket.AF_PACKET, socket.SOCK_RAW, socket.htons(3))
        s.close()
        return True
    except (PermissionError, OSError):
        return False


live = pytest.mark.skipif(not _sockets_allowed(), reason="AF_PACKET needs CAP_NET_RAW")


def _tagged(frames, tag):
    """Frames re-addressed from a test MAC (so other loopback traffic is
    ignored). 802.1Q frames are left out: the kernel moves a VLAN tag into the
    packet metadata on receive for recvfrom (the reference's path) and the
    ring alike, so the bytes delivered differ from the bytes sent."""
    return [f[:6] + MAC_SRC[:5] + bytes([tag]) + f[12:] for f in frames
            if len(f) >= 14 and f[12:14] not in (b"\x81\x00", b"\x88\xa8", b"\x91\x00")]


def _send(frames):
    from nex_amd.datalink import RawSender
    data = np.frombuffer(b"".join(frames), np.uint8)
    offs = np.cumsum([0] + [len(f) for f in frames]).astype(np.uint64)
    with RawSender("lo") as tx:
        assert tx.send_batch(data, offs) == len(frames)


def _drain(rx, tag):
    got = []
    while True:
        d, o = rx.next_batch()
        if len(o) <= 1:
            return got
        got += [bytes(d[int(a):int(b)]) for a, b in zip(o[:-1], o[1:])]
        got = [g for g in got if g[6:12] == MAC_SRC[:5] + bytes([tag])]


@live
@pytest.mark.parametrize("mode", [0, 1], ids=["tpacket_v3", "recvmmsg"])
def test_loopback_batch_roundtrip(frames, mode):
    from nex_amd.datalink import Config, RawReceiver
    fr = _tagged([f for f in frames if len(f) >= 14] * 20, 10 + mode)
    with RawReceiver("lo", Config(read_timeout_ms=300, mode=mode, skip_outgoing=True)) as rx:
        _send(fr)
        assert _drain(rx, 10 + mode) == fr
    with RawReceiver("lo", Config(read_timeout_ms=300, mode=mode)) as rx:  # the reference keeps both copies
        _send(fr[:50])
        got = _drain(rx, 10 + mode)
        assert len(got) == 100 and sorted(got) == sorted(fr[:50] * 2)


@live
def test_loopback_truncation_and_fanout(frames):
    """read_buffer_size truncation; two receivers in one PACKET_FANOUT group
    (the per-GPU ingest of SURVEY.md 8(e)) split the frames without loss."""
    from nex_amd.datalink import FANOUT_HASH, Config, FanoutOption, RawReceiver
    fr = _tagged([f for f in frames if len(f) >= 14] * 30, 20)
    with RawReceiver("lo", Config(read_timeout_ms=300, read_buffer_size=64, skip_outgoing=True)) as rx:
        _send(fr)
        assert _drain(rx, 20) == [f[:64] for f in fr]
    grp = 0x4E00 | (os.getpid() & 0xFF)
    cfg = Config(read_timeout_ms=300, skip_outgoing=True, linux_fanout=FanoutOption(grp, FANOUT_HASH))
    with RawReceiver("lo", cfg) as a, RawReceiver("lo", cfg) as b:
        _send(fr)
        ga, gb = _drain(a, 20), _drain(b, 20)
    assert sorted(ga + gb) == sorted(fr)
    assert ga and gb  # both members of the group receive a share


def test_open_errors():
    from nex_amd.datalink import Config, DatalinkError, RawReceiver
    with pytest.raises((DatalinkError, PermissionError)):
        RawReceiver("no-such-if0", Config())
    with pytest.raises((DatalinkError, PermissionError)):
        RawReceiver("lo", Config(read_buffer_size=0))


@live
@pytest.mark.parametrize("mode", [0, 1], ids=["tpacket_v3", "recvmmsg"])
@pytest.mark.timeout(60)
def test_rx_buffer_too_small_fails_instead_of_spinning(frames, mode):
    """a data_cap that cannot hold the next frame (ring) or
    one read_buffer_size slot (recvmmsg) returns NEXG_ERANGE instead of
    polling a readable socket forever (read_timeout -1 = wait); a retry with
    a large buffer then resumes at that frame, losing nothing."""
    from nex_amd.datalink import Config, DatalinkError, RawReceiver
    fr = _tagged([f for f in frames if len(f) >= 100] * 4, 30 + mode)
    with RawReceiver("lo", Config(read_timeout_ms=-1, mode=mode, skip_outgoing=True)) as rx:
        _send(fr)
        time.sleep(0.05)
        with pytest.raises(DatalinkError):
            for _ in range(100):  # other loopback traffic may fit first; ours never does
                d, o = rx.next_batch(data_cap=40)
                assert len(o) > 1
        got = []
        while len(got) < len(fr):
            d, o = rx.next_batch()
            got += [bytes(d[int(a):int(b)]) for a, b in zip(o[:-1], o[1:])]
            got = [g for g in got if g[6:12] == MAC_SRC[:5] + bytes([30 + mode])]
        assert got == fr
