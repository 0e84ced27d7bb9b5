"""nex_amd.parse_frame: the batched counterpart of examples/parse_frame.rs.

CPU: display_frame's layout (parse_frame.rs:76-131) on Frames materialised
from oracle records of the reference's own fixtures. GPU: capture file ->
GPU batches -> display lines == the same lines built from oracle records."""
import numpy as np
import pytest

from nex_amd import abi
from nex_amd.frame import frame_from_record
from nex_amd.parse_frame import display_frame, display_records
from tests import helpers


def _golden(name):
    for v in helpers.golden()["frames"]:
        if v["name"] == name:
            return bytes.fromhex(v["frame"])
    raise KeyError(name)


def test_display_udp_frame(oracle):
    fr = _golden("udp_basic_parse")  # udp.rs:511-527 fixture in a frame
    lines = display_frame(frame_from_record(oracle.parse_frame(fr), fr))
    assert lines[0] == f"Packet Frame ({len(fr)} bytes)"
    assert lines[1].startswith("  Ethernet: ") and lines[1].endswith("(Ipv4)")
    assert lines[2].startswith("  IPv4: ") and lines[2].endswith("(protocol: Udp)")
    assert lines[3] == "  UDP: 4660 -> 43981"
    assert lines[4] == "  Payload: 4 bytes"
    assert len(lines) == 5


def test_display_other_layers(oracle):
    fr = _golden("icmpv6_echo_request_lo")  # icmpv6.rs:606-631
    lines = display_frame(frame_from_record(oracle.parse_frame(fr), fr))
    assert "  IPv6: ::1 -> ::1 (next header: Icmpv6)" in lines
    assert "  ICMPv6: present" in lines
    fr = _golden("unknown_ethertype_keeps_payload")  # frame.rs:665-680
    lines = display_frame(frame_from_record(oracle.parse_frame(fr), fr))
    assert lines[1].endswith("(Unknown(34997))") and lines[-1] == "  Payload: 4 bytes"  # 0x88b5
    fr = _golden("tcp_basic_parse")  # tcp.rs:1276-1314
    lines = display_frame(frame_from_record(oracle.parse_frame(fr), fr))
    assert "  TCP: 49511 -> 9000" in lines


def test_display_records_failed_frame(oracle):
    frames = [b"\x01" * 10, _golden("udp_basic_parse")]  # < 14 B: Err(BufferTooShort)
    recs = oracle.parse_frames(frames)
    lines = list(display_records(recs, frames, 1, "cap"))
    assert lines[0] == "---- Interface: cap, No.: 1, Total Length: 10 bytes ----"
    assert lines[1] == "Failed to parse packet as Frame"
    assert lines[2].startswith("---- Interface: cap, No.: 2,")


@pytest.mark.gpu
def test_parse_capture_on_gpu(engine, oracle, tmp_path):
    from nex_amd.parse_frame import parse_capture
    from tests import pcapfile
    frames = ([bytes.fromhex(v["frame"]) for v in helpers.golden()["frames"] if v["parse_flags"] == 0] +
              helpers.crafted_frames() + [oracle.gen_frame(abi.WL_IMIX, i) for i in range(300)])
    path = tmp_path / "cap.pcap"
    path.write_bytes(pcapfile.classic(frames))
    got = list(parse_capture(str(path), engine=engine, batch_frames=128))
    want = list(display_records(oracle.parse_frames(frames), frames, 1, str(path)))
    assert got == want
    assert len(list(parse_capture(str(path), engine=engine, batch_frames=64, limit=70))) == \
        len(list(display_records(oracle.parse_frames(frames[:70]), frames[:70], 1, str(path))))


@pytest.mark.gpu
def test_cpp_parse_frame_matches_python(engine, oracle, tmp_path):
    """tools/parse_frame (C++ host API) prints exactly what nex_amd.parse_frame
    prints for the same capture (both: capture -> GPU batches -> display_frame)."""
    import os
    import subprocess
    from nex_amd.parse_frame import parse_capture
    from tests import pcapfile
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "parse_frame")
    assert os.path.exists(exe), "build tools/parse_frame first (make -C tools parse_frame)"
    mapped = (bytes(12) + b"\x86\xdd" + bytes([0x60, 0, 0, 0, 0, 8, 17, 64]) +
              bytes(10) + b"\xff\xff" + bytes([1, 2, 3, 4]) + bytes(15) + b"\x01" +
              bytes([0x12, 0x34, 0, 53, 0, 8, 0, 0]))  # IPv6/UDP from ::ffff:1.2.3.4 to ::1
    frames = ([bytes.fromhex(v["frame"]) for v in helpers.golden()["frames"] if v["parse_flags"] == 0] +
              helpers.crafted_frames() + [oracle.gen_frame(abi.WL_IMIX, i) for i in range(500)] + [mapped])
    path = tmp_path / "cap.pcap"
    path.write_bytes(pcapfile.classic(frames))
    want = list(parse_capture(str(path), engine=engine, batch_frames=256))
    assert "  IPv6: ::ffff:1.2.3.4 -> ::1 (next header: Udp)" in want
    r = subprocess.run([exe, str(path), "256"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = r.stdout.splitlines()
    assert len(got) == len(want)
    bad = [(i, g, w) for i, (g, w) in enumerate(zip(got, want)) if g != w]
    assert not bad, bad[:5]
