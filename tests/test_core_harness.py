"""CPU: the engine's device parse core (frame_core.hpp, the code the gfx950
kernels run) executed on the host via tests/native/core_harness.hip, checked
bit-exactly against the oracle on crafted, mutated and generated frames across
parse modes, frame alignments and LDS window sizes. This is the pre-GPU gate;
tests/test_gpu_parity.py repeats the comparison on the device."""
import os

import numpy as np
import pytest

from nex_amd import abi
from tests import helpers
from tests.native import harness


def pack(frames, align=1, base_off=0):
    offs, pos = [], base_off
    for f in frames:
        offs.append(pos)
        pos += (len(f) + align - 1) // align * align
    buf = np.zeros(pos + 16, np.uint8)
    for f, p in zip(frames, offs):
        buf[p:p + len(f)] = np.frombuffer(f, np.uint8)
    return buf, np.array(offs, np.uint64), np.array([len(f) for f in frames], np.uint32)


@pytest.fixture(scope="module")
def corpus(oracle):
    g = helpers.golden()
    base = ([bytes.fromhex(v["frame"]) for v in g["frames"]] + helpers.crafted_frames() +
            [oracle.gen_frame(abi.WL_IMIX, i) for i in range(60)] +
            [oracle.gen_frame(abi.WL_UDP64, i) for i in range(20)])
    rng = np.random.default_rng(2024)
    return base + helpers.mutate_frames(rng, base, 12000)


@pytest.mark.parametrize("flags", [0, abi.PARSE_STRICT, abi.PARSE_FROM_IP,
                                   abi.PARSE_FROM_IP | abi.PARSE_STRICT])
@pytest.mark.parametrize("layout", [(1, 0), (1, 3), (4, 0), (16, 0)], ids=str)
def test_core_matches_oracle(oracle, corpus, flags, layout):
    buf, offs, lens = pack(corpus, *layout)
    ipo = 14 if flags & abi.PARSE_FROM_IP else 0
    want = oracle.parse_packed(buf, offs, lens, flags=flags, ip_offset=ipo)
    for window in (128, 64, 0):
        for mode in (0, 4, 5):  # WinFrame / canonical fast path / span prefix-sum tail
            got = harness.parse_packed(buf, offs, lens, flags=flags, ip_offset=ipo, window=window,
                                       use_fast=mode)
            helpers.records_equal(got, want, [buf[p:p + l] for p, l in zip(offs, lens)],
                                  f"flags={flags} layout={layout} window={window} mode={mode}")
    # a second poison past len: the unmasked span window must not depend on it
    got = harness.parse_packed(buf, offs, lens, flags=flags, ip_offset=ipo, use_fast=5, poison=0xFF)
    helpers.records_equal(got, want, None, f"flags={flags} layout={layout} poison=0xFF")


def test_core_bad_extent(oracle):
    buf = np.zeros(100, np.uint8)
    got = harness.parse_packed(buf, np.array([0, 90, 200], np.uint64), np.array([64, 20, 4], np.uint32))
    st = abi.status_of(got["flags"])
    assert list(st) == [0, abi.ERR_BAD_EXTENT, abi.ERR_BAD_EXTENT]


def test_core_max_size_frames(oracle):
    """65535-byte frames (the ABI maximum): IPv4 zero total length, UDP and
    TCP spanning the whole frame, IPv6 jumbo-ish payload."""
    rng = np.random.default_rng(7)
    body = bytes(rng.integers(0, 256, 65535 - 14 - 20 - 8, dtype=np.uint8))
    frames = [
        helpers._eth(helpers._ipv4(helpers._udp(body), 17, total=0)),
        helpers._eth(helpers._ipv4(helpers._tcp(body[:-12]), 6, total=0)),
        helpers._eth(helpers._ipv6(helpers._udp(body[:-20]), 17, plen=65535), 0x86DD),
        helpers._eth(helpers._ipv4(body + bytes(8), 1, total=0)),
    ]
    frames = [f[:65535] for f in frames]
    buf, offs, lens = pack(frames, 1, 1)
    want = oracle.parse_packed(buf, offs, lens)
    for mode in (0, 4, 5):
        got = harness.parse_packed(buf, offs, lens, use_fast=mode)
        helpers.records_equal(got, want, None, f"max-size mode={mode}")
    assert (want["flags"] & abi.C_L4_CHECKED).all()


def test_fast_path_udp64_matches_oracle(oracle):
    """fast_udp4_64 (register path of the TileStride64 kernel) vs the oracle on
    64-B frames: generated ones (fast path taken) and single-field mutations of
    them (fast path taken or declined; the result must not depend on which)."""
    rng = np.random.default_rng(64)
    base = [oracle.gen_frame(abi.WL_UDP64, i) for i in range(2000)]
    frames = list(base)
    for f in base[:1500]:
        fr = bytearray(f)
        j = int(rng.choice([12, 13, 14, 16, 17, 23, 38, 39, int(rng.integers(64))]))
        fr[j] = int(rng.choice([0, 0x45, 17, 30, 50, int(rng.integers(256))]))
        frames.append(bytes(fr))
    buf = np.frombuffer(b"".join(frames), np.uint8).copy()
    for flags in (0, abi.PARSE_STRICT, abi.PARSE_FROM_IP):
        ipo = 14 if flags & abi.PARSE_FROM_IP else 0
        want = oracle.parse_packed(buf, stride=64, flags=flags, ip_offset=ipo)
        got = harness.parse_packed(buf, stride=64, flags=flags, ip_offset=ipo, use_fast=True)
        helpers.records_equal(got, want, frames, f"fast path flags={flags}")


def test_canonical_fast_path_on_imix(oracle):
    """fast_canonical80 on generated IMIX frames (all six shapes, every length
    class) and single-byte mutations of them."""
    rng = np.random.default_rng(80)
    base = [oracle.gen_frame(abi.WL_IMIX, i) for i in range(3000)]
    frames = list(base)
    for f in base[:2500]:
        fr = bytearray(f)
        j = int(rng.choice([12, 13, 14, 16, 17, 18, 19, 20, 23, 38, 39, 46, 58, 59, 66, 67,
                            int(rng.integers(len(f)))]))
        fr[min(j, len(fr) - 1)] = int(rng.choice([0, 0x45, 0x60, 6, 17, 58, 1, 0x50, int(rng.integers(256))]))
        frames.append(bytes(fr))
        frames.append(f[: int(rng.integers(30, len(f) + 1))])
    # the App. C kinds the fast path now keeps: Ethernet padding (IP end at
    # the frame end, inside the window, at the span's second prefix value, or
    # in 80..83 where it must decline), declared IP lengths past the frame
    # (clamped unless strict) or 0, UDP length words that do not fit (Q14)
    for f in base[:1500]:
        v4 = f[12:14] == b"\x08\x00"
        frames.append(f + bytes(rng.integers(0, 256, int(rng.integers(1, 64)), dtype=np.uint8)))
        fr = bytearray(f)
        j = 16 if v4 else 18
        fr[j:j + 2] = int(rng.choice([0, int(rng.integers(0, 1 << 16)), len(f) - (14 if v4 else 54) + 1])
                          ).to_bytes(2, "big")
        frames.append(bytes(fr))
        fr = bytearray(f)
        l4 = 34 if v4 else 54
        fr[l4 + 4] = int(rng.integers(256))
        frames.append(bytes(fr))
    frames += helpers.tcp_ts_frames(oracle, base[:1500], rng)  # TCP timestamps (register fast path)
    frames += helpers.tcp_ts_frames(oracle, base[1500:2000], rng, fix_checksums=False)
    frames += helpers.tcp_option_frames(oracle, base[:2500], rng)  # one-TLV option lists and near misses
    frames += helpers.tcp_option_sweep(oracle, rng, base[:600])  # ... for every data offset 6..15
    for e in (64, 79, 80, 81, 83, 84, 85, 100):  # IPv4/UDP of IP end e, padded by 1..40
        for pad in (1, 3, 4, 17, 40):
            body = bytes(rng.integers(0, 256, e - 42, dtype=np.uint8))
            frames.append(helpers._eth(helpers._ipv4(helpers._udp(body), 17)) + bytes(pad))
            frames.append(helpers._eth(helpers._ipv6(helpers._udp(bytes(max(0, e - 62))), 17), 0x86DD) + bytes(pad))
    buf, offs, lens = pack(frames, 4)
    for flags in (0, abi.PARSE_STRICT):
        want = oracle.parse_packed(buf, offs, lens, flags=flags)
        got = harness.parse_packed(buf, offs, lens, flags=flags, use_fast=4)
        helpers.records_equal(got, want, frames, f"canonical flags={flags}")
    # k_parse_span's arithmetic at every byte alignment (odd frames: x256
    # tail for the fast path, SpanFrame for the declined ones)
    for shift in (1, 2, 3):
        buf, offs, lens = pack(frames, 1, shift)
        want = oracle.parse_packed(buf, offs, lens)
        got = harness.parse_packed(buf, offs, lens, use_fast=5)
        helpers.records_equal(got, want, frames, f"span arithmetic shift={shift}")


@pytest.mark.parametrize("flags,ipo", [(0, 0), (abi.PARSE_FROM_IP, 14), (abi.PARSE_FROM_IP, 0),
                                       (abi.PARSE_FROM_IP | abi.PARSE_STRICT, 14)])
@pytest.mark.parametrize("layout", [(1, 0), (1, 3), (4, 0)], ids=str)
def test_slice_core_matches_oracle(oracle, corpus, flags, ipo, layout):
    """FrameSlice core (slice_frame) on the host vs the oracle's FrameSlice."""
    frames = corpus + helpers.slice_frames()
    buf, offs, lens = pack(frames, *layout)
    want = oracle.slice_packed(buf, offs, lens, flags=flags, ip_offset=ipo)
    for window in (128, 64, 0):
        got = harness.slice_packed(buf, offs, lens, flags=flags, ip_offset=ipo, window=window)
        bad = np.nonzero(got != want)[0]
        assert len(bad) == 0, (window, bad[:5], got[bad[:3]], want[bad[:3]])
    st = abi.status_of(want["flags"])
    assert (st == 0).sum() > 1000 and len(set(st.tolist())) >= 4  # both outcomes well covered


@pytest.mark.parametrize("flags", [abi.PARSE_VLAN, abi.PARSE_VLAN | abi.PARSE_STRICT])
@pytest.mark.parametrize("layout", [(1, 0), (4, 0)], ids=str)
def test_vlan_core_matches_oracle(oracle, corpus, flags, layout):
    frames = corpus[:3000] + helpers.vlan_frames()
    buf, offs, lens = pack(frames, *layout)
    want = oracle.parse_packed(buf, offs, lens, flags=flags)
    for mode in (0, 4, 5):
        got = harness.parse_packed(buf, offs, lens, flags=flags, use_fast=mode)
        helpers.records_equal(got, want, None, f"vlan flags={flags} mode={mode}")
    assert (want["flags"] & abi.L_VLAN).sum() >= len(helpers.vlan_frames()) - 3


def test_parse_core_memory_safe_random_inputs(tmp_path, oracle):
    """SURVEY.md §4 item 4 (the reference's panic_free_parsing.rs): random
    0..2048-B inputs and mutated frames through the device parse core and the
    oracle built with AddressSanitizer + UBSan (tests/native/parse_fuzz): each
    frame alone in a heap block ending at its last 16-B load granule, three
    alignments, six parse modes, four staging variants — no out-of-bounds
    access, no UB, and every record / FrameSlice equal to the oracle's."""
    import struct
    import subprocess
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")
    subprocess.check_call(["make", "-s", "-C", here, "parse_fuzz"])
    rng = np.random.default_rng(2048)
    frames = [bytes(rng.integers(0, 256, int(rng.integers(0, 2049)), dtype=np.uint8)) for _ in range(3000)]
    base = ([bytes.fromhex(v["frame"]) for v in helpers.golden()["frames"]] + helpers.crafted_frames() +
            [oracle.gen_frame(abi.WL_IMIX, i) for i in range(200)])
    frames += base + helpers.mutate_frames(rng, base, 6000)
    path = tmp_path / "frames.bin"
    path.write_bytes(b"".join(struct.pack("<I", len(f)) + f for f in frames))
    r = subprocess.run([os.path.join(here, "parse_fuzz"), str(path)], capture_output=True, text=True,
                       timeout=600, env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
                                             UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1"))
    assert r.returncode == 0, (r.stdout[-500:], r.stderr[-3000:])
    assert "mismatches 0" in r.stdout


@pytest.mark.parametrize("kinds", [None, ("l4_length", "ver_ihl", "ipv6_hbh"), ("tcp_sack", "tcp_ts", "pad")])
def test_span_groups_match_oracle(oracle, kinds):
    """k_parse_span's fast path and generic section emulated per 256-frame
    group (80-B slots, bucketed items, deferred ranges) over the malformed
    mix, at two byte alignments of the batch: every record equals the
    oracle's."""
    data, offs, _ = helpers.host_malformed_mix(oracle, 6000, seed=77, kinds=kinds)
    frames = [bytes(data[a:b]) for a, b in zip(offs[:-1], offs[1:])]
    want = oracle.parse_frames(frames)
    for shift in (0, 5):
        buf = np.zeros(len(data) + shift + 16, np.uint8)
        buf[shift:shift + len(data)] = data
        got = harness.span_groups(buf, offs + shift)
        helpers.records_equal(got, want, frames, f"span groups shift {shift}")


def test_fastpath_edge_shapes_match_oracle(oracle):
    """The fast path's round-3 shapes (Q2 short frames, one IPv6 extension
    header, TCP option walks failing at the first TLV) and their near misses,
    lenient and strict, through the lane kernel's path (aligned) and the span
    kernel's arithmetic at every byte alignment, and through the span-group
    emulation: records equal the oracle's."""
    frames = helpers.fastpath_edge_frames(np.random.default_rng(31))
    assert len(frames) > 1500
    buf, offs, lens = pack(frames, 4)
    for flags in (0, abi.PARSE_STRICT):
        want = oracle.parse_packed(buf, offs, lens, flags=flags)
        got = harness.parse_packed(buf, offs, lens, flags=flags, use_fast=4)
        helpers.records_equal(got, want, frames, f"edge shapes flags={flags}")
    for shift in (1, 2, 3):
        buf, offs, lens = pack(frames, 1, shift)
        for flags in (0, abi.PARSE_STRICT):
            got = harness.parse_packed(buf, offs, lens, use_fast=5, flags=flags)
            helpers.records_equal(got, oracle.parse_packed(buf, offs, lens, flags=flags), frames,
                                  f"edge span shift={shift} flags={flags}")
    po = np.zeros(len(frames) + 1, np.int64)
    np.cumsum([len(x) for x in frames], out=po[1:])
    data = np.frombuffer(b"".join(frames) + bytes(16), np.uint8)
    helpers.records_equal(harness.span_groups(data, po), oracle.parse_frames(frames), frames, "edge span groups")


def test_ipv4_options_span_groups(oracle):
    """IPv4 option lists (helpers.ipv4_option_frames: the walk of
    ipv4.rs:442-508, the re-serialised header checksum with Q16 / Q17),
    lenient and strict, at four byte alignments, through the span kernel's
    emulation (fast path + generic section) equal the oracle."""
    frames = helpers.ipv4_option_frames(np.random.default_rng(7))
    assert len(frames) > 15000
    for shift in (0, 1, 2, 3):
        po = np.zeros(len(frames) + 1, np.int64)
        np.cumsum([len(x) for x in frames], out=po[1:])
        data = np.frombuffer(bytes(shift) + b"".join(frames) + bytes(16), np.uint8)
        for flags in (0, abi.PARSE_STRICT):
            got = harness.span_groups(data, po + shift, flags=flags)
            helpers.records_equal(got, oracle.parse_frames(frames, flags=flags), frames,
                                  f"ipv4 options span groups shift={shift} flags={flags}")


def test_tcp_option_walk_span_groups(oracle):
    """TCP option lists beyond the fast path's one-TLV shapes
    (helpers.tcp_walk_frames: SYN lists of common stacks, EOL with junk after
    it, Q13 cuts after the first option) at four byte alignments, lenient and
    strict, through the span kernel's emulation equal the oracle; the
    declined ones are counted by the emulation."""
    frames = helpers.tcp_walk_frames(np.random.default_rng(9))
    for shift in (0, 1, 2, 3):
        po = np.zeros(len(frames) + 1, np.int64)
        np.cumsum([len(x) for x in frames], out=po[1:])
        data = np.frombuffer(bytes(shift) + b"".join(frames) + bytes(16), np.uint8)
        for flags in (0, abi.PARSE_STRICT):
            dec = np.zeros(len(frames), np.uint8)
            got = harness.span_groups(data, po + shift, flags=flags, declined=dec)
            want = oracle.parse_frames(frames, flags=flags)
            helpers.records_equal(got, want, frames, f"tcp walk span groups shift={shift} flags={flags}")
            assert dec.sum() > 0  # multi-option lists go to the generic walk
            q13 = ((want["flags"] & abi.L_TRANSPORT) != 0) & ((want["flags"] & abi.L_TCP) == 0)
            assert q13.sum() > 20


@pytest.mark.parametrize("order", [0, 1, 2, 3, 8, 16, 64, 1 << 20, 0xFFFFFFFF, 0x80000001, 0x80000004, 0x80000000])
def test_tile_map_is_a_permutation(order):
    """tile_of (nexg_internal.hpp), the workgroup -> tile map every tile
    kernel uses: a permutation of [0, nb) for every grid size, ragged tails
    included; order 16 gives each XCD (workgroup % 8) runs of 16 consecutive
    tiles."""
    for nb in list(range(0, 300)) + [1023, 1024, 1025, 4096 + 127, 65536, 212993]:
        m = harness.tile_map(nb, order)
        assert np.array_equal(np.sort(m), np.arange(nb, dtype=np.uint64)), (nb, order)
    if order == 0x80000004:  # CU-affine runs of 32 x 4: the c-th workgroup of XCD x's round takes 4 tiles
        m = harness.tile_map(65536, order).reshape(-1, 8)
        for x in range(8):
            for c in range(32):
                assert np.array_equal(m[c::32, x][:4], x * 128 + c * 4 + np.arange(4))
    if order == 16:
        m = harness.tile_map(65536, 16).reshape(-1, 8)  # row i: the i-th workgroup of each XCD
        for x in range(8):
            run = m[:16, x]
            assert np.array_equal(run, np.arange(x * 16, x * 16 + 16))
