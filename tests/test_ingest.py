"""Capture-file batch ingest (nexg_pcap_*, nex_amd/csrc/nexg_pcap.cpp) on the
host: classic pcap in both byte orders and resolutions, pcapng with EPB / SPB /
OPB blocks, interface timestamp resolutions, skipped blocks, sections that
change byte order, batch boundaries, truncated and malformed files. The GPU
half (device_batches -> nexg_parse_batch) is in tests/test_gpu_parity.py."""
import os

import numpy as np
import pytest

from nex_amd import abi
from nex_amd.ingest import PcapError, PcapReader
from tests import helpers, pcapfile

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "nex_amd", "libnexg.so")
pytestmark = pytest.mark.skipif(not os.path.exists(LIB), reason="libnexg.so not built")


@pytest.fixture(scope="module")
def frames(oracle):
    rng = np.random.default_rng(5)
    base = helpers.crafted_frames() + [oracle.gen_frame(abi.WL_IMIX, i) for i in range(200)]
    return [f for f in base if len(f) > 0] + [bytes(rng.integers(0, 256, 9000, dtype=np.uint8))]


def _write(tmp_path, name, blob):
    p = tmp_path / name
    p.write_bytes(blob)
    return str(p)


@pytest.mark.parametrize("big_endian", [False, True])
@pytest.mark.parametrize("nsec", [False, True])
def test_classic_pcap(tmp_path, frames, big_endian, nsec):
    ts = [i * 1_234_567_891 + 17_000 for i in range(len(frames))]
    path = _write(tmp_path, "a.pcap", pcapfile.classic(frames, ts, big_endian, nsec, linktype=1))
    with PcapReader(path) as r:
        assert r.linktype == 1
        data, offs, t = r.read_batch(max_frames=len(frames) + 5)
        got = [bytes(data[int(a):int(b)]) for a, b in zip(offs[:-1], offs[1:])]
        assert got == frames
        want_ts = ts if nsec else [x // 1000 * 1000 for x in ts]
        assert list(t) == want_ts
        assert len(r.read_batch()[1]) == 1  # end of file


def test_batch_boundaries(tmp_path, frames):
    path = _write(tmp_path, "b.pcap", pcapfile.classic(frames))
    with PcapReader(path) as r:
        got = []
        while True:
            data, offs, _ = r.read_batch(max_frames=7, data_cap=12000)  # both limits bind
            if len(offs) == 1:
                break
            assert len(offs) - 1 <= 7 and offs[-1] <= 12000
            got += [bytes(data[int(a):int(b)]) for a, b in zip(offs[:-1], offs[1:])]
    assert got == frames
    with PcapReader(path) as r, pytest.raises(PcapError):
        for _ in range(1000):  # a record larger than data_cap can never be delivered
            r.read_batch(max_frames=4, data_cap=2000)


@pytest.mark.parametrize("big_endian", [False, True])
def test_pcapng(tmp_path, frames, big_endian):
    be = big_endian
    fr = frames[:60]
    blob = pcapfile.ng_shb(be) + pcapfile.ng_idb(1, 0, None, be) + pcapfile.ng_idb(1, 0, 9, be)
    want_ts = []
    for i, f in enumerate(fr):
        kind = i % 4
        if kind == 0:
            blob += pcapfile.ng_epb(f, 1000 * i + 7, 0, big_endian=be)  # µs ticks (default resolution)
            want_ts.append((1000 * i + 7) * 1000)
        elif kind == 1:
            blob += pcapfile.ng_epb(f, 10**9 * i + 3, 1, big_endian=be)  # ns ticks (if_tsresol 9)
            want_ts.append(10**9 * i + 3)
        elif kind == 2:
            blob += pcapfile.ng_spb(f, be)
            want_ts.append(0)
        else:
            blob += pcapfile.ng_nrb(be) + pcapfile.ng_opb(f, 5 * i, 0, be)
            want_ts.append(5 * i * 1000)
    # a second section in the other byte order
    blob += pcapfile.ng_shb(not be) + pcapfile.ng_idb(1, 0, None, not be)
    blob += pcapfile.ng_epb(fr[0], 42, 0, big_endian=not be)
    path = _write(tmp_path, "c.pcapng", blob)
    with PcapReader(path) as r:
        assert r.linktype == 1
        data, offs, t = r.read_batch(max_frames=1000)
        got = [bytes(data[int(a):int(b)]) for a, b in zip(offs[:-1], offs[1:])]
        assert got == fr + [fr[0]]
        assert list(t) == want_ts + [42000]


def test_caplen_truncated_records(tmp_path, frames):
    caps = [max(1, len(f) // 2) for f in frames]
    path = _write(tmp_path, "d.pcap", pcapfile.classic(frames, caplens=caps))
    with PcapReader(path) as r:
        got = list(r.frames())
    assert got == [f[:c] for f, c in zip(frames, caps)]


def test_truncated_and_bad_files(tmp_path, frames):
    blob = pcapfile.classic(frames[:10])
    path = _write(tmp_path, "e.pcap", blob[:-5])
    with PcapReader(path) as r:
        data, offs, _ = r.read_batch(max_frames=100)
        assert len(offs) - 1 == 9  # the complete records first ...
        with pytest.raises(PcapError):  # ... then the damage
            r.read_batch()
    with pytest.raises(PcapError):
        PcapReader(_write(tmp_path, "f.pcap", b"not a capture file at all"))
    with pytest.raises(PcapError):
        PcapReader(str(tmp_path / "missing.pcap"))
    raw = _write(tmp_path, "g.pcap", pcapfile.classic(frames[:3], linktype=101))
    with PcapReader(raw) as r:
        assert r.linktype == 101


def _all_variants(tmp_path, frames):
    fr = frames[:80]
    out = {"classic_le": pcapfile.classic(fr), "classic_be_ns": pcapfile.classic(fr, big_endian=True, nsec=True)}
    blob = pcapfile.ng_shb() + pcapfile.ng_idb(1, 0, 9)
    for i, f in enumerate(fr):
        blob += (pcapfile.ng_epb(f, i), pcapfile.ng_spb(f), pcapfile.ng_nrb() + pcapfile.ng_opb(f, i))[i % 3]
    out["pcapng"] = blob + pcapfile.ng_shb(True) + pcapfile.ng_idb(1, 0, None, True) + pcapfile.ng_epb(fr[1], 5, big_endian=True)
    return out, fr


@pytest.mark.parametrize("cap", [1 << 22, 20000, 9100])
def test_raw_shape_matches_packed(tmp_path, frames, cap):
    from nex_amd.ingest import raw_frames
    files, fr = _all_variants(tmp_path, frames)
    for name, blob in files.items():
        path = _write(tmp_path, name, blob)
        with PcapReader(path) as r:
            packed = list(r.frames())
        with PcapReader(path) as r:
            raw = list(raw_frames(r, cap=cap, max_frames=13))
        assert raw == packed, name
        assert packed[:len(fr)] == fr


def test_raw_shape_errors(tmp_path, frames):
    from nex_amd.ingest import raw_frames
    path = _write(tmp_path, "t.pcap", pcapfile.classic(frames[:10])[:-3])
    with PcapReader(path) as r:
        got = []
        with pytest.raises(PcapError):
            for f in raw_frames(r, cap=1 << 20):
                got.append(f)
        assert got == frames[:9]
    path = _write(tmp_path, "big.pcap", pcapfile.classic(frames[-1:]))  # a 9000-B record
    with PcapReader(path) as r, pytest.raises(PcapError):
        list(raw_frames(r, cap=4096))


def test_malformed_captures_are_memory_safe(tmp_path, frames):
    """Random corruptions of valid pcap / pcapng files through the reader
    built with AddressSanitizer + UBSan (tests/native/pcap_fuzz): every call
    returns (frames or an error), nothing reads or writes out of bounds."""
    import subprocess
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")
    subprocess.check_call(["make", "-s", "-C", here, "pcap_fuzz"])
    rng = np.random.default_rng(77)
    files, _ = _all_variants(tmp_path, frames)
    paths = []
    for name, blob in files.items():
        for k in range(60):
            b = bytearray(blob)
            for _ in range(int(rng.integers(1, 8))):
                op = rng.integers(0, 3)
                i = int(rng.integers(0, len(b)))
                if op == 0:
                    b[i] = int(rng.integers(0, 256))  # byte flip (lengths, magics, caplens ...)
                elif op == 1:
                    b[i:i + 4] = int(rng.integers(0, 2**32)).to_bytes(4, "little")
                else:
                    del b[i:]  # truncation
                    break
            p = tmp_path / f"{name}_{k}.bin"
            p.write_bytes(bytes(b))
            paths.append(str(p))
    r = subprocess.run([os.path.join(here, "pcap_fuzz")] + paths, capture_output=True, text=True,
                       timeout=300, env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
                                             UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1"))
    assert r.returncode == 0, r.stderr[-3000:]


@pytest.mark.parametrize("threads", [2, 5])
def test_raw_shape_parallel_reads(tmp_path, frames, threads):
    """nexg_pcap_set_read_threads: read_raw's parallel preads (>= 4-MiB
    pieces) deliver exactly the sequential reader's frames, chunk edges and
    carries included, on a ~22 MB classic capture and on pcapng."""
    from nex_amd.ingest import raw_frames
    rep = frames * (22_000_000 // sum(len(f) for f in frames) + 1)
    for name, blob in (("big.pcap", pcapfile.classic(rep)),
                       ("big.pcapng", pcapfile.ng_shb() + pcapfile.ng_idb(1) +
                        b"".join(pcapfile.ng_epb(f, i) for i, f in enumerate(rep[:20000])))):
        path = _write(tmp_path, name, blob)
        with PcapReader(path) as r:
            want = list(raw_frames(r, cap=9 << 20, max_frames=1 << 16))
        for cap in (9 << 20, 17 << 20 | 5):
            with PcapReader(path) as r:
                r.set_read_threads(threads)
                got = list(raw_frames(r, cap=cap, max_frames=1 << 16))
            assert got == want, (name, cap)
        with PcapReader(path) as r:  # the setting leaves the packed shape unchanged
            r.set_read_threads(threads)
            assert list(r.frames()) == want, name
    with PcapReader(path) as r:
        with pytest.raises(PcapError):
            r.set_read_threads(0)


def test_oversized_record_passes_through(tmp_path, frames):
    """A legal record longer than 65535 B (loopback / GRO captures) in the
    middle of a file: both shapes deliver every frame in order, the big one
    included (the parse kernels flag it NEXG_ERR_BAD_EXTENT), and the reader
    never gets stuck (it used to fail every later call)."""
    from nex_amd.ingest import raw_frames
    big = bytes(range(256)) * 274  # 70144 B
    fr = frames[:20] + [big] + frames[20:40]
    for name, blob in (("classic", pcapfile.classic(fr)),
                       ("ng", pcapfile.ng_shb() + pcapfile.ng_idb(1) + b"".join(pcapfile.ng_epb(f, i)
                                                                               for i, f in enumerate(fr)))):
        path = _write(tmp_path, name, blob)
        with PcapReader(path) as r:
            assert list(r.frames(max_frames=7, data_cap=1 << 20)) == fr, name
        with PcapReader(path) as r:
            assert list(raw_frames(r, cap=1 << 20, max_frames=5)) == fr, name


def test_raw_retry_after_erange_resumes(tmp_path, frames):
    """read_raw with a buffer smaller than the next record returns ERANGE and
    keeps every byte it took (carry + file): retrying with a larger buffer
    yields exactly the frames one large read gives."""
    fr = frames[:30] + [frames[-1]] + frames[30:50]  # a 9000-B record in the middle
    path = _write(tmp_path, "r.pcap", pcapfile.classic(fr))
    got = []
    with PcapReader(path) as r:
        small = np.empty(4096, np.uint8)
        big = np.empty(1 << 20, np.uint8)
        offs = np.empty(64, np.uint64)
        lens = np.empty(64, np.uint32)
        errors = 0
        while True:
            try:
                n, used = r.read_raw_into(small, offs, lens)
                buf = small
            except PcapError:
                errors += 1
                n, used = r.read_raw_into(big, offs, lens)
                buf = big
            if n == 0 and used == 0:
                break
            got += [bytes(buf[int(offs[k]):int(offs[k]) + int(lens[k])]) for k in range(n)]
        assert errors >= 1
    assert got == fr


@pytest.mark.parametrize("threads", [3, 8])
def test_raw_parallel_walk_against_lookalike_headers(tmp_path, threads):
    """read_raw's parallel record walk (classic pcap, >= 8 MiB read) starts
    chunks at speculated record boundaries; payloads made of chained,
    plausible-looking 16-B record headers must not fool it: the frames, their
    lengths and the bytes consumed equal the sequential walk's, in both byte
    orders and with the frame limit cutting inside a chunk."""
    import struct

    from nex_amd.ingest import raw_frames
    rng = np.random.default_rng(5)
    fr = []
    for i in range(60000):
        n = int(rng.integers(20, 400))
        if i % 3 == 0:  # a payload of fake headers, each "caplen" pointing at the next
            fake = b""
            while len(fake) + 16 + 24 <= n:
                fake += struct.pack("<IIII", 1_700_000_000, 123456, 24, 24) + bytes(24)
            fr.append(fake + bytes(n - len(fake)))
        else:
            fr.append(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
    for big_endian in (False, True):
        path = _write(tmp_path, f"look{int(big_endian)}.pcap", pcapfile.classic(fr, big_endian=big_endian))
        with PcapReader(path) as r:
            want = list(raw_frames(r, cap=10 << 20, max_frames=1 << 15))
        assert want == fr
        for cap, maxf in ((10 << 20, 1 << 15), (12 << 20 | 3, 1 << 20)):
            with PcapReader(path) as r:
                r.set_read_threads(threads)
                got = list(raw_frames(r, cap=cap, max_frames=maxf))
            assert got == want, (big_endian, cap, maxf)


@pytest.mark.parametrize("window", [1 << 22, 20000, 9100])
def test_mapped_shape_matches_packed(tmp_path, frames, window):
    """nexg_pcap_map + nexg_pcap_walk_mapped (zero-copy shape) describe the
    same frames as the packed reader, for classic pcap in both byte orders /
    resolutions and pcapng, at window sizes that cut records."""
    from nex_amd.ingest import mapped_frames
    files, fr = _all_variants(tmp_path, frames)
    for name, blob in files.items():
        path = _write(tmp_path, name, blob)
        with PcapReader(path) as r:
            packed = list(r.frames())
        with PcapReader(path) as r:
            got = list(mapped_frames(r, window=window, max_frames=13))
        assert got == packed, name


def test_mapped_shape_errors_and_layout(tmp_path, frames):
    """Records are described in place (offsets relative to the window start,
    16-B classic record headers between them, monotone); a truncated file
    raises after its complete records; a window smaller than a record raises
    ERANGE; an empty capture maps to nothing."""
    from nex_amd.ingest import mapped_frames
    path = _write(tmp_path, "m.pcap", pcapfile.classic(frames[:20]))
    with PcapReader(path) as r:
        arr, first = r.map()
        assert first == 24 and len(arr) == os.path.getsize(path)
        offs, lens = np.empty(64, np.uint64), np.empty(64, np.uint32)
        n, nxt = r.walk_mapped(first, 1 << 20, offs, lens)
        assert n == 20 and nxt == len(arr)
        assert int(offs[0]) == 16 and (np.diff(offs[:n].astype(np.int64)) == lens[:n - 1].astype(np.int64) + 16).all()
    path = _write(tmp_path, "mt.pcap", pcapfile.classic(frames[:10])[:-3])
    with PcapReader(path) as r:
        got = []
        with pytest.raises(PcapError):
            for f in mapped_frames(r, window=1 << 20):
                got.append(f)
        assert got == frames[:9]
    path = _write(tmp_path, "mb.pcap", pcapfile.classic(frames[-1:]))  # a 9000-B record
    with PcapReader(path) as r, pytest.raises(PcapError):
        list(mapped_frames(r, window=4096))
    path = _write(tmp_path, "me.pcap", pcapfile.classic([]))
    with PcapReader(path) as r:
        assert list(mapped_frames(r)) == []


@pytest.mark.parametrize("threads", [1, 4])
def test_mapped_parallel_walk(tmp_path, threads):
    """The mapped walk uses the parallel classic walk for windows >= 8 MiB and
    gives the sequential result for any thread count."""
    from nex_amd.ingest import mapped_frames
    rng = np.random.default_rng(9)
    fr = [bytes(rng.integers(0, 256, int(rng.integers(14, 1600)), dtype=np.uint8)) for _ in range(12000)]
    path = _write(tmp_path, "p.pcap", pcapfile.classic(fr))
    with PcapReader(path) as r:
        r.set_read_threads(threads)
        assert list(mapped_frames(r, window=9 << 20, max_frames=1 << 15)) == fr


@pytest.mark.parametrize("shape", ["raw", "mapped"])
def test_parallel_walk_large_final_record(tmp_path, shape):
    """a chunk with no plausible header start (all its bytes
    inside one record larger than a chunk) is never live in the interleaved
    walk; when the buffer ends on a record boundary right after it, the walk
    must still report the whole buffer as consumed, not offset 0 (which made
    read_raw hand the same frames back forever and walk_mapped never
    advance). 16 threads = 128 chunks of ~66 KB over a buffer just over
    8 MiB whose last record is 300 KB of 0xFF (no look-alike header)."""
    import itertools

    from nex_amd.ingest import mapped_frames, raw_frames
    rng = np.random.default_rng(11)
    fr, total = [], 24
    while total < (8 << 20) + 4096 - 300_000:
        f = rng.integers(0, 256, int(rng.integers(60, 1500)), dtype=np.uint8).tobytes()
        fr.append(f)
        total += 16 + len(f)
    fr.append(b"\xff" * 300_000)
    fr_mid = fr[:-1] + [b"\xff" * 140_000] + fr[-1:]  # and a chunk-spanning record in the middle
    for name, frs in (("end", fr), ("mid", fr_mid)):
        path = _write(tmp_path, f"big_{name}.pcap", pcapfile.classic(frs))
        with PcapReader(path) as r:
            r.set_read_threads(16)
            if shape == "raw":
                it = raw_frames(r, cap=os.path.getsize(path) + 64, max_frames=1 << 15)
            else:
                it = mapped_frames(r, window=os.path.getsize(path) + 64, max_frames=1 << 15)
            got = list(itertools.islice(it, len(frs) + 8))
        assert len(got) == len(frs) and got == frs, (name, len(got), len(frs))
