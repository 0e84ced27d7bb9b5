"""NEXG_OUT_SPARSE encoding (include/nexg.h), no GPU: the kernels' encoder
(frame_core.hpp sparse_encode, run on the host by the core harness) over the
oracle's records, decoded three independent ways — the kernels' device
decoder, the C header's nexg_sparse_decode and numpy (abi.sparse_to_desc) —
must give back every descriptor exactly, in every parse mode; the synthetic
workloads must need no exceptions at all (their 1-B-per-frame size)."""
import numpy as np
import pytest

from nex_amd import abi
from tests import helpers
from tests.native import harness

MODES = [(0, 0), (abi.PARSE_STRICT, 0), (abi.PARSE_FROM_IP, 14), (abi.PARSE_FROM_IP | abi.PARSE_STRICT, 14),
         (abi.PARSE_VLAN, 0), (abi.PARSE_FROM_IP, 0)]


def desc_of(recs):
    d = np.zeros(len(recs), abi.DESC_DTYPE)
    for n in abi.DESC_DTYPE.names:
        d[n] = recs[n]
    return d


def host_sparse_buffer(codes, recs):
    """The NEXG_OUT_SPARSE byte layout a kernel writes for these codes."""
    n = len(codes)
    buf = np.zeros(abi.sparse_bytes(n), np.uint8)
    buf[:n] = codes
    exc = buf[abi.sparse_exc_offset(n):].view(abi.DESC_DTYPE)
    d = desc_of(recs)
    for g in range(0, n, 64):
        idx = [i for i in range(g, min(g + 64, n)) if codes[i] == 0]
        for k, i in enumerate(idx):
            exc[g + k] = d[i]
    return buf


@pytest.fixture(scope="module")
def corpus(oracle):
    base = ([bytes.fromhex(v["frame"]) for v in helpers.golden()["frames"]] + helpers.crafted_frames() +
            helpers.vlan_frames() + helpers.slice_frames() +
            [oracle.gen_frame(abi.WL_IMIX, i) for i in range(300)] +
            [oracle.gen_frame(abi.WL_UDP64, i) for i in range(50)])
    return base + helpers.mutate_frames(np.random.default_rng(77), base, 20000)


@pytest.mark.parametrize("flags,ip_offset", MODES)
def test_sparse_roundtrip_all_decoders(oracle, corpus, flags, ip_offset):
    recs = oracle.parse_frames(corpus, flags, ip_offset)
    codes, dev, hdr = harness.sparse(recs, flags, ip_offset)
    want = desc_of(recs)
    ok = codes != 0
    assert ok.mean() > 0.5, ok.mean()  # most frames, even mutated ones, have a shape code
    helpers.records_equal(dev[ok], want[ok], None, "device decoder")
    helpers.records_equal(hdr[ok], want[ok], None, "header decoder")
    lens = np.array([len(f) for f in corpus])
    got = abi.sparse_to_desc(host_sparse_buffer(codes, recs), len(corpus), lens, flags, ip_offset)
    helpers.records_equal(got, want, corpus, "numpy decoder incl. exceptions")
    # every code that decodes is one the table defines: shape 1..15, tags <= 2
    assert ((codes[ok] & 0xF) >= 1).all() and ((codes >> 6) <= 2).all()


def test_sparse_every_code_and_length():
    """All 256 code bytes x lengths: the C header decoder, the kernels'
    decoder and numpy agree wherever a code decodes (pure table check)."""
    codes = np.repeat(np.arange(256, dtype=np.uint8), 9)
    lens = np.tile(np.array([0, 14, 42, 60, 64, 74, 100, 1500, 65535]), 256)
    for flags, ip_offset in ((0, 0), (abi.PARSE_FROM_IP, 6), (abi.PARSE_VLAN, 0)):
        buf = np.zeros(abi.sparse_bytes(len(codes)), np.uint8)
        buf[:len(codes)] = codes
        out = abi.sparse_to_desc(buf, len(codes), lens, flags, ip_offset)
        dev, hdr = harness.sparse_decode(codes, lens, flags, ip_offset)
        ok = codes & 15 != 0
        assert (dev["flags"][~ok] == 0xFFFFFFFF).all()
        helpers.records_equal(dev[ok], out[ok], None, "device decoder vs numpy")
        helpers.records_equal(hdr[ok], out[ok], None, "header decoder vs numpy")


@pytest.mark.parametrize("workload", [abi.WL_UDP64, abi.WL_IMIX])
def test_synthetic_workloads_need_no_exceptions(oracle, workload):
    frames = [oracle.gen_frame(workload, i) for i in range(4000)]
    recs = oracle.parse_frames(frames)
    codes, dev, _ = harness.sparse(recs)
    assert (codes != 0).all()
    helpers.records_equal(dev, desc_of(recs), frames, "synthetic")
    if workload == abi.WL_UDP64:
        assert set(np.unique(codes & 0xF)) == {1}  # NEXG_SHAPE_V4_UDP


def host_grouped_buffer(codes, recs, tile_run=False):
    """The NEXG_OUT_GROUPED byte layout a kernel writes for these codes
    (include/nexg.h): uniform 64-frame groups as head + verdict masks, the
    rest as NEXG_OUT_SPARSE codes and exceptions past them. tile_run: the
    packed-batch kernel's form, every group mixed with head
    NEXG_GROUPED_TILE_RUN and each 256-frame tile's exceptions in one run."""
    n = len(codes)
    mask, code, exc_off, total = abi.grouped_offsets(n)
    buf = np.zeros(total, np.uint8)
    exc = buf[exc_off:].view(abi.DESC_DTYPE)
    d = desc_of(recs)
    if tile_run:
        buf[:(n + 63) // 64] = abi.GROUPED_TILE_RUN
        buf[code:code + n] = np.asarray(codes, np.uint8)
        for t in range(0, n, 256):
            for k, i in enumerate([i for i in range(t, min(t + 256, n)) if codes[i] == 0]):
                exc[t + k] = d[i]
        return buf
    for g in range(0, n, 64):
        c = np.asarray(codes[g:g + 64], np.int64)
        base = c & ~(abi.SPARSE_IP_OK | abi.SPARSE_L4_OK)
        if (base == base[0]).all() and (base[0] & 0xF) != 0:
            buf[g // 64] = base[0]
            ip = sum(1 << k for k in range(len(c)) if c[k] & abi.SPARSE_IP_OK)
            l4 = sum(1 << k for k in range(len(c)) if c[k] & abi.SPARSE_L4_OK)
            buf[mask + 16 * (g // 64):mask + 16 * (g // 64) + 16] = np.frombuffer(
                ip.to_bytes(8, "little") + l4.to_bytes(8, "little"), np.uint8)
            continue
        buf[code + g:code + g + len(c)] = c
        for k, i in enumerate([i for i in range(g, min(g + 64, n)) if codes[i] == 0]):
            exc[g + k] = d[i]
    return buf


def test_grouped_roundtrip_both_decoders(oracle, corpus, tmp_path):
    """NEXG_OUT_GROUPED over uniform groups (64-B UDP frames, both verdicts
    varying), groups one frame off uniform, partial last groups and the mixed
    corpus: the numpy decoder restores every descriptor and the header's
    inline nexg_grouped_code gives every frame's NEXG_OUT_SPARSE code."""
    import os
    import subprocess
    rng = np.random.default_rng(5)
    udp = [bytearray(oracle.gen_frame(abi.WL_UDP64, i)) for i in range(64 * 5 + 40)]
    for f in udp[::3]:
        f[rng.integers(42, 64)] ^= 0x5A  # UDP checksum fails: L4 verdict varies inside a group
    for f in udp[1::7]:
        f[24] ^= 0x01  # IPv4 header checksum fails
    udp[64 * 2 + 9] = bytearray(oracle.gen_frame(abi.WL_IMIX, 3))  # one group no longer uniform
    frames = [bytes(f) for f in udp] + corpus[:1000]
    recs = oracle.parse_frames(frames)
    codes, _, _ = harness.sparse(recs, 0, 0)
    buf = host_grouped_buffer(codes, recs)
    assert (buf[:5] != 0).sum() >= 3  # uniform groups present
    lens = np.array([len(f) for f in frames])
    helpers.records_equal(abi.grouped_to_desc(buf, len(frames), lens), desc_of(recs), frames, "grouped numpy")
    assert (abi.grouped_codes(buf, len(frames)) == codes).all()
    src = tmp_path / "g.c"
    src.write_text('#include <stdio.h>\n#include <stdlib.h>\n#include "%s"\n'
                   'int main(int c, char** v) { FILE* f = fopen(v[1], "rb"); static unsigned char b[1 << 22];'
                   ' if (!f || fread(b, 1, sizeof b, f) == 0) return 2; unsigned long long n = strtoull(v[2], 0, 10);'
                   ' for (unsigned long long i = 0; i < n; i++) printf("%%u %%llu\\n", nexg_grouped_code(b, n, i),'
                   ' (unsigned long long)nexg_grouped_exc_slot(b, n, i));'
                   ' return 0; }\n' % os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                   "include", "nexg.h"))
    subprocess.check_call(["gcc", "-O1", "-std=c99", "-Wall", "-Werror", "-o", str(tmp_path / "g"), str(src)])
    buf.tofile(tmp_path / "b.bin")
    out = subprocess.check_output([str(tmp_path / "g"), str(tmp_path / "b.bin"), str(len(frames))]).split()
    assert [int(x) for x in out[0::2]] == [int(x) for x in codes]
    # per-group exception slots (heads 0): the group's base + the rank among its code-0 frames
    ex = [i for i in range(len(frames)) if codes[i] == 0]
    want = {i: i // 64 * 64 + sum(1 for j in ex if i // 64 * 64 <= j < i) for i in ex}
    assert all(int(out[2 * i + 1]) == want[i] for i in ex)


def test_grouped_tile_run_both_decoders(oracle, corpus, tmp_path):
    """The packed-batch kernel's grouped form (heads NEXG_GROUPED_TILE_RUN,
    each 256-frame tile's exceptions in one run) over the mixed corpus with a
    partial last tile: the numpy decoder restores every descriptor, and the
    header's nexg_grouped_exc_slot names each exception's slot."""
    import os
    import subprocess
    frames = corpus[:1000] + corpus[:77]
    recs = oracle.parse_frames(frames)
    codes, _, _ = harness.sparse(recs, 0, 0)
    assert 50 < int((np.asarray(codes) == 0).sum()) < len(frames)  # exceptions in most tiles
    buf = host_grouped_buffer(codes, recs, tile_run=True)
    lens = np.array([len(f) for f in frames])
    helpers.records_equal(abi.grouped_to_desc(buf, len(frames), lens), desc_of(recs), frames, "grouped tile run")
    assert (abi.grouped_codes(buf, len(frames)) == codes).all()
    src = tmp_path / "s.c"
    src.write_text('#include <stdio.h>\n#include <stdlib.h>\n#include "%s"\n'
                   'int main(int c, char** v) { FILE* f = fopen(v[1], "rb"); static unsigned char b[1 << 22];'
                   ' if (!f || fread(b, 1, sizeof b, f) == 0) return 2; unsigned long long n = strtoull(v[2], 0, 10);'
                   ' for (unsigned long long i = 0; i < n; i++) if (nexg_grouped_code(b, n, i) == 0)'
                   ' printf("%%llu %%llu\\n", i, (unsigned long long)nexg_grouped_exc_slot(b, n, i));'
                   ' return 0; }\n' % os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                    "include", "nexg.h"))
    subprocess.check_call(["gcc", "-O1", "-std=c99", "-Wall", "-Werror", "-o", str(tmp_path / "s"), str(src)])
    buf.tofile(tmp_path / "b.bin")
    out = subprocess.check_output([str(tmp_path / "s"), str(tmp_path / "b.bin"), str(len(frames))]).split()
    pairs = [(int(out[k]), int(out[k + 1])) for k in range(0, len(out), 2)]
    ex = [i for i in range(len(frames)) if codes[i] == 0]
    want = [(i, i // 256 * 256 + sum(1 for j in ex if i // 256 * 256 <= j < i)) for i in ex]
    assert pairs == want
