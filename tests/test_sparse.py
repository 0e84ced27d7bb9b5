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
