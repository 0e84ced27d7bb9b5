"""GPU parity of the FrameSlice output (NEXG_OUT_SLICE, frame.rs:84-287)
against the oracle's FrameSlice on the same batch layout, in every staging the
kernels use: fixed 64-B and 128-B strides (tile staging), explicit lengths and
packed offset tables (per-lane 128-B window + HBM), parse options."""
import numpy as np
import pytest

from nex_amd import abi
from nex_amd.engine import FrameBatch
from tests import helpers

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def frames(oracle):
    rng = np.random.default_rng(31)
    g = helpers.golden()
    base = ([bytes.fromhex(v["frame"]) for v in g["frames"]] + helpers.crafted_frames() +
            helpers.slice_frames() + [oracle.gen_frame(abi.WL_IMIX, i) for i in range(100)] +
            [oracle.gen_frame(abi.WL_UDP64, i) for i in range(20)])
    return base + helpers.mutate_frames(rng, base, 12000)


def _cmp(got, want, what):
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, f"{what}: {len(bad)} differ, first {bad[:5]}: {got[bad[:2]]} vs {want[bad[:2]]}"


@pytest.mark.parametrize("flags,ipo", [(0, 0), (abi.PARSE_FROM_IP, 14), (abi.PARSE_FROM_IP, 0)])
def test_slice_offset_layouts(engine, oracle, frames, flags, ipo):
    from nex_amd.frame import ParseMode, ParseOption
    opt = ParseOption(bool(flags & abi.PARSE_FROM_IP), ipo)
    for batch in (FrameBatch.from_frames(frames, pad_to=4), FrameBatch.from_packed(frames, pad_to=1)):
        data = batch.data.cpu().numpy()
        offs = batch.offsets.cpu().numpy().astype(np.uint64)
        lens = None if batch.lengths is None else batch.lengths.cpu().numpy().astype(np.uint32)
        want = oracle.slice_packed(data, offs, lens, flags=flags, ip_offset=ipo)
        got = engine.parse_to_numpy(batch, opt, ParseMode.Lenient, abi.OUT_SLICE)
        _cmp(got, want, f"lengths={lens is not None} flags={flags}")


@pytest.mark.parametrize("stride", [64, 128, 200])
def test_slice_strided(engine, oracle, frames, stride):
    rng = np.random.default_rng(stride)
    sel = [f for f in frames if len(f) <= stride][:8000]
    arr = rng.integers(0, 256, (len(sel), stride), dtype=np.uint8)
    for i, f in enumerate(sel):
        arr[i, :len(f)] = np.frombuffer(f, np.uint8)
    want = oracle.slice_packed(arr.reshape(-1), stride=stride)
    got = engine.parse_to_numpy(FrameBatch.from_strided(arr), out_kind=abi.OUT_SLICE)
    _cmp(got, want, f"stride={stride}")


def test_slice_goldens_on_gpu(engine, oracle):
    for v in helpers.golden()["frames"]:
        fr = bytes.fromhex(v["frame"])
        from nex_amd.frame import ParseOption
        opt = ParseOption(bool(v["parse_flags"] & abi.PARSE_FROM_IP), v["ip_offset"])
        got = engine.parse_to_numpy(FrameBatch.from_frames([fr]), opt, out_kind=abi.OUT_SLICE)[0]
        want = oracle.slice_frame(fr, v["parse_flags"] & abi.PARSE_FROM_IP, v["ip_offset"])
        assert got.tobytes() == want.tobytes(), v["name"]
