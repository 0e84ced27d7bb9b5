"""NEXG_OUT_VERDICT encoding (include/nexg.h): the 2-B verdict is lossless
for the flags word. Checked on the oracle's flags over golden, crafted and
mutated frames in every parse mode, with the encoder written here as the
kernel's store_result<NEXG_OUT_VERDICT> states it (no GPU)."""
import re
from pathlib import Path

import numpy as np

from nex_amd import abi
from tests import helpers

ROOT = Path(__file__).resolve().parents[1]


def encode(flags):
    flags = flags.astype(np.uint32)
    st = (flags >> abi.STATUS_SHIFT) & 7
    return np.where(st != 0, abi.VERDICT_ERR | (st << 3), flags & 0xFFFF).astype(np.uint16)


def test_header_constants_match():
    h = (ROOT / "include" / "nexg.h").read_text()
    assert int(re.search(r"#define NEXG_OUT_VERDICT (\d+)", h).group(1)) == abi.OUT_VERDICT
    assert "#define NEXG_VERDICT_ERR (NEXG_L_ARP | NEXG_L_IP)" in h
    assert abi.VERDICT_ERR == abi.L_ARP | abi.L_IP


def test_verdict_round_trip_on_oracle_flags(oracle):
    g = helpers.golden()
    base = [bytes.fromhex(v["frame"]) for v in g["frames"]] + helpers.crafted_frames()
    frames = base + helpers.mutate_frames(np.random.default_rng(5), base, 4000)
    seen_err = 0
    for flags in (0, abi.PARSE_STRICT, abi.PARSE_FROM_IP, abi.PARSE_FROM_IP | abi.PARSE_STRICT,
                  abi.PARSE_VLAN):
        f = oracle.parse_frames(frames, flags, 14)["flags"].astype(np.uint32)
        ok = (f >> abi.STATUS_SHIFT) == 0
        # the properties the encoding relies on
        assert ((f & 0x00FF0000) == 0).all()
        assert ((f[ok] & abi.VERDICT_ERR) != abi.VERDICT_ERR).all()
        assert ((f[~ok] & 0xFFFF) == 0).all()
        assert (abi.verdict_to_flags(encode(f)) == f).all(), flags
        seen_err += int((~ok).sum())
    assert seen_err > 0
    for st in (1, 2, 3, 4, 7):
        assert abi.verdict_to_flags(encode(np.array([st << abi.STATUS_SHIFT])))[0] == st << abi.STATUS_SHIFT
