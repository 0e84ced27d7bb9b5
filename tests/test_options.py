"""Option lists (nexg_options / nexg_decode_options):
Ipv4Header.options (ipv4.rs:442-508) and TcpHeader.options (tcp.rs:767-818)
decoded on the device as positions.

CPU: the oracle's lists against the reference's own option fixtures
(ipv4.rs:944-1020 NOP / RR(len 4, data 12 34) / EOL; tcp.rs:1276-1314
NOP, NOP, TS(0x2c57cda5, 0x02a04192)), against the host's independent walk
(frame.py) on a mutated corpus, and the struct layout against the C header.
GPU: the device decode == the oracle in every parse mode."""
import subprocess

import numpy as np
import pytest

from nex_amd import abi
from nex_amd.frame import (_ipv4_options, _tcp_options, frame_from_record, ipv4_options_at,
                           tcp_options_at)
from tests import helpers

MODES = [(0, 0), (abi.PARSE_STRICT, 0), (abi.PARSE_FROM_IP, 14), (abi.PARSE_FROM_IP | abi.PARSE_STRICT, 14)]


def _golden(name):
    for v in helpers.golden()["frames"]:
        if v["name"] == name:
            return v
    raise KeyError(name)


def test_reference_option_fixtures(oracle):
    v = _golden("ipv4_with_options")
    fr = bytes.fromhex(v["frame"])
    o = oracle.decode_options(fr, v["parse_flags"], v["ip_offset"])
    opts = ipv4_options_at(fr, int(o["ip_opt_off"]), o["ip_pos"][:o["n_ip"]])
    assert [x[2] for x in opts] == [1, 7, 0]  # NOP, RecordRoute, EOL
    assert opts[1][3] == 4 and opts[1][4] == bytes([0x12, 0x34])
    v = _golden("tcp_basic_parse")
    fr = bytes.fromhex(v["frame"])
    o = oracle.decode_options(fr, v["parse_flags"], v["ip_offset"])
    opts = tcp_options_at(fr, int(o["tcp_opt_off"]), o["tcp_pos"][:o["n_tcp"]])
    assert [x[0] for x in opts] == [1, 1, 8]  # NOP, NOP, Timestamp
    assert opts[2][1] == 10 and opts[2][2] == bytes.fromhex("2c57cda502a04192")


@pytest.fixture(scope="module")
def option_corpus(oracle):
    base = [bytes.fromhex(v["frame"]) for v in helpers.golden()["frames"]] + helpers.crafted_frames()
    with_opts = [f for f in base if len(f) > 34 and ((f[14] & 0xF) > 5 or len(f) > 54)]
    rng = np.random.default_rng(17)
    return base + helpers.mutate_frames(rng, with_opts or base, 6000)


@pytest.mark.parametrize("flags,ip_offset", MODES)
def test_oracle_lists_match_host_walk(oracle, option_corpus, flags, ip_offset):
    """Two restatements of the walks agree: the oracle's positions vs the
    host's own walk (frame.py) on every frame with an IPv4 / TCP header."""
    recs = oracle.parse_frames(option_corpus, flags, ip_offset)
    seen_ip = seen_tcp = 0
    for fr, rec in zip(option_corpus, recs):
        o = oracle.decode_options(fr, flags, ip_offset)
        f = int(rec["flags"])
        if abi.status_of(f):
            assert o["n_ip"] == 0 and o["n_tcp"] == 0
            continue
        assert int(o["n_ip"]) == (int(rec["ip_nopt"]) if f & abi.L_IPV4 else 0)
        assert int(o["n_tcp"]) == (int(rec["l4_nopt"]) if f & abi.L_TCP else 0)
        a = frame_from_record(rec, fr)
        b = frame_from_record(rec, fr, options=o)
        if f & abi.L_IPV4:
            assert b.ip.ipv4.options == a.ip.ipv4.options
            seen_ip += int(o["n_ip"]) > 0
        if f & abi.L_TCP:
            assert b.transport.tcp.options == a.transport.tcp.options
            seen_tcp += int(o["n_tcp"]) > 0
    assert seen_ip > 10 and seen_tcp > 10, (seen_ip, seen_tcp)


def test_options_layout_matches_c(tmp_path):
    from tests.test_abi import HDR
    names = ["n_ip", "n_tcp", "ip_opt_off", "tcp_opt_off", "reserved", "ip_pos", "tcp_pos", "pad"]
    src = tmp_path / "po.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "%s"\nint main(void){\n'
                   'printf("%%zu\\n", sizeof(nexg_options));\n%s\nreturn 0;}\n'
                   % (HDR, "\n".join(f'printf("%zu\\n", offsetof(nexg_options, {n}));' for n in names)))
    exe = tmp_path / "po"
    subprocess.check_call(["gcc", str(src), "-o", str(exe)])
    got = [int(x) for x in subprocess.check_output([str(exe)], text=True).split()]
    assert got == [abi.OPTIONS_DTYPE.itemsize] + [abi.OPTIONS_DTYPE.fields[n][1] for n in names]


@pytest.mark.gpu
@pytest.mark.parametrize("flags,ip_offset", MODES)
def test_decode_options_on_gpu(engine, oracle, option_corpus, flags, ip_offset):
    from nex_amd.engine import FrameBatch
    from nex_amd.frame import ParseMode, ParseOption
    import torch
    opt = ParseOption(bool(flags & abi.PARSE_FROM_IP), ip_offset)
    mode = ParseMode.Strict if flags & abi.PARSE_STRICT else ParseMode.Lenient
    for batch in (FrameBatch.from_frames(option_corpus, pad_to=4), FrameBatch.from_packed(option_corpus)):
        recs = engine.parse(batch, opt, mode, abi.OUT_RECORD)
        out = engine.decode_options(batch, recs)
        torch.cuda.synchronize()
        got = out.cpu().numpy()[: len(option_corpus) * 96].view(abi.OPTIONS_DTYPE)
        want = np.array([oracle.decode_options(f, flags, ip_offset) for f in option_corpus], abi.OPTIONS_DTYPE)
        helpers.records_equal(got, want, option_corpus, f"options flags={flags}")
