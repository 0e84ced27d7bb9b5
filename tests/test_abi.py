"""CPU: the C-ABI library loads and exports every symbol include/nexg.h
declares, and the Python struct mirrors match the C layout. No compute calls
(there is no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

from nex_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "nexg.h")
LIB = os.path.join(ROOT, "nex_amd", "libnexg.so")


def declared_functions():
    text = open(HDR).read()
    inline = set(re.findall(r"static inline [\w\s*]*?\b(nexg_[a-z0-9_]+)\s*\(", text))
    assert inline == set(abi.HEADER_INLINE)
    return sorted(set(re.findall(r"\b(nexg_[a-z0-9_]+)\s*\(", text)) - inline)


def test_header_declares_exported_list():
    assert declared_functions() == sorted(abi.EXPORTED_SYMBOLS)


@pytest.mark.skipif(not os.path.exists(LIB), reason="libnexg.so not built")
def test_library_exports_every_symbol():
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [s for s in declared_functions() if s not in exported]
    assert not missing, missing
    lib = ctypes.CDLL(LIB)
    for s in declared_functions():
        assert getattr(lib, s) is not None
    lib.nexg_abi_version.restype = ctypes.c_int
    assert lib.nexg_abi_version() == abi.ABI_VERSION


@pytest.mark.skipif(not os.path.exists(LIB), reason="libnexg.so not built")
def test_library_has_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", LIB], capture_output=True, text=True)
    assert ".hip_fatbin" in out.stdout
    blob = open(LIB, "rb").read()
    assert b"gfx950" in blob


def test_struct_layouts_match_c(tmp_path):
    """Compile a probe against include/nexg.h and compare sizes/offsets."""
    fields = abi.RECORD_DTYPE.names
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HDR}"', 'int main(void){',
             'printf("%zu %zu %zu %zu %zu\\n", sizeof(nexg_record), sizeof(nexg_desc), '
             'sizeof(nexg_frames), sizeof(nexg_parse_option), sizeof(nexg_udp4_build));']
    for f in fields:
        lines.append(f'printf("%zu\\n", offsetof(nexg_record, {f}));')
    for f, _ in abi.Udp4Build._fields_:
        lines.append(f'printf("%zu\\n", offsetof(nexg_udp4_build, {f}));')
    lines.append("return 0;}")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.check_call(["gcc", "-std=c11", "-o", str(exe), str(src)])
    out = subprocess.check_output([str(exe)], text=True).split()
    sizes = list(map(int, out[:5]))
    assert sizes == [64, 8, ctypes.sizeof(abi.Frames), ctypes.sizeof(abi.ParseOptionC),
                     ctypes.sizeof(abi.Udp4Build)]
    offs = list(map(int, out[5:5 + len(fields)]))
    assert offs == [abi.RECORD_DTYPE.fields[f][1] for f in fields]
    boffs = list(map(int, out[5 + len(fields):]))
    assert boffs == [getattr(abi.Udp4Build, f).offset for f, _ in abi.Udp4Build._fields_]


def test_udp6_build_layout_matches_c(tmp_path):
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HDR}"', 'int main(void){',
             'printf("%zu\\n", sizeof(nexg_udp6_build));']
    for f, _ in abi.Udp6Build._fields_:
        lines.append(f'printf("%zu\\n", offsetof(nexg_udp6_build, {f}));')
    lines.append("return 0;}")
    src = tmp_path / "probe6.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe6"
    subprocess.check_call(["gcc", "-std=c11", "-o", str(exe), str(src)])
    out = list(map(int, subprocess.check_output([str(exe)], text=True).split()))
    assert out[0] == ctypes.sizeof(abi.Udp6Build)
    assert out[1:] == [getattr(abi.Udp6Build, f).offset for f, _ in abi.Udp6Build._fields_]


def test_engine_refuses_without_library(monkeypatch, tmp_path):
    """The product path fails loudly when the HIP library is missing."""
    from nex_amd import _lib
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(_lib.NexgLibraryMissing):
        _lib.load()


def test_slice_layout_matches_c(tmp_path):
    names = abi.SLICE_DTYPE.names
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HDR}"', 'int main(void){',
             'printf("%zu\\n", sizeof(nexg_slice));']
    lines += [f'printf("%zu\\n", offsetof(nexg_slice, {f}));' for f in names]
    lines += [f'printf("%u\\n", (unsigned)({m}));' for m in
              ("NEXG_OUT_SLICE", "NEXG_S_DATALINK", "NEXG_S_NETWORK", "NEXG_S_TRANSPORT",
               "NEXG_S_ETHERTYPE", "NEXG_S_IP_PROTOCOL", "NEXG_S_PROTO_SHIFT")]
    lines.append("return 0;}")
    src = tmp_path / "probes.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probes"
    subprocess.check_call(["gcc", "-std=c11", "-o", str(exe), str(src)])
    out = list(map(int, subprocess.check_output([str(exe)], text=True).split()))
    assert out[0] == abi.SLICE_DTYPE.itemsize
    assert out[1:1 + len(names)] == [abi.SLICE_DTYPE.fields[f][1] for f in names]
    assert out[1 + len(names):] == [abi.OUT_SLICE, abi.S_DATALINK, abi.S_NETWORK, abi.S_TRANSPORT,
                                    abi.S_ETHERTYPE, abi.S_IP_PROTOCOL, abi.S_PROTO_SHIFT]


@pytest.mark.parametrize("cname,cls", [("nexg_ip_build", abi.IpBuild), ("nexg_tcp_build", abi.TcpBuild),
                                       ("nexg_icmp_echo_build", abi.IcmpEchoBuild)])
def test_l4_build_layouts_match_c(tmp_path, cname, cls):
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HDR}"', 'int main(void){',
             f'printf("%zu\\n", sizeof({cname}));']
    lines += [f'printf("%zu\\n", offsetof({cname}, {f}));' for f, _ in cls._fields_]
    lines.append("return 0;}")
    src = tmp_path / "probe_l4.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe_l4"
    subprocess.check_call(["gcc", "-std=c11", "-o", str(exe), str(src)])
    out = list(map(int, subprocess.check_output([str(exe)], text=True).split()))
    assert out[0] == ctypes.sizeof(cls)
    assert out[1:] == [getattr(cls, f).offset for f, _ in cls._fields_]


def test_error_contexts_match_header():
    """NEXG_CTX_* values and the context strings they name (include/nexg.h)
    are the table the Python / C++ host layers report ParseError with."""
    text = open(HDR).read()
    pairs = re.findall(r'NEXG_CTX_\w+ = (\d+),?\s*/\* "([^"]+)"', text)
    assert len(pairs) == len(abi.ERR_CONTEXTS) - 1
    for v, ctx in pairs:
        assert abi.ERR_CONTEXTS[int(v)] == ctx


def test_offsets32_table_roundtrip():
    """abi.offsets32_table / offsets32_decode (include/nexg.h
    NEXG_FRAMES_OFFSETS32): under 4 GiB the table is the low 32 bits alone;
    over 4 GiB the u64 group bases at the next 8-B boundary restore every
    offset, including groups that straddle a 4-GiB multiple."""
    import numpy as np
    from nex_amd import abi
    rng = np.random.default_rng(3)
    for count, start, data_bytes in ((1, 0, 100), (255, 7, 1 << 20), (256, 0, 1 << 20), (1000, 0, 1 << 20),
                                     (70_000, (1 << 32) - 3_000_000, 9 << 30)):
        lens = rng.integers(0, 1500, count, dtype=np.uint64)
        offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64) + np.uint64(start)
        t = abi.offsets32_table(offs, data_bytes)
        with_bases = data_bytes > 0xFFFFFFFF
        n, base_off, nb, total = abi.offsets32_layout(count, with_bases)
        assert len(t) == total and n == count + 1
        assert (t[: 4 * n].view(np.uint32) == (offs & np.uint64(0xFFFFFFFF))).all()
        if with_bases:
            assert base_off % 8 == 0 and nb == (count + 256) // 256
            assert int(offs[-1]) > (1 << 32) > int(offs[0])  # the case crosses 4 GiB
        assert (abi.offsets32_decode(t, count, data_bytes) == offs).all()
