"""The C++ host API (include/nexg.hpp: nexg::Engine, Frame, ParseOption,
ParseMode, ParseError, frame_from_record) under the reference's own unit-test
assertions (tests/native/cpp_frame_test.cpp), in the reference's words:
CPU mode materialises Frames from oracle records (the C++ reading of
records), GPU mode runs Engine::try_from_bufs on the device."""
import json
import os
import subprocess

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")
EXE = os.path.join(HERE, "cpp_frame_test")
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_vectors.json")


def _fixture(tmp_path):
    g = json.load(open(GOLDEN))
    p = tmp_path / "fixtures.txt"
    p.write_text("".join(f"{v['name']} {v['parse_flags']} {v['ip_offset']} {v['frame']}\n" for v in g["frames"]))
    return str(p)


def test_cpp_api_cpu(tmp_path):
    subprocess.check_call(["make", "-s", "-C", HERE, "cpp_frame_test"])
    r = subprocess.run([EXE, "--cpu", _fixture(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout


@pytest.mark.gpu
def test_cpp_api_gpu(tmp_path):
    assert os.path.exists(EXE), "build tests/native first (__graft_entry__.build())"
    r = subprocess.run([EXE, "--gpu", _fixture(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "gpu:" in r.stdout and "0 failures" in r.stdout
