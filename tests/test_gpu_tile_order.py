"""Tile order (tile_index, nex_amd/csrc/nexg_internal.hpp): which workgroup
handles which tile must never change a result. Each order is a permutation of
the tiles; a wrong one skips some frames and parses others twice.

- the default order (XCD-local runs of 16 tiles for fixed strides) on a
  mutated-frame batch with whole runs and a ragged tail, every record against
  the oracle;
- every order the env overrides of the measurement build
  (nex_amd/libnexg_knobs.so, -DNEXG_AB_KNOBS; the product library reads no
  environment) select (grid, contiguous eighths, runs of 3 / 8 / 16 / 64) in
  a child process per order: the parse outputs of fixed
  64-B and 96-B strides and of a packed IMIX batch (span kernel), and the
  udp_ping / udp6 / tcp_ping / icmp_ping builds, hashed and compared with
  the grid-order run."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from nex_amd import abi
from nex_amd.engine import FrameBatch
from tests import helpers

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KNOBS_LIB = os.path.join(ROOT, "nex_amd", "libnexg_knobs.so")

# 1172 64-B tiles: 1152 in whole groups of 8 x 16 (and of 8 x 3, 8 x 8), a 20-tile tail
N_FIXED = 1171 * 256 + 7
N_IMIX = 200_003

CHILD = r'''
import hashlib, json, sys
import torch
from nex_amd import _lib, abi
_lib.LIB_PATH = sys.argv[3]  # the -DNEXG_AB_KNOBS build: it reads the order overrides
from nex_amd.engine import Engine, FrameBatch
e = Engine(0)
h = {}
def put(name, t):
    torch.cuda.synchronize()
    h[name] = hashlib.sha256(t.cpu().numpy().tobytes()).hexdigest()
nf, ni = int(sys.argv[1]), int(sys.argv[2])
b = e.gen_batch(abi.WL_UDP64, nf, first_index=11)
for k in (abi.OUT_RECORD, abi.OUT_DESC, abi.OUT_GROUPED):
    put(f"udp64.{k}", e.parse(b, out_kind=k))
wide = torch.zeros((nf, 96), dtype=torch.uint8, device="cuda")
wide[:, :64] = b.data[: nf * 64].view(nf, 64)
wide[::5, 70] = 0x5A  # junk past some frames
put("stride96", e.parse(FrameBatch(data=wide.view(-1), count=nf, stride=96), out_kind=abi.OUT_RECORD))
im = e.gen_batch(abi.WL_IMIX, ni, first_index=5)
for k in (abi.OUT_RECORD, abi.OUT_GROUPED):
    put(f"imix.{k}", e.parse(im, out_kind=k))
p = e.gen_udp4_params(nf, first_index=3)
put("build.full", e.build_udp4(*p))
put("build.probe", e.build_udp4(None, p[1], def_src_ip=0x0A000001, def_src_port=40000, def_dst_port=33435))
put("build.tuples", e.build_udp4_tuples(e.pack_udp4_tuples(*p)))
g = torch.Generator(device="cuda").manual_seed(9)
rb = lambda *s: torch.randint(0, 256, s, dtype=torch.uint8, device="cuda", generator=g)
r16 = lambda: torch.randint(-32768, 32767, (nf,), dtype=torch.int16, device="cuda", generator=g)
a4s, a4d, a6s, a6d, sp, dp = rb(nf, 4), rb(nf, 4), rb(nf, 16), rb(nf, 16), r16(), r16()
seq = torch.randint(-2**31, 2**31 - 1, (nf,), dtype=torch.int32, device="cuda", generator=g)
opts = bytes.fromhex("020405b4040201010303 07".replace(" ", ""))
put("build.udp6", e.build_udp6(a6s, a6d, sp, dp))
put("build.tcp4", e.build_tcp(4, a4s, a4d, sp, dp, seq, None, flags=0x02, window=64240))
put("build.tcp4_opts", e.build_tcp(4, a4s, a4d, sp, dp, seq, None, flags=0x02, window=64240, options=opts))
put("build.tcp6", e.build_tcp(6, a6s, a6d, sp, dp, seq, None, flags=0x12, window=1024))
put("build.icmp4", e.build_icmp_echo(4, a4s, a4d, sp, dp))
put("build.icmp6", e.build_icmp_echo(6, a6s, a6d, sp, dp))
from nex_amd import probes  # the probe batches: k_build_probe (tcp_ping, udp6) and k_build_lane (icmp_ping)
for shape in ("tcp_ping", "udp6", "icmp_ping"):
    put("probe." + shape, probes.build(e, shape, a6d if probes.dst_bytes(shape) == 16 else a4d))
print(json.dumps(h))
'''


def run_child(order):
    env = dict(os.environ, NEXG_TILE_ORDER=order, NEXG_BUILD_ORDER=order, NEXG_L4_ORDER=order, NEXG_PROBE_ORDER=order)
    r = subprocess.run([sys.executable, "-c", CHILD, str(N_FIXED), str(N_IMIX), KNOBS_LIB], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_every_tile_order_gives_the_same_bytes():
    want = run_child("linear")
    for order in ("xcd", "xcd3", "xcd8", "xcd16", "xcd64", "cu1", "cu4"):
        got = run_child(order)
        diff = sorted(k for k in want if got[k] != want[k])
        assert not diff, (order, diff)


def test_default_order_mutated_fixed_stride(engine, oracle):
    """Default order at 64-B stride over 300k mutated frames (whole runs of
    16 tiles plus a tail): every record bit-exact against the oracle."""
    g = helpers.golden()
    base = ([bytes.fromhex(v["frame"]) for v in g["frames"]] + helpers.crafted_frames() +
            [oracle.gen_frame(abi.WL_IMIX, i) for i in range(60)])
    rng = np.random.default_rng(1172)
    sel = [f[:64] for f in helpers.mutate_frames(rng, base, N_FIXED)]
    arr = np.zeros((N_FIXED, 64), np.uint8)
    for i, f in enumerate(sel):
        arr[i, :len(f)] = np.frombuffer(f, np.uint8)
    full = [bytes(r) for r in arr]
    want = oracle.parse_frames(full)
    got = engine.parse_to_numpy(FrameBatch.from_strided(arr))
    helpers.records_equal(got, want, full, "default tile order, stride 64")
