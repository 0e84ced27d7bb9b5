"""bench.py --gpus 2 on the GPU box: the self-launch (nex_amd/launch.py)
starts two ranks as a child torch.distributed.run (gloo, both ranks on the one
visible GPU: RCCL refuses two ranks per device) and relays rank 0's line,
which reports n_gpus 2 with every rank's kernel time. VERDICT r03 next 1."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_gpus2_self_launch():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(NEXG_DIST_BACKEND="gloo", OMP_NUM_THREADS="4")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--frames", str(1 << 20), "--no-imix", "--no-malformed", "--no-real", "--no-large", "--no-ser",
           "--no-cpu-baseline"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["frames_per_gpu"] == 1 << 20
    assert len(res["per_rank"]["kernel_ms"]) == 2 and all(k > 0 for k in res["per_rank"]["kernel_ms"])
    assert res["value"] > 0 and res["roofline"]["frac"] > 0
