"""bench.py's self-launch (nex_amd/launch.py): `python bench.py --gpus N`
outside torchrun starts N ranks as a child process and relays rank 0's line;
it never runs one rank and reports n_gpus 1. CPU only: the decision is a pure
function, and the spawn leg runs torch.distributed.run over a stub script."""
import io
import os
import subprocess
import sys

from nex_amd import launch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_launcher_imports_no_torch():
    code = "import sys; from nex_amd import launch; assert 'torch' not in sys.modules, 'torch imported'"
    subprocess.run([sys.executable, "-c", code], cwd=ROOT, check=True)


def test_one_gpu_runs_in_process():
    assert launch.decide(["--steps", "5"], {}, 1, n_devices=lambda: 1 / 0) == ("run", None)


def test_rank_under_torchrun_runs():
    env = {"WORLD_SIZE": "8", "RANK": "3", "LOCAL_RANK": "3"}
    assert launch.decide(["--gpus", "8"], env, 8, n_devices=lambda: 1 / 0) == ("run", None)


def test_rank_world_mismatch_is_an_error():
    action, msg = launch.decide(["--gpus", "8"], {"WORLD_SIZE": "1"}, 8)
    assert action == "error" and "WORLD_SIZE=1" in msg
    action, msg = launch.decide(["--gpus=2"], {"WORLD_SIZE": "8"}, 2)
    assert action == "error" and "WORLD_SIZE=8" in msg


def test_torchrun_without_gpus_takes_world_size():
    """`torchrun --nproc-per-node 8 bench.py` with --gpus left at its default:
    the ranks run (world size from the launcher), no refusal."""
    env = {"WORLD_SIZE": "8", "RANK": "0", "LOCAL_RANK": "0"}
    assert launch.decide(["--steps", "5"], env, 1, n_devices=lambda: 1 / 0) == ("run", None)


def test_spawn_command():
    argv = ["--gpus", "8", "--steps", "20", "--warmup", "5"]
    action, cmd = launch.decide(argv, {}, 8, n_devices=8, script="/x/bench.py", python="py", port=29999)
    assert action == "spawn"
    assert cmd == ["py", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
                   "--master-addr=127.0.0.1", "--master-port=29999", "/x/bench.py"] + argv


def test_too_few_devices_is_an_error():
    for n in (0, 1, 7):
        action, msg = launch.decide(["--gpus", "8"], {}, 8, n_devices=n)
        assert action == "error" and f"{n} GPU(s) visible" in msg


def test_gloo_rehearsal_folds_ranks_without_counting():
    action, cmd = launch.decide(["--gpus", "2"], {"NEXG_DIST_BACKEND": "gloo"}, 2,
                                n_devices=lambda: 1 / 0, port=1)
    assert action == "spawn" and "--nproc-per-node=2" in cmd


def test_zero_gpus_is_an_error():
    assert launch.decide([], {}, 0)[0] == "error"


def test_relay_passes_line_and_exit_code():
    buf = io.StringIO()
    rc = launch.relay([sys.executable, "-c", "print('{\"value\": 1}')"], dict(os.environ), out=buf)
    assert rc == 0 and buf.getvalue().strip() == '{"value": 1}'
    rc = launch.relay([sys.executable, "-c", "import sys; sys.exit(3)"], dict(os.environ), out=io.StringIO())
    assert rc == 3
    # exit 0 without a result line is a failure, not a silent empty record
    rc = launch.relay([sys.executable, "-c", "print('hello')"], dict(os.environ), out=io.StringIO())
    assert rc == 1


STUB = r'''
import json, os, sys
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
import torch.distributed as dist
dist.init_process_group("gloo")
t = [None] * world
dist.all_gather_object(t, rank)
if rank == 0:
    print(json.dumps({"n_gpus": world, "ranks": t, "argv": sys.argv[1:]}), flush=True)
dist.destroy_process_group()
'''


def test_spawned_ranks_report_world(tmp_path):
    """The spawn leg end to end: torch.distributed.run starts 2 gloo ranks of
    a stub with bench.py's argv; the parent relays rank 0's line."""
    stub = tmp_path / "stub.py"
    stub.write_text(STUB)
    argv = ["--gpus", "2", "--steps", "3"]
    action, cmd = launch.decide(argv, {"NEXG_DIST_BACKEND": "gloo"}, 2, script=str(stub))
    assert action == "spawn"
    buf = io.StringIO()
    env = launch.child_env(dict(os.environ, NEXG_DIST_BACKEND="gloo", OMP_NUM_THREADS="1"))
    for k in launch.RANK_ENV:
        env.pop(k, None)
    rc = launch.relay(cmd, env, out=buf)
    assert rc == 0, buf.getvalue()
    import json
    line = [ln for ln in buf.getvalue().splitlines() if ln.startswith("{")]
    assert len(line) == 1
    res = json.loads(line[0])
    assert res["n_gpus"] == 2 and res["ranks"] == [0, 1] and res["argv"] == argv


def test_bench_refuses_gpus_without_devices():
    """bench.py --gpus 2 in this GPU-less container: exits non-zero with a
    message, prints no result line."""
    env = {k: v for k, v in os.environ.items() if k not in launch.RANK_ENV + ("NEXG_DIST_BACKEND",)}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 2, r.stderr
    assert "GPU(s) visible" in r.stderr and "{" not in r.stdout


def test_relay_forwards_sigterm(tmp_path):
    """A SIGTERM to the launcher reaches the child (torch.distributed.run
    stops its ranks on it): the child sees it and exits with its own code."""
    child = tmp_path / "child.py"
    child.write_text("import signal, sys, time\n"
                     "signal.signal(signal.SIGTERM, lambda *a: (print('got term', flush=True), sys.exit(7)))\n"
                     "print('ready', flush=True)\n"
                     "time.sleep(60)\n")
    parent = tmp_path / "parent.py"
    parent.write_text("import os, sys\n"
                      f"sys.path.insert(0, {ROOT!r})\n"
                      "from nex_amd import launch\n"
                      f"sys.exit(launch.relay([sys.executable, {str(child)!r}], dict(os.environ)))\n")
    import signal
    import time
    p = subprocess.Popen([sys.executable, str(parent)], stdout=subprocess.PIPE, text=True)
    assert p.stdout.readline().strip() == "ready"
    time.sleep(0.2)
    p.send_signal(signal.SIGTERM)
    rest = p.stdout.read()
    assert p.wait(timeout=30) == 7 and "got term" in rest
