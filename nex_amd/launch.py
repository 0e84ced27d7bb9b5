"""bench.py's self-launch for `--gpus N > 1` (one process per GPU).

`python bench.py --gpus 8 ...` without torchrun's environment must not run one
rank and report `n_gpus: 1`. The parent process makes no GPU call at all: it
counts the visible devices in a throw-away child interpreter, starts
`python -m torch.distributed.run --nproc-per-node N bench.py <same args>` as a
fresh child process (never exec: a process that has touched the GPU must not
replace itself), relays the children's stdout line by line (rank 0 prints the
one JSON line) and exits with the child's exit code.

The reference's scale-out analogue is one receiver per queue in a
PACKET_FANOUT group (nex-datalink/src/linux.rs:154-193, lib.rs:119-131): the
shards never exchange data, so neither do the ranks here.

Nothing in this module imports torch; `decide` is a pure function of argv,
env and a device count so the CPU tests can check every branch.
"""
import os
import signal
import socket
import subprocess
import sys

#: env a rank of torch.distributed.run always has
RANK_ENV = ("WORLD_SIZE", "RANK", "LOCAL_RANK")


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def count_devices(python=sys.executable) -> int:
    """Visible GPUs, counted in a separate interpreter so this process never
    initialises the HIP runtime."""
    try:
        out = subprocess.run([python, "-c", "import torch; print(torch.cuda.device_count())"],
                             capture_output=True, text=True, timeout=600)
        return int(out.stdout.strip().splitlines()[-1])
    except (OSError, ValueError, IndexError, subprocess.TimeoutExpired):
        return 0


def decide(argv, env, gpus: int, n_devices=None, script="bench.py", python=sys.executable, port=None):
    """What `bench.py argv` does in this environment.

    Returns ("run", None) when this process is the bench itself (a rank under
    torchrun, or --gpus 1), ("spawn", cmd) with the torchrun command line to
    start as a child, or ("error", message). `n_devices` is a count or a
    callable returning one (only called when it matters).
    """
    in_rank = "WORLD_SIZE" in env
    if gpus < 1:
        return "error", f"--gpus {gpus}: need at least one rank"
    if in_rank:
        world = int(env["WORLD_SIZE"])
        # `torchrun --nproc-per-node 8 bench.py` (no --gpus): the launcher's
        # world is the rank count; only an explicit --gpus that disagrees is refused
        explicit = any(a == "--gpus" or a.startswith("--gpus=") for a in argv)
        if world != gpus and explicit:
            return "error", (f"WORLD_SIZE={world} but --gpus {gpus}: launch one rank per GPU "
                             f"(torch.distributed.run --nproc-per-node {gpus}) or drop the launcher "
                             "and let bench.py start the ranks itself")
        return "run", None
    if gpus == 1:
        return "run", None
    gloo = env.get("NEXG_DIST_BACKEND", "") == "gloo"
    if not gloo:
        n = n_devices() if callable(n_devices) else n_devices
        if n is None or n < gpus:
            return "error", (f"--gpus {gpus} but {n or 0} GPU(s) visible: one rank per GPU needs "
                             f"{gpus} devices (NEXG_DIST_BACKEND=gloo folds ranks onto fewer "
                             "devices for a rehearsal)")
    cmd = [python, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port or free_port()}", script] + list(argv)
    return "spawn", cmd


def child_env(env):
    """The ranks' environment: the caller's, with the dmabuf IPC mode RCCL
    needs on this host kept on."""
    e = dict(env)
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return e


def relay(cmd, env, out=None) -> int:
    """Run `cmd` as a child, copy its stdout through line by line (stderr is
    inherited), return its exit code. Non-zero as well when the ranks exited
    0 without rank 0 printing a JSON line."""
    out = out or sys.stdout
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, bufsize=1)
    # a SIGTERM / SIGINT to this process goes on to the launcher, which stops
    # its ranks (no orphaned ranks holding GPUs when a driver times the run out)
    forward = lambda sig, _frame: proc.send_signal(sig)
    old = {sig: signal.signal(sig, forward) for sig in (signal.SIGTERM, signal.SIGINT)}
    try:
        saw_json = False
        for line in proc.stdout:
            out.write(line)
            out.flush()
            saw_json |= line.lstrip().startswith("{")
        rc = proc.wait()
    finally:
        for sig, h in old.items():
            signal.signal(sig, h)
    if rc == 0 and not saw_json:
        print("bench launcher: the ranks exited 0 but rank 0 printed no result line", file=sys.stderr)
        return 1
    return rc


def main_or_spawn(argv, gpus: int, script: str):
    """bench.py's first step. Returns normally when this process should run
    the bench; otherwise runs the ranks (or reports the error) and exits."""
    action, what = decide(argv, os.environ, gpus, n_devices=count_devices, script=script)
    if action == "run":
        return
    if action == "error":
        print(f"bench.py: {what}", file=sys.stderr, flush=True)
        sys.exit(2)
    print(f"bench.py: --gpus {gpus}: starting {gpus} ranks: {' '.join(what)}", file=sys.stderr, flush=True)
    sys.exit(relay(what, child_env(os.environ)))
