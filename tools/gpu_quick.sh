#!/bin/bash
# Short GPU session: GPU tests, default bench (UDP64 + IMIX lines), flags output, kbench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping at $name rc=$rc"; exit $rc; fi
}
step pytest_gpu 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
step bench_default 400 python bench.py
step bench_flags 300 python bench.py --out flags --no-cpu-baseline
[ -x tools/kbench ] && step kbench 200 ./tools/kbench
echo done
