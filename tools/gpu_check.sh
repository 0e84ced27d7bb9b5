#!/bin/bash
# One GPU session: smoke, GPU parity tests, benches, rocprofv3 kernel trace.
# Every GPU step has its own time limit; a fault/abort/timeout ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/session.log
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc, stopping"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-all}
rocminfo 2>/dev/null | grep -m1 -E "gfx9" > gpurun_out/arch.txt
if [[ $STEPS == *smoke* || $STEPS == all ]]; then
  step smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $STEPS == *pytest* || $STEPS == all ]]; then
  step pytest_gpu 900 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread
fi
if [[ $STEPS == *bench* || $STEPS == all ]]; then
  step bench_udp64 400 python bench.py --steps 50 --warmup 5 --cpu-seconds 5
  step bench_imix 400 python bench.py --workload imix --steps 20 --warmup 3 --cpu-seconds 5
  step bench_ser 300 python bench.py --workload ser --steps 50 --warmup 5 --no-cpu-baseline
  step bench_udp64_record 300 python bench.py --out record --steps 20 --warmup 3 --no-cpu-baseline
  step bench_imix_record 300 python bench.py --workload imix --out record --steps 10 --warmup 2 --no-cpu-baseline
fi
if [[ $STEPS == *prof* || $STEPS == all ]]; then
  step prof_udp64 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_udp64 -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline
  step prof_imix 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_imix -o run -- python3 bench.py --workload imix --steps 10 --warmup 2 --no-cpu-baseline
  step prof_ser 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ser -o run -- python3 bench.py --workload ser --steps 20 --warmup 2 --no-cpu-baseline
fi
echo done
