#!/bin/bash
# HBM traffic per launch from PMC counters (separate passes: FETCH_SIZE and
# WRITE_SIZE do not fit one pass on gfx950). See MI355X_MICROARCH.md §HBM.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
run() { local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/pmc/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi; }
run list 120 rocprofv3 -L
for wl in udp64 imix ser; do
  for c in FETCH_SIZE WRITE_SIZE; do
    run ${wl}_$c 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc/${wl}_$c -o run -- python3 bench.py --workload $wl --steps 5 --warmup 1 --no-cpu-baseline
  done
done
echo done
