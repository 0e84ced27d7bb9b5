#!/bin/bash
# GPU tests, then an in-process A/B of a baseline library build against the
# tree's (tools/bench_malformed.py --libs), then the default bench line.
# usage: BASE=abtmp/libnexg_base.so KINDS=clean,all,tcp_ts bash tools/gpu_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$BASE" ]; then
  timeout -k 10 600 python -u tools/bench_malformed.py --libs $BASE,nex_amd/libnexg.so --kinds ${KINDS:-clean,all} > gpurun_out/ab.log 2>&1
  rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab.log | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 600 python -u bench.py --steps 50 --cpu-seconds 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; exit $rc
fi
