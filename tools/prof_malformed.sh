#!/bin/bash
# rocprofv3 kernel trace of tools/bench_malformed.py (one library) per kind,
# then per-kernel durations by kind (tools/trace_by_kind.py).
# usage: KINDS=clean,all,ipv6_hbh bash tools/prof_malformed.sh [tag]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
tag=${1:-prof}
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag -o run -- python3 tools/bench_malformed.py --kinds ${KINDS:-clean,all} --steps 10 --warmup 5 > gpurun_out/$tag.log 2>&1
rc=$?; echo "prof rc=$rc"; grep -v amdgpu.ids gpurun_out/$tag.log
python3 tools/trace_by_kind.py gpurun_out/$tag/run_kernel_trace.csv ${KINDS:-clean,all} 15
