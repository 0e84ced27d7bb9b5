#!/bin/bash
# Named GPU test files under one time limit: FILES="tests/a.py tests/b.py" bash tools/gpu_quick_tests.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 ${SECS:-600} python -u -m pytest ${FILES:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/quick_tests.log; exit $rc
