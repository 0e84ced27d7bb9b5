export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_abi.py -k "build_udp4 or abi" -q --timeout 120 --timeout-method thread > gpurun_out/pt_build.log 2>&1; echo pytest rc=$?; tail -3 gpurun_out/pt_build.log
STEPS="ser" bash tools/gpu_session.sh || exit 1
timeout -k 10 500 python -u tools/bench_malformed.py --libs abtmp/libnexg_base.so,abtmp/libnexg_pf1.so,abtmp/libnexg_pf2.so --kinds clean,all > gpurun_out/ab_pf.log 2>&1; echo ab rc=$?; grep -v amdgpu.ids gpurun_out/ab_pf.log | tail -12
