export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_grouped.py tests/test_gpu_sparse.py tests/test_gpu_malformed.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_grouped.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/pt_grouped.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for o in grouped sparse; do timeout -k 10 400 python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so --out $o --workloads udp64,imix --rounds 3 >> gpurun_out/ab_grouped.log 2>&1; echo ab rc=$?; done; done
grep -v amdgpu.ids gpurun_out/ab_grouped.log
