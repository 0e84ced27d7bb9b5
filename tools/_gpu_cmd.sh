export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_grouped.py tests/test_gpu_malformed.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_grouped.log 2>&1; rc=$?; echo pytest rc=$rc; tail -2 gpurun_out/pt_grouped.log; [ $rc -ne 0 ] && exit $rc
for o in sparse grouped; do timeout -k 10 500 python -u tools/bench_malformed.py --out $o --kinds clean,l4_length,ipv6_hbh,truncate,all > gpurun_out/mal_$o.log 2>&1; echo $o rc=$?; grep -v amdgpu.ids gpurun_out/mal_$o.log | cut -c1-110; done
