cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tcp_options.py tests/test_gpu_sparse.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > gpurun_out/new_tests.log 2>&1
rc=$?; echo "new tests rc=$rc"; tail -5 gpurun_out/new_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
[ -f mutcheck/libnexg.so ] || { echo "no mutant library (build one with the one-TLV test perturbed into mutcheck/)"; exit 0; }
cp mutcheck/libnexg.so nex_amd/libnexg.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_tcp_options.py -x -q --timeout 300 --timeout-method thread -k "every_layout or fixed_stride" > gpurun_out/mutcheck.log 2>&1
echo "mutant rc=$? (expected 1: the perturbed one-TLV branch must fail)"; grep -m3 "AssertionError\|differ" gpurun_out/mutcheck.log
