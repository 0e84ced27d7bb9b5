cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/sq
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d gpurun_out/sq/imix -o run -- python3 bench.py --workload imix --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/sq/imix.log 2>&1
echo rc=$?
