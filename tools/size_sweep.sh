#!/bin/bash
# Headline kernel (UDP64 desc) and IMIX over batch sizes: is 16M representative?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/sweep
for n in 1048576 4194304 16777216 67108864 268435456; do
  timeout -k 10 200 python bench.py --frames $n --steps 20 --warmup 5 --no-cpu-baseline --no-imix > gpurun_out/sweep/udp64_$n.json 2> gpurun_out/sweep/udp64_$n.err || exit 1
done
for n in 1048576 4194304 16777216 67108864; do
  timeout -k 10 200 python bench.py --workload imix --frames $n --steps 10 --no-cpu-baseline > gpurun_out/sweep/imix_$n.json 2> gpurun_out/sweep/imix_$n.err || exit 1
done
echo done
