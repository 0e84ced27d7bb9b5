#!/bin/bash
# Headline kernel (UDP64, grouped) and IMIX over batch sizes: is 16M
# representative, and what does IMIX run at when the batch fits the 256-MiB
# Infinity Cache (262144 frames = 93 MB) — the kernel's non-HBM floor.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/sweep
summ() { python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], sys.argv[3], r['kernel_ms'], r['frac'], flush=True)" "$@"; }
for n in 1048576 4194304 16777216 67108864 268435456; do
  timeout -k 10 200 python bench.py --frames $n --steps 20 --warmup 5 --no-cpu-baseline --no-imix > gpurun_out/sweep/udp64_$n.json 2> gpurun_out/sweep/udp64_$n.err || exit 1
  summ gpurun_out/sweep/udp64_$n.json udp64 $n
done
for n in 131072 262144 1048576 4194304 16777216 67108864; do
  timeout -k 10 200 python bench.py --workload imix --frames $n --steps 40 --no-cpu-baseline > gpurun_out/sweep/imix_$n.json 2> gpurun_out/sweep/imix_$n.err || exit 1
  summ gpurun_out/sweep/imix_$n.json imix $n
done
echo done
