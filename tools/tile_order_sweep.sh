#!/bin/bash
# Tile orders (NEXG_TILE_ORDER) over batch sizes, UDP64 and IMIX, and the GPU
# parity tests with the XCD order forced.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/order
NEXG_TILE_ORDER=xcd timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/order/pytest_xcd.log 2>&1 || exit 1
tail -1 gpurun_out/order/pytest_xcd.log
for n in 16777216 33554432 67108864; do
  for o in linear xcd; do
    NEXG_TILE_ORDER=$o timeout -k 10 200 python bench.py --lib nex_amd/libnexg_knobs.so --frames $n --steps 20 --warmup 5 --no-cpu-baseline --no-imix > gpurun_out/order/udp64_${o}_$n.json 2> gpurun_out/order/udp64_${o}_$n.err || exit 1
  done
done
for n in 4194304 16777216; do
  for o in linear xcd; do
    NEXG_TILE_ORDER=$o timeout -k 10 200 python bench.py --lib nex_amd/libnexg_knobs.so --workload imix --frames $n --steps 20 --no-cpu-baseline > gpurun_out/order/imix_${o}_$n.json 2> gpurun_out/order/imix_${o}_$n.err || exit 1
  done
done
echo done
