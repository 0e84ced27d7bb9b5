#!/bin/bash
# UDP64 headline kernel by tile order (NEXG_TILE_ORDER), 16M and 52M frames,
# grouped output, one process per setting, order of settings alternated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tileorder
for rnd in 1 2; do
  if [ $rnd = 1 ]; then L="${ORDERS:-linear xcd8 xcd16 xcd32}"; else L=$(echo ${ORDERS:-linear xcd8 xcd16 xcd32} | tr " " "\n" | tac | tr "\n" " "); fi
  for o in $L; do
    for f in 16777216 54525952; do
      NEXG_TILE_ORDER=$o timeout -k 10 120 python bench.py --lib nex_amd/libnexg_knobs.so --frames $f --steps 50 --warmup 25 --no-cpu-baseline --no-imix > gpurun_out/tileorder/${o}_${f}_$rnd.json 2>/dev/null
      rc=$?; [ $rc -ne 0 ] && { echo "$o $f rc=$rc"; exit $rc; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['roofline']['kernel_ms'], d['roofline']['frac'])" gpurun_out/tileorder/${o}_${f}_$rnd.json $o $f
    done
  done
done
