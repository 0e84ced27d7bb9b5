#!/bin/bash
# UDP64 headline kernel with its workgroups per CU capped by dynamic LDS
# (NEXG_TILE_LDS_PAD: 0 -> 6 per CU from its VGPRs, 12000 -> 5, 20000 -> 4,
# 33000 -> 3), 16M and 52M frames, settings' order reversed in a second round.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tilelds
for rnd in 1 2; do
  if [ $rnd = 1 ]; then L="0 12000 20000 33000"; else L="33000 20000 12000 0"; fi
  for p in $L; do
    for f in 16777216 54525952; do
      NEXG_TILE_LDS_PAD=$p timeout -k 10 120 python bench.py --frames $f --steps 50 --warmup 25 --no-cpu-baseline --no-imix > gpurun_out/tilelds/${p}_${f}_$rnd.json 2>/dev/null
      rc=$?; [ $rc -ne 0 ] && { echo "$p $f rc=$rc"; exit $rc; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['roofline']['kernel_ms'], d['roofline']['frac'], flush=True)" gpurun_out/tilelds/${p}_${f}_$rnd.json $p $f
    done
  done
done
