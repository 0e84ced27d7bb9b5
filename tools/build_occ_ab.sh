#!/bin/bash
# udp_ping builder: tile order (NEXG_BUILD_ORDER) x workgroups per CU capped by
# dynamic LDS (NEXG_BUILD_LDS_PAD beside the 16-KiB static tile: 6500 -> 7,
# 10500 -> 6, 16000 -> 5, 24000 -> 4 per CU), one bench process per setting,
# two rounds in opposite orders. Prints: order pad probe write_only_gbs / tuples
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/buildocc
S="${SETTINGS:-linear:24000 xcd:6500 xcd:10500 xcd:16000 xcd:24000 xcd4:24000 xcd16:24000 xcd:0}"
for rnd in 1 2; do
  if [ $rnd = 1 ]; then L="$S"; else L=$(echo $S | tr ' ' '\n' | tac | tr '\n' ' '); fi
  for c in $L; do
    o=${c%:*}; p=${c#*:}
    for shape in probe tuples; do
      NEXG_BUILD_ORDER=$o NEXG_BUILD_LDS_PAD=$p timeout -k 10 180 python bench.py --lib nex_amd/libnexg_knobs.so --workload ser --ser-shape $shape --steps 50 --warmup 25 \
        --no-cpu-baseline > gpurun_out/buildocc/${shape}_${o}_${p}_$rnd.json 2>/dev/null
      rc=$?; [ $rc -ne 0 ] && { echo "$c rc=$rc"; exit $rc; }
      python -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(sys.argv[2], sys.argv[3], sys.argv[4], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['stream_ceilings']['write_only_gbs'], flush=True)" gpurun_out/buildocc/${shape}_${o}_${p}_$rnd.json $o $p $shape
    done
  done
done
