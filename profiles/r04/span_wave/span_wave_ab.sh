#!/bin/bash
# Span kernel A/B: workgroup sub-tiles (NEXG_SPAN_WAVE=0, 4 barriers per
# 20-KiB sub-tile) against wave-private spans (1, no barrier in the loop).
# One bench process per setting, alternated. Prints: setting imix malformed real.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/spanwave
for rnd in 1 2 3; do
  for w in 0 1; do
    NEXG_SPAN_WAVE=$w timeout -k 10 240 python bench.py --steps 40 --warmup 20 --no-cpu-baseline --no-large --no-ser \
      > gpurun_out/spanwave/${w}_$rnd.json 2>/dev/null
    rc=$?; [ $rc -ne 0 ] && { echo "$w rc=$rc"; exit $rc; }
    python - gpurun_out/spanwave/${w}_$rnd.json $w <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
f = lambda o: (o["roofline"]["kernel_ms"], o["roofline"]["frac"])
print(sys.argv[2], f(d["imix"]), f(d["malformed"]), f(d["real_traffic"]), flush=True)
PY
  done
done
