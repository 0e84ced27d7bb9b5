#!/bin/bash
# Tile order A/B for the span kernel (IMIX, malformed, real traffic) and the
# udp_ping builder: NEXG_TILE_ORDER / NEXG_BUILD_ORDER per setting, one bench
# process per setting, order of settings reversed in the second round.
# Prints: order imix malformed real ser.probe ser.tuples (roofline fractions).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tileorder2
ORDERS="${ORDERS:-linear xcd xcd2 xcd4 xcd8 xcd16}"
REV=$(echo $ORDERS | tr ' ' '\n' | tac | tr '\n' ' ')
for rnd in 1 2; do
  if [ $rnd = 1 ]; then L="$ORDERS"; else L="$REV"; fi
  for o in $L; do
    NEXG_TILE_ORDER=$o NEXG_BUILD_ORDER=$o timeout -k 10 240 python bench.py --lib nex_amd/libnexg_knobs.so --steps 40 --warmup 20 \
      --no-cpu-baseline --no-large > gpurun_out/tileorder2/${o}_$rnd.json 2>/dev/null
    rc=$?; [ $rc -ne 0 ] && { echo "$o rc=$rc"; exit $rc; }
    python - gpurun_out/tileorder2/${o}_$rnd.json $o <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
f = lambda o: o["roofline"]["frac"]
print(sys.argv[2], f(d), f(d["imix"]), f(d["malformed"]), f(d["real_traffic"]), f(d["ser"]), f(d["ser"]["tuples"]), flush=True)
EOF
  done
done
