#!/bin/bash
# udp_ping builder tile order A/B (NEXG_BUILD_ORDER), one bench process per
# setting, order of settings reversed in the second round. The write-only
# ceiling probe follows the same order. Prints: order udp64 probe
# write_ceiling_gbs tuples tuples_aos (roofline fractions).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tileorder3
ORDERS="${ORDERS:-linear xcd xcd16 xcd32 xcd64}"
REV=$(echo $ORDERS | tr ' ' '\n' | tac | tr '\n' ' ')
for rnd in 1 2; do
  if [ $rnd = 1 ]; then L="$ORDERS"; else L="$REV"; fi
  for o in $L; do
    NEXG_BUILD_ORDER=$o timeout -k 10 180 python bench.py --lib nex_amd/libnexg_knobs.so --steps 50 --warmup 25 --no-cpu-baseline \
      --no-imix --no-malformed --no-real --no-large > gpurun_out/tileorder3/${o}_$rnd.json 2>/dev/null
    rc=$?; [ $rc -ne 0 ] && { echo "$o rc=$rc"; exit $rc; }
    python - gpurun_out/tileorder3/${o}_$rnd.json $o <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
s = d["ser"]
f = lambda o: o["roofline"]["frac"]
print(sys.argv[2], f(d), f(s), s["roofline"]["stream_ceilings"]["write_only_gbs"], f(s["tuples"]),
      f(s["tuples_aos"]), flush=True)
EOF
  done
done
