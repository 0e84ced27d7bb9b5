#!/bin/bash
# Capture-file ingest, in-place (raw) shape: parallel preads + parallel record
# walk over reader thread counts, IMIX and UDP64; packed shape for reference.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/ingest && export TMPDIR=/tmp
for wl in imix udp64; do
  for cfg in "packed 1" "raw 1" "raw 4" "raw 8" "raw 16"; do
    set -- $cfg
    timeout -k 10 200 python tools/bench_ingest.py --workload $wl --shape $1 --threads $2 \
      > gpurun_out/ingest/${wl}_$1_t$2.json 2> gpurun_out/ingest/${wl}_$1_t$2.err || exit 1
    echo "$wl $1 t$2: $(python3 -c "import json;d=json.load(open('gpurun_out/ingest/${wl}_$1_t$2.json'));print(d['value'], d['gib_s'], d['reader_busy_s'])")"
  done
done
echo done
