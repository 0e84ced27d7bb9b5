#!/bin/bash
# Capture-file ingest rate (tools/bench_ingest.py) over reader thread counts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/ingest && export TMPDIR=/tmp
for wl in imix udp64; do
  for t in 1 2 4 8; do
    timeout -k 10 150 python tools/bench_ingest.py --workload $wl --shape packed --threads $t \
      > gpurun_out/ingest/${wl}_packed_t$t.json 2> gpurun_out/ingest/${wl}_packed_t$t.err || exit 1
  done
done
echo done
