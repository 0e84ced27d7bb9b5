#!/bin/bash
# HBM traffic per launch from PMC counters (separate passes: FETCH_SIZE and
# WRITE_SIZE do not fit one pass on gfx950). See MI355X_MICROARCH.md §HBM.
# Pass directories are named <workload>.<output>_<COUNTER> for tools/pmc_summary.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
run() { local name=$1 secs=$2; shift 2
  timeout -s KILL "$secs" "$@" > "gpurun_out/pmc/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
CONFIGS=${CONFIGS:-"udp64.grouped imix.grouped imix_pcap.grouped malformed.grouped real_traffic.grouped udp64_large.grouped udp64.sparse imix.sparse udp64.desc ser.desc ser_probe.desc ser_aos.desc"}
for cfg in $CONFIGS; do
  wl=${cfg%.*}; out=${cfg#*.}; extra=""
  # ser = the full-tuple build, ser_probe = the udp_ping probe batch (bench.py --ser-shape)
  case $wl in ser) extra="--ser-shape tuples" ;; ser_probe) wl=ser; extra="--ser-shape probe" ;;
    ser_aos) wl=ser; extra="--ser-shape tuples_aos" ;;
    udp64_large) wl=udp64; extra="--frames $((52 << 20))" ;; esac
  for c in FETCH_SIZE WRITE_SIZE; do
    case $wl in
      ser_tcp_ping|ser_icmp_ping|ser_udp6)  # bench.py's ser.<shape> probe objects
        run ${cfg}_$c 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc/${cfg}_$c -o run -- python3 tools/probe_run.py --shape ${wl#ser_} ;;
      *)
        run ${cfg}_$c 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc/${cfg}_$c -o run -- python3 bench.py --workload $wl --out $out --steps 5 --warmup 1 --no-cpu-baseline --no-imix --no-malformed --no-real --no-large --no-ser $extra ;;
    esac
  done
done
echo done
