#!/bin/bash
# One GPU session of named steps (each under its own time limit; a fault,
# abort or timeout ends the session). Usage: STEPS="kbench tests bench" bash tools/gpu_session.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/session.log
  tail -4 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc=$rc, stopping"; exit $rc; fi
  return 0
}
for s in ${STEPS:-tests}; do
  case $s in
    kbench) step kbench 300 ./tools/kbench ;;
    probetests) step pytest_probe 600 python -u -m pytest tests/test_gpu_probe_batches.py tests/test_gpu_build_l4.py tests/test_gpu_parity.py -k "probe or build or fixed_stride" -q -x --timeout 300 --timeout-method thread ;;
    probebench) step probe_bench 600 bash -c 'for r in 1 2; do python tools/bench_builders.py --probe || exit 1; python tools/bench_builders.py --probe --lib abvar/libnexg_noprobe.so || exit 1; NEXG_BUILD_LDS_PAD=0 python tools/bench_builders.py --probe --lib abvar/libnexg_noprobe.so || exit 1; done' ;;
    probewgs) step probe_wgs 900 bash -c 'for cfg in "0 def" "1 def" "1 0"; do set -- $cfg; export NEXG_PROBE_ICMP=$1; if [ $2 = 0 ]; then export NEXG_BUILD_LDS_PAD=0; fi; echo "cfg $cfg"; for l in nex_amd/libnexg.so abvar/libnexg_noprobe.so; do python tools/bench_builders.py --probe --lib $l || exit 1; done; done' ;;
       probetime) step probe_time 600 bash -c 'python -u tools/probe_timing.py --lib abvar/libnexg_ptime.so && NEXG_PROBE_WAVES=4 NEXG_PROBE_WGS=5 python -u tools/probe_timing.py --lib abvar/libnexg_ptime.so && python -u tools/probe_timing.py --lib abvar/libnexg_ptime_noprobe.so' ;;
    nodev) step nodev 600 bash -c 'for w in 1 4; do for l in nex_amd/libnexg.so abvar/libnexg_nodev.so; do NEXG_PROBE_WAVES=$w NEXG_PROBE_WGS=5 python tools/bench_builders.py --probe --lib $l || exit 1; done; done' ;;
    mixprobe) step mix_probe 400 python3 bench.py --steps 20 --warmup 5 --no-large --no-ser --no-cpu-baseline ;;
    headab) step head_ab 600 python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so,abvar/libnexg_headlate.so --workloads imix,mix,real --out grouped --check --rounds 4 ;;
    r04ab) step r04_ab 900 env NEXG_AB_LIB_LENIENT=1 python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so,abvar/libnexg_head.so,abvar/libnexg_r04.so --workloads imix,mix,real --out grouped --check --rounds 4 ;;
    sparseab) step sparse_ab 600 env NEXG_AB_LIB_LENIENT=1 python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so,abvar/libnexg_head.so --workloads mix --out sparse --check --rounds 4 ;;
    placement) step placement 600 bash -c 'python -u tools/placement_ab.py --workload real && python -u tools/placement_ab.py --workload mix --copies 4 && python -u tools/placement_ab.py --workload imix --copies 4' ;;
    counters) step counters 120 bash -c 'rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || rocprofv3 --list-avail > gpurun_out/rocprof_counters.txt 2>&1; true' ;;
    drift) step drift 600 bash -c 'python -u tools/placement_ab.py --workload mix --drift 8 && python -u tools/placement_ab.py --workload real --drift 6' ;;
    tlb) step tlb 900 bash tools/tlb_pmc.sh ;;
    stride) step stride 600 bash -c 'python -u tools/stride_probe.py && NEXG_AB_LIB_LENIENT=1 python -u tools/stride_probe.py --lib abvar/libnexg_head.so' ;;
    tstride) step template_stride 600 python -u tools/template_stride.py ;;
    fresh) step fresh 600 bash -c 'python -u tools/placement_ab.py --workload real --fresh 8' ;;
    reserve) step reserve 900 bash -c 'python -u tools/placement_ab.py --workload real --fresh 6 --reserve 32 && python -u tools/placement_ab.py --workload imix --fresh 6 && python -u tools/placement_ab.py --workload imix --fresh 6 --reserve 32' ;;
    freshpmc) step fresh_pmc 1000 bash tools/fresh_pmc.sh ;;
    subab4) step sub_ab4 700 python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so,abvar/libnexg_sub20480w5.so,abvar/libnexg_sub16384w5.so,abvar/libnexg_sub20480.so --workloads imix,mix,real --out grouped --check --rounds 3 ;;
    pmcspan) step pmc_span 1100 env CONFIGS="imix.grouped imix_pcap.grouped malformed.grouped real_traffic.grouped imix.sparse" bash tools/pmc.sh ;;
    spantests) step pytest_span 600 python -u -m pytest tests/test_gpu_span.py -q -x --timeout 300 --timeout-method thread ;;
    contigvmm) step contig_vmm 700 bash -c 'python -u tools/contig_ab.py --workload real --vmm 8' ;;
    freshtcp) step fresh_tcp 1100 bash -c 'SET="TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum TD_TD_BUSY_sum" bash tools/fresh_pmc.sh && SET="TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_THRASHING_STALL_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum TA_TA_BUSY_sum" bash tools/fresh_pmc.sh' ;;
    freshsq) step fresh_sq 1100 bash -c 'SET="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" bash tools/fresh_pmc.sh && SET="SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD" bash tools/fresh_pmc.sh' ;;
    boundsab) step bounds_ab 700 python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so,abvar/libnexg_lanebounds.so --workloads imix,mix,real --out grouped --check --rounds 4 ;;
    phasesab) step phases_ab 600 python -u tools/span_phases_ab.py --libs nex_amd/libnexg.so,abvar/libnexg_sub24w4.so ;;
    subab3) step sub_ab3 600 python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so,abvar/libnexg_sub28672.so,abvar/libnexg_sub24w4.so --workloads imix,mix,real --out grouped --check --rounds 3 ;;
    subab2) step sub_ab2 600 bash -c 'python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so,abvar/libnexg_sub20480.so --workloads imix,real --out desc --check --rounds 3 && python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so,abvar/libnexg_sub20480.so --workloads imix,mix,real --out grouped --check --rounds 3' ;;
    subab) step sub_ab 600 python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so,abvar/libnexg_sub24576.so,abvar/libnexg_sub16384.so --workloads imix,mix,real --out grouped --check --rounds 4 ;;
    contigclk) step contig_clk 600 bash -c 'python -u tools/contig_ab.py --workload real --map 12 --clock' ;;
    contiglat) step contig_lat 600 bash -c 'python -u tools/contig_ab.py --workload real --map 12 --latency' ;;
    contigout) step contig_out 600 bash -c 'python -u tools/contig_ab.py --workload real --map 12 --outs flags,desc,sparse,fresh_grouped' ;;
    contignt) step contig_nt 600 bash -c 'python -u tools/contig_ab.py --workload real --map 16 --libs abvar/libnexg_sub20480.so' ;;
    contigspan) step contig_span 600 bash -c 'python -u tools/contig_ab.py --workload real --map 24' ;;
    contigsub) step contig_sub 600 bash -c 'python -u tools/contig_ab.py --workload real --map 24 --libs abvar/libnexg_sub20480.so,abvar/libnexg_sub28672.so' ;;
    contigmap) step contig_map 600 bash -c 'python -u tools/contig_ab.py --workload real --map 32' ;;
    contig) step contig 600 bash -c 'python -u tools/contig_ab.py --workload real --copies 4 && python -u tools/contig_ab.py --workload imix --copies 3' ;;
    icmpab) step icmp_ab 600 bash -c 'python tools/bench_builders.py --probe && NEXG_PROBE_ICMP=1 python tools/bench_builders.py --probe && NEXG_PROBE_ICMP=1 NEXG_PROBE_WAVES=8 python tools/bench_builders.py --probe && NEXG_PROBE_ICMP=1 NEXG_PROBE_WAVES=8 NEXG_PROBE_WGS=3 python tools/bench_builders.py --probe && NEXG_PROBE_ICMP=1 NEXG_PROBE_WAVES=8 NEXG_PROBE_WGS=0 python tools/bench_builders.py --probe' ;;
    spanorder) step span_order 1000 bash -c 'for o in linear xcd xcd2 xcd8; do echo "order $o"; NEXG_TILE_ORDER=$o python -u tools/placement_ab.py --workload real --fresh 4 || exit 1; done' ;;
    freshpmc2) step fresh_pmc 1000 env SET="TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_GMI_CREDIT_STALL_sum TCC_EA0_RDREQ_IO_CREDIT_STALL_sum TCC_EA0_RDREQ_LEVEL_sum" bash tools/fresh_pmc.sh ;;
    serab) step ser_ab 300 python -u tools/bench_ser_ab.py --libs nex_amd/libnexg.so,abvar/libnexg_noprobe.so --shape probe --rounds 4 ;;
    descab) step desc_ab 600 python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so,abvar/libnexg_desc1.so,abvar/libnexg_desc0.so --workloads udp64,imix --out desc --rounds 3 ;;
    newtests) step pytest_new 600 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_fixup.py -q -x --timeout 300 --timeout-method thread ;;
    tests) step pytest_gpu 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench_udp64 500 python bench.py --steps 50 --cpu-seconds 5 ;;
    driverbench) step bench_driver 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 ;;
    malformedtests) step pytest_malformed 600 python -u -m pytest tests/test_gpu_malformed.py tests/test_gpu_span.py -q -x --timeout 300 --timeout-method thread ;;
    newtests4) step pytest_new4 600 python -u -m pytest tests/test_gpu_launch.py tests/test_gpu_tcp_options.py tests/test_gpu_build_probe.py "tests/test_gpu_parity.py::test_build_udp4_tuples_aos" tests/test_cpp_api.py -q -x --timeout 300 --timeout-method thread ;;
    malformed) step bench_malformed 500 python tools/bench_malformed.py ;;
    benchpcap) step bench_pcap 400 python bench.py --workload imix_pcap --steps 20 --cpu-seconds 5 ;;
    ser) step bench_ser 300 python bench.py --workload ser --steps 50 --no-cpu-baseline
         step bench_ser_tuples 300 python bench.py --workload ser --ser-shape tuples --steps 50 --no-cpu-baseline
         step bench_ser_aos 300 python bench.py --workload ser --ser-shape tuples_aos --steps 50 --no-cpu-baseline ;;
    e2e) step bench_e2e 400 python bench.py --e2e --steps 5 --warmup 2 --no-cpu-baseline
         step bench_e2e_imix 400 python bench.py --e2e --workload imix --steps 3 --warmup 1 --no-cpu-baseline ;;
    # bench.py --gpus N starts its own N ranks (nex_amd/launch.py); gloo folds them onto the one GPU
    rehearse2) step rehearse2 600 env NEXG_DIST_BACKEND=gloo python bench.py --gpus 2 --steps 20 --warmup 5 --cpu-seconds 2 ;;
    rehearse8) step rehearse8 900 env NEXG_DIST_BACKEND=gloo python bench.py --gpus 8 --steps 10 --warmup 3 --cpu-seconds 2 --no-large ;;
    benchimix) step bench_imix 400 python bench.py --workload imix --steps 20 --warmup 3 --cpu-seconds 5 ;;
    pmc) step pmc 900 bash tools/pmc.sh ;;
    sqkinds) step sqkinds 900 bash tools/sq_kinds.sh ;;
    tileorder) step tileorder 900 bash tools/tile_order_ab.sh ;;
    tileorder2) step tileorder2 1000 bash tools/tile_order_ab2.sh ;;
    orderbench) step orderbench 300 ./tools/orderbench
                step orderbench52 300 ./tools/orderbench 54525952 ;;
    buildocc) step buildocc 900 bash tools/build_occ_ab.sh ;;
    spantiming) step spantiming 300 python -u tools/span_timing.py abvar/libnexg_timing.so ;;
    builders) step builders_tests 600 python -u -m pytest tests/test_gpu_build_l4.py tests/test_gpu_build_probe.py tests/test_gpu_parity.py -k "build or udp_ping or probe" -q -x --timeout 300 --timeout-method thread
              step builders_ab 600 bash -c 'for r in 1 2; do NEXG_BUILD_LDS_PAD=0 python tools/bench_builders.py || exit 1; python tools/bench_builders.py || exit 1; done' ;;
    buildorder) step builders_tests 600 python -u -m pytest tests/test_gpu_build_l4.py tests/test_gpu_tile_order.py tests/test_gpu_parity.py -k "build or udp_ping or probe or order" -q -x --timeout 300 --timeout-method thread
                step builders_order_ab 600 bash -c 'for r in 1 2 3; do python tools/bench_builders.py || exit 1; done' ;;
    sizesweep) step sizesweep 900 bash tools/size_sweep.sh ;;
    tileorder3) step tileorder3 900 bash tools/tile_order_ab3.sh ;;
    ordertests) step ordertests 600 python -u -m pytest tests/test_gpu_tile_order.py -x -v --timeout 300 --timeout-method thread ;;
    abser) step ab_ser 300 python -u tools/bench_ser_ab.py --libs ${LIBS} --shape ${SHAPE:-tuples} --rounds 4 ;;
    # in-process A/B of library variants under abvar/ (LIBS=a,b,...): IMIX with an output check, then the mixes
    abspan) step ab_imix 600 python -u tools/bench_parse_ab.py --libs ${LIBS} --workloads imix,udp64 --out grouped --check --rounds 4
            step ab_mixes 600 python -u tools/bench_malformed.py --libs ${LIBS} --kinds ${KINDS:-clean,all,tcp_ts} --out grouped ;;
    lanetests) step pytest_lane 600 python -u -m pytest tests/test_gpu_probe_batches.py tests/test_gpu_build_l4.py tests/test_gpu_tile_order.py tests/test_gpu_build_probe.py -q -x --timeout 300 --timeout-method thread ;;
    laneab) step lane_ab 900 bash -c 'for r in 1 2; do for cfg in "" "NEXG_PROBE_ICMP=2" "NEXG_PROBE_ICMP=1" "NEXG_PROBE_LANE_TCP=1" "NEXG_PROBE_WGS=3" "NEXG_PROBE_WGS=4" "NEXG_PROBE_WGS=8" "NEXG_PROBE_WGS=0"; do env $cfg python tools/bench_builders.py --probe || exit 1; done; done' ;;
    laneab2) step lane_ab2 900 bash -c 'for r in 1 2; do for cfg in "" "NEXG_PROBE_ICMP=2" "NEXG_LANE_WGS=3" "NEXG_LANE_WGS=5" "NEXG_LANE_WGS=6" "NEXG_PROBE_LANE_TCP=1" "NEXG_PROBE_LANE_TCP=1 NEXG_LANE_WGS=5"; do env $cfg python tools/bench_builders.py --probe || exit 1; done; done' ;;
    o32tests) step pytest_o32 600 python -u -m pytest tests/test_gpu_span.py tests/test_gpu_grouped.py tests/test_gpu_sparse.py tests/test_gpu_fixup.py -q -x --timeout 300 --timeout-method thread ;;
    o32ab) step o32_ab 900 python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so --tables 64,32 --workloads imix,mix,real --out grouped --check --rounds 4 ;;
    depthab) step depth_ab 1100 python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so,abx/libnexg_d2w4.so,abx/libnexg_d2w4s16.so,abx/libnexg_d2w4s20.so,abx/libnexg_d1w4.so --workloads imix,mix,real --out grouped --check --rounds 3 ;;
    mixkinds) step mix_kinds 900 python -u tools/bench_malformed.py --libs nex_amd/libnexg.so,abx/libnexg_d1w4.so --kinds clean,truncate,pad,ip_length,ver_ihl,l4_length,ipv6_hbh,vlan,proto200,random --out grouped
              step mix_phases 600 python -u tools/span_phases_ab.py --libs nex_amd/libnexg.so,abx/libnexg_d1w4.so --workloads imix,mix ;;
    slotab) step slot_ab 1100 python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so,abx/libnexg_s96w5.so,abx/libnexg_s96w4.so,abx/libnexg_s128w4.so,abx/libnexg_d1w4.so --workloads imix,mix,real --out grouped --check --rounds 3
            step slot_kinds 900 python -u tools/bench_malformed.py --libs nex_amd/libnexg.so,abx/libnexg_s96w5.so,abx/libnexg_s128w4.so,abx/libnexg_d1w4.so --kinds clean,ver_ihl,l4_length,ipv6_hbh,truncate,pad --out grouped ;;
    cuorder) step cu_order 1100 bash -c 'for o in cu1 cu4 cu16; do echo "order $o"; NEXG_TILE_ORDER=$o python -u tools/contig_ab.py --workload real --map 10 --libs nex_amd/libnexg_knobs.so || exit 1; done' ;;
    spanorder2) step span_order2 1100 bash -c 'for o in xcd32 xcd64 xcd128 xcd16; do echo "order $o"; NEXG_TILE_ORDER=$o python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so,nex_amd/libnexg_knobs.so --workloads imix,mix,real --out grouped --check --rounds 3 || exit 1; done' ;;
    orderconfirm) step order_confirm 900 bash -c 'NEXG_TILE_ORDER=linear python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so,nex_amd/libnexg_knobs.so --workloads imix,mix,real --out grouped --check --rounds 4 && python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so --tables 64,32 --workloads imix,mix,real --out grouped --check --rounds 3' ;;
    subab64) step sub_ab64 1100 python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so,abx/libnexg_s20.so,abx/libnexg_s16.so,abx/libnexg_w4.so,abx/libnexg_s28w4.so --workloads imix,mix,real --out grouped --check --rounds 3 ;;
    pfab) step pf_ab 1100 python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so,abx/libnexg_pf40.so,abx/libnexg_pf160.so,abx/libnexg_pf320.so,abx/libnexg_pf640.so --workloads imix,mix,real --out grouped --check --rounds 3 ;;
    buildorder2) step build_order2 1100 bash -c 'for o in xcd xcd16 xcd64 cu1; do echo "order $o"; NEXG_BUILD_ORDER=$o python -u tools/bench_ser_ab.py --libs nex_amd/libnexg.so,nex_amd/libnexg_knobs.so --shape probe --rounds 3 || exit 1; NEXG_BUILD_ORDER=$o NEXG_L4_ORDER=$o python -u tools/bench_builders.py --probe || exit 1; done; python -u tools/bench_builders.py --probe --lib nex_amd/libnexg.so' ;;
    shortab) step short_ab 1100 python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so,abx/libnexg_noshort.so --workloads imix,mix,real --out grouped --check --rounds 4
             step short_kinds 900 python -u tools/bench_malformed.py --libs nex_amd/libnexg.so,abx/libnexg_noshort.so --kinds clean,ver_ihl,l4_length,ipv6_hbh --out grouped ;;
    w6ab) step w6_ab 900 python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so,abx/libnexg_s20w6.so,abx/libnexg_s16w6.so --workloads imix,mix,real --out grouped --check --rounds 3 ;;
    udptests) step pytest_udp 600 python -u -m pytest tests/test_gpu_probe_batches.py tests/test_gpu_parity.py tests/test_gpu_fixup.py tests/test_gpu_tile_order.py -q -x --timeout 300 --timeout-method thread ;;
    udpab) step udp_ab 900 bash -c 'for r in 1 2; do for cfg in "" "NEXG_LANE_WGS=4" "NEXG_LANE_WGS=5" "NEXG_LANE_WGS=2"; do env $cfg python tools/bench_builders.py --probe || exit 1; done; done' ;;
    realkinds) step real_kinds 900 python -u tools/bench_malformed.py --libs nex_amd/libnexg.so --kinds clean,tcp_ts,tcp_sack,tcp_mss --share 0.7 --out grouped ;;
    pmc32) mkdir -p gpurun_out/pmc32 && export TMPDIR=/tmp && for c in FETCH_SIZE WRITE_SIZE; do for t in 64 32; do
        step pmc32_${t}_$c 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc32/t${t}_$c -o run -- python3 tools/bench_parse_ab.py --libs nex_amd/libnexg.so --tables $t --workloads imix --out grouped --rounds 1 --steps 5 --warmup 1 || exit 1; done; done ;;
    realout) for o in grouped verdict desc; do step real_out_$o 600 python -u tools/bench_malformed.py --kinds clean,tcp_ts,clean,tcp_ts --share 0.7 --out $o; done ;;
    padab) step pad_ab 900 python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so,abx/libnexg_pad1.so,abx/libnexg_pad2.so --workloads real,mix,imix --out grouped --rounds 3 &&
        step pad_kinds 900 python -u tools/bench_malformed.py --libs nex_amd/libnexg.so,abx/libnexg_pad1.so,abx/libnexg_pad2.so --kinds clean,tcp_ts,truncate,pad,ver_ihl --out grouped ;;
    excab) step exc_ab 900 python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so,abx/libnexg_skip.so,abx/libnexg_e9.so --workloads real,mix,imix --out grouped --rounds 3 && step exc_kinds 900 python -u tools/bench_malformed.py --libs nex_amd/libnexg.so,abx/libnexg_skip.so,abx/libnexg_e9.so --kinds clean,tcp_ts --share 0.7 --out grouped ;;
    codeab) step code_ab 900 python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so,abx/libnexg_p7.so,abx/libnexg_p1.so,abx/libnexg_p2.so,abx/libnexg_p3.so,abx/libnexg_p4.so,abx/libnexg_p5.so,abx/libnexg_p6.so --workloads imix,real --out grouped --rounds 3 ;;
    tpwab) step tpw_ab 900 python -u tools/bench_parse_ab.py --libs abx/libnexg_t1.so,abx/libnexg_t2.so,abx/libnexg_t1s.so,abx/libnexg_t2s.so --workloads imix,real --out grouped --rounds 3 ;;
    codeat) step code_at 900 python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so,abx/libnexg_at1.so,abx/libnexg_at2.so,abx/libnexg_at3.so --workloads imix,real --out grouped --rounds 3 ;;
    runtests) step pytest_run 900 python -u -m pytest tests/test_gpu_grouped.py tests/test_gpu_malformed.py tests/test_gpu_span.py tests/test_gpu_tcp_options.py tests/test_gpu_clocks.py tests/test_gpu_tile_order.py tests/test_gpu_parity.py tests/test_cpp_api.py -q -x --timeout 300 --timeout-method thread ;;
    offnt) step offnt_ab 900 python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so,abx/libnexg_vote.so --tables 32 --workloads imix,imix --out grouped --check --rounds 4 &&
        step offnt_ab2 900 python -u tools/bench_parse_ab.py --libs nex_amd/libnexg.so,abx/libnexg_vote.so --workloads real,mix --out grouped --check --rounds 4 ;;
    driverbench2) step bench_driver_2 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 && step bench_driver_3 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 ;;
    # the driver's own command under the kernel trace: a row for every object of its line (tools/line_trace.py)
    lineprof) step lineprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lineprof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 ;;
    prof) step prof_udp64 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_udp64 -o run -- python3 bench.py --steps 60 --warmup 25 --no-cpu-baseline --no-imix --no-malformed --no-real --no-large --no-ser
          step prof_pcap 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pcap -o run -- python3 bench.py --workload imix_pcap --steps 60 --warmup 25 --no-cpu-baseline
          step prof_imix 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_imix -o run -- python3 bench.py --workload imix --steps 60 --warmup 25 --no-cpu-baseline
          step prof_malformed 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_malformed -o run -- python3 bench.py --workload malformed --steps 60 --warmup 25 --no-cpu-baseline
          step prof_real 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_real -o run -- python3 bench.py --workload real_traffic --steps 60 --warmup 25 --no-cpu-baseline
          step prof_large 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_large -o run -- python3 bench.py --frames 54525952 --steps 60 --warmup 25 --no-cpu-baseline --no-imix
          step prof_ser 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ser -o run -- python3 bench.py --workload ser --steps 60 --warmup 25 --no-cpu-baseline
          step prof_ser_tuples 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ser_tuples -o run -- python3 bench.py --workload ser --ser-shape tuples --steps 60 --warmup 25 --no-cpu-baseline
          step prof_ser_aos 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ser_aos -o run -- python3 bench.py --workload ser --ser-shape tuples_aos --steps 60 --warmup 25 --no-cpu-baseline ;;
  esac
done
echo done
