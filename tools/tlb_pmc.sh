#!/bin/bash
# Address-translation counters of the span kernel on the App. C mix built two
# ways (tools/kind_parse.py: workloads.tiled's one allocation filled in place,
# or round 4's repeat + cat), one rocprofv3 --pmc pass per counter set, plus a
# kernel-trace pass for the durations; 60 launches each (the first ~30 ms of
# a process run slower). Summary: tools/tlb_summary.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tlb
export TMPDIR=/tmp
for mode in new old; do
  flag=""; [ $mode = old ] && flag="--old-tiled"
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tlb/${mode}_trace -o run -- python3 tools/kind_parse.py --kind all --launches 60 $flag > gpurun_out/tlb/${mode}_trace.log 2>&1
  rc=$?; echo "$mode trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
  for set in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" \
             "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_HIT_sum" \
             "GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"; do
    tag=$(echo $set | cut -d' ' -f1 | tr 'A-Z' 'a-z')
    timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/tlb/${mode}_$tag -o run -- python3 tools/kind_parse.py --kind all --launches 60 $flag > gpurun_out/tlb/${mode}_$tag.log 2>&1
    rc=$?; echo "$mode $tag rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
echo done
