#!/bin/bash
# Counters of the span kernel on one batch held in 8 live allocations
# (tools/placement_ab.py --fresh 8: the first copies run slower than the later
# ones in one process): address translation, TCP->L2 read latency, L2 / DRAM
# request counters, one rocprofv3 --pmc pass per set. Summary:
# tools/fresh_summary.py (dispatches grouped per copy in launch order).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fresh_pmc
export TMPDIR=/tmp
# SET="<counters>" runs that one set only
sets=("TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum"
      "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_HIT_sum TCC_MISS_sum"
      "GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE")
[ -n "$SET" ] && sets=("$SET")
for set in "${sets[@]}"; do
  tag=$(echo $set | cut -d' ' -f1 | tr 'A-Z' 'a-z')
  timeout -s KILL 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/fresh_pmc/$tag -o run -- python3 tools/placement_ab.py --workload real --fresh 8 > gpurun_out/fresh_pmc/$tag.log 2>&1
  rc=$?; echo "$tag rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
echo done
