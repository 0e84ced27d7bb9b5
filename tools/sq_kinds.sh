#!/bin/bash
# SQ counters of the span kernel per App. C mutation kind (tools/kind_parse.py),
# one rocprofv3 pass of 8 SQ counters per kind. KINDS="clean ver_ihl ..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sqk
export TMPDIR=/tmp
for k in ${KINDS:-clean ver_ihl l4_length}; do
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
             "SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
    tag=$(echo $set | cut -d' ' -f1 | tr 'A-Z' 'a-z')
    timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/sqk/${k}_$tag -o run -- python3 tools/kind_parse.py --kind $k > gpurun_out/sqk/${k}_$tag.log 2>&1
    rc=$?; echo "$k $tag rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
echo done
