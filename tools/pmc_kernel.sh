#!/usr/bin/env bash
# SQ counter passes (one rocprofv3 --pmc pass each) over the kernels matching a regex.
#   tools/pmc_kernel.sh <outdir> <kernel regex> <command...>   (GPU box, repo root)
set -eu
out=$1; re=$2; shift 2
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "$re" -d $out -o p$i --output-format csv -- "$@" > $out.p$i.log 2>&1
done
