#!/usr/bin/env bash
# SQ counter passes over k_csv_parse (load path), one rocprofv3 --pmc pass each.
#   tools/pmc_csv.sh <outdir> [libmq path]   (run on the GPU box from the repo root)
set -eu
out=$1; lib=${2:-}
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH"; do
  i=$((i+1))
  MQ_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex k_csv_parse -d $out -o p$i --output-format csv -- python3 tools/load_bench.py 100000000 4 1 > $out.p$i.log 2>&1
done
