# SQ counters (two passes) of the 2^28 joins' partition, window and gather kernels:
#   tools/sq_join.sh <tag> [dup]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; D=$2
mkdir -p gpurun_out/$T
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
SQ2="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH"
tools/gpu_steps.sh \
  "90|$T/sq1|timeout -s KILL 80 rocprofv3 --pmc $SQ1 --kernel-include-regex 'k_win|k_pwin' -d gpurun_out/$T/sq -o sq1 --output-format csv -- python3 tools/join_bench.py 28 $D" \
  "90|$T/sq2|timeout -s KILL 80 rocprofv3 --pmc $SQ2 --kernel-include-regex 'k_win|k_pwin' -d gpurun_out/$T/sq -o sq2 --output-format csv -- python3 tools/join_bench.py 28 $D"
