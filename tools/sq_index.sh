# SQ counters (two passes) and HBM bytes of the 1e9 index build's counting finisher:
#   tools/sq_index.sh <tag> [lib]   (lib: another libmq through MQ_LIB)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; L=${2:-}
mkdir -p gpurun_out/$T
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
SQ2="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH"
P="--kernel-include-regex finish_count"
tools/gpu_steps.sh \
  "90|$T/sq1|MQ_LIB=$L timeout -s KILL 80 rocprofv3 --pmc $SQ1 $P -d gpurun_out/$T/sq -o sq1 --output-format csv -- python3 tools/index_bench.py 1000000000 2" \
  "90|$T/sq2|MQ_LIB=$L timeout -s KILL 80 rocprofv3 --pmc $SQ2 $P -d gpurun_out/$T/sq -o sq2 --output-format csv -- python3 tools/index_bench.py 1000000000 2" \
  "90|$T/fetch|MQ_LIB=$L timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE $P -d gpurun_out/$T/sq -o fetch --output-format csv -- python3 tools/index_bench.py 1000000000 2" \
  "90|$T/write|MQ_LIB=$L timeout -s KILL 80 rocprofv3 --pmc WRITE_SIZE $P -d gpurun_out/$T/sq -o write --output-format csv -- python3 tools/index_bench.py 1000000000 2"
