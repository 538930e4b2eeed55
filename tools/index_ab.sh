# A/B of two libmq builds on the 1e9 index build, alternating on one box:
#   tools/index_ab.sh <tag> <lib B>   (A = the in-tree libmq.so); then B's kernel stats
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; LB=$2
mkdir -p gpurun_out/$T
tools/gpu_steps.sh \
  "120|$T/a1|python3 tools/index_bench.py 1000000000 5" \
  "120|$T/b1|MQ_LIB=$LB python3 tools/index_bench.py 1000000000 5" \
  "120|$T/a2|python3 tools/index_bench.py 1000000000 5" \
  "120|$T/b2|MQ_LIB=$LB python3 tools/index_bench.py 1000000000 5" \
  "150|$T/bprof|MQ_LIB=$LB rocprofv3 --kernel-trace --stats -d gpurun_out/$T/bix -o s --output-format csv -- python3 tools/index_bench.py 1000000000 3"
