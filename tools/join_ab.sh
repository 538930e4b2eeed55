# A/B of two libmq builds on the 2^28 joins (unique, many-to-many), alternating on one box:
#   tools/join_ab.sh <tag> <lib B> [pmc]  (A = the in-tree libmq.so); then B's kernel stats,
#   and with "pmc" B's FETCH_SIZE / WRITE_SIZE per kernel
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; LB=$2
mkdir -p gpurun_out/$T
tools/gpu_steps.sh \
  "120|$T/au1|python3 tools/join_bench.py 28" \
  "120|$T/bu1|MQ_LIB=$LB python3 tools/join_bench.py 28" \
  "120|$T/ad1|python3 tools/join_bench.py 28 dup" \
  "120|$T/bd1|MQ_LIB=$LB python3 tools/join_bench.py 28 dup" \
  "120|$T/au2|python3 tools/join_bench.py 28" \
  "120|$T/bu2|MQ_LIB=$LB python3 tools/join_bench.py 28" \
  "120|$T/ad2|python3 tools/join_bench.py 28 dup" \
  "120|$T/bd2|MQ_LIB=$LB python3 tools/join_bench.py 28 dup" \
  "150|$T/bprof_u|MQ_LIB=$LB rocprofv3 --kernel-trace --stats -d gpurun_out/$T/bju -o s --output-format csv -- python3 tools/join_bench.py 28" \
  "150|$T/bprof_d|MQ_LIB=$LB rocprofv3 --kernel-trace --stats -d gpurun_out/$T/bjd -o s --output-format csv -- python3 tools/join_bench.py 28 dup" || exit $?
if [ "$3" = pmc ]; then
tools/gpu_steps.sh \
  "90|$T/fetch_ju|MQ_LIB=$LB timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/$T/ju -o fetch --output-format csv -- python3 tools/join_bench.py 28" \
  "90|$T/write_ju|MQ_LIB=$LB timeout -s KILL 80 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/$T/ju -o write --output-format csv -- python3 tools/join_bench.py 28" \
  "90|$T/fetch_jd|MQ_LIB=$LB timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/$T/jd -o fetch --output-format csv -- python3 tools/join_bench.py 28 dup" \
  "90|$T/write_jd|MQ_LIB=$LB timeout -s KILL 80 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/$T/jd -o write --output-format csv -- python3 tools/join_bench.py 28 dup"
fi
