# A/B of the in-tree libmq against <lib B> on the 2^28 joins and the 1e9 index build,
# alternating on one box, then the join parity subset and the index tests (in-tree lib).
#   tools/hist_ab.sh <tag> <lib B>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; LB=$2
mkdir -p gpurun_out/$T
tools/gpu_steps.sh \
  "120|$T/A_ix1|python3 tools/index_bench.py 1000000000 5" \
  "120|$T/B_ix1|MQ_LIB=$LB python3 tools/index_bench.py 1000000000 5" \
  "120|$T/A_ix2|python3 tools/index_bench.py 1000000000 5" \
  "120|$T/B_ix2|MQ_LIB=$LB python3 tools/index_bench.py 1000000000 5" || exit $?
timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_index.py > gpurun_out/$T/pytest_index.log 2>&1
echo "index pytest rc=$?"; tail -1 gpurun_out/$T/pytest_index.log
exec bash tools/join_abc.sh $T $LB
