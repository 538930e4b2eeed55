# Alternating A/B/C... of libmq builds on the 2^28 joins: tools/join_abc.sh <tag> <lib B> [<lib C> ...]
# (A = the in-tree libmq.so), two rounds of unique + many-to-many; then the in-tree library's
# join parity subset.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; shift
mkdir -p gpurun_out/$T
steps=()
for r in 1 2; do
  steps+=("120|$T/A_u$r|python3 tools/join_bench.py 28" "120|$T/A_d$r|python3 tools/join_bench.py 28 dup")
  i=0
  for L in "$@"; do i=$((i+1))
    steps+=("120|$T/L${i}_u$r|MQ_LIB=$L python3 tools/join_bench.py 28" "120|$T/L${i}_d$r|MQ_LIB=$L python3 tools/join_bench.py 28 dup")
  done
done
tools/gpu_steps.sh "${steps[@]}" || exit $?
timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k 'join and (dup or partitioned or golden)' > gpurun_out/$T/pytest_join.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/$T/pytest_join.log
