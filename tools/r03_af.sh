# round-3 GPU call AF: the many-to-many write with more run reads in flight: parity, A/B
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "400|r03/jw_pytest|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k 'dup or join_vs'" \
  "300|r03/jw_ab|for r in 1 2 3; do for f in 8 4 1; do echo write=\$f; MQ_JOIN_WRITE=\$f python -u tools/join_bench.py 28 dup || exit 1; done; done" \
  "200|r03/jw_prof|rocprofv3 --kernel-trace --stats -d gpurun_out/r03/jwprof -o run --output-format csv -- python -u tools/join_bench.py 28 dup"
