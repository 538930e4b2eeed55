# round-3 GPU call AH: the windowed runs build for duplicate keys: parity (all join paths), timing
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "600|r03/wr16b_pytest|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shards.py -m gpu -x -q --timeout 300 --timeout-method thread -k 'join'" \
  "300|r03/wr16b_bench|for r in 1 2 3; do for f in 1 0; do echo slot16=\$f; MQ_JOIN_SLOT16=\$f python -u tools/join_bench.py 28 dup || exit 1; done; done" \
  "200|r03/wr16b_prof|rocprofv3 --kernel-trace --stats -d gpurun_out/r03/wr16bprof -o run --output-format csv -- python -u tools/join_bench.py 28 dup"
