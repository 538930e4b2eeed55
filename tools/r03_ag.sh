# round-3 GPU call AG: per-word run lengths summed by the many-to-many probe (k_runs_count gone)
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "400|r03/jp_pytest|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shards.py -m gpu -x -q --timeout 300 --timeout-method thread -k 'join and not 2e28'" \
  "300|r03/jp_bench|for r in 1 2 3; do python -u tools/join_bench.py 28 dup || exit 1; python -u tools/join_bench.py 28 || exit 1; done" \
  "200|r03/jp_prof|rocprofv3 --kernel-trace --stats -d gpurun_out/r03/jpprof -o run --output-format csv -- python -u tools/join_bench.py 28 dup"
