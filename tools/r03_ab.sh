# round-3 GPU call AB: the counting finisher of the MSD index sort: parity, timing, size sweep
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "400|r03/pytest_isort11|python -u -m pytest tests/test_gpu_index.py -m gpu -x -v --timeout 200 --timeout-method thread -k 'wide_range or one_output or form_boundary'" \
  "200|r03/isort11_prof|rocprofv3 --kernel-trace --stats -d gpurun_out/r03/isortprof11 -o run --output-format csv -- python -u tools/index_bench.py 1000000000 2" \
  "400|r03/isort11_sweep|env SWEEP_N='1000000000' tools/index_sweep.sh"
