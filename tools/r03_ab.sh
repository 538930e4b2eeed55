# round-3 GPU call AB: the counting finisher of the MSD index sort: parity, timing, size sweep
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "400|r03/pytest_isort2|python -u -m pytest tests/test_gpu_index.py -m gpu -x -v --timeout 200 --timeout-method thread -k 'wide_range or index_build_vs_oracle or 1e9_properties'" \
  "200|r03/isort2_prof|rocprofv3 --kernel-trace --stats -d gpurun_out/r03/isortprof2 -o run --output-format csv -- python -u tools/index_bench.py 1000000000 2" \
  "400|r03/isort2_sweep|tools/index_sweep.sh"
