# round-3 GPU call AA: the MSD + LDS-finisher index sort (mq_isort.hip): parity, 1e9 timing vs the 4-pass LSD
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "300|r03/pytest_isort|python -u -m pytest tests/test_gpu_index.py -m gpu -x -v --timeout 200 --timeout-method thread -k 'wide_range or index_build_vs_oracle or 1e9_properties'" \
  "120|r03/isort_msd|python -u tools/index_bench.py 1000000000 5" \
  "120|r03/isort_lsd4|env MQ_INDEX_SORT=lsd4 python -u tools/index_bench.py 1000000000 5" \
  "200|r03/isort_prof|rocprofv3 --kernel-trace --stats -d gpurun_out/r03/isortprof -o run --output-format csv -- python -u tools/index_bench.py 1000000000 2"
tools/gpu_steps.sh \
  "200|r03/isort_prof_lsd4|env MQ_INDEX_SORT=lsd4 rocprofv3 --kernel-trace --stats -d gpurun_out/r03/isortprof4 -o run --output-format csv -- python -u tools/index_bench.py 1000000000 2"
