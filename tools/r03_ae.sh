# round-3 GPU call AE: counting-finisher shapes (MQ_ISORT_FIN 1/2/3), 1e9 rows, alternating
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "200|r03/fin_pytest|env MQ_ISORT_FIN=2 python -u -m pytest tests/test_gpu_index.py -m gpu -x -q --timeout 200 --timeout-method thread -k 'wide_range'" \
  "200|r03/fin_pytest3|env MQ_ISORT_FIN=3 python -u -m pytest tests/test_gpu_index.py -m gpu -x -q --timeout 200 --timeout-method thread -k 'wide_range'" \
  "300|r03/fin_ab|for r in 1 2; do for f in 1 2 3; do echo fin=\$f; MQ_ISORT_FIN=\$f python -u tools/index_bench.py 1000000000 5 || exit 1; done; done" \
  "200|r03/fin_prof|env MQ_ISORT_FIN=2 rocprofv3 --kernel-trace --stats -d gpurun_out/r03/finprof -o run --output-format csv -- python -u tools/index_bench.py 1000000000 2"
