# round-3 final evidence of the tree (MSD index sort, windowed join runs): -m gpu suite, smoke, bench line, kernel stats, PMC
# traffic of the headline, the N = 2 rehearsal
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03g
tools/gpu_steps.sh \
  "1000|r03g/pytest_gpu_all|python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -s" \
  "120|r03g/smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "300|r03g/bench|python3 bench.py" \
  "300|r03g/prof_bench|rocprofv3 --kernel-trace --stats -d gpurun_out/r03g/prof -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu" \
  "120|r03g/pmc_fetch|timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/r03g/pmc -o fetch --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extra" \
  "120|r03g/pmc_write|timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/r03g/pmc -o write --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extra" \
  "200|r03g/bench_n2|MQ_BENCH_BACKEND=gloo MQ_BENCH_ONE_DEVICE=1 python3 bench.py --gpus 2 --no-extra --no-cpu"
