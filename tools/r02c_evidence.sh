# round-2 final evidence of the tree: -m gpu suite, smoke, bench line, kernel stats,
# PMC traffic (headline and CSV parse), the N = 2 rehearsal
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02c
tools/gpu_steps.sh \
  "900|r02c/pytest_gpu_all|python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -s" \
  "120|r02c/smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "300|r02c/bench|python3 bench.py" \
  "300|r02c/prof_bench|rocprofv3 --kernel-trace --stats -d gpurun_out/r02c/prof -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu" \
  "120|r02c/pmc_fetch|timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/r02c/pmc -o fetch --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extra" \
  "120|r02c/pmc_write|timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/r02c/pmc -o write --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extra" \
  "120|r02c/pmc_fetch_csv|timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --kernel-trace --kernel-include-regex k_csv -d gpurun_out/r02c/pmc_csv -o fetch --output-format csv -- python3 tools/load_bench.py 100000000 4 1" \
  "120|r02c/pmc_write_csv|timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --kernel-trace --kernel-include-regex k_csv -d gpurun_out/r02c/pmc_csv -o write --output-format csv -- python3 tools/load_bench.py 100000000 4 1" \
  "200|r02c/bench_n2|MQ_BENCH_BACKEND=gloo MQ_BENCH_ONE_DEVICE=1 python3 bench.py --gpus 2 --no-extra --no-cpu"
