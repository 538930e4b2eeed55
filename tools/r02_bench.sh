# round-2 GPU evidence, part 2: bench line, kernel stats, PMC traffic passes
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02
tools/gpu_steps.sh \
  "300|r02/bench|python3 bench.py" \
  "300|r02/prof_bench|rocprofv3 --kernel-trace --stats -d gpurun_out/r02/prof -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu" \
  "120|r02/pmc_fetch|timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/r02/pmc -o fetch --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extra" \
  "120|r02/pmc_write|timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/r02/pmc -o write --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extra" \
  "120|r02/pmc_fetch_ss|timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/r02/pmc_ss -o fetch --output-format csv -- python3 tools/shared_prof.py 150 2" \
  "120|r02/pmc_write_ss|timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/r02/pmc_ss -o write --output-format csv -- python3 tools/shared_prof.py 150 2" \
  "120|r02/pmc_fetch_jd|timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/r02/pmc_jd -o fetch --output-format csv -- python3 tools/join_bench.py 28 dup" \
  "120|r02/pmc_write_jd|timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/r02/pmc_jd -o write --output-format csv -- python3 tools/join_bench.py 28 dup" \
  "200|r02/bench_n2|MQ_BENCH_BACKEND=gloo MQ_BENCH_ONE_DEVICE=1 python3 bench.py --gpus 2 --no-extra --no-cpu"
