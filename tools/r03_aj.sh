# round-3 GPU call AJ: windowed runs build with the coalesced run-array copy: parity, timing, SQ counters
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "600|r03/wc_pytest|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k 'dup or join_vs or clustered'" \
  "300|r03/wc_bench|for r in 1 2 3; do python -u tools/join_bench.py 28 dup || exit 1; done" \
  "200|r03/wc_prof|rocprofv3 --kernel-trace --stats -d gpurun_out/r03/wcprof -o run --output-format csv -- python -u tools/join_bench.py 28 dup" \
  "300|r03/wc_pmc|tools/pmc_kernel.sh gpurun_out/r03/pmc_winruns2 'k_win_build_runs|k_join_write_runs_mlp' python -u tools/join_bench.py 28 dup"
