# Round-6 join work: the join parity tests, the shard joins, then the 2^28 joins' kernel stats.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-r06b}
mkdir -p gpurun_out/$T
tools/gpu_steps.sh \
  "150|$T/jb_u|rocprofv3 --kernel-trace --stats -d gpurun_out/$T/ju -o s --output-format csv -- python3 tools/join_bench.py 28" \
  "150|$T/jb_d|rocprofv3 --kernel-trace --stats -d gpurun_out/$T/jd -o s --output-format csv -- python3 tools/join_bench.py 28 dup" \
  "700|$T/pytest_join|python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k join" \
  "400|$T/pytest_pjoin|python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_pjoin.py"
