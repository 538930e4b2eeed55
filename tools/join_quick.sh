# Round-6 join iteration: the 2^28 joins' kernel stats, then a quick parity subset.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-r06c}
mkdir -p gpurun_out/$T
tools/gpu_steps.sh \
  "120|$T/jb_u_plain|python3 tools/join_bench.py 28" \
  "120|$T/jb_d_plain|python3 tools/join_bench.py 28 dup" \
  "150|$T/jb_u|rocprofv3 --kernel-trace --stats -d gpurun_out/$T/ju -o s --output-format csv -- python3 tools/join_bench.py 28" \
  "150|$T/jb_d|rocprofv3 --kernel-trace --stats -d gpurun_out/$T/jd -o s --output-format csv -- python3 tools/join_bench.py 28 dup" \
  "400|$T/pytest_join|python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k 'join and (dup or partitioned or golden)'"
