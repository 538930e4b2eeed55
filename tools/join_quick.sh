# Round-6 join iteration: the 2^28 joins' kernel stats, then a quick parity subset.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-r06c}
mkdir -p gpurun_out/$T
tools/gpu_steps.sh \
  "120|$T/jb_u_plain|python3 tools/join_bench.py 28" \
  "120|$T/jb_d_plain|python3 tools/join_bench.py 28 dup" \
  "150|$T/jb_u|rocprofv3 --kernel-trace --stats -d gpurun_out/$T/ju -o s --output-format csv -- python3 tools/join_bench.py 28" \
  "150|$T/jb_d|rocprofv3 --kernel-trace --stats -d gpurun_out/$T/jd -o s --output-format csv -- python3 tools/join_bench.py 28 dup" \
  "400|$T/pytest_join|python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k 'join and (dup or partitioned or golden)'" || exit 1
if [ -n "$2" ]; then  # read/write bytes per kernel as well
tools/gpu_steps.sh \
  "90|$T/fetch_ju|timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/$T/ju -o fetch --output-format csv -- python3 tools/join_bench.py 28" \
  "90|$T/write_ju|timeout -s KILL 80 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/$T/ju -o write --output-format csv -- python3 tools/join_bench.py 28" \
  "90|$T/fetch_jd|timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/$T/jd -o fetch --output-format csv -- python3 tools/join_bench.py 28 dup" \
  "90|$T/write_jd|timeout -s KILL 80 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/$T/jd -o write --output-format csv -- python3 tools/join_bench.py 28 dup"
fi
