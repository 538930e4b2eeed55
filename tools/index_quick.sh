# Round-6 index iteration: the index tests (all green, else stop), then the 1e9 build's
# time and kernel stats.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-r06ix}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_index.py > gpurun_out/$T/pytest_index.log 2>&1
rc=$?
tail -3 gpurun_out/$T/pytest_index.log
[ $rc -eq 0 ] || { echo "index tests rc=$rc: stopping"; exit $rc; }
tools/gpu_steps.sh \
  "150|$T/ix_plain|python3 tools/index_bench.py 1000000000 5" \
  "150|$T/ix|rocprofv3 --kernel-trace --stats -d gpurun_out/$T/ix -o s --output-format csv -- python3 tools/index_bench.py 1000000000 3"
