# round-2 re-entry check of the current tree: -m gpu suite, smoke, bench line
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02b
tools/gpu_steps.sh \
  "900|r02b/pytest_gpu_all|python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -s" \
  "120|r02b/smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "300|r02b/bench|python3 bench.py"
