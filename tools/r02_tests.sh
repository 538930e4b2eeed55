# round-2 GPU evidence, part 1: the whole -m gpu suite (incl. big) and smoke
set -u
mkdir -p gpurun_out/r02
tools/gpu_steps.sh \
  "1000|r02/pytest_gpu_all|python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -s" \
  "120|r02/smoke|python -c 'import __graft_entry__ as g; g.smoke()'"
