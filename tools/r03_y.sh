# round-3 GPU call Y: exact index, doubling with 8 entries in flight per lane; walk limits
set -u
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "400|r03/pytest_index9|python -u -m pytest tests/test_gpu_index.py -m gpu -x -q --timeout 300 --timeout-method thread -k 'lomuto'" \
  "120|r03/ld9|python -u tools/lomuto_prof.py 27 3" \
  "200|r03/ld9_prof|rocprofv3 --kernel-trace --stats -d gpurun_out/r03/ld9prof -o run --output-format csv -- python -u tools/lomuto_prof.py 27 2"
