# round-3 GPU call T: exact index, round-major placement: parity + time + profile
set -u
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "400|r03/pytest_index5|python -u -m pytest tests/test_gpu_index.py -m gpu -x -q --timeout 300 --timeout-method thread -k 'lomuto'" \
  "120|r03/ld4|python -u tools/lomuto_prof.py 27 3" \
  "200|r03/ld4_prof|rocprofv3 --kernel-trace --stats -d gpurun_out/r03/ld4prof -o run --output-format csv -- python -u tools/lomuto_prof.py 27 2"
