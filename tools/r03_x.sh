# round-3 GPU call X: exact index, doubling with 8 entries in flight per lane; walk limits
set -u
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "400|r03/pytest_index8|python -u -m pytest tests/test_gpu_index.py -m gpu -x -q --timeout 300 --timeout-method thread -k 'lomuto'" \
  "120|r03/ld8|python -u tools/lomuto_prof.py 27 3" \
  "120|r03/ld8_cap256|env MQ_LQ_CAP=256 python -u tools/lomuto_prof.py 27 3" \
  "120|r03/ld8_cap1k|env MQ_LQ_CAP=1024 python -u tools/lomuto_prof.py 27 3" \
  "200|r03/ld8_prof|rocprofv3 --kernel-trace --stats -d gpurun_out/r03/ld8prof -o run --output-format csv -- python -u tools/lomuto_prof.py 27 2"
