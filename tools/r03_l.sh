# round-3 GPU call L: exact index with zone-restricted doubling: parity, time, stats
set -u
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "400|r03/pytest_index|python -u -m pytest tests/test_gpu_index.py -m gpu -q --timeout 300 --timeout-method thread" \
  "120|r03/lomuto_time|python -u tools/lomuto_prof.py 27 3" \
  "120|r03/lomuto_stats2|env MQ_LQ_STATS=1 python -u tools/lomuto_prof.py 27 1"
