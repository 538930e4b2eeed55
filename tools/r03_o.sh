# round-3 GPU call O: speculative select payload: API parity + A/B
set -u
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "600|r03/pytest_api|python -u -m pytest tests/test_gpu_residency.py tests/test_gpu_shards.py tests/test_e2e.py tests/test_gpu_parity.py -m gpu -k 'api or residency or shard or e2e or server' -q --timeout 300 --timeout-method thread" \
  "120|r03/spec_off|env MQ_SPECULATE=0 python -u tools/api_timing.py --reps 6" \
  "120|r03/spec_on|python -u tools/api_timing.py --reps 6" \
  "120|r03/spec_trace|env MQ_TRACE=1 python -u tools/api_timing.py --reps 3"
