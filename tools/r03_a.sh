# round-3 GPU call A: the new correctness tests, the PCIe probe, the API trace
set -u
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "600|r03/pytest_new|python -u -m pytest tests/test_gpu_shards.py tests/test_gpu_index.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k 'shards or index or fullsize or 1e9 or combine' -m gpu -v --timeout 300 --timeout-method thread" \
  "120|r03/pcie_probe|tools/pcie_probe 40000000 268435456" \
  "180|r03/api_trace|env MQ_TRACE=1 python -u tools/api_timing.py --reps 4"
