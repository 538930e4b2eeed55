# round-3 GPU call G: many-to-many join with per-word run lengths: parity + timing
set -u
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "600|r03/pytest_join|python -u -m pytest tests/test_gpu_parity.py -m gpu -k 'join' -v --timeout 300 --timeout-method thread" \
  "120|r03/join_dup|python -u tools/join_bench.py 28 dup" \
  "120|r03/join_uni|python -u tools/join_bench.py 28"
