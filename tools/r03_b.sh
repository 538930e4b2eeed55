# round-3 GPU call B: host-memory probe + the full bench (new legs)
set -u
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "180|r03/payload_probe|tools/payload_probe 40000000 1073741824" \
  "600|r03/bench_b|python -u bench.py"
