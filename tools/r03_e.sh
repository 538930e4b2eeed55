# round-3 GPU call E: random reads vs table size; upload trace
set -u
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "180|r03/random_read_ic|python -u tools/random_read_ic.py" \
  "120|r03/up_trace2|env MQ_TRACE=1 python -u tools/api_timing.py --reps 2"
