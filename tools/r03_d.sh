# round-3 GPU call D: column upload A/B (guard armed concurrently; copy threads)
set -u
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "120|r03/up_sync_c4|env MQ_GUARD_ASYNC=0 python -u tools/api_timing.py --reps 3" \
  "120|r03/up_async_c4|python -u tools/api_timing.py --reps 3" \
  "120|r03/up_async_c8|env MQ_COPY_THREADS=8 python -u tools/api_timing.py --reps 3" \
  "120|r03/up_async_c12|env MQ_COPY_THREADS=12 python -u tools/api_timing.py --reps 3" \
  "120|r03/up_sync_c8|env MQ_GUARD_ASYNC=0 MQ_COPY_THREADS=8 python -u tools/api_timing.py --reps 3" \
  "120|r03/up_trace|env MQ_TRACE=1 python -u tools/api_timing.py --reps 2"
