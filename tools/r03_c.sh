# round-3 GPU call C: A/B of the staged D2H with background page population
set -u
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "120|r03/api_prefault_off|env MQ_PREFAULT=0 python -u tools/api_timing.py --reps 6" \
  "120|r03/api_prefault_on|python -u tools/api_timing.py --reps 6" \
  "120|r03/api_prefault_f2|env MQ_FAULT_THREADS=2 python -u tools/api_timing.py --reps 6" \
  "120|r03/api_prefault_f8|env MQ_FAULT_THREADS=8 python -u tools/api_timing.py --reps 6" \
  "120|r03/api_prefault_c8|env MQ_COPY_THREADS=8 python -u tools/api_timing.py --reps 6" \
  "120|r03/api_prefault_f4c6|env MQ_COPY_THREADS=6 MQ_FAULT_THREADS=6 python -u tools/api_timing.py --reps 6" \
  "120|r03/api_trace2|env MQ_TRACE=1 python -u tools/api_timing.py --reps 4"
