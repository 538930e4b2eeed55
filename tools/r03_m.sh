# round-3 GPU call M: exact index, chain walk cap A/B
set -u
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "120|r03/lq_cap8|env MQ_LQ_CAP=8 python -u tools/lomuto_prof.py 27 3" \
  "120|r03/lq_cap16|env MQ_LQ_CAP=16 python -u tools/lomuto_prof.py 27 3" \
  "120|r03/lq_cap32|env MQ_LQ_CAP=32 python -u tools/lomuto_prof.py 27 3" \
  "120|r03/lq_cap64|env MQ_LQ_CAP=64 python -u tools/lomuto_prof.py 27 3" \
  "200|r03/lq_prof|rocprofv3 --kernel-trace --stats -d gpurun_out/r03/lqprof -o lq --output-format csv -- python3 tools/lomuto_prof.py 27 1"
