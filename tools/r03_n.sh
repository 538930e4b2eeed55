# round-3 GPU call N: exact index, larger chain walk caps
set -u
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "120|r03/lq_cap64b|env MQ_LQ_CAP=64 python -u tools/lomuto_prof.py 27 3" \
  "120|r03/lq_cap128|env MQ_LQ_CAP=128 python -u tools/lomuto_prof.py 27 3" \
  "120|r03/lq_cap256|env MQ_LQ_CAP=256 python -u tools/lomuto_prof.py 27 3" \
  "120|r03/lq_cap512|env MQ_LQ_CAP=512 python -u tools/lomuto_prof.py 27 3"
