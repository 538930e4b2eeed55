# round-3 GPU call U: exact index, chain walk limits after the round-major placement
set -u
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "120|r03/ld5_cap128|env MQ_LQ_CAP=128 python -u tools/lomuto_prof.py 27 3" \
  "120|r03/ld5_cap512|env MQ_LQ_CAP=512 python -u tools/lomuto_prof.py 27 3" \
  "120|r03/ld5_cap2k|env MQ_LQ_CAP=2048 python -u tools/lomuto_prof.py 27 3" \
  "120|r03/ld5_cap8k|env MQ_LQ_CAP=8192 python -u tools/lomuto_prof.py 27 3" \
  "120|r03/ld5_capinf|env MQ_LQ_CAP=1000000 python -u tools/lomuto_prof.py 27 3"
bash tools/pmc_kernel.sh gpurun_out/r03/pmc_small k_ld_small python3 tools/lomuto_prof.py 27 1
