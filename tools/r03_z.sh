# round-3 GPU call Z: exact index, small-range limit sweep after the pull placement
set -u
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "120|r03/ld10_t256|env MQ_LQ_SMALL=256 python -u tools/lomuto_prof.py 27 3" \
  "120|r03/ld10_t512|env MQ_LQ_SMALL=512 python -u tools/lomuto_prof.py 27 3" \
  "120|r03/ld10_t1024|env MQ_LQ_SMALL=1024 python -u tools/lomuto_prof.py 27 3" \
  "120|r03/ld10_t2048|env MQ_LQ_SMALL=2048 python -u tools/lomuto_prof.py 27 3" \
  "200|r03/ld10_prof512|MQ_LQ_SMALL=512 rocprofv3 --kernel-trace --stats -d gpurun_out/r03/ld10prof -o run --output-format csv -- python -u tools/lomuto_prof.py 27 2"
