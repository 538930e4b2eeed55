# round-3 GPU call P: exact index, large ranges level by level + wave finisher: parity, time per threshold
set -u
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "400|r03/pytest_index2|python -u -m pytest tests/test_gpu_index.py -m gpu -x -q --timeout 300 --timeout-method thread" \
  "120|r03/ld_t1024|python -u tools/lomuto_prof.py 27 3" \
  "120|r03/ld_t512|env MQ_LQ_SMALL=512 python -u tools/lomuto_prof.py 27 3" \
  "120|r03/ld_t2048|env MQ_LQ_SMALL=2048 python -u tools/lomuto_prof.py 27 3" \
  "120|r03/ld_stats|env MQ_LQ_STATS=1 python -u tools/lomuto_prof.py 27 1" \
  "200|r03/ld_prof|rocprofv3 --kernel-trace --stats -d gpurun_out/r03/ldprof -o run -- python -u tools/lomuto_prof.py 27 2"
