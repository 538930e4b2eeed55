# round-3 GPU call V: exact index, single-buffer finisher: parity + time per threshold
set -u
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "400|r03/pytest_index6|python -u -m pytest tests/test_gpu_index.py -m gpu -x -q --timeout 300 --timeout-method thread -k 'lomuto'" \
  "120|r03/ld6_t1024|python -u tools/lomuto_prof.py 27 3" \
  "120|r03/ld6_t512|env MQ_LQ_SMALL=512 python -u tools/lomuto_prof.py 27 3" \
  "120|r03/ld6_t512_8|env MQ_LQ_SMALL=512 MQ_LQ_TINY=8 python -u tools/lomuto_prof.py 27 3" \
  "200|r03/ld6_prof|rocprofv3 --kernel-trace --stats -d gpurun_out/r03/ld6prof -o run --output-format csv -- python -u tools/lomuto_prof.py 27 2"
