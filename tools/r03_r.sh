# round-3 GPU call R: exact index, batched doubling + folded memsets; finisher tiny threshold A/B
set -u
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "400|r03/pytest_index4|python -u -m pytest tests/test_gpu_index.py -m gpu -x -q --timeout 300 --timeout-method thread -k 'lomuto'" \
  "120|r03/ld3_t16|python -u tools/lomuto_prof.py 27 3" \
  "120|r03/ld3_t8|env MQ_LQ_TINY=8 python -u tools/lomuto_prof.py 27 3" \
  "120|r03/ld3_t32|env MQ_LQ_TINY=32 python -u tools/lomuto_prof.py 27 3" \
  "120|r03/ld3_t32_s512|env MQ_LQ_TINY=32 MQ_LQ_SMALL=512 python -u tools/lomuto_prof.py 27 3" \
  "200|r03/ld3_prof|rocprofv3 --kernel-trace --stats -d gpurun_out/r03/ld3prof -o run --output-format csv -- python -u tools/lomuto_prof.py 27 2"
tools/gpu_steps.sh \
  "200|r03/inproc1|python -u bench.py --inproc --gpus 1" \
  "200|r03/inproc2_one|env MQ_BENCH_ONE_DEVICE=1 python -u bench.py --inproc --gpus 2"
