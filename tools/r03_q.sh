# round-3 GPU call Q: exact index with interleaved chains + flagged-range doubling: parity, time, profile
set -u
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "400|r03/pytest_index3|python -u -m pytest tests/test_gpu_index.py -m gpu -x -q --timeout 300 --timeout-method thread" \
  "120|r03/ld2_t1024|python -u tools/lomuto_prof.py 27 3" \
  "120|r03/ld2_t512|env MQ_LQ_SMALL=512 python -u tools/lomuto_prof.py 27 3" \
  "120|r03/ld2_cap1k|env MQ_LQ_CAP=1024 python -u tools/lomuto_prof.py 27 3" \
  "120|r03/ld2_cap64|env MQ_LQ_CAP=64 python -u tools/lomuto_prof.py 27 3" \
  "200|r03/ld2_prof|rocprofv3 --kernel-trace --stats -d gpurun_out/r03/ld2prof -o run --output-format csv -- python -u tools/lomuto_prof.py 27 2"
