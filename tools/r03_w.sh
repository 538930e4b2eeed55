# round-3 GPU call W: exact index, back-map pull placement: parity + time + profile
set -u
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "400|r03/pytest_index7|python -u -m pytest tests/test_gpu_index.py -m gpu -x -q --timeout 300 --timeout-method thread -k 'lomuto'" \
  "120|r03/ld7|python -u tools/lomuto_prof.py 27 3" \
  "120|r03/ld7_cap512|env MQ_LQ_CAP=512 python -u tools/lomuto_prof.py 27 3" \
  "120|r03/ld7_cap2k|env MQ_LQ_CAP=2048 python -u tools/lomuto_prof.py 27 3" \
  "200|r03/ld7_prof|rocprofv3 --kernel-trace --stats -d gpurun_out/r03/ld7prof -o run --output-format csv -- python -u tools/lomuto_prof.py 27 2"
