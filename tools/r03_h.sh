# round-3 GPU call H: shared_select k-major count pass: parity, A/B, kernel times
set -u
mkdir -p gpurun_out/r03
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "600|r03/pytest_ss|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_shards.py -m gpu -k 'shared' -v --timeout 300 --timeout-method thread" \
  "120|r03/ss_new|python -u tools/shared_prof.py 2,16,150,256 7" \
  "120|r03/ss_old|env MQ_SS_COUNT=filter python -u tools/shared_prof.py 2,16,150,256 7" \
  "200|r03/ss_prof|rocprofv3 --kernel-trace --stats -d gpurun_out/r03/ssprof -o ss --output-format csv -- python3 tools/shared_prof.py 16,150 5"
