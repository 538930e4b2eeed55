# round-3 GPU call J: shared_select count pass, 4096-cell table (4 blocks a CU)
set -u
mkdir -p gpurun_out/r03
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "300|r03/pytest_ss2|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -k 'shared' -q --timeout 300 --timeout-method thread" \
  "120|r03/ss_new2|python -u tools/shared_prof.py 2,16,150,256 7" \
  "120|r03/ss_old2|env MQ_SS_COUNT=filter python -u tools/shared_prof.py 2,16,150,256 7" \
  "200|r03/ss_prof2|rocprofv3 --kernel-trace --stats -d gpurun_out/r03/ssprof2 -o ss --output-format csv -- python3 tools/shared_prof.py 16,150 5"
