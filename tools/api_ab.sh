# A/B of the in-tree libmq against <lib B> on the config-3 API chain (tools/api_timing.py,
# 8 reps a process), three processes each, alternating; then the API / e2e tests.
#   tools/api_ab.sh <tag> <lib B>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; LB=$2
mkdir -p gpurun_out/$T
tools/gpu_steps.sh \
  "150|$T/A1|python3 tools/api_timing.py --reps 8" "150|$T/B1|MQ_LIB=$LB python3 tools/api_timing.py --reps 8" \
  "150|$T/A2|python3 tools/api_timing.py --reps 8" "150|$T/B2|MQ_LIB=$LB python3 tools/api_timing.py --reps 8" \
  "150|$T/A3|python3 tools/api_timing.py --reps 8" "150|$T/B3|MQ_LIB=$LB python3 tools/api_timing.py --reps 8" || exit $?
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_residency.py tests/test_e2e.py tests/test_gpu_parity.py -k "select_column or residency or e2e or pipe or api" > gpurun_out/$T/pytest_api.log 2>&1
echo "pytest rc=$?"; tail -1 gpurun_out/$T/pytest_api.log
