# round-3 GPU call F: where the exact index path spends its time
set -u
mkdir -p gpurun_out/r03
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "120|r03/lomuto_wall|env MQ_TRACE=1 python -u tools/lomuto_prof.py 27 2" \
  "200|r03/lomuto_prof|rocprofv3 --kernel-trace --stats -d gpurun_out/r03/lomuto_rocprof -o lomuto -- python3 tools/lomuto_prof.py 27 1"
