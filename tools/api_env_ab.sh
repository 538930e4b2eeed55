# A/B of an environment setting on the config-3 API chain (tools/api_timing.py, 8 reps a
# process), three processes each, alternating:  tools/api_env_ab.sh <tag> "<VAR=value ...>"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; EB=$2
mkdir -p gpurun_out/$T
tools/gpu_steps.sh \
  "150|$T/A1|python3 tools/api_timing.py --reps 8" "150|$T/B1|env $EB python3 tools/api_timing.py --reps 8" \
  "150|$T/A2|python3 tools/api_timing.py --reps 8" "150|$T/B2|env $EB python3 tools/api_timing.py --reps 8" \
  "150|$T/A3|python3 tools/api_timing.py --reps 8" "150|$T/B3|env $EB python3 tools/api_timing.py --reps 8"
