# round-3 GPU call K: exact index per-level stats, then the evidence run
set -u
mkdir -p gpurun_out/r03
tools/gpu_steps.sh "120|r03/lomuto_stats|env MQ_LQ_STATS=1 python -u tools/lomuto_prof.py 27 1" && bash tools/r03_evidence.sh
