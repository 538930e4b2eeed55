# round-3 GPU call I: SQ counters, new (k_ssk_count) vs old (k_ssp_count) count pass at Q = 150
set -u
mkdir -p gpurun_out/r03
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 bash tools/pmc_kernel.sh gpurun_out/r03/pmc_ssk 'k_ssk_count' python3 tools/shared_prof.py 150 2 && \
MQ_SS_COUNT=filter timeout -k 10 300 bash tools/pmc_kernel.sh gpurun_out/r03/pmc_ssp 'k_ssp_count' python3 tools/shared_prof.py 150 2
