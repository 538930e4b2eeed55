# round-3 GPU call AD: SQ counters of the MSD index sort's finisher and scatters at 1e9 rows
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03
timeout -k 10 300 tools/pmc_kernel.sh gpurun_out/r03/pmc_isort9 'k_msd_finish_count|k_msd_scatter' python -u tools/index_bench.py 1000000000 1
