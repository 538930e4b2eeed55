# round-3 GPU call AC: SQ counters of the MSD index sort's kernels at 2^28 rows
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03
timeout -k 10 300 tools/pmc_kernel.sh gpurun_out/r03/pmc_isort 'k_msd' python -u tools/index_bench.py 268435456 1
