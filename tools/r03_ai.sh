# round-3 GPU call AI: SQ counters of the windowed runs build and the m2m write at 2^28
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03
timeout -k 10 300 tools/pmc_kernel.sh gpurun_out/r03/pmc_winruns 'k_win_build_runs|k_join_write_runs_mlp' python -u tools/join_bench.py 28 dup
