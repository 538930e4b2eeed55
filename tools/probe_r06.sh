# Round-6 probes: SQ counters of the join's window kernels and fused write, the API
# select's phase trace, the index build's kernel stats.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-r06h}
mkdir -p gpurun_out/$T
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
SQ2="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH"
tools/gpu_steps.sh \
  "90|$T/sq1_ju|timeout -s KILL 80 rocprofv3 --pmc $SQ1 --kernel-include-regex 'k_win_join|k_pwin_gather_write|k_pwin_scatter' -d gpurun_out/$T/sq -o sq1 --output-format csv -- python3 tools/join_bench.py 28" \
  "90|$T/sq2_ju|timeout -s KILL 80 rocprofv3 --pmc $SQ2 --kernel-include-regex 'k_win_join|k_pwin_gather_write|k_pwin_scatter' -d gpurun_out/$T/sq -o sq2 --output-format csv -- python3 tools/join_bench.py 28" \
  "90|$T/fetch_ju|timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/$T/ju -o fetch --output-format csv -- python3 tools/join_bench.py 28" \
  "90|$T/write_ju|timeout -s KILL 80 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/$T/ju -o write --output-format csv -- python3 tools/join_bench.py 28" \
  "90|$T/fetch_jd|timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/$T/jd -o fetch --output-format csv -- python3 tools/join_bench.py 28 dup" \
  "90|$T/write_jd|timeout -s KILL 80 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/$T/jd -o write --output-format csv -- python3 tools/join_bench.py 28 dup" \
  "200|$T/api_trace|MQ_TRACE=1 python3 tools/api_timing.py --reps 5" \
  "150|$T/ix|rocprofv3 --kernel-trace --stats -d gpurun_out/$T/ix -o s --output-format csv -- python3 tools/index_bench.py 1000000000 3"
