set -u
timeout -k 10 200 python -u -m pytest tests/test_gpu_load.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/load_tests3.log 2>&1; rc=$?; tail -3 gpurun_out/load_tests3.log; [ $rc -eq 0 ] || exit $rc
tools/csv_ab.sh 250000000 base new || exit 1
for g in 1024 3072 6144; do MQ_CSV_GRID=$g MQ_LIB=$GRAFT_REPO_ROOT/gpurun_ab/libmq_new.so timeout -k 10 120 python3 tools/load_bench.py 250000000 4 5 > gpurun_out/grid_$g.log 2>&1 || exit 1; echo "grid $g $(grep '^{' gpurun_out/grid_$g.log | cut -c1-200)"; done
