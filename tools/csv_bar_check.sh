set -u
timeout -k 10 200 python -u -m pytest tests/test_gpu_load.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/load_tests4.log 2>&1; rc=$?; tail -3 gpurun_out/load_tests4.log; [ $rc -eq 0 ] || exit $rc
tools/csv_ab.sh 250000000 base bar
