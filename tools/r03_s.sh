# round-3 GPU call S: shard residency fix: shard tests + inproc rehearsal
set -u
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "300|r03/pytest_shards2|python -u -m pytest tests/test_gpu_shards.py tests/test_gpu_residency.py -m gpu -x -q --timeout 200 --timeout-method thread" \
  "200|r03/inproc1b|python -u bench.py --inproc --gpus 1" \
  "200|r03/inproc2b|env MQ_BENCH_ONE_DEVICE=1 python -u bench.py --inproc --gpus 2" \
  "200|r03/inproc4b|env MQ_BENCH_ONE_DEVICE=1 python -u bench.py --inproc --gpus 4"
