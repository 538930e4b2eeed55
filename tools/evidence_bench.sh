#!/usr/bin/env bash
# The round's bench evidence without the test suite: smoke, the bench line, its kernel stats,
# the headline's PMC traffic passes, the N = 2 gloo rehearsal.   tools/evidence_bench.sh <tag>
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag="$1"; out="gpurun_out/$tag"; mkdir -p "$out"
exec tools/gpu_steps.sh \
  "120|$tag/smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "420|$tag/bench|python3 -u bench.py" \
  "420|$tag/prof_bench|rocprofv3 --kernel-trace --stats -d $out/prof -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu" \
  "120|$tag/pmc_fetch|timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $out/pmc -o fetch --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extra" \
  "120|$tag/pmc_write|timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $out/pmc -o write --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extra" \
  "200|$tag/bench_n2|MQ_BENCH_BACKEND=gloo MQ_BENCH_ONE_DEVICE=1 python3 bench.py --gpus 2 --no-extra --no-cpu"
