#!/usr/bin/env bash
# GPU evidence runs, one script for every round (replaces the per-call r0N_*.sh launchers).
#   tools/evidence.sh <tag> final            -m gpu suite, smoke, bench line, kernel stats, PMC traffic
#                                           of the headline, the N = 2 gloo rehearsal
#   tools/evidence.sh <tag> tests [pytest-args...]   a pytest -m gpu selection (e.g. -k join)
#   tools/evidence.sh <tag> bench [bench-args...]    one bench line (+ its rocprof kernel stats)
#   tools/evidence.sh <tag> pmc <kernel-regex> <cmd...>  FETCH_SIZE / WRITE_SIZE + SQ passes of one command
#   tools/evidence.sh <tag> steps "<secs>|<name>|<cmd>" ...  anything else (tools/gpu_steps.sh)
# Logs go to gpurun_out/<tag>/; each step runs under its own limit and the first fault stops the call.
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag="$1"; what="$2"; shift 2
out="gpurun_out/$tag"
mkdir -p "$out"
py="python3 -u"
case "$what" in
  final)
    exec tools/gpu_steps.sh \
      "1000|$tag/pytest_gpu_all|python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -s" \
      "120|$tag/smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
      "300|$tag/bench|$py bench.py" \
      "300|$tag/prof_bench|rocprofv3 --kernel-trace --stats -d $out/prof -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu" \
      "120|$tag/pmc_fetch|timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $out/pmc -o fetch --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extra" \
      "120|$tag/pmc_write|timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $out/pmc -o write --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extra" \
      "200|$tag/bench_n2|MQ_BENCH_BACKEND=gloo MQ_BENCH_ONE_DEVICE=1 python3 bench.py --gpus 2 --no-extra --no-cpu"
    ;;
  tests)
    exec tools/gpu_steps.sh "900|$tag/pytest|python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread -s ${*:-tests}"
    ;;
  bench)
    exec tools/gpu_steps.sh \
      "300|$tag/bench|$py bench.py $*" \
      "300|$tag/prof_bench|rocprofv3 --kernel-trace --stats -d $out/prof -o bench --output-format csv -- python3 bench.py --no-cpu $*"
    ;;
  pmc)
    shift  # (kernel regex: kept in the call for the log; the fold covers every kernel)
    exec tools/gpu_steps.sh \
      "120|$tag/pmc_fetch|timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $out/pmc -o fetch --output-format csv -- $*" \
      "120|$tag/pmc_write|timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $out/pmc -o write --output-format csv -- $*" \
      "120|$tag/pmc_sq|timeout -s KILL 110 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace -d $out/pmc -o sq --output-format csv -- $*" \
      "60|$tag/pmc_fold|$py tools/pmc_traffic.py $out/pmc --out $out/pmc_traffic.json"
    ;;
  steps)
    exec tools/gpu_steps.sh "$@"
    ;;
  *)
    echo "unknown recipe: $what" >&2
    exit 2
    ;;
esac
