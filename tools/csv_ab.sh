#!/usr/bin/env bash
# k_csv_parse A/B over libmq variants in gpurun_ab/ (tools/csv_variants.sh), alternating
# on one box; prints ms_count / ms_parse (HIP events, median of reps) per run.
#   tools/csv_ab.sh <rows> <variant>...     (GPU box, repo root)
set -eu
rows=$1; shift
for r in 1 2; do
  for v in "$@"; do
    MQ_LIB=$GRAFT_REPO_ROOT/gpurun_ab/libmq_$v.so timeout -k 10 120 python3 tools/load_bench.py $rows 4 5 > gpurun_out/csvab_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/csvab_$v.log; exit 1; }
    echo "$r $v $(grep '^{' gpurun_out/csvab_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ok"], d["ms_count"], d["ms_parse"])')"
  done
done
