# A/B of a join variant switched by an env var ($1=VAR, $2 = join_bench arg), alternating, same box
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
var=$1
for v in 1 0 1 0; do
  export $var=$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/jab_$v -o j --output-format csv -- python3 tools/join_bench.py 28 ${2:-} > gpurun_out/jab_$v.log 2>&1 || exit 1
  echo "== $var=$v"; grep "^{" gpurun_out/jab_$v.log | cut -c1-140
  python3 - gpurun_out/jab_$v/j_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if any(k in r['Name'] for k in ('probe_unique', 'win_build', 'join_write')):
        print("  ", r['Name'][:50], r['Calls'], round(float(r['AverageNs']) / 1e6, 3))
PY
done
