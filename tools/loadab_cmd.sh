# k_csv_parse A/B: gpurun_ab/libmq_base.so vs the tree's libmq.so, alternating, same box
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rows=${1:-250000000}
for v in base new base new; do
  if [ $v = base ]; then export MQ_LIB=$GRAFT_REPO_ROOT/gpurun_ab/libmq_base.so; else unset MQ_LIB; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/lab_$v -o l --output-format csv -- python3 tools/load_bench.py $rows 4 3 > gpurun_out/lab_$v.log 2>&1 || exit 1
  echo "== $v"; grep "^{" gpurun_out/lab_$v.log | cut -c1-160
  python3 - gpurun_out/lab_$v/l_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'csv' in r['Name']:
        print("  ", r['Name'][:50], r['Calls'], round(float(r['AverageNs']) / 1e6, 3))
PY
done
