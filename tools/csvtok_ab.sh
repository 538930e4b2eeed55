# k_csv_parse A/B on one box: MQ_CSV_TOKENS=0 (row-wise only) vs 1 (token-parallel), alternating
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rows=${1:-250000000}
for v in 0 1 0 1; do
  MQ_CSV_TOKENS=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ctab_$v -o l --output-format csv -- python3 tools/load_bench.py $rows 4 3 > gpurun_out/ctab_$v.log 2>&1 || exit 1
  echo "== MQ_CSV_TOKENS=$v"; grep "^{" gpurun_out/ctab_$v.log | cut -c1-200
  python3 - gpurun_out/ctab_$v/l_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'csv' in r['Name']:
        print("  ", r['Name'][:50], r['Calls'], round(float(r['AverageNs']) / 1e6, 3))
PY
done
