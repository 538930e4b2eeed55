# the 2^28 joins (unique and many-to-many) under rocprofv3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
stats() { python3 - "$1" <<'PY'
import csv, sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:10]:
    print("  ", r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6, 3), round(float(r['TotalDurationNs'])/1e6, 2))
PY
}
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ju -o j --output-format csv -- python3 tools/join_bench.py 28 > gpurun_out/ju.log 2>&1 || exit 1
echo "== join unique"; grep "^{" gpurun_out/ju.log; stats gpurun_out/ju/j_kernel_stats.csv
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/jp -o j --output-format csv -- python3 tools/join_bench.py 28 dup > gpurun_out/jp.log 2>&1 || exit 1
echo "== join dup"; grep "^{" gpurun_out/jp.log; stats gpurun_out/jp/j_kernel_stats.csv
