# index build (onesweep vs classic sort) and the many-to-many join under rocprofv3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
stats() { python3 - "$1" <<'PY'
import csv, sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:14]:
    print("  ", r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6, 3), round(float(r['TotalDurationNs'])/1e6, 2))
PY
}
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sp1 -o s --output-format csv -- python3 tools/index_bench.py 1000000000 3 > gpurun_out/sp1.log 2>&1 || exit 1
echo "== onesweep"; grep "^{" gpurun_out/sp1.log; stats gpurun_out/sp1/s_kernel_stats.csv
MQ_SORT_IMPL=classic timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sp2 -o s --output-format csv -- python3 tools/index_bench.py 1000000000 3 > gpurun_out/sp2.log 2>&1 || exit 1
echo "== classic"; grep "^{" gpurun_out/sp2.log; stats gpurun_out/sp2/s_kernel_stats.csv
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/jp -o j --output-format csv -- python3 tools/join_bench.py 28 dup > gpurun_out/jp.log 2>&1 || exit 1
echo "== join dup"; grep "^{" gpurun_out/jp.log; stats gpurun_out/jp/j_kernel_stats.csv
