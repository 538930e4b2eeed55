# index build with and without the digit-byte histograms, under rocprofv3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
stats() { python3 - "$1" <<'PY'
import csv, sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:8]:
    print("  ", r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6, 3), round(float(r['TotalDurationNs'])/1e6, 2))
PY
}
for d in 1 0 1 0; do
MQ_SORT_DIGITS=$d timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sd$d -o s --output-format csv -- python3 tools/index_bench.py 1000000000 3 > gpurun_out/sd$d.log 2>&1 || exit 1
echo "== digits=$d"; grep "^{" gpurun_out/sd$d.log; stats gpurun_out/sd$d/s_kernel_stats.csv
done
