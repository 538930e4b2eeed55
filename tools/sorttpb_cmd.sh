# index build (1e9 rows) at sort tiles of 256/512/1024 x 16 words, under rocprofv3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for cfg in 512:16 512:8 1024:8 512:16 512:8 1024:8; do t=${cfg%:*}; export MQ_SORT_IT=${cfg#*:}
MQ_SORT_TPB=$t timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/st${t}_$MQ_SORT_IT -o s --output-format csv -- python3 tools/index_bench.py 1000000000 3 > gpurun_out/st${t}_$MQ_SORT_IT.log 2>&1 || exit 1
echo "== tpb=$t it=$MQ_SORT_IT"; grep "^{" gpurun_out/st${t}_$MQ_SORT_IT.log
python3 - gpurun_out/st${t}_$MQ_SORT_IT/s_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'sortw' in r['Name'] or 'tile_s' in r['Name']:
        print("  ", r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e6, 3))
PY
done
