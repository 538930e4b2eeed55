# shared_select single pass: k_ssp_count vs the lane-contiguous k_ssp_count_lc (timing)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 0 1; do
  export MQ_SSP_LC=$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sslc$v -o ss --output-format csv -- python3 tools/shared_prof.py 16,150 3 > gpurun_out/sslc$v.log 2>&1 || exit 1
  echo "== MQ_SSP_LC=$v"; grep "^q=" gpurun_out/sslc$v.log
  python3 - $v <<'PY'
import csv, sys
rows=list(csv.DictReader(open(f'gpurun_out/sslc{sys.argv[1]}/ss_kernel_stats.csv')))
for r in rows:
    if 'k_ss' in r['Name'] and 'totals' not in r['Name']:
        print(r['Name'][:45], r['Calls'], round(float(r['AverageNs'])/1e6, 3))
PY
done
