# shared_select pair-listing A/B (timing only): full, no stores, no prefix/stores, two-pass
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 0 1 2 tp; do
  if [ $v = tp ]; then export MQ_SS_TWOPASS=1; unset MQ_SSP_DEBUG; else export MQ_SSP_DEBUG=$v; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ssdbg$v -o ss --output-format csv -- python3 tools/shared_prof.py 16,150 3 > gpurun_out/ssdbg$v.log 2>&1 || exit 1
  echo "== variant $v"; grep "^q=" gpurun_out/ssdbg$v.log
  python3 - $v <<'PY'
import csv, sys
rows=list(csv.DictReader(open(f'gpurun_out/ssdbg{sys.argv[1]}/ss_kernel_stats.csv')))
for r in rows:
    if 'k_ss' in r['Name'] and 'totals' not in r['Name']:
        print(r['Name'][:45], r['Calls'], round(float(r['AverageNs'])/1e6, 3))
PY
done
