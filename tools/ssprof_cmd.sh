cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ssprof -o ss --output-format csv -- python3 tools/shared_prof.py 2,16,150 5 > gpurun_out/ssprof.log 2>&1 && python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/ssprof/ss_kernel_trace.csv')))
for r in rows:
    n=r['Kernel_Name']
    if 'k_ss' in n and 'totals' not in n:
        print(n[:48], (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6)
PY
grep "^q=" gpurun_out/ssprof.log
