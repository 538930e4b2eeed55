# column upload (2 x 4 GB memfd-backed) and the config-3 API chain: staged H2D vs plain
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 1 0 1 0; do
  echo "== MQ_H2D_STAGED=$v"
  MQ_TRACE=1 MQ_H2D_STAGED=$v timeout -k 10 200 python3 tools/api_timing.py --reps 5 > gpurun_out/h2d_$v.out 2> gpurun_out/h2d_$v.err || exit 1
  grep -E "upload|rep" gpurun_out/h2d_$v.out
done
