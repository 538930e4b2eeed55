# Per-kernel HBM traffic (separate FETCH_SIZE / WRITE_SIZE passes) and kernel stats of
# the 2^28 unique and many-to-many joins (tools/join_bench.py).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcj6
tools/gpu_steps.sh \
  "150|pmcj6/stats_ju|timeout -s KILL 140 rocprofv3 --kernel-trace --stats -d gpurun_out/pmcj6/sju -o s --output-format csv -- python3 tools/join_bench.py 28" \
  "150|pmcj6/stats_jd|timeout -s KILL 140 rocprofv3 --kernel-trace --stats -d gpurun_out/pmcj6/sjd -o s --output-format csv -- python3 tools/join_bench.py 28 dup" \
  "150|pmcj6/fetch_ju|timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcj6/ju -o fetch --output-format csv -- python3 tools/join_bench.py 28" \
  "150|pmcj6/write_ju|timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcj6/ju -o write --output-format csv -- python3 tools/join_bench.py 28" \
  "150|pmcj6/fetch_jd|timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcj6/jd -o fetch --output-format csv -- python3 tools/join_bench.py 28 dup" \
  "150|pmcj6/write_jd|timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcj6/jd -o write --output-format csv -- python3 tools/join_bench.py 28 dup"
