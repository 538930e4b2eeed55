# PMC traffic (separate FETCH_SIZE / WRITE_SIZE passes) of the 2^28 joins and of the
# random-read probes (tools/random_read: 16/32/64-B random reads of a 4 GB table)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcj
tools/gpu_steps.sh \
  "120|pmcj/fetch_ju|timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcj/ju -o fetch --output-format csv -- python3 tools/join_bench.py 28" \
  "120|pmcj/write_ju|timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcj/ju -o write --output-format csv -- python3 tools/join_bench.py 28" \
  "120|pmcj/fetch_jd|timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcj/jd -o fetch --output-format csv -- python3 tools/join_bench.py 28 dup" \
  "120|pmcj/write_jd|timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcj/jd -o write --output-format csv -- python3 tools/join_bench.py 28 dup" \
  "120|pmcj/fetch_rr|timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcj/rr -o fetch --output-format csv -- tools/random_read 29 28" \
  "120|pmcj/write_rr|timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcj/rr -o write --output-format csv -- tools/random_read 29 28"
