# round-3 GPU call AK: m2m write with 16 words in flight vs 8 (A/B, alternating)
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03
tools/gpu_steps.sh \
  "300|r03/w16_pytest|env MQ_JOIN_WRITE=16 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k 'dup_goldens or dups_short'" \
  "300|r03/w16_ab|for r in 1 2 3; do for f in 16 8; do echo write=\$f; MQ_JOIN_WRITE=\$f python -u tools/join_bench.py 28 dup || exit 1; done; done"
