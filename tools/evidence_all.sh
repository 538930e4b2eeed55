#!/usr/bin/env bash
# The round's whole evidence in one call: the -m gpu suite, then tools/evidence_bench.sh.
#   tools/evidence_all.sh <tag>
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag="$1"; mkdir -p "gpurun_out/$tag"
tools/gpu_steps.sh "900|$tag/pytest_gpu_all|python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread" || exit $?
exec tools/evidence_bench.sh "$tag"
