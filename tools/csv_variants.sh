#!/usr/bin/env bash
# Build libmq variants that differ only in mq_csv.hip compile flags (A/B on the GPU box):
#   tools/csv_variants.sh <name> "<-D flags>" ...   -> gpurun_ab/libmq_<name>.so
set -eu
cd "$(dirname "$0")/.."
make -C analytical-database_amd -s
B=analytical-database_amd/build
mkdir -p gpurun_ab /tmp/csvvar
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Iinclude $flags \
    -c analytical-database_amd/csrc/mq_csv.hip -o /tmp/csvvar/mq_csv_$name.o
  objs=$(ls $B/*.o | grep -v '/mq_csv.o$')
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread -Wl,-soname,libmq.so \
    -o gpurun_ab/libmq_$name.so $objs /tmp/csvvar/mq_csv_$name.o
  echo "built gpurun_ab/libmq_$name.so ($flags)"
done
