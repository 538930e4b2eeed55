# index build (mq_index_build) at several sizes: the MSD form (forced) vs the LSD form
set -u
for n in ${SWEEP_N:-4194304 16777216 67108864 134217728 268435456 1000000000}; do
  echo "== n=$n"
  MQ_INDEX_MSD_MIN=0 timeout -k 10 100 python -u tools/index_bench.py $n 5 || exit 1
  MQ_INDEX_SORT=lsd timeout -k 10 100 python -u tools/index_bench.py $n 5 || exit 1
done
