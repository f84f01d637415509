set -e
for i in 1 2 3; do
  for p in none teacher; do
    CLSKD_STREAM_PRIO=$p timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/ab_$p_$i.log 2>&1
    v=$(grep -o '"value": [0-9.]*' gpurun_out/ab_$p_$i.log)
    echo "$p $v"
  done
done
