mkdir -p gpurun_out/ring_ab
for rep in 1 2 3; do
  for nw in 3 4; do
    out=gpurun_out/ring_ab/files_w${nw}_r${rep}.log
    KRK_STAGING_WINDOWS=$nw timeout -k 10 300 python bench.py --workload files --steps 2 --warmup 1 --no-cpu-baseline > $out 2>&1 || { echo "failed $out"; exit 1; }
    echo "files w=$nw rep=$rep $(grep -o '"value": [0-9.]*' $out | head -1) $(grep -o '"peak": [0-9.]*' $out | head -1)"
  done
done
