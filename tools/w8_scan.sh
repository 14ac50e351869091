mkdir -p gpurun_out
for n in 1000 2048 3072 4096; do
  timeout -k 10 200 python -u bench.py --workload small --blobs $n --no-e2e --no-cpu-baseline --no-offload --steps 3 --warmup 1 > gpurun_out/w8_$n.log 2>&1 || exit $?
  echo "done $n"
done
