#!/bin/bash
# Every shard of an emulated 8-GPU C3 run, one after another on one MI355X (bench.py
# --emulate-rank K for K = 0..7), so the emulated job's time is the max over all eight shards
# rather than rank 0's (which holds the longest blob).
#   bash tools/c3_w8_all_shards.sh          the tail handoff alone (--c3-tail-only)
#   bash tools/c3_w8_all_shards.sh gpu      the GPU-only windows (the bench `value`)
mkdir -p gpurun_out
mode=${1:-tail}
for k in 0 1 2 3 4 5 6 7; do
  if [ "$mode" = gpu ]; then
    timeout -k 10 150 python -u bench.py --workload c3 --emulate-world 8 --emulate-rank $k --no-e2e \
        --no-cpu-baseline > gpurun_out/c3_w8_gpu_rank$k.log 2>&1 || exit $?
    grep '^{' gpurun_out/c3_w8_gpu_rank$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($k, d['config']['longest_blob'], d['value'], d['ms_per_step'])"
  else
    timeout -k 10 150 python -u bench.py --workload c3 --emulate-world 8 --emulate-rank $k --c3-tail-only --no-e2e \
        --no-cpu-baseline > gpurun_out/c3_w8_rank$k.log 2>&1 || exit $?
    grep '^{' gpurun_out/c3_w8_rank$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['tail_handoff']; print($k, d['config']['longest_blob'], t.get('value'), t.get('ms_per_step'), t.get('measured_over_model'))"
  fi
done
