#!/bin/bash
# Every shard of an emulated W-GPU C3 run (W = 8 by default), one after another on one MI355X
# (bench.py --emulate-rank K for K = 0..W-1), so the emulated job's time is the max over all
# shards rather than rank 0's (which holds the longest blob).
#   bash tools/c3_w8_all_shards.sh [tail|gpu] [W]
#     tail: the tail handoff alone (--c3-tail-only); gpu: the GPU-only windows (the bench `value`)
mkdir -p gpurun_out
mode=${1:-tail}
W=${2:-8}
for k in $(seq 0 $((W - 1))); do
  if [ "$mode" = gpu ]; then
    log=gpurun_out/c3_w${W}_gpu_rank$k.log
    timeout -k 10 150 python -u bench.py --workload c3 --emulate-world $W --emulate-rank $k --no-e2e \
        --no-cpu-baseline > $log 2>&1 || exit $?
    grep '^{' $log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($k, d['config']['longest_blob'], d['value'], d['ms_per_step'])"
  else
    log=gpurun_out/c3_w${W}_rank$k.log
    timeout -k 10 150 python -u bench.py --workload c3 --emulate-world $W --emulate-rank $k --c3-tail-only --no-e2e \
        --no-cpu-baseline > $log 2>&1 || exit $?
    grep '^{' $log | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['tail_handoff']; print($k, d['config']['longest_blob'], t.get('value'), t.get('ms_per_step'), t.get('measured_over_model'))"
  fi
done
