#!/bin/bash
# The SHA offload's D2H copies on dedicated copy queues (default) vs each thread's own
# normal streams (KRK_OFFLOAD_COPY_QUEUES=0): C3 rank 0's shard of 8 GPUs with the host lane.
for r in 1 2; do
  for q in 1 0; do
    KRK_OFFLOAD_COPY_QUEUES=$q timeout -k 10 500 python bench.py --workload c3 --emulate-world 8 --host-lane --no-cpu-baseline --no-e2e > gpurun_out/lane_q${q}_$r.log 2>&1 || { echo "fail q=$q"; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/lane_q${q}_$r.log') if l.startswith('{')][-1]); h=d['host_offload']; print('queues=$q', d['value'], h['value'], h['lane_s'], h['modelled_s'], h['matches_gpu_only'])
"
  done
done
