#!/bin/bash
# Engine crossover numbers (printed by the 256-digester test) and the C3 bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_engine.py \
    > gpurun_out/engine_test.log 2>&1 || { tail -30 gpurun_out/engine_test.log; exit 1; }
grep -E "single GPU digester|passed|failed" gpurun_out/engine_test.log
./tools/gpu_r02.sh bc3
python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/bench_c3.log') if l.startswith('{')][-1]); print(d['value'], json.dumps(d['roofline']))"
