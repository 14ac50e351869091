# host-lane probes (tools/lane_probe.py) beside the windows: s_a (the SHA-256 launches) at
# normal / low / high priority (KRK_SA_PRIO: hardware queues of its own)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export KRK_TRACE=1 && \
timeout -k 10 200 python tools/lane_probe.py --mode windows --k 480 > gpurun_out/lane0.log 2>&1 && \
KRK_SA_PRIO=1 timeout -k 10 200 python tools/lane_probe.py --mode windows --k 480 > gpurun_out/lane1.log 2>&1 && \
KRK_SA_PRIO=-1 timeout -k 10 200 python tools/lane_probe.py --mode windows --k 480 > gpurun_out/lane2.log 2>&1
