# host-lane probes (tools/lane_probe.py) beside the windows: lane streams at high / low priority
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export KRK_TRACE=1 && \
timeout -k 10 200 python tools/lane_probe.py --mode windows --k 480 --lane-prio -1 > gpurun_out/lane1.log 2>&1 && \
timeout -k 10 200 python tools/lane_probe.py --mode windows --k 480 --lane-prio 1 > gpurun_out/lane2.log 2>&1
