# round 4: the module at C2's real rate on its own ticker (tools/bench_module.py --realtime):
# relayed packets/s and the RTSPIncomingData -> QTSS_Write latency per RTP packet, fixed 20-ms
# ticks against reflect-on-arrival at 2 and 1 ms.  Logs under gpurun_out/$1 (default r04_latency).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r04_latency}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python tools/bench_module.py --realtime --tick-ms 20 --seconds 5 > $O/bench_module_realtime.json \
    2> $O/bench_module_realtime.err; r=$?
echo "realtime rc=$r"; cat $O/bench_module_realtime.json
exit $r
