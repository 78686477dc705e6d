# round 5: the module with its threads on the GPU's NUMA node (EDGPU_QTSS_AFFINITY, default on) and
# tools/bench_module.py --affinity gpu-node (every side on that node) against --affinity none and
# the module's own pinning off.  Module tests first.  Logs under gpurun_out/$1.
# (EDGPU_QTSS_AFFINITY was removed after this run: the module's own pinning measured no gain.)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05z9}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu \
    tests/test_gpu_qtss_module.py tests/test_gpu_engine_api.py > $O/gputests.log 2>&1; r=$?
tail -2 $O/gputests.log; [ $r -eq 0 ] || exit $r
run() {   # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err; local r=$?
  echo "$n rc=$r"; python -c "
import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); m=d.get('module')
if m: print(round(m['relayed_per_s']/1e6,1), 'M', m['per_tick_ms'], 'push_s', m['push_s'], 'tick_s', m['tick_s'], 'vs ref module', d.get('module_vs_reference_module'), 'vs ref', d.get('module_vs_reference'), 'ref', (d.get('reference') or {}).get('relayed_per_s'), 'refmod', (d.get('reference_module') or {}).get('relayed_per_s'))
else: print([(r['reflect_on_arrival_ms'], r['latency_ms']['mean'], r['latency_ms']['p99']) for r in d['runs']])"
  return $r
}
run t100_node 400 python tools/bench_module.py --tick-ms 100 && \
run t100_none 400 python tools/bench_module.py --tick-ms 100 --affinity none && \
EDGPU_QTSS_AFFINITY=0 run t100_none_nopin 200 python tools/bench_module.py --tick-ms 100 --affinity none --no-reference && \
EDGPU_QTSS_TICK_MSEC=20 run t20_node 400 python tools/bench_module.py --tick-ms 20 && \
run realtime_node 300 python tools/bench_module.py --realtime --tick-ms 20 --seconds 5
exit $?
