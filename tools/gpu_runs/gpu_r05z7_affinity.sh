# round 5: the module's C2 line (100-ms ticks, no reference) with the whole process on the GPU's
# NUMA node, on the other node, and unpinned (the default: 256 CPUs allowed).  Logs under
# gpurun_out/$1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05z7}
O=gpurun_out/$TAG
mkdir -p $O
GPU_BDF=$(python -c "
import torch; p = torch.cuda.get_device_properties(0)
print('%04x:%02x:%02x.0' % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id))")
NODE=$(cat /sys/bus/pci/devices/$GPU_BDF/numa_node)
LOCAL=$(cat /sys/bus/pci/devices/$GPU_BDF/local_cpulist)
echo "gpu $GPU_BDF node $NODE local $LOCAL"; [ -n "$LOCAL" ] || exit 3
L16=$(python -c "
s='$LOCAL'; c=[]
for r in s.split(','):
    a,_,b=r.partition('-'); c+=list(range(int(a),int(b or a)+1))
print(','.join(map(str,c[:16])))")
R16=$(python -c "
s='$LOCAL'; c=set()
for r in s.split(','):
    a,_,b=r.partition('-'); c|=set(range(int(a),int(b or a)+1))
print(','.join(map(str,[x for x in range(256) if x not in c][:16])))")
echo "local16 $L16 remote16 $R16"
run() {   # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err; local r=$?
  echo "$n rc=$r"; python -c "
import json,sys; d=json.load(open('$O/$n.json')); m=d['module']
print(round(m['relayed_per_s']/1e6,1), 'M', m['per_tick_ms'], 'push_s', m['push_s'], 'tick_s', m['tick_s'])"
  return $r
}
L32=$(python -c "print(','.join('$L16'.split(',') + [str(int(x)+128) for x in '$L16'.split(',')]))")
echo "local32 $L32"
run unpinned 200 python tools/bench_module.py --no-reference && \
run localnode 200 taskset -c $LOCAL python tools/bench_module.py --no-reference && \
run local16 200 taskset -c $L16 python tools/bench_module.py --no-reference && \
run local32 200 taskset -c $L32 python tools/bench_module.py --no-reference && \
run remote16 200 taskset -c $R16 python tools/bench_module.py --no-reference && \
run unpinned2 200 python tools/bench_module.py --no-reference
exit $?
