# round 5: the C4 burst (tools/bench_c4.py) through the measurement build's fan-out variants
# (EDGPU_FANOUT), the default k_fanout6<1024,16,nt,dyn> first and last.  Logs under gpurun_out/$1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05zi}
O=gpurun_out/$TAG
mkdir -p $O
export EDGPU_LIB=$GRAFT_REPO_ROOT/easydarwin_amd/ab/libedgpu_ab.so
for v in 40 39 53 41 44 51 32 31 40; do
  EDGPU_FANOUT=$v timeout -k 10 200 python tools/bench_c4.py > $O/c4_v$v.json 2> $O/c4_v$v.err || exit $?
  python -c "
import json; d=json.load(open('$O/c4_v$v.json')); r=d['roofline']
print('$v', r['kernel'], 'burst copy', d.get('copy_ms'), 'frac', r['frac'], 'end to end', d['burst_ms'])"
done
