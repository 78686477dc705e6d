# round 3, run ad: the fan-out's dynamic-schedule tail, measured (measurement build: each
# k_fanout6 workgroup's start / exit by s_memrealtime; EDGPU_FAN_TAIL=1 prints the last tick's
# span and first exit; and the same for k_ingest), C2 and C3's per-GPU shape
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03ad
mkdir -p $O
export EDGPU_LIB=easydarwin_amd/ab/libedgpu_ab.so EDGPU_FAN_TAIL=1
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/c2.json 2> $O/c2.err && grep "fan tail" $O/c2.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --subs 64 > $O/c3.json 2> $O/c3.err && grep "fan tail" $O/c3.err && \
python -c "
import json
for n in ['c2','c3']:
    d=json.load(open('$O/'+n+'.json')); print(n, d['kernel_ms'])"
