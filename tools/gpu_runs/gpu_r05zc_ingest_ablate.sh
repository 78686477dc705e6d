# round 5: where k_ingest's time goes -- the measurement build with the per-sender scans skipped
# -- measured, but it leaves the rings inconsistent and the engine stops --, the slot copy skipped (32), descriptor and interleaved lines.
# Timing experiments only (--ablation-study: the lines say so).  Logs under gpurun_out/$1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05zc}
O=gpurun_out/$TAG
mkdir -p $O
export EDGPU_LIB=$GRAFT_REPO_ROOT/easydarwin_amd/ab/libedgpu_ab.so
for ing in desc tcp; do
  for abl in 0 32; do
    n=${ing}_abl$abl
    if [ $abl = 0 ]; then unset EDGPU_ABLATE; else export EDGPU_ABLATE=$abl; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --ablation-study --ingest $ing > $O/$n.json 2> $O/$n.err || exit $?
    python -c "
import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1])
print('$n', d['ms_per_step'], 'ingest', d['ingest']['avg_ms'], 'fanout', d['roofline']['avg_kernel_ms'])"
  done
done
exit 0
