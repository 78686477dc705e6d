# round 5: k_ingest's per-sender scans in one pass (DPP wave scans, one barrier) instead of a block
# scan per sender and per track.  The whole GPU suite, the descriptor and interleaved lines, and
# the header phase alone (measurement build, slot copy skipped).  Logs under gpurun_out/$1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05zd}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 150 --timeout-method thread -p no:cacheprovider -m gpu -x tests > $O/gputests.log 2>&1; rc=$?
tail -2 $O/gputests.log; [ $rc -eq 0 ] || exit $rc
for ing in desc tcp; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --ingest $ing > $O/bench_$ing.json 2> $O/bench_$ing.err || exit $?
  python -c "
import json; d=json.loads(open('$O/bench_$ing.json').read().strip().splitlines()[-1])
print('$ing', round(d['value']/1e9,3), d['ms_per_step'], 'ingest', d['ingest']['avg_ms'], d['ingest']['frac'], 'fanout', d['roofline']['avg_kernel_ms'])"
done
EDGPU_LIB=$GRAFT_REPO_ROOT/easydarwin_amd/ab/libedgpu_ab.so EDGPU_ABLATE=32 timeout -k 10 200 python bench.py --no-cpu-baseline --ablation-study > $O/hdr_only.json 2> $O/hdr_only.err || exit $?
python -c "
import json; d=json.loads(open('$O/hdr_only.json').read().strip().splitlines()[-1]); print('header phase alone', d['ingest']['avg_ms'])"
