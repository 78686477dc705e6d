# round 2, run z18: FanSub records loaded one window ahead (variants 60 / 61) against 40 / 31,
# identity and rewriting, C2; then the parity subset under 60
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02z18
mkdir -p $O
bash tools/ab_fanout.sh r02z18_ab 40 60 31 61 40 60 31 61 || { echo AB_FAIL; exit 1; }
BENCH_EXTRA=--rewrite TAGSUF=_rw bash tools/ab_fanout.sh r02z18_ab 40 60 31 61 60 61 || { echo AB_FAIL; exit 1; }
for f in gpurun_out/r02z18_ab/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['roofline']['avg_kernel_ms'], d['roofline']['frac'], d['ms_per_step'])"; done
EDGPU_FANOUT=60 timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "parity or scale or configs or rewrite or random or interleave or egress" > $O/gputest60.log 2>&1; rc=$?
echo "v60 tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest60.log | tail -5; [ $rc -ne 0 ] && exit $rc
echo ALL_OK
