# round 2, run z7: full suite (batched work-item reservations), parity of k_fanout6 (two LDS
# images, one barrier per item; variant 39), then A/B 31 / 39 / 40 on C2 (x3) and with the rewrite
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02z7
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/gputest.log | tail -8; [ $rc -ne 0 ] && exit $rc
EDGPU_FANOUT=39 timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "parity or scale or configs or rewrite or random or interleave or egress" > $O/gputest39.log 2>&1; rc=$?
echo "v39 tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest39.log | tail -5; [ $rc -ne 0 ] && exit $rc
bash tools/ab_fanout.sh r02z7_ab 31 39 40 31 39 40 31 39 40 || { echo AB_FAIL; exit 1; }
BENCH_EXTRA=--rewrite TAGSUF=_rw bash tools/ab_fanout.sh r02z7_ab 31 39 31 39 || { echo AB_FAIL; exit 1; }
BENCH_EXTRA="--subs 64" TAGSUF=_c3 bash tools/ab_fanout.sh r02z7_ab 31 39 || { echo AB_FAIL; exit 1; }
for f in gpurun_out/r02z7_ab/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['roofline']['avg_kernel_ms'], d['roofline']['frac'], d['ms_per_step'], round(d['kernel_ms']['tick_plan_plus_fanout']-d['kernel_ms']['fanout'],4))"; done
echo ALL_OK
