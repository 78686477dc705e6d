# round 2, run z5: full suite (k_ingest's per-socket newest-accepted by atomicMax), parity of the
# two-windows-at-once fan-out (variant 37), then A/B 31 / 37 / 38 on C2 (x3) and with the rewrite
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02z5
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/gputest.log | tail -8; [ $rc -ne 0 ] && exit $rc
EDGPU_FANOUT=37 timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "parity or scale or configs or rewrite or random" > $O/gputest37.log 2>&1; rc=$?
echo "v37 tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest37.log | tail -5; [ $rc -ne 0 ] && exit $rc
bash tools/ab_fanout.sh r02z5_ab 31 37 38 31 37 38 31 37 38 || { echo AB_FAIL; exit 1; }
BENCH_EXTRA=--rewrite TAGSUF=_rw bash tools/ab_fanout.sh r02z5_ab 31 37 31 37 || { echo AB_FAIL; exit 1; }
for f in gpurun_out/r02z5_ab/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['roofline']['avg_kernel_ms'], d['roofline']['frac'], d['ms_per_step'], d['kernel_ms']['ingest'])"; done
echo ALL_OK
