# round 2, run x: dynamic work-item claiming (variants 31, 32) -- parity, then A/B vs 10
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02x
mkdir -p $O
for v in 31 32; do
  EDGPU_FANOUT=$v timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "(engine_matches_reference) or rewrite or random or configs" > $O/gputest_$v.log 2>&1; rc=$?
  echo "variant $v tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest_$v.log | tail -4; [ $rc -ne 0 ] && exit 1
done
bash tools/ab_fanout.sh r02x_ab 10 31 32 10 31 32 || { echo AB_FAIL; exit 1; }
BENCH_EXTRA=--rewrite TAGSUF=_rw bash tools/ab_fanout.sh r02x_ab 10 31 || { echo AB_FAIL; exit 1; }
for f in gpurun_out/r02x_ab/*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['roofline']['kernel'], d['roofline']['avg_kernel_ms'], d['roofline']['frac'], d['ms_per_step'])"; done
echo ALL_OK
