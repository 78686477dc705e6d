# round 2, run z3: newest-chunks-first work order (EDGPU_FAN_ORDER=1) -- parity subset under
# the order, then A/B against sender-major on C2 (x3) and the C3 shape
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02z3
mkdir -p $O
EDGPU_FAN_ORDER=1 timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "parity or scale or configs or rewrite or random" > $O/gputest.log 2>&1; rc=$?
echo "order-1 tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest.log | tail -5; [ $rc -ne 0 ] && exit $rc
k=0
for o in 0 1 0 1 0 1; do
  k=$((k+1))
  EDGPU_FAN_ORDER=$o timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/o${o}_$k.json 2> $O/o${o}_$k.err || { echo BENCH_FAIL; tail -3 $O/o${o}_$k.err; exit 1; }
done
for o in 0 1; do
  EDGPU_FAN_ORDER=$o timeout -k 10 300 python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --subs 64 > $O/c3_o$o.json 2> $O/c3_o$o.err || { echo BENCH_FAIL; exit 1; }
done
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['roofline']['avg_kernel_ms'], d['roofline']['frac'], d['ms_per_step'], d['kernel_ms'])"; done
echo ALL_OK
