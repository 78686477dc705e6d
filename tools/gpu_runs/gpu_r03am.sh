# round 3, run am: edgpu_set_timing -- the bench's timed steps record only the fan-out kernel's
# event pair (the other timings from 3 steps after them): the full GPU suite, smoke, then the
# default and interleaved lines against --all-timing-events (the previous behaviour), 3 pairs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03am
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests > $O/gputests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "FAIL|ERROR" $O/gputests.log | head -20; tail -1 $O/gputests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rs=$?
echo "smoke rc=$rs"; tail -2 $O/smoke.log
[ $rs -ne 0 ] && exit $rs
for k in 1 2 3; do
  for v in all fan; do
    for m in desc tcp; do
      f=""; [ $v = all ] && f="--all-timing-events"
      timeout -k 10 200 python bench.py --no-cpu-baseline --ingest $m $f > $O/${v}_${m}_$k.json 2> $O/${v}_${m}_$k.err; r=$?
      echo "$v $m /$k rc=$r $(python -c "import json;d=json.load(open('$O/${v}_${m}_$k.json'));print(d['ms_per_step'], round(d['value']/1e9,3), d['roofline']['frac'], d['kernel_ms'])" 2>/dev/null)"
      [ $r -ne 0 ] && exit $r
    done
  done
done
exit 0
