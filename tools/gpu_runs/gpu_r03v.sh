# round 3, run v: module -- FlushIngest's descriptors by a counting sort, the tick's readback
# gathered in four parts by a gather thread while the write threads deliver the earlier parts;
# module parity (whole / parts), adapter, random traces; then the module bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03v
mkdir -p $O
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_qtss_module.py \
  tests/test_gpu_adapter.py tests/test_gpu_random.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAIL|ERROR|passed|failed" $O/tests.log | tail -12
[ $rc -ne 0 ] && exit $rc
for k in 1 2; do
  timeout -k 10 200 python tools/bench_module.py --no-reference > $O/module_$k.json 2> $O/module_$k.err; r=$?
  echo "module/$k rc=$r $(python -c "import json;d=json.load(open('$O/module_$k.json'))['module'];print(d['relayed_per_s'], round(d['push_s']/d['ticks_timed']*1e3,3), d['per_tick_ms'])")"
  [ $r -ne 0 ] && exit $r
done
exit 0
