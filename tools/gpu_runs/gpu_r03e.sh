# round 3, run e: the module after the push-path lock split (slot reserved under the lock,
# copied outside it; route table shared by pushers) and with parallel QTSS_Write threads:
# module + adapter + random-trace parity, the threaded default mode (with diagnostics), and the
# module bench at C2 with 1 / 4 / 8 write threads; the interleaved-frame slot copy specialised on
# the frame's word offset: interleave + parity tests and the --ingest tcp / desc lines
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03e
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_qtss_module.py \
  tests/test_gpu_adapter.py tests/test_gpu_random.py tests/test_gpu_interleave.py tests/test_gpu_parity.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAIL|ERROR|passed|failed|Error|threaded:" $O/tests.log | tail -40
[ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc
for w in 1 4 8; do
  EDGPU_QTSS_WRITE_THREADS=$w timeout -k 10 300 python tools/bench_module.py $([ $w -ne 4 ] && echo --no-reference) \
    > $O/bench_module_w$w.json 2> $O/bench_module_w$w.err; r=$?
  echo "module bench w=$w rc=$r"; tail -2 $O/bench_module_w$w.err; cat $O/bench_module_w$w.json
  [ $r -ne 0 ] && exit $r
done
for m in tcp desc; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --ingest $m > $O/bench_$m.json 2> $O/bench_$m.err; r=$?
  echo "bench $m rc=$r"; cat $O/bench_$m.json
  [ $r -ne 0 ] && exit $r
done
exit $rc
