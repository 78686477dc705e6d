# round 3, run g: the module's write threads split by session (cache locality) -- module and
# adapter parity, the module bench with 4 / 8 write threads; a kernel trace of the
# RTSP-interleaved ingest line after the deframe fusions
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03g
mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_qtss_module.py \
  tests/test_gpu_adapter.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAIL|ERROR|passed|failed|Error|threaded:" $O/tests.log | tail -20
[ $rc -ne 0 ] && exit $rc
for w in 4 8; do
  EDGPU_QTSS_WRITE_THREADS=$w timeout -k 10 300 python tools/bench_module.py --no-reference > $O/bench_module_w$w.json 2> $O/bench_module_w$w.err; r=$?
  echo "module bench w=$w rc=$r"; cat $O/bench_module_w$w.json
  [ $r -ne 0 ] && exit $r
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/kt_tcp -o kt -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --ingest tcp > $O/kt_tcp.json 2> $O/kt_tcp.err; r=$?
echo "tcp trace rc=$r"; cat $O/kt_tcp.json
exit $r
