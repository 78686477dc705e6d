# round 3, run b: session lifecycle (edgpu_session_remove, repush golden through the engine,
# pinned ingest, interleaved push and the adapter), then the whole GPU suite, smoke and the
# default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lifecycle.py \
  "tests/test_gpu_parity.py::test_engine_matches_reference[repush-serial]" \
  "tests/test_gpu_parity.py::test_engine_matches_reference[repush-overlap]" \
  "tests/test_gpu_parity.py::test_pinned_host_ingest_matches_reference[repush]" \
  "tests/test_gpu_adapter.py" > $O/lifecycle.log 2>&1; rc=$?
echo "lifecycle tests rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" $O/lifecycle.log | tail -40
[ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/gputest.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest.log | tail -12; [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -2 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic_source'], d['cpu_baseline']['value'])"
echo ALL_OK
