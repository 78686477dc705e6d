# round 3, run c: the QTSS module with session lifecycle (repush) and in its default threaded
# mode (tick thread + UDP reader + two pusher threads), interleaved-push repush, replica skips
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c
mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 150 --timeout-method thread -m gpu tests/test_gpu_qtss_module.py \
  "tests/test_gpu_interleave.py::test_interleaved_push_matches_reference[1-repush]" \
  "tests/test_gpu_interleave.py::test_interleaved_push_matches_reference[2-repush]" \
  "tests/test_gpu_interleave.py::test_interleaved_push_matches_reference[1-threaded]" \
  tests/test_gpu_replica.py > $O/module.log 2>&1; rc=$?
echo "module tests rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed|SKIP" $O/module.log | tail -60
exit $rc
