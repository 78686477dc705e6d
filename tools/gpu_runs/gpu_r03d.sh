# round 3, run d: run c's tests again (the interleaved-push selections by -k); the module bench
# at C2 scale next to the reference (tools/bench_module.py); the RTSP-interleaved ingest line:
# kernel trace + FETCH_SIZE / WRITE_SIZE passes (tools/profile.sh), one SQ pass of k_ingest and
# the deframe kernels in both ingest modes, and the --ingest tcp bench line with its CPU baseline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03d
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_qtss_module.py \
  tests/test_gpu_random.py tests/test_gpu_multiprocess.py tests/test_gpu_replica.py \
  tests/test_gpu_interleave.py -k "not test_interleaved_push_matches_reference or repush or threaded" \
  "tests/test_gpu_egress.py::test_udp_overload_loses_datagrams_without_reordering" > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAIL|ERROR|passed|failed|Error" $O/tests.log | tail -30
[ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc
timeout -k 10 400 python tools/bench_module.py > $O/bench_module_c2.json 2> $O/bench_module_c2.err; rc3=$?
echo "module bench rc=$rc3"; tail -3 $O/bench_module_c2.err; cat $O/bench_module_c2.json
[ $rc3 -eq 124 ] || [ $rc3 -eq 137 ] && exit $rc3
timeout -k 10 900 bash tools/profile.sh r03d/tcp "--ingest tcp"; rc4=$?
echo "tcp profile rc=$rc4"
[ $rc4 -ne 0 ] && exit $rc4
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
for m in tcp desc; do
  timeout -k 10 120 rocprofv3 --pmc $SQ -T --output-format csv --kernel-include-regex 'k_ingest|k_tcp' -d $O/sq_$m -o sq \
    -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --ingest $m > $O/sq_$m.json 2> $O/sq_$m.err; r=$?
  echo "sq $m rc=$r"; [ $r -ne 0 ] && exit $r
done
timeout -k 10 400 python bench.py --ingest tcp > $O/bench_tcp.json 2> $O/bench_tcp.err; rc5=$?
echo "tcp bench rc=$rc5"; cat $O/bench_tcp.json
exit $(( rc || rc3 || rc5 ))
