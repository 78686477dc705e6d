# round 3, run c: the QTSS module with session lifecycle (repush) and in its default threaded
# mode, random differential traces with lifecycle (engine, interleaved, adapter, module), the
# interleaved-push repush, replica skips; two engine processes (shards, image exchange); UDP
# overload ordering; bench.py's RCCL path at world 1; the module bench at C2 scale
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_qtss_module.py \
  tests/test_gpu_random.py tests/test_gpu_multiprocess.py \
  "tests/test_gpu_interleave.py::test_interleaved_push_matches_reference[1-repush]" \
  "tests/test_gpu_interleave.py::test_interleaved_push_matches_reference[2-repush]" \
  "tests/test_gpu_interleave.py::test_interleaved_push_matches_reference[1-threaded]" \
  "tests/test_gpu_egress.py::test_udp_overload_loses_datagrams_without_reordering" \
  tests/test_gpu_replica.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAIL|ERROR|passed|failed|Error" $O/tests.log | tail -30
[ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc
EDGPU_BENCH_FORCE_PG=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline \
  > $O/bench_rccl_world1.json 2> $O/bench_rccl_world1.err; rc2=$?
echo "rccl world-1 bench rc=$rc2"; tail -2 $O/bench_rccl_world1.err; head -c 400 $O/bench_rccl_world1.json; echo
[ $rc2 -eq 124 ] || [ $rc2 -eq 137 ] && exit $rc2
EDGPU_QTSS_ARENA_MB=2048 EDGPU_QTSS_MAX_OUT_PACKETS=2000000 timeout -k 10 300 tools/qtss_replay \
  easydarwin_amd/libQTSSReflectorModule.so --bench 1024 16 3 100 8 > $O/bench_module_c2.json 2> $O/bench_module_c2.err; rc3=$?
echo "module bench rc=$rc3"; tail -3 $O/bench_module_c2.err; cat $O/bench_module_c2.json
exit $(( rc || rc2 || rc3 ))
