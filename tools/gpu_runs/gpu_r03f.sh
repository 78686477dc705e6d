# round 3, run f: interleaved ingest -- emit's read lookup in LDS, the session scan folded into
# k_tcp_resolve and the finish into k_tcp_emit, four frames per k_ingest copy round
# (EDGPU_TCP_TD=4) vs 2 / 3 (A/B libraries, alternating); the module's push path striped by
# session; interleave, random-trace and module parity on the product build; module bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03f
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_interleave.py \
  tests/test_gpu_random.py tests/test_gpu_qtss_module.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAIL|ERROR|passed|failed|Error|threaded:" $O/tests.log | tail -30
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in td4 td2 td3; do
    L=easydarwin_amd/libedgpu.so; [ $v != td4 ] && L=easydarwin_amd/ab/libedgpu_$v.so
    EDGPU_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --ingest tcp > $O/tcp_${v}_$rep.json 2> $O/tcp_${v}_$rep.err; r=$?
    echo "$v/$rep rc=$r $(python -c "import json;d=json.load(open('$O/tcp_${v}_$rep.json'));print(d['kernel_ms'], d['value'])")"
    [ $r -ne 0 ] && exit $r
  done
done
EDGPU_QTSS_WRITE_THREADS=8 timeout -k 10 300 python tools/bench_module.py > $O/bench_module_w8.json 2> $O/bench_module_w8.err; r=$?
echo "module bench rc=$r"; cat $O/bench_module_w8.json
exit $r
