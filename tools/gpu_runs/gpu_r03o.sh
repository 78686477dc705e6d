# round 3, run o: tick_regions with flat per-sender tables, pinned output buffers grown geometrically; the
# the pinned buffer, large edgpu_copy_to_host reads into pinned memory by a copy kernel): egress,
# adapter, module and engine-API tests, then the module bench (16 write threads) and the egress bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03o
mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_egress.py \
  tests/test_gpu_adapter.py tests/test_gpu_qtss_module.py tests/test_gpu_engine_api.py tests/test_gpu_random.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAIL|ERROR|passed|failed" $O/tests.log | tail -12
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/bench_module.py --no-reference > $O/module_w16.json 2> $O/module_w16.err && \
python -c "import json;d=json.load(open('$O/module_w16.json'))['module'];print(d['relayed_per_s'], d['per_tick_ms'])" && \
timeout -k 10 200 python tools/bench_egress.py > $O/egress.json 2> $O/egress.err && head -c 700 $O/egress.json
