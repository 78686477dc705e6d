# round 3, run ap: the module's batch streamed ahead of the tick (adapter stager +
# edgpu_ingest_prestage): module / adapter / random / lifecycle suites (with the heavy-trace
# prestage test), then the module bench, EDGPU_PRESTAGE_BYTES=0 vs default, 6-s runs, three pairs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03ap
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_qtss_module.py tests/test_gpu_adapter.py tests/test_gpu_random.py tests/test_gpu_lifecycle.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAIL|ERROR" $O/tests.log | head -20; tail -1 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for k in 1 2 3; do
  for p in 0 def; do
    if [ $p = 0 ]; then export EDGPU_PRESTAGE_BYTES=0; else unset EDGPU_PRESTAGE_BYTES; fi
    timeout -k 10 300 python tools/bench_module.py --no-reference --seconds 6 > $O/m_${p}_$k.json 2> $O/m_${p}_$k.err; r=$?
    echo "prestage=$p /$k rc=$r $(python -c "import json;d=json.load(open('$O/m_${p}_$k.json'))['module'];print(round(d['relayed_per_s']/1e6,1), d['per_tick_ms'], d['per_tick_bytes']['prestaged'])" 2>/dev/null)"
    [ $r -ne 0 ] && exit $r
  done
done
exit 0
