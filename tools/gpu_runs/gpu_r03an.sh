# round 3, run an: the module's batch streamed to the device while it fills (edgpu_ingest_prestage
# from the adapter's stager thread): the adapter / module / random / parity suites, then the
# module bench with EDGPU_PRESTAGE_BYTES=0 (whole-batch copy at the tick) vs the default, both
# push modes, two pairs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03an
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_qtss_module.py tests/test_gpu_adapter.py tests/test_gpu_random.py tests/test_gpu_lifecycle.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAIL|ERROR" $O/tests.log | head -20; tail -1 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for k in 1 2; do
  for p in 0 def; do
    for m in alt conc; do
      f=""; [ $m = conc ] && f="--concurrent-push"
      if [ $p = 0 ]; then export EDGPU_PRESTAGE_BYTES=0; else unset EDGPU_PRESTAGE_BYTES; fi
      timeout -k 10 300 python tools/bench_module.py --no-reference --seconds 4 $f > $O/m_${p}_${m}_$k.json 2> $O/m_${p}_${m}_$k.err; r=$?
      echo "prestage=$p $m /$k rc=$r $(python -c "import json;d=json.load(open('$O/m_${p}_${m}_$k.json'))['module'];print(round(d['relayed_per_s']/1e6,1), d['wall_s'], d['push_s'], d['tick_s'], d['per_tick_ms'])" 2>/dev/null)"
      [ $r -ne 0 ] && exit $r
    done
  done
done
exit 0
