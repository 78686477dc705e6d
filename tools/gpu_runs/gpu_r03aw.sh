# round 3, run aw: the module's readback gathered in 8 parts instead of 4 (EDGPU_GATHER_PARTS):
# the module suite with 8 parts, then the module bench 4 vs 8 parts, 6-s runs, three pairs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03aw
mkdir -p $O
EDGPU_GATHER_PARTS=8 timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_qtss_module.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAIL|ERROR" $O/tests.log | head -20; tail -1 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for k in 1 2 3; do
  for g in 4 8; do
    EDGPU_GATHER_PARTS=$g timeout -k 10 300 python tools/bench_module.py --no-reference --seconds 6 > $O/m_g${g}_$k.json 2> $O/m_g${g}_$k.err; r=$?
    echo "parts=$g /$k rc=$r $(python -c "import json;d=json.load(open('$O/m_g${g}_$k.json'))['module'];print(round(d['relayed_per_s']/1e6,1), d['per_tick_ms'])" 2>/dev/null)"
    [ $r -ne 0 ] && exit $r
  done
done
exit 0
