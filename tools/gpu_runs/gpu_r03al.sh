# round 3, run al: timing events recorded by the kernels' own dispatches (hipExtLaunchKernel)
# instead of separate event markers: the engine API tests, then the default and interleaved lines
# against the previous library (easydarwin_amd/ab_base, built from the parent commit), 3 pairs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03al
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine_api.py tests/test_gpu_parity.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAIL|ERROR" $O/tests.log | head; tail -1 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for k in 1 2 3; do
  for v in base new; do
    for m in desc tcp; do
      if [ $v = base ]; then L=$GRAFT_REPO_ROOT/easydarwin_amd/ab_base/libedgpu.so; else L=$GRAFT_REPO_ROOT/easydarwin_amd/libedgpu.so; fi
      EDGPU_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --ingest $m --steps 30 --warmup 5 > $O/${v}_${m}_$k.json 2> $O/${v}_${m}_$k.err; r=$?
      echo "$v $m /$k rc=$r $(python -c "import json;d=json.load(open('$O/${v}_${m}_$k.json'));print(d['ms_per_step'], round(d['value']/1e9,3), d['kernel_ms'])" 2>/dev/null)"
      [ $r -ne 0 ] && exit $r
    done
  done
done
exit 0
