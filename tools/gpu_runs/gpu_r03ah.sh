# round 3, run ah: the deferred ingest (packet pass beside the previous fan-out, flat slot copy
# after it): its parity tests and the suites that run it, then A/B bench lines (descriptor and
# RTSP-interleaved ingest, EDGPU_INGEST_DEFER=0 / default) and a kernel trace of the default line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03ah
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_deferred_ingest.py tests/test_gpu_random.py tests/test_gpu_parity.py tests/test_gpu_interleave.py tests/test_gpu_engine_api.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAIL|ERROR|Error" $O/tests.log | head -20; tail -1 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for k in 1 2; do
  for m in desc tcp; do
    for d in 0 1; do
      EDGPU_INGEST_DEFER=$d timeout -k 10 200 python bench.py --no-cpu-baseline --ingest $m > $O/${m}_d${d}_$k.json 2> $O/${m}_d${d}_$k.err; r=$?
      echo "$m defer=$d /$k rc=$r $(python -c "import json;d=json.load(open('$O/${m}_d${d}_$k.json'));print(d['value']/1e9, d['ms_per_step'], d['kernel_ms'])" 2>/dev/null)"
      [ $r -ne 0 ] && exit $r
    done
  done
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/kt -o kt -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/kt.json 2> $O/kt.err; r=$?
echo "kt rc=$r"; grep -h -E "k_ingest|k_fanout|k_keyframe" $O/kt/kt_kernel_stats.csv | cut -d, -f1-5
exit $r
