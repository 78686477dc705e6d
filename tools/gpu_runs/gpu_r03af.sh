# round 3, run af: the interleaved deframe on its own stream, overlapping the previous tick's
# fan-out (k_ingest waits for it; the deframe waits for the last keyframe index): interleave,
# parity, random-trace and lifecycle tests, then the --ingest tcp line twice and a kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03af
mkdir -p $O
timeout -k 10 500 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_interleave.py \
  tests/test_gpu_parity.py tests/test_gpu_random.py tests/test_gpu_lifecycle.py tests/test_gpu_engine_api.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 $O/tests.log)"; grep -E "FAIL|Error" $O/tests.log | head -10
[ $rc -ne 0 ] && exit $rc
for k in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --ingest tcp > $O/tcp_$k.json 2> $O/tcp_$k.err; r=$?
  echo "tcp/$k rc=$r $(python -c "import json;d=json.load(open('$O/tcp_$k.json'));print(d['value'], d['ms_per_step'], d['kernel_ms'])")"
  [ $r -ne 0 ] && exit $r
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/kt_tcp -o kt -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --ingest tcp > $O/kt_tcp.json 2> $O/kt_tcp.err
