# round 3, run r: k_ingest finds the interleaved frames itself (chunk from the per-chunk frame ends, start
# from the walk records, length and channel from the header) -- the per-chunk emit replaced by a per-session
# k_tcp_finish; interleave + random + module parity, the --ingest tcp line twice, a kernel trace of it
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03r
mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_interleave.py \
  tests/test_gpu_random.py tests/test_gpu_qtss_module.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAIL|ERROR|passed|failed|Error" $O/tests.log | tail -20
[ $rc -ne 0 ] && exit $rc
for k in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --ingest tcp > $O/tcp_$k.json 2> $O/tcp_$k.err; r=$?
  echo "tcp/$k rc=$r $(python -c "import json;d=json.load(open('$O/tcp_$k.json'));print(d['kernel_ms'], d['value'])")"
  [ $r -ne 0 ] && exit $r
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/kt_tcp -o kt -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --ingest tcp > $O/kt_tcp.json 2> $O/kt_tcp.err; r=$?
echo "tcp trace rc=$r"
exit $r
