# round 3, run y: C4 burst with the bench's host bookkeeping out of the timed region (and the
# binding's per-session track counts cached); replica / multi-process tests (session images);
# FETCH_SIZE / WRITE_SIZE passes of the C5 fan-out (tools/summarize_pmc_c5.py afterwards)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03y
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_replica.py \
  tests/test_gpu_multiprocess.py tests/test_gpu_configs.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 $O/tests.log)"
[ $rc -ne 0 ] && exit $rc
for k in 1 2; do
  timeout -k 10 300 python tools/bench_c4.py > $O/c4_$k.json 2> $O/c4_$k.err; r=$?
  echo "c4/$k rc=$r $(python -c "import json;d=json.load(open('$O/c4_$k.json'));print({k:d[k] for k in ['burst_ms','image_export_copy_import_ms','join_calls_ms','burst_fanout_ms']})")"
  [ $r -ne 0 ] && exit $r
done
mkdir -p $O/c5pmc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv --kernel-include-regex 'k_fanout' -d $O/c5pmc/fetch -o fetch \
  -- python3 tools/bench_c5.py > $O/c5pmc/c5.json 2> $O/c5pmc/fetch.err && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T --output-format csv --kernel-include-regex 'k_fanout' -d $O/c5pmc/write -o write \
  -- python3 tools/bench_c5.py > $O/c5pmc/c5_write.json 2> $O/c5pmc/write.err
