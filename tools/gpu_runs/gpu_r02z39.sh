# round 2, run z39 (the change it measured was reverted): k_tcp_emit with 4 independent waves (one chunk each) per workgroup instead of
# one-wave workgroups (~16k of them: is the walk's neighbour limited by workgroup slots per CU?)
# vs the r02z38 library (head); interleave / random / module parity under the default and
# interleave parity under head; --ingest tcp x2 each; kernel trace of the default
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02z39
mkdir -p $O
cp easydarwin_amd/libedgpu.so $O/../libedgpu_default.so.bak
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "interleave or random or module" > $O/gputest_default.log 2>&1; rc=$?
echo "default tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest_default.log | tail -3; [ $rc -ne 0 ] && exit $rc
for c in default head; do
  if [ $c = default ]; then cp $O/../libedgpu_default.so.bak easydarwin_amd/libedgpu.so; else cp easydarwin_amd/ab/libedgpu_$c.so easydarwin_amd/libedgpu.so; fi
  if [ $c != default ]; then
    timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "interleave" > $O/gputest_$c.log 2>&1; rc=$?
    echo "$c tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest_$c.log | tail -3; [ $rc -ne 0 ] && exit $rc
  fi
  for r in 1 2; do
    timeout -k 10 300 python3 bench.py --ingest tcp --no-cpu-baseline > $O/tcp_${c}_$r.json 2> $O/tcp_${c}_$r.err || { echo FAIL; tail -5 $O/tcp_${c}_$r.err; exit 1; }
  done
done
cp $O/../libedgpu_default.so.bak easydarwin_amd/libedgpu.so
rm -f $O/../libedgpu_default.so.bak
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/kt -o kt -- python3 bench.py --ingest tcp --no-cpu-baseline --steps 5 --warmup 2 > $O/kt_bench.json 2> $O/kt_bench.err || { echo PROF_FAIL; exit 1; }
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['kernel_ms']['ingest'])"; done
echo ALL_OK
