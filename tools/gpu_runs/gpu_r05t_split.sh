# round 5: the split ingest -- the full GPU suite, then the default and interleaved lines with the
# split ingest and with the fused one (EDGPU_INGEST_SPLIT=0), and a kernel trace of each line.
set -o pipefail
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$R/gpurun_out/${1:-r05t}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rf --timeout 150 --timeout-method thread -p no:cacheprovider > $O/gputests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "FAILED|Timeout" $O/gputests.log | head -20; tail -1 $O/gputests.log
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for ing in desc tcp; do
    for sp in 1 0; do
      EDGPU_INGEST_SPLIT=$sp timeout -k 10 120 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --ingest $ing > $O/${ing}_s${sp}_r$rep.json 2> $O/${ing}_s${sp}_r$rep.err || exit 1
      python3 -c "import json; d=json.load(open('$O/${ing}_s${sp}_r$rep.json')); print('$ing split=$sp r$rep', d['value'], d['ms_per_step'], d['kernel_ms'], d['ingest']['frac'])"
    done
  done
done
for ing in desc tcp; do
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/kt_$ing -o kt -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --ingest $ing > /dev/null 2> $O/kt_$ing.err || exit 1
done
echo done
