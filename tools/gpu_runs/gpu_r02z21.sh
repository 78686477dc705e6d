# round 2, run z21: four TCP frames per wave round in k_ingest (EDGPU_INGEST_TCP=3, its own
# instantiation) against two (default), --ingest tcp x2; interleave parity under 3
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02z21
mkdir -p $O
EDGPU_INGEST_TCP=3 timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "interleave or module" > $O/gputest_tcp3.log 2>&1; rc=$?
echo "tcp3 tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest_tcp3.log | tail -5; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for m in 2 3; do
    EDGPU_INGEST_TCP=$m timeout -k 10 300 python3 bench.py --ingest tcp --no-cpu-baseline > $O/tcp${m}_$r.json 2> $O/tcp${m}_$r.err || { echo FAIL; tail -5 $O/tcp${m}_$r.err; exit 1; }
  done
done
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['kernel_ms'])"; done
echo ALL_OK
