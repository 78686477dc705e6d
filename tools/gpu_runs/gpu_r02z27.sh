# round 2, run z27: TCP-frame copy with the frame state in SGPRs (EDGPU_INGEST_TCP=3: two frames
# per round, 4: four at a forced 4 waves/SIMD) against the default (2); interleave parity under 3, 4
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02z27
mkdir -p $O
for m in 3 4; do
  EDGPU_INGEST_TCP=$m timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "interleave or module" > $O/gputest_tcp$m.log 2>&1; rc=$?
  echo "tcp$m tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest_tcp$m.log | tail -3; [ $rc -ne 0 ] && exit $rc
done
for r in 1 2; do
  for m in 2 3 4; do
    EDGPU_INGEST_TCP=$m timeout -k 10 300 python3 bench.py --ingest tcp --no-cpu-baseline > $O/tcp${m}_$r.json 2> $O/tcp${m}_$r.err || { echo FAIL; tail -5 $O/tcp${m}_$r.err; exit 1; }
  done
done
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['kernel_ms']['ingest'])"; done
echo ALL_OK
