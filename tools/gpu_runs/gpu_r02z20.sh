# round 2, run z20: tick pipelining on the C2 packet-ingest line with the current copy kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02z20
mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/desc_$r.json 2> $O/desc_$r.err || { echo FAIL; tail -5 $O/desc_$r.err; exit 1; }
  timeout -k 10 300 python3 bench.py --overlap --no-cpu-baseline > $O/desc_ov_$r.json 2> $O/desc_ov_$r.err || { echo FAIL; tail -5 $O/desc_ov_$r.err; exit 1; }
done
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['kernel_ms'])"; done
echo ALL_OK
