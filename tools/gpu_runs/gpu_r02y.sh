# round 2, run y: dynamic-claim variants head to head (identity x3, rewrite x2), C3 shape, TCP push
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_fanout.sh r02y_ab 31 32 33 34 10 31 32 33 34 31 32 || { echo AB_FAIL; exit 1; }
BENCH_EXTRA=--rewrite TAGSUF=_rw bash tools/ab_fanout.sh r02y_ab 31 32 34 31 32 34 || { echo AB_FAIL; exit 1; }
BENCH_EXTRA="--subs 64" TAGSUF=_c3 bash tools/ab_fanout.sh r02y_ab 10 31 32 || { echo AB_FAIL; exit 1; }
for f in gpurun_out/r02y_ab/*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['roofline']['kernel'], d['roofline']['avg_kernel_ms'], d['roofline']['frac'], d['ms_per_step'])"; done
echo ALL_OK
