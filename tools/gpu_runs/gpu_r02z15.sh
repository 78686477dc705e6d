# round 2, run z15: k_fanout6 chunk sizes around the 16-packet optimum (14 / 20 / 22 / 23 against
# 16 and 18) on C2 identity, x2, and with every sub-stream rewriting
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_fanout.sh r02z15_ab 40 52 41 53 54 55 40 52 41 53 54 55 || { echo AB_FAIL; exit 1; }
BENCH_EXTRA=--rewrite TAGSUF=_rw bash tools/ab_fanout.sh r02z15_ab 31 53 54 55 || { echo AB_FAIL; exit 1; }
for f in gpurun_out/r02z15_ab/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['roofline']['avg_kernel_ms'], d['roofline']['frac'], d['ms_per_step'])"; done
echo ALL_OK
