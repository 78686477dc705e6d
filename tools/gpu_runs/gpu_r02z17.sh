# round 2, run z17: k_fanout6 at 768 / 896 threads (a C2 window of 16 packets in two fuller
# rows) against the 1024-thread default, C2 identity x2 and rewriting
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_fanout.sh r02z17_ab 40 56 57 58 59 40 56 57 58 59 || { echo AB_FAIL; exit 1; }
BENCH_EXTRA=--rewrite TAGSUF=_rw bash tools/ab_fanout.sh r02z17_ab 31 56 58 || { echo AB_FAIL; exit 1; }
for f in gpurun_out/r02z17_ab/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['roofline']['avg_kernel_ms'], d['roofline']['frac'], d['ms_per_step'])"; done
echo ALL_OK
