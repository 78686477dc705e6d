# round 2, run z11: is the 16-packet chunks' slow patch path the per-lane bitmap test?  A/B of
# 40 (k_fanout6<16>), 46 (k_fanout4<16>), 47 (46 + row-mask patch), 48 / 49 (24 packets, without /
# with row mask) and 31 on identity, with every sub-stream rewriting, and on C5 (TCP patch)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02z11
mkdir -p $O
bash tools/ab_fanout.sh r02z11_ab 40 46 47 48 49 31 40 46 47 48 49 31 || { echo AB_FAIL; exit 1; }
BENCH_EXTRA=--rewrite TAGSUF=_rw bash tools/ab_fanout.sh r02z11_ab 46 47 48 49 31 47 49 31 || { echo AB_FAIL; exit 1; }
for v in 31 47 49; do EDGPU_FANOUT=$v timeout -k 10 300 python3 tools/bench_c5.py > $O/c5_v$v.json 2> $O/c5_v$v.err || { echo C5_FAIL; exit 1; }; done
for f in gpurun_out/r02z11_ab/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['roofline']['avg_kernel_ms'], d['roofline']['frac'], d['ms_per_step'])"; done
for f in $O/c5_*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['fanout_kernel'], d['fanout_ms'], d['ms_per_step'])"; done
echo ALL_OK
