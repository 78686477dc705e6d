# round 2, run z9: why is k_fanout6<1024,16> (variant 40) slow with the rewrite stage?  A/B of
# 31 / 40 / 44 (40 at one workgroup per CU) / 45 (18 packets, one per CU) / 39 with every
# sub-stream rewriting and on identity, and C5 (half the sub-streams TCP: channel-byte patch)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02z9
mkdir -p $O
BENCH_EXTRA=--rewrite TAGSUF=_rw bash tools/ab_fanout.sh r02z9_ab 31 40 44 45 39 31 40 44 45 || { echo AB_FAIL; exit 1; }
bash tools/ab_fanout.sh r02z9_ab 31 40 44 45 31 40 44 45 || { echo AB_FAIL; exit 1; }
for v in 31 40 44; do EDGPU_FANOUT=$v timeout -k 10 300 python3 tools/bench_c5.py > $O/c5_v$v.json 2> $O/c5_v$v.err || { echo C5_FAIL; exit 1; }; done
for f in gpurun_out/r02z9_ab/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['roofline']['avg_kernel_ms'], d['roofline']['frac'], d['ms_per_step'])"; done
for f in $O/c5_*.json; do echo $f; cut -c1-600 $f; done
echo ALL_OK
