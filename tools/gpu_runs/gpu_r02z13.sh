# round 2, run z13: k_fanout6 with the patch as per-packet fix-ups (variants 50 / 51): parity of
# 50 over the golden / rewrite / TCP / random / C5-mix tests, then A/B against 40 / 31 on
# identity, with every sub-stream rewriting, and on C5
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02z13
mkdir -p $O
EDGPU_FANOUT=50 timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "parity or scale or configs or rewrite or random or interleave or egress or module or adapter" > $O/gputest50.log 2>&1; rc=$?
echo "v50 tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest50.log | tail -8; [ $rc -ne 0 ] && exit $rc
bash tools/ab_fanout.sh r02z13_ab 40 50 51 31 40 50 || { echo AB_FAIL; exit 1; }
BENCH_EXTRA=--rewrite TAGSUF=_rw bash tools/ab_fanout.sh r02z13_ab 50 51 31 50 51 31 || { echo AB_FAIL; exit 1; }
for v in 31 50 51; do EDGPU_FANOUT=$v timeout -k 10 300 python3 tools/bench_c5.py > $O/c5_v$v.json 2> $O/c5_v$v.err || { echo C5_FAIL; exit 1; }; done
for f in gpurun_out/r02z13_ab/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['roofline']['avg_kernel_ms'], d['roofline']['frac'], d['ms_per_step'])"; done
for f in $O/c5_*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['fanout_kernel'], d['fanout_ms'], d['ms_per_step'])"; done
echo ALL_OK
