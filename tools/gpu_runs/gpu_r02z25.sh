# round 2, run z25: the patch as a divergent branch on the slot-start test (variants 62 / 63)
# against 40 / 31: identity, rewriting, C5; parity of 62 over the rewrite / TCP / golden tests
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02z25
mkdir -p $O
EDGPU_FANOUT=62 timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "parity or rewrite or random or interleave or egress or module or adapter or configs" > $O/gputest62.log 2>&1; rc=$?
echo "v62 tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest62.log | tail -5; [ $rc -ne 0 ] && exit $rc
BENCH_EXTRA=--rewrite TAGSUF=_rw bash tools/ab_fanout.sh r02z25_ab 40 62 31 63 40 62 31 63 || { echo AB_FAIL; exit 1; }
bash tools/ab_fanout.sh r02z25_ab 40 62 31 63 || { echo AB_FAIL; exit 1; }
for v in 31 62 63; do EDGPU_FANOUT=$v timeout -k 10 300 python3 tools/bench_c5.py > $O/c5_v$v.json 2> $O/c5_v$v.err || { echo C5_FAIL; exit 1; }; done
for f in gpurun_out/r02z25_ab/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['roofline']['avg_kernel_ms'], d['roofline']['frac'], d['ms_per_step'])"; done
for f in $O/c5_*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['fanout_kernel'], d['fanout_ms'], d['ms_per_step'])"; done
echo ALL_OK
