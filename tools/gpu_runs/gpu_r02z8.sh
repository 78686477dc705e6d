# round 2, run z8: A/B of the k_fanout6 chunk sizes (31 = default, 40 = 16 packets, 41 = 18,
# 42 = 12, 43 = 16 at 512 threads) on C2 x2, then parity of variant 40 and its rewrite / C3 lines
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02z8
mkdir -p $O
timeout -k 10 120 tools/store_peak6 > $O/store_peak6.json || { echo SP6_FAIL; exit 1; }; cat $O/store_peak6.json
bash tools/ab_fanout.sh r02z8_ab 31 40 41 42 43 31 40 41 42 43 || { echo AB_FAIL; exit 1; }
BENCH_EXTRA=--rewrite TAGSUF=_rw bash tools/ab_fanout.sh r02z8_ab 40 || { echo AB_FAIL; exit 1; }
BENCH_EXTRA="--subs 64" TAGSUF=_c3 bash tools/ab_fanout.sh r02z8_ab 31 40 || { echo AB_FAIL; exit 1; }
for f in gpurun_out/r02z8_ab/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['roofline']['avg_kernel_ms'], d['roofline']['frac'], d['ms_per_step'])"; done
EDGPU_FANOUT=40 timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "parity or scale or configs or rewrite or random or interleave or egress" > $O/gputest40.log 2>&1; rc=$?
echo "v40 tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest40.log | tail -5; [ $rc -ne 0 ] && exit $rc
echo ALL_OK
