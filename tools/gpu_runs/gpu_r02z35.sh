# round 2, run z35: verification of the committed tree after the two-chunks-per-wave RTSP-interleaved walk --
# full suite + smoke, headline profile (kernel trace + PMC),
# the headline with its CPU baseline, and the other bench lines of this round's final code
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02z35
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/gputest.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -2 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
bash tools/profile.sh r02z35_prof || { echo PROF_FAIL; exit 1; }
run() { tag=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAIL"; tail -5 $O/$tag.err; exit 1; }; python -c "import json; d=json.load(open('$O/$tag.json')); r=d['roofline']; print('$tag', d['value'], d['ms_per_step'], r['avg_kernel_ms'], r['frac'], r['traffic'], d['kernel_ms'])"; }
run headline
run rewrite --rewrite --no-cpu-baseline
run tcp --ingest tcp --no-cpu-baseline
run c3 --subs 64 --no-cpu-baseline
run host --ingest host --no-cpu-baseline --steps 6 --warmup 2
run tcp_overlap --ingest tcp --overlap --no-cpu-baseline
timeout -k 10 300 python tools/bench_c5.py > $O/c5.json 2> $O/c5.err || { echo C5_FAIL; tail -5 $O/c5.err; exit 1; }; tail -c 400 $O/c5.json
timeout -k 10 300 python tools/bench_c4.py > $O/c4.json 2> $O/c4.err || { echo C4_FAIL; tail -5 $O/c4.err; exit 1; }; tail -c 400 $O/c4.json
echo ALL_OK
