# round 2, run l: new module tests + the bench lines of this round's final code
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "interleaved_pushers" > $O/gputest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest.log | tail -5; [ $rc -ge 124 ] && exit 1
run() { tag=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAIL"; tail -5 $O/$tag.err; exit 1; }; python -c "import json; d=json.load(open('$O/$tag.json')); r=d['roofline']; print('$tag', d['value'], d['ms_per_step'], r['avg_kernel_ms'], r['frac'], r['traffic'], d['kernel_ms'])"; }
run headline
run rewrite --rewrite --no-cpu-baseline
run tcp --ingest tcp --no-cpu-baseline
run c3 --subs 64 --no-cpu-baseline
timeout -k 10 300 python tools/bench_c5.py > $O/c5.json 2> $O/c5.err || { echo C5_FAIL; tail -5 $O/c5.err; exit 1; }; cat $O/c5.json
timeout -k 10 300 python tools/bench_c4.py > $O/c4.json 2> $O/c4.err || { echo C4_FAIL; tail -5 $O/c4.err; exit 1; }; tail -c 600 $O/c4.json
echo ALL_OK
