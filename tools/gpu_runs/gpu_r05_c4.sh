# round 5: replica / ring-growth / parity GPU tests, then the C4 burst in both layouts and its
# rocprofv3 kernel trace + PMC passes.  Logs under gpurun_out/$1 (default r05j).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05j}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_replica.py tests/test_gpu_ring_growth.py tests/test_gpu_parity.py \
    -v -rf --timeout 150 --timeout-method thread -p no:cacheprovider > $O/gputest.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "FAILED|Timeout" $O/gputest.log | head -20; tail -1 $O/gputest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/bench_c4.py > $O/c4_merged.json 2> $O/c4_merged.err; r=$?
echo "c4 merged rc=$r"; cat $O/c4_merged.json; [ $r -ne 0 ] && exit $r
timeout -k 10 200 python tools/bench_c4.py --contexts 2 > $O/c4_two.json 2> $O/c4_two.err; r=$?
echo "c4 two rc=$r"; cat $O/c4_two.json; [ $r -ne 0 ] && exit $r
bash tools/profile_c4.sh $TAG/prof_c4 && python tools/summarize_pmc_c4.py $O/prof_c4 r05_c4
