# round 2, run z: the dynamic-claim default (variant 31) end to end -- full GPU suite + smoke,
# rocprof kernel trace/stats + PMC passes of the headline, the headline line with its CPU baseline
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02z
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/gputest.log | tail -12; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -2 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
bash tools/profile.sh r02z_prof || { echo PROF_FAIL; exit 1; }
timeout -k 10 400 python bench.py > $O/headline.json 2> $O/headline.err || { echo HEADLINE_FAIL; tail -5 $O/headline.err; exit 1; }
cat $O/headline.json
timeout -k 10 120 ./tools/store_peak5 > $O/store_peak5.json || { echo SP5_FAIL; exit 1; }; cat $O/store_peak5.json
echo ALL_OK
