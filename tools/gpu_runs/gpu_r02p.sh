# round 2, run p: interleave parity with the default TCP copy, then fan-out ablation (loads vs stores)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02p
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "interleav" > gpurun_out/r02p/gputest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/r02p/gputest.log | tail -5; [ $rc -ne 0 ] && exit 1
ABL="0 1 4 5 0" bash tools/ab_ablate.sh r02p_abl 10 || { echo ABL_FAIL; exit 1; }
echo ALL_OK
