set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "configs or engine_api" > gpurun_out/r02a_newtests.log 2>&1 || { echo NEWTESTS_FAIL; tail -30 gpurun_out/r02a_newtests.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02a_gputest.log 2>&1 || { echo GPUTEST_FAIL; tail -30 gpurun_out/r02a_gputest.log; exit 1; }
bash tools/ab_fanout.sh r02a_ab 10 20 21 22 10 || { echo AB_FAIL; exit 1; }
echo ALL_OK
