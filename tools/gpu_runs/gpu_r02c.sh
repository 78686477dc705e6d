set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "qtss_module" > gpurun_out/r02c_module.log 2>&1; echo "module tests rc=$?"; tail -30 gpurun_out/r02c_module.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not qtss_module" > gpurun_out/r02c_gputest.log 2>&1 || { echo GPUTEST_FAIL; tail -40 gpurun_out/r02c_gputest.log; exit 1; }
tail -3 gpurun_out/r02c_gputest.log
bash tools/ab_fanout.sh r02c_ab 10 26 22 23 24 25 10 || { echo AB_FAIL; exit 1; }
BENCH_EXTRA=--rewrite TAGSUF=_rw bash tools/ab_fanout.sh r02c_ab 10 26 23 25 || { echo AB_FAIL; exit 1; }
for f in gpurun_out/r02c_ab/*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['roofline']['kernel'], d['roofline']['avg_kernel_ms'], d['roofline']['frac'], d['ms_per_step'], d['config']['rewrite'][:8])"; done
echo ALL_OK
