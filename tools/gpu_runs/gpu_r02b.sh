set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "configs or engine_api or rewrite" > gpurun_out/r02b_newtests.log 2>&1 || { echo NEWTESTS_FAIL; tail -40 gpurun_out/r02b_newtests.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02b_gputest.log 2>&1 || { echo GPUTEST_FAIL; tail -30 gpurun_out/r02b_gputest.log; exit 1; }
tail -3 gpurun_out/r02b_gputest.log
bash tools/ab_fanout.sh r02b_ab 10 20 21 22 10 || { echo AB_FAIL; exit 1; }
timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --rewrite > gpurun_out/r02b_ab/rewrite.json 2> gpurun_out/r02b_ab/rewrite.err || { echo RW_FAIL; exit 1; }
timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/r02b_ab/identity.json 2> gpurun_out/r02b_ab/identity.err || { echo ID_FAIL; exit 1; }
for f in gpurun_out/r02b_ab/*.json; do echo $f; python -c "import json,sys; d=json.load(open('$f')); print(d['roofline']['kernel'], d['roofline']['avg_kernel_ms'], d['roofline']['frac'], d['ms_per_step'], d['value'])"; done
echo ALL_OK
