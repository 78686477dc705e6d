set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05k
timeout -k 10 300 python -u -m pytest tests/test_gpu_replica.py tests/test_gpu_ring_growth.py -q -x --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/r05k/gputest.log 2>&1 || { tail -30 gpurun_out/r05k/gputest.log; exit 1; }
tail -1 gpurun_out/r05k/gputest.log
timeout -k 10 200 python tools/bench_c4.py > gpurun_out/r05k/c4_merged.json 2> gpurun_out/r05k/c4.err || exit $?
head -c 600 gpurun_out/r05k/c4_merged.json; echo
timeout -k 10 400 python tools/bench_module.py --tick-ms 100 > gpurun_out/r05k/bench_module_t100.json 2> gpurun_out/r05k/t100.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/r05k/bench_module_t100.json')); print(d['module']['relayed_per_s'], d.get('module_vs_reference_module'), d.get('module_vs_reference'), d.get('reference_module_push_us_per_packet'), d.get('reference_module_push_vs_harness'), d['reference'].get('push_us_per_packet_per_process'))"
bash tools/gpu_runs/gpu_r05_tcp.sh r05k
