# round 5: the interleaved ingest's report read after the deframe (aux stream) instead of after
# k_ingest; frame counts from k_tcp_finish.  Interleave tests, then the tcp and desc lines, then
# the tcp kernel trace.  Logs under gpurun_out/$1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05z2}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_interleave.py tests/test_gpu_engine_api.py tests/test_gpu_random.py tests/test_gpu_passes.py \
    tests/test_gpu_ring_growth.py > $O/gputests.log 2>&1; r=$?
tail -3 $O/gputests.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python bench.py --no-cpu-baseline --ingest tcp > $O/bench_tcp.json 2> $O/bench_tcp.err && \
tail -c 600 $O/bench_tcp.json && \
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_desc.json 2> $O/bench_desc.err && \
tail -c 300 $O/bench_desc.json && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -- python bench.py --no-cpu-baseline --ingest tcp --steps 10 > $O/kt.log 2>&1
exit $?
