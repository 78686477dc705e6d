# round 5: the interleaved ingest enqueues k_ingest after the host has read the deframe's report
# (no cross-stream wait on the context stream).  Interleave tests, the tcp and desc lines, then
# the tcp profile (kernel trace + FETCH/WRITE passes).  Logs under gpurun_out/$1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05z3}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_interleave.py tests/test_gpu_engine_api.py tests/test_gpu_random.py tests/test_gpu_passes.py \
    tests/test_gpu_ring_growth.py tests/test_gpu_qtss_module.py > $O/gputests.log 2>&1; r=$?
tail -3 $O/gputests.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python bench.py --no-cpu-baseline --ingest tcp > $O/bench_tcp.json 2> $O/bench_tcp.err && \
tail -c 300 $O/bench_tcp.json && \
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_desc.json 2> $O/bench_desc.err && \
tail -c 200 $O/bench_desc.json && \
bash tools/profile.sh $TAG/prof_tcp "--ingest tcp" > $O/prof.log 2>&1
exit $?
