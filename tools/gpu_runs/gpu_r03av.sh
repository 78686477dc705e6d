# round 3, run av: the shipped library with the ingest experiments moved to the measurement
# build (k_ingest<4,256> only): the GPU suite and the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03av
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests > $O/gputests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "FAIL|ERROR" $O/gputests.log | head -20; tail -1 $O/gputests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err; rb=$?
echo "bench rc=$rb $(python -c "import json;d=json.load(open('$O/bench.json'));print(d['value']/1e9, d['ms_per_step'], d['kernel_ms'])")"
exit $rb
