# round 2, run o: DPP-neighbour TCP slot copy -- interleave parity, then A/B on --ingest tcp
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02o
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "interleav" > $O/gputest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest.log | tail -8; [ $rc -ne 0 ] && exit 1
for v in 2; do EDGPU_INGEST_TCP=$v timeout -k 10 300 python bench.py --ingest tcp --no-cpu-baseline > $O/tcp_$v.json 2> $O/tcp_$v.err || { echo BENCH_FAIL; tail -5 $O/tcp_$v.err; exit 1; }; python -c "import json; d=json.load(open('$O/tcp_$v.json')); print('tcp_copy=$v', d['value'], d['ms_per_step'], d['kernel_ms'])"; done
echo ALL_OK
