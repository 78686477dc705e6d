# round 2, run e: full GPU suite, the r01 intermittent bisect, profiles + PMC, bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02e
mkdir -p $O
fatal() { [ $1 -ge 124 ]; }          # timeout / abort / segfault: stop using the GPU
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -5 $O/gputest.log; fatal $rc && exit 1
timeout -k 10 400 bash tools/fpi_bisect.sh > $O/bisect.jsonl 2>&1; rc=$?; cat $O/bisect.jsonl; fatal $rc && exit 1
bash tools/profile.sh r02e_prof || { echo PROF_FAIL; exit 1; }
python tools/summarize_profile.py gpurun_out/r02e_prof r02e || echo SUMMARY_FAIL
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -T --output-format csv -d $O/host_kt -o kt -- python3 bench.py --ingest host --steps 6 --warmup 2 --no-cpu-baseline > $O/bench_host.json 2> $O/bench_host.err || { echo HOST_FAIL; tail -20 $O/bench_host.err; exit 1; }
cat $O/bench_host.json
for d in 0 1; do timeout -k 10 300 python tools/bench_egress.py --dedup $d > $O/egress_dedup$d.json 2> $O/egress_dedup$d.err || { echo EGRESS_FAIL; tail -20 $O/egress_dedup$d.err; exit 1; }; cat $O/egress_dedup$d.json; done
echo ALL_OK
