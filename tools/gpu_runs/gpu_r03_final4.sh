# round 3, final run 4 (the tree after timing levels and the module's prestaging): the full GPU
# suite, smoke(), every bench line, and rocprofv3 kernel trace + PMC passes of the default and
# RTSP-interleaved lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03_final4
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests > $O/gputests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "FAIL|ERROR" $O/gputests.log | head -20; tail -1 $O/gputests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rs=$?
echo "smoke rc=$rs"; tail -2 $O/smoke.log
[ $rs -ne 0 ] && exit $rs
run() {   # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err; local r=$?
  echo "$n rc=$r"; head -c 700 $O/$n.json; echo
  return $r
}
run bench_default 500 python bench.py && \
run bench_tcp 500 python bench.py --ingest tcp && \
run bench_rewrite 300 python bench.py --no-cpu-baseline --rewrite && \
run bench_c3 300 python bench.py --no-cpu-baseline --subs 64 && \
run bench_host 300 python bench.py --no-cpu-baseline --ingest host && \
run bench_c5 300 python tools/bench_c5.py && \
run bench_c4 300 python tools/bench_c4.py && \
run bench_module 300 python tools/bench_module.py && \
run bench_module_conc 300 python tools/bench_module.py --no-reference --concurrent-push && \
run bench_egress 300 python tools/bench_egress.py && \
bash tools/profile.sh r03_final4/prof_desc "" && bash tools/profile.sh r03_final4/prof_tcp "--ingest tcp"
exit $?
