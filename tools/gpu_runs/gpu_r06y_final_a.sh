#!/bin/bash
# Round 6 final measurements on the committed tree, part 1: the whole GPU suite, smoke(), the
# default line (with its CPU baseline), the interleaved line, the 100- and 20-ms tick lines with
# their kernel traces and the 100-ms line's PMC passes.  Logs under gpurun_out/r06y_final.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06y_final
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gputests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --ingest tcp > $O/bench_tcp.json 2> $O/bench_tcp.err || exit $?
bash tools/tick_sweep.sh r06y_final/ticks > $O/ticks.log 2>&1 || exit $?
bash tools/profile.sh r06y_final/prof_t100 "--tick-ms 100 --steps 100 --warmup 30" > $O/prof.log 2>&1
