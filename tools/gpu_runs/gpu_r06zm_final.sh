#!/bin/bash
# Round 6, the final tree: the whole GPU suite (every golden also with the speculative ingest forced
# on), smoke(), the default line with its CPU baseline, the interleaved line, the 100- and 20-ms lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06zm_final
mkdir -p $O
timeout -k 10 800 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests > $O/gputests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --ingest tcp > $O/bench_tcp.json 2> $O/bench_tcp.err || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --tick-ms 100 --steps 100 --warmup 30 > $O/bench_t100.json 2> $O/bench_t100.err || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --tick-ms 20 --steps 500 --warmup 150 > $O/bench_t20.json 2> $O/bench_t20.err || exit $?
echo done
