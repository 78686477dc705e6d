#!/bin/bash
# The committed tree with the libraries as built for the round end: the whole GPU suite, smoke(),
# the default line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06zq_head
mkdir -p $O
timeout -k 10 800 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests > $O/gputests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
echo done
