#!/bin/bash
# Profiles of the speculative-copy ingest (the new default): the C2 descriptor line and the 100-ms
# line (kernel trace, FETCH_SIZE and WRITE_SIZE passes, tools/profile.sh), smoke(), the tick sweep.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06zh
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
bash tools/profile.sh r06zh/prof_desc > $O/prof_desc.log 2>&1 || exit $?
bash tools/profile.sh r06zh/prof_t100 "--tick-ms 100 --steps 100 --warmup 30" > $O/prof_t100.log 2>&1 || exit $?
bash tools/tick_sweep.sh r06zh/ticks > $O/ticks.log 2>&1 || exit $?
echo done
