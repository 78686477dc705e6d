#!/bin/bash
# The 20-ms tick line's trace and PMC passes (tools/profile.sh), for the registry bench.py reads
# roofline.traffic from.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r06zo
bash tools/profile.sh r06zo/prof_t20 "--tick-ms 20 --steps 500 --warmup 150" > gpurun_out/r06zo/prof_t20.log 2>&1 || exit $?
echo done
