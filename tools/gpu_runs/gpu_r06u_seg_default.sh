#!/bin/bash
# The segmented deframe walk as the default: the whole GPU suite, then the interleaved C2 line's
# profile (kernel trace, FETCH_SIZE, WRITE_SIZE passes) and both C2 bench lines.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06u
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gputests.log 2>&1 && \
timeout -k 10 900 bash tools/profile.sh r06u_tcp "--ingest tcp" > $O/profile.log 2>&1 && \
timeout -k 10 200 python bench.py --ingest tcp > $O/bench_tcp.json 2> $O/bench_tcp.err && \
timeout -k 10 200 python bench.py > $O/bench.json 2> $O/bench.err
