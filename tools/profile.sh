#!/bin/bash
# Profiling recipe (run on the GPU box through gpurun): kernel trace + stats, then one PMC
# pass per counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-prof}
ARGS="--steps 5 --warmup 2 --no-cpu-baseline ${2:-}"     # $2: extra bench flags, e.g. "--ingest tcp"
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/kt -o kt -- python3 $R/bench.py $ARGS > $OUT/kt_bench.json 2> $OUT/kt_bench.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv --kernel-include-regex 'k_fanout|k_ingest|k_tcp' -d $OUT/fetch -o fetch -- python3 $R/bench.py $ARGS > $OUT/fetch_bench.json 2> $OUT/fetch_bench.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T --output-format csv --kernel-include-regex 'k_fanout|k_ingest|k_tcp' -d $OUT/write -o write -- python3 $R/bench.py $ARGS > $OUT/write_bench.json 2> $OUT/write_bench.err
echo done
