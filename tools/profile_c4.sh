#!/bin/bash
# rocprofv3 of tools/bench_c4.py (run on the GPU box through gpurun): kernel trace + stats, then one
# PMC pass per counter (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).  Then
# python tools/summarize_pmc_c4.py gpurun_out/<run> <tag> writes profiles/pmc_c4.json.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-prof_c4}
ARGS="${2:-}"
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/kt -o kt -- python3 $R/tools/bench_c4.py $ARGS > $OUT/c4.json 2> $OUT/kt.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv --kernel-include-regex 'k_fanout' -d $OUT/fetch -o fetch -- python3 $R/tools/bench_c4.py $ARGS > $OUT/fetch_c4.json 2> $OUT/fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T --output-format csv --kernel-include-regex 'k_fanout' -d $OUT/write -o write -- python3 $R/tools/bench_c4.py $ARGS > $OUT/write_c4.json 2> $OUT/write.err
echo done
