#!/bin/bash
# Calibrates FETCH_SIZE for narrow loads (tools/fetch_calib.hip) and reads the raw TCC request
# counters of the interleaved ingest chain and of the descriptor ingest.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06o_calib
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $R
RAW="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_DRAM_sum"
timeout -k 10 120 tools/fetch_calib 4 10 > $O/time.jsonl 2> $O/time.err && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/p_fetch -o f -- tools/fetch_calib 4 2 > /dev/null 2> $O/p_fetch.err && \
timeout -s KILL 120 rocprofv3 --pmc $RAW -T --output-format csv -d $O/p_raw -o r -- tools/fetch_calib 4 2 > /dev/null 2> $O/p_raw.err && \
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -T --output-format csv -d $O/p_hit -o h -- tools/fetch_calib 4 2 > /dev/null 2> $O/p_hit.err && \
timeout -s KILL 180 rocprofv3 --pmc $RAW -T --output-format csv --kernel-include-regex 'k_ingest|k_tcp' -d $O/tcp_raw -o r -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --ingest tcp > $O/tcp_raw.json 2> $O/tcp_raw.err && \
timeout -s KILL 180 rocprofv3 --pmc $RAW -T --output-format csv --kernel-include-regex 'k_ingest' -d $O/desc_raw -o r -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/desc_raw.json 2> $O/desc_raw.err
