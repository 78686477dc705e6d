# round 2, run z16: kernel trace of the RTSP-interleaved push line (--ingest tcp)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02z16
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/kt -o kt -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --ingest tcp > $O/kt_bench.json 2> $O/kt_bench.err || { echo PROF_FAIL; tail -5 $O/kt_bench.err; exit 1; }
f=$(find $O/kt -name "kt_kernel_stats.csv" | head -1); cut -d, -f1-8 $f | head -20
echo ALL_OK
