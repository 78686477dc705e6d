# round 2, run z26: where the RTSP-interleaved ingest's extra time goes -- k_ingest with and
# without its slot copy (EDGPU_ABLATE=32, timing only) on --ingest tcp and on packet ingest
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02z26
mkdir -p $O
for m in desc tcp; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/${m}_full -o kt -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --ingest $m > $O/${m}_full.json 2> $O/${m}_full.err || { echo FAIL; exit 1; }
  EDGPU_ABLATE=32 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/${m}_nocopy -o kt -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --ablation-study --ingest $m > $O/${m}_nocopy.json 2> $O/${m}_nocopy.err || { echo FAIL; exit 1; }
done
for d in $O/*_full $O/*_nocopy; do f=$(find $d -name "kt_kernel_stats.csv" | head -1); echo $d; grep -E "k_ingest|k_tcp" $f | cut -d, -f1,2,4; done
echo ALL_OK
