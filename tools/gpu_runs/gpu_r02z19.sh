# round 2, run z19: tick pipelining on the RTSP-interleaved push line: the deframe kernels are
# latency-bound, so they might hide under the previous tick's fan-out
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02z19
mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --ingest tcp --no-cpu-baseline > $O/tcp_$r.json 2> $O/tcp_$r.err || { echo FAIL; tail -5 $O/tcp_$r.err; exit 1; }
  timeout -k 10 300 python3 bench.py --ingest tcp --overlap --no-cpu-baseline > $O/tcp_ov_$r.json 2> $O/tcp_ov_$r.err || { echo FAIL; tail -5 $O/tcp_ov_$r.err; exit 1; }
done
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['kernel_ms'])"; done
echo ALL_OK
