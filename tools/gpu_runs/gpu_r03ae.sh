# round 3, run ae: k_ingest with 512-thread workgroups (one round per C2 session, two workgroups
# per CU, so the second half of the sessions starts as the first finish) vs the default 256, A/B
# in one call, descriptor and RTSP-interleaved ingest
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03ae
mkdir -p $O
for k in 1 2; do
  for t in 256 512; do
    for m in desc tcp; do
      EDGPU_INGEST_THREADS=$t timeout -k 10 200 python bench.py --no-cpu-baseline --ingest $m > $O/${m}_t${t}_$k.json 2> $O/${m}_t${t}_$k.err; r=$?
      echo "$m t=$t /$k rc=$r $(python -c "import json;d=json.load(open('$O/${m}_t${t}_$k.json'));print(d['kernel_ms']['ingest'], d['ms_per_step'])")"
      [ $r -ne 0 ] && exit $r
    done
  done
done
exit 0
