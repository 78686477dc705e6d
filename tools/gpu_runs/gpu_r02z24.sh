# round 2, run z24: is the 16-packet patch path's cost the patch arithmetic or the bytes?  The
# same patch path with an SSRC override equal to the stream's own SSRC (identity bytes)
set -o pipefail
cd $GRAFT_REPO_ROOT
BENCH_EXTRA=--rewrite-same-ssrc TAGSUF=_same bash tools/ab_fanout.sh r02z24_ab 40 31 40 31 || { echo AB_FAIL; exit 1; }
BENCH_EXTRA=--rewrite TAGSUF=_rw bash tools/ab_fanout.sh r02z24_ab 40 31 || { echo AB_FAIL; exit 1; }
bash tools/ab_fanout.sh r02z24_ab 40 31 || { echo AB_FAIL; exit 1; }
for f in gpurun_out/r02z24_ab/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['roofline']['avg_kernel_ms'], d['roofline']['frac'], d['ms_per_step'], d['config']['rewrite'][:20])"; done
echo ALL_OK
