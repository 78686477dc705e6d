# round 2, run r: A/B of tick pipelining (--overlap) and the flat ingest copy kernel (EDGPU_INGEST=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02r
mkdir -p $O
run() { tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAIL"; tail -5 $O/$tag.err; exit 1; }; python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['value'], d['ms_per_step'], d['kernel_ms'])"; }
run base
run overlap --overlap
run base2
run overlap2 --overlap
EDGPU_INGEST=1 run flatcopy
EDGPU_INGEST=1 run flatcopy2
echo ALL_OK
