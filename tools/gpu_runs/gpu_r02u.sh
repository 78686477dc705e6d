# round 2, run u: k_ingest with 512-thread workgroups (one round per C2 session) -- parity, A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02u
mkdir -p $O
EDGPU_INGEST_THREADS=512 timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "(engine_matches_reference and serial) or interleaved_push or random or pinned" > $O/gputest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest.log | tail -4; [ $rc -ne 0 ] && exit 1
run() { tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAIL"; tail -5 $O/$tag.err; exit 1; }; python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['value'], d['ms_per_step'], d['kernel_ms'])"; }
run t256
EDGPU_INGEST_THREADS=512 run t512
run t256b
EDGPU_INGEST_THREADS=512 run t512b
EDGPU_INGEST_THREADS=512 run t512tcp --ingest tcp
run t256tcp --ingest tcp
echo ALL_OK
