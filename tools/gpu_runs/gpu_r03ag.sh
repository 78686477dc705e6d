# round 3, run ag: how much of k_ingest is its per-round metadata chain and how long a flat copy
# takes on its own (measurement build): kernel traces of the default ingest, EDGPU_INGEST=1 (k_ingest
# writes copy jobs, k_ingest_copy copies over a flat grid) and EDGPU_ABLATE=32 (no slot copy)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export EDGPU_LIB=$GRAFT_REPO_ROOT/easydarwin_amd/ab/libedgpu_ab.so
O=gpurun_out/r03ag
mkdir -p $O
run() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 240 env "$@" rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/$name -o kt -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 $BARGS > $O/$name.json 2> $O/$name.err; local r=$?
  echo "$name rc=$r $(python -c "import json;d=json.load(open('$O/$name.json'));print(d['kernel_ms'], d['ms_per_step'])" 2>/dev/null)"
  grep -h -E "k_ingest|k_tcp|k_fanout" $O/$name/kt_kernel_stats.csv 2>/dev/null | cut -d, -f1-5
  return $r
}
BARGS="" run base EDGPU_INGEST=0 && \
BARGS="" run flat EDGPU_INGEST=1 && \
BARGS="--ablation-study" run nocopy EDGPU_ABLATE=32
