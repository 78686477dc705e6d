# round 3, run ak: what the engine's per-launch timing events cost a step (measurement build):
# the default line with every timing event vs only the fan-out's two (EDGPU_MARKS_FAN_ONLY), 3 pairs
set -o pipefail
# (EDGPU_MARKS_FAN_ONLY was a temporary switch of that build, superseded by edgpu_set_timing: gpu_r03am.sh)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export EDGPU_LIB=$GRAFT_REPO_ROOT/easydarwin_amd/ab/libedgpu_ab.so
O=gpurun_out/r03ak
mkdir -p $O
for k in 1 2 3; do
  for m in 0 1; do
    EDGPU_MARKS_FAN_ONLY=$m timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --warmup 5 > $O/m${m}_$k.json 2> $O/m${m}_$k.err; r=$?
    echo "fan_only=$m /$k rc=$r $(python -c "import json;d=json.load(open('$O/m${m}_$k.json'));print(d['ms_per_step'], d['kernel_ms'])" 2>/dev/null)"
    [ $r -ne 0 ] && exit $r
  done
done
exit 0
