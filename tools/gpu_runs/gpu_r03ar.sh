# round 3, run ar: fan-out chunk size on C3's per-GPU shape (1024 x 64 subs), measurement build:
# k_fanout6 with 16 (default, variant 40), 32 (39), 18 (41), 12 (42) and 20 (53) packets per item, two passes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export EDGPU_LIB=$GRAFT_REPO_ROOT/easydarwin_amd/ab/libedgpu_ab.so
O=gpurun_out/r03ar
mkdir -p $O
for k in 1 2; do
  for v in 40 39 41 42 53; do
    EDGPU_FANOUT=$v timeout -k 10 200 python bench.py --no-cpu-baseline --subs 64 > $O/v${v}_$k.json 2> $O/v${v}_$k.err; r=$?
    echo "v$v /$k rc=$r $(python -c "import json;d=json.load(open('$O/v${v}_$k.json'));print(d['ms_per_step'], d['kernel_ms']['fanout'], d['roofline']['frac'], d['roofline']['kernel'])" 2>/dev/null)"
    [ $r -ne 0 ] && exit $r
  done
done
exit 0
