# round 3, run w: module bench A/B in one call -- readback gathered whole before the writes
# (EDGPU_GATHER_SPLIT_BYTES huge) vs in four parts overlapped with the writes (default), 3 each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03w
mkdir -p $O
for k in 1 2 3; do
  for m in whole parts; do
    if [ $m = whole ]; then export EDGPU_GATHER_SPLIT_BYTES=1099511627776; else unset EDGPU_GATHER_SPLIT_BYTES; fi
    timeout -k 10 200 python tools/bench_module.py --no-reference > $O/module_${m}_$k.json 2> $O/module_${m}_$k.err; r=$?
    echo "$m/$k rc=$r $(python -c "import json;d=json.load(open('$O/module_${m}_$k.json'))['module'];print(round(d['relayed_per_s']/1e6,1), round(d['push_s']/d['ticks_timed']*1e3,3), d['per_tick_ms'])")"
    [ $r -ne 0 ] && exit $r
  done
done
exit 0
