# round 3, run ai: the drop-in module's throughput with the pushers running while a tick runs
# (EDGPU_BENCH_CONCURRENT_PUSH) against pushing and ticking alternating, two pairs in one call
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03ai
mkdir -p $O
for k in 1 2; do
  for m in alt conc; do
    f=""; [ $m = conc ] && f="--concurrent-push"
    timeout -k 10 300 python tools/bench_module.py --no-reference $f > $O/module_${m}_$k.json 2> $O/module_${m}_$k.err; r=$?
    echo "$m /$k rc=$r $(python -c "import json;d=json.load(open('$O/module_${m}_$k.json'))['module'];print(d['relayed_per_s']/1e6, d['wall_s'], d['push_s'], d['tick_s'], d['per_tick_ms'])" 2>/dev/null)"
    [ $r -ne 0 ] && exit $r
  done
done
exit 0
