# round 3, run aj: the drop-in module, 6-s runs, pushers alternating with / concurrent with the
# ticks (two pairs), then one concurrent run next to the reference on the same box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03aj
mkdir -p $O
for k in 1 2; do
  for m in alt conc; do
    f=""; [ $m = conc ] && f="--concurrent-push"
    timeout -k 10 300 python tools/bench_module.py --no-reference --seconds 6 $f > $O/module_${m}_$k.json 2> $O/module_${m}_$k.err; r=$?
    echo "$m /$k rc=$r $(python -c "import json;d=json.load(open('$O/module_${m}_$k.json'))['module'];print(d['relayed_per_s']/1e6, d['wall_s'], d['push_s'], d['tick_s'], d['per_tick_ms'])" 2>/dev/null)"
    [ $r -ne 0 ] && exit $r
  done
done
timeout -k 10 400 python tools/bench_module.py --seconds 6 --concurrent-push > $O/module_conc_ref.json 2> $O/module_conc_ref.err; r=$?
echo "conc+ref rc=$r $(python -c "import json;d=json.load(open('$O/module_conc_ref.json'));print(d['module']['relayed_per_s']/1e6, d.get('reference'), d.get('module_vs_reference'))" 2>/dev/null)"
exit $r
