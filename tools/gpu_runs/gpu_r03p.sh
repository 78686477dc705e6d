# round 3, run p: module bench with the replay's clock advanced once per frame (it was a CAS on
# one shared line per packet), 8 and 16 pusher threads
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03p
mkdir -p $O
for t in 8 16; do
  timeout -k 10 200 python tools/bench_module.py --no-reference --threads $t > $O/module_p$t.json 2> $O/module_p$t.err; r=$?
  echo "pushers=$t rc=$r $(python -c "import json;d=json.load(open('$O/module_p$t.json'))['module'];print(d['relayed_per_s'], round(d['push_s']/d['ticks_timed']*1e3,3), d['per_tick_ms'])")"
  [ $r -ne 0 ] && exit $r
done
exit 0
