# round 3, run k: module bench after the write threads' per-worker results moved to their own
# cache lines (a per-packet counter shared a line across the write threads); 4 / 8 / 16 write threads
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03k
mkdir -p $O
for w in 4 8 16; do
  EDGPU_QTSS_WRITE_THREADS=$w timeout -k 10 200 python tools/bench_module.py --no-reference > $O/module_w$w.json 2> $O/module_w$w.err; r=$?
  echo "w=$w rc=$r $(python -c "import json;d=json.load(open('$O/module_w$w.json'))['module'];print(d['relayed_per_s'], d['per_tick_ms'])")"
  [ $r -ne 0 ] && exit $r
done
exit 0
