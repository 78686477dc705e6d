# round 3, run ab: module soak -- the module bench at 20-ms ticks for 10 s of virtual time (500
# ticks: push stripes, batch swaps, split gathers and 16 write threads hundreds of times), then
# the threaded-mode parity test five times in a row, and module parity (whole / parts gathers)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03ab
mkdir -p $O
timeout -k 10 400 python tools/bench_module.py --no-reference --seconds 10 --tick-ms 20 > $O/module_soak.json 2> $O/module_soak.err; r=$?
echo "soak rc=$r $(python -c "import json;d=json.load(open('$O/module_soak.json'))['module'];print(d['ticks_timed'], d['relayed_per_s'], d['per_tick_ms'])")"
[ $r -ne 0 ] && exit $r
for k in 1 2 3 4 5; do
  timeout -k 10 200 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu \
    "tests/test_gpu_qtss_module.py::test_module_threaded_default_mode_matches_reference" > $O/threaded_$k.log 2>&1; r=$?
  echo "threaded/$k rc=$r $(tail -1 $O/threaded_$k.log)"
  [ $r -ne 0 ] && exit $r
done
timeout -k 10 300 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_qtss_module.py > $O/module.log 2>&1; r=$?
echo "module rc=$r $(tail -1 $O/module.log)"
exit $r
