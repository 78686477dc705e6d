# round 2, run g: module transmit-time debugging + instrumented bisect (small outputs only)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02g
mkdir -p $O
fatal() { [ $1 -ge 124 ]; }
for n in tiny backpressure; do
  python -c "import sys; sys.path[:0]=['.','tests']; from scenarios import SCENARIOS; SCENARIOS['$n']().write('$O/$n.edtr')"
  EDGPU_TT_OUT=$O/$n.edtt timeout -k 10 120 ./tools/qtss_replay easydarwin_amd/libQTSSReflectorModule.so $O/$n.edtr $O/$n.edcp > $O/$n.log 2>&1; rc=$?
  echo "$n rc=$rc"; tail -3 $O/$n.log; fatal $rc && exit 1
  rm -f $O/$n.edtr
done
VARIANTS="Bi" RUNS=30 timeout -k 10 300 bash tools/fpi_bisect.sh > $O/bisect.jsonl 2>&1; rc=$?; cat $O/bisect.jsonl; fatal $rc && exit 1
du -sh gpurun_out
echo ALL_OK
