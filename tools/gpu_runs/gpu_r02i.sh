set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02i
mkdir -p $O
python -c "import sys; sys.path[:0]=['.','tests']; from scenarios import SCENARIOS; SCENARIOS['rtpinfo']().write('$O/rtpinfo.edtr')"
EDGPU_TT_OUT=$O/rtpinfo.edtt timeout -k 10 120 ./tools/qtss_replay easydarwin_amd/libQTSSReflectorModule.so $O/rtpinfo.edtr $O/rtpinfo.edcp > $O/rtpinfo.log 2>&1; rc=$?
rm -f $O/rtpinfo.edtr $O/rtpinfo.edcp
echo rc=$rc; tail -3 $O/rtpinfo.log; exit $rc
