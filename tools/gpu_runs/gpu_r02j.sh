set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02j
mkdir -p $O
python -c "import sys; sys.path[:0]=['.','tests']; from scenarios import SCENARIOS; SCENARIOS['rtpinfo']().write('$O/rtpinfo.edtr')"
for k in 1; do
  EDGPU_QTSS_DEBUG=1 EDGPU_DEBUG_PLAY=1 EDGPU_TT_OUT=$O/rtpinfo_$k.edtt timeout -k 10 120 ./tools/qtss_replay easydarwin_amd/libQTSSReflectorModule.so $O/rtpinfo.edtr $O/c.edcp > $O/rtpinfo_$k.log 2>&1; rc=$?
  echo "run $k rc=$rc $(sha256sum $O/c.edcp | cut -c1-16) $(tail -1 $O/rtpinfo_$k.log)"; [ $rc -ge 124 ] && exit 1
done
rm -f $O/rtpinfo.edtr $O/c.edcp
exit 0
