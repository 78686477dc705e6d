# round 3, final run C: rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of the default
# and the RTSP-interleaved line (tools/profile.sh), summarised into profiles/ afterwards
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/profile.sh r03_final/prof_desc "" && bash tools/profile.sh r03_final/prof_tcp "--ingest tcp"
