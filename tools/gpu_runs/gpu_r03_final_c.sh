# round 3, final run C: rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes (tools/profile.sh)
# of the default line, the RTSP-interleaved line, every sub-stream rewriting and C3's per-GPU
# shape; summarised into profiles/ afterwards (tools/summarize_profile.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/profile.sh r03_final/prof_desc "" && bash tools/profile.sh r03_final/prof_tcp "--ingest tcp" && \
bash tools/profile.sh r03_final/prof_rw "--rewrite" && bash tools/profile.sh r03_final/prof_c3 "--subs 64"
