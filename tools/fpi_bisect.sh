#!/bin/bash
# The r01 stale RTP-Info intermittent, bisected (built by tools/fpi_bisect_build.sh): the C++ adapter replays the
# rtpinfo trace 20 times per build of the engine as it was before commit 085e3ba --
#   A  unchanged (per-call hipMallocAsync query buffers, ingest returns before its pageable copies)
#   B  A + edgpu_ingest waits for its pageable host->device copies
#   C  A + RTP-Info query buffers from hipMalloc (no stream-ordered pool)
#   D  B + C
#   F  B + pinned host staging for the query and the result (pool device buffers kept)
#   Bi B + a second, synchronous read of the result / query buffers before they are freed
#      (stderr lines "FPI ..." into gpurun_out/bisect/Bi_<k>.log)
# and counts captures that differ from the reference fixture.
cd "$(dirname "$0")/_bisect"
want=$(cat rtpinfo.sha)
mkdir -p ../../gpurun_out/bisect
for v in ${VARIANTS:-A B C}; do
  bad=0
  for k in $(seq 1 ${RUNS:-20}); do
    timeout -k 5 60 ./$v/tools/adapter_replay rtpinfo.edtr /tmp/bisect_$v.edcp > /dev/null 2> /tmp/bisect_$v.log || { echo "{\"variant\": \"$v\", \"error\": $?}"; exit 1; }
    got=$(sha256sum /tmp/bisect_$v.edcp | cut -d' ' -f1)
    [ "$got" = "$want" ] || { bad=$((bad+1)); cp /tmp/bisect_$v.log ../../gpurun_out/bisect/${v}_$k.log;
                              [ $bad = 1 ] && cp /tmp/bisect_$v.edcp ../../gpurun_out/bisect/${v}_first.edcp; }
    [ "$got" = "$want" ] && [ $k = 1 ] && cp /tmp/bisect_$v.log ../../gpurun_out/bisect/${v}_good.log
  done
  echo "{\"variant\": \"$v\", \"runs\": ${RUNS:-20}, \"mismatches\": $bad}"
done
