# round 5: the drop-in's push path (RTSPIncomingData -> Reflector::PushPacket) against pusher threads,
# and the reference module's, in the fake server at C2 scale (100-ms ticks, 4 s, the first ticks untimed).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05n}
mkdir -p $O
for so in easydarwin_amd/libQTSSReflectorModule.so oracle/_ref/libQTSSReflectorModule_ref.so; do
  for th in 1 2 4 8 16; do
    n=$(basename $so .so)_t$th
    EDGPU_REF_TICK_THREADS=16 EDGPU_QTSS_WRITE_THREADS=16 EDGPU_QTSS_ARENA_MB=4096 EDGPU_QTSS_MAX_OUT_PACKETS=4194304 \
      timeout -k 10 120 $R/tools/qtss_replay $R/$so --bench 1024 16 4 100 $th > $O/$n.json 2> $O/$n.err || exit 1
    python3 -c "import json; d=json.loads([l for l in open('$O/$n.json') if 'relayed_per_s' in l][-1]); print('$n', d['push_us_per_packet'], d['push_s'], d['relayed_per_s'])"
  done
done
