# round 5: the drop-in's push path (RTSPIncomingData -> Reflector::PushPacket) against pusher threads,
# with streaming and with cached slot stores, and the reference module's, in the fake server at C2
# scale (100-ms ticks, 4 s, the first ticks untimed).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05n}
mkdir -p $O
run() {   # name, module, threads, extra env...
  local n=$1 so=$2 th=$3; shift 3
  env "$@" EDGPU_REF_TICK_THREADS=16 EDGPU_QTSS_WRITE_THREADS=16 EDGPU_QTSS_ARENA_MB=4096 EDGPU_QTSS_MAX_OUT_PACKETS=4194304 \
    timeout -k 10 120 $R/tools/qtss_replay $R/$so --bench 1024 16 4 100 $th > $O/$n.json 2> $O/$n.err || return 1
  python3 -c "import json; d=json.loads([l for l in open('$O/$n.json') if 'relayed_per_s' in l][-1]); print('$n', d['push_us_per_packet'], d['push_s'], d['relayed_per_s'])"
}
for th in 1 8 16; do
  run drop_stream_t$th easydarwin_amd/libQTSSReflectorModule.so $th EDGPU_PUSH_STREAMING=1 || exit 1
  run drop_cached_t$th easydarwin_amd/libQTSSReflectorModule.so $th EDGPU_PUSH_STREAMING=0 || exit 1
  run ref_t$th oracle/_ref/libQTSSReflectorModule_ref.so $th X=1 || exit 1
done
