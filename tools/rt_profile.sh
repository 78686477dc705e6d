#!/bin/bash
# Kernel timeline of the QTSS module at its real rate (tools/qtss_replay --bench, EDGPU_BENCH_REALTIME=1,
# the default reflect-on-arrival ticker): rocprofv3 kernel trace + stats.  Usage:
#   tools/rt_profile.sh <out tag> [sessions] [seconds]
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-rt_prof}
mkdir -p $OUT
export EDGPU_BENCH_REALTIME=1 EDGPU_QTSS_REFLECT_ON_ARRIVAL=2 EDGPU_QTSS_WRITE_THREADS=16
export EDGPU_QTSS_ARENA_MB=4096 EDGPU_QTSS_MAX_OUT_PACKETS=4194304
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/kt -o kt -- \
    $R/tools/qtss_replay $R/easydarwin_amd/libQTSSReflectorModule.so --bench ${2:-2048} 16 ${3:-4} 100 8 > $OUT/rt.json 2> $OUT/rt.err
echo done
