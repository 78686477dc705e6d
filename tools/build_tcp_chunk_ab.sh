#!/bin/bash
# A/B builds of libedgpu.so with another RTSP-interleaved walk chunk size (EDGPU_TCP_CHUNK):
# easydarwin_amd/ab/libedgpu_w<N>x2_8.so.  Since round 3 k_ingest finds frames by chunk too, so
# every TU that knows the chunk size is rebuilt: this is tools/build_tcp_walk4_ab.sh N:2.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
args=()
for n in "$@"; do args+=("$n:2"); done
exec bash "$R/tools/build_tcp_walk4_ab.sh" "${args[@]}"
