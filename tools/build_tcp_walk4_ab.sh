#!/bin/bash
# A/B builds of libedgpu.so with another RTSP-interleaved walk shape: arguments CHUNK:CPW[:WPE]
# (walk chunk bytes, chunks per walking wave, waves per SIMD the walk's registers must allow),
# e.g. 16384:4:7 -> easydarwin_amd/ab/libedgpu_w16384x4_7.so.
# Every TU that knows the chunk size is rebuilt (k_ingest finds frames by chunk since round 3).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
S=$R/easydarwin_amd/csrc
mkdir -p $R/easydarwin_amd/ab /tmp/tcpab
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I$R/include -I$S"
for v in "$@"; do
  IFS=: read -r n c e <<< "$v"; e=${e:-8}
  D="-DEDGPU_TCP_CHUNK=$n -DEDGPU_TCP_WALK_CPW=$c -DEDGPU_TCP_WALK_WPE=$e"; t=w${n}x${c}_$e
  /opt/rocm/bin/hipcc $F $D -c $S/edgpu_kernels.hip -o /tmp/tcpab/kernels_$t.o &
  /opt/rocm/bin/hipcc $F $D -c $S/edgpu_deframe.hip -o /tmp/tcpab/deframe_$t.o &
  /opt/rocm/bin/hipcc $F $D -c $S/edgpu_engine.cpp -o /tmp/tcpab/engine_$t.o &
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/easydarwin_amd/ab/libedgpu_$t.so \
      /tmp/tcpab/kernels_$t.o /tmp/tcpab/deframe_$t.o $S/edgpu_egress.o /tmp/tcpab/engine_$t.o $S/reflector_adapter.o -pthread
done
