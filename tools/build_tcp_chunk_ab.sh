#!/bin/bash
# A/B builds of libedgpu.so with another RTSP-interleaved walk chunk size (EDGPU_TCP_CHUNK):
# easydarwin_amd/ab/libedgpu_chunk<N>.so.  A GPU run copies one over easydarwin_amd/libedgpu.so
# in its scratch tree before benchmarking.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
S=$R/easydarwin_amd/csrc
mkdir -p $R/easydarwin_amd/ab /tmp/tcpab
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I$R/include -I$S"
for n in "$@"; do
  /opt/rocm/bin/hipcc $F -DEDGPU_TCP_CHUNK=$n -c $S/edgpu_deframe.hip -o /tmp/tcpab/deframe_$n.o
  /opt/rocm/bin/hipcc $F -DEDGPU_TCP_CHUNK=$n -c $S/edgpu_engine.cpp -o /tmp/tcpab/engine_$n.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/easydarwin_amd/ab/libedgpu_chunk$n.so \
      $S/edgpu_kernels.o /tmp/tcpab/deframe_$n.o $S/edgpu_egress.o /tmp/tcpab/engine_$n.o $S/reflector_adapter.o -pthread
done
