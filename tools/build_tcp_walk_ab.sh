#!/bin/bash
# A/B builds of libedgpu.so with other RTSP-interleaved walk settings: each argument is
# tag=compiler flags, e.g. cpw1="-DEDGPU_TCP_WALK_CPW=1 -DEDGPU_TCP_WALK_WPE=1" ->
# easydarwin_amd/ab/libedgpu_cpw1.so.  A GPU run copies one over easydarwin_amd/libedgpu.so in
# its scratch tree before benchmarking.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
S=$R/easydarwin_amd/csrc
mkdir -p $R/easydarwin_amd/ab /tmp/tcpab
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I$R/include -I$S"
for a in "$@"; do
  tag=${a%%=*}; flags=${a#*=}
  # edgpu_kernels.hip with the same flags: k_ingest finds interleaved frames by chunk (round 3)
  /opt/rocm/bin/hipcc $F $flags -c $S/edgpu_kernels.hip -o /tmp/tcpab/kernels_$tag.o &
  /opt/rocm/bin/hipcc $F $flags -c $S/edgpu_deframe.hip -o /tmp/tcpab/deframe_$tag.o &
  /opt/rocm/bin/hipcc $F $flags -c $S/edgpu_engine.cpp -o /tmp/tcpab/engine_$tag.o &
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/easydarwin_amd/ab/libedgpu_$tag.so \
      /tmp/tcpab/kernels_$tag.o /tmp/tcpab/deframe_$tag.o $S/edgpu_egress.o /tmp/tcpab/engine_$tag.o $S/reflector_adapter.o -pthread
done
