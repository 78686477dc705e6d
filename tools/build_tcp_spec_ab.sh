#!/bin/bash
# A/B builds of libedgpu.so with a number of guessed frame headers per burst of the
# RTSP-interleaved walk (EDGPU_TCP_SPEC, 0 = the sequential walk):
# easydarwin_amd/ab/libedgpu_spec<N>.so.  A GPU run copies one over easydarwin_amd/libedgpu.so
# in its scratch tree before benchmarking.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
S=$R/easydarwin_amd/csrc
mkdir -p $R/easydarwin_amd/ab /tmp/tcpab
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I$R/include -I$S"
for n in "$@"; do
  /opt/rocm/bin/hipcc $F -DEDGPU_TCP_SPEC=$n -c $S/edgpu_deframe.hip -o /tmp/tcpab/deframe_spec$n.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/easydarwin_amd/ab/libedgpu_spec$n.so \
      $S/edgpu_kernels.o /tmp/tcpab/deframe_spec$n.o $S/edgpu_egress.o $S/edgpu_engine.o $S/reflector_adapter.o -pthread
done
