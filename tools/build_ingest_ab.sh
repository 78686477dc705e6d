#!/bin/bash
# A/B builds of libedgpu.so with other ingest kernel settings: each argument is tag=compiler
# flags, e.g. td2="-DEDGPU_TCP_TD=2" -> easydarwin_amd/ab/libedgpu_td2.so (EDGPU_LIB selects
# it for bench.py and the Python mirror).  Needs the product objects (make) first.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
S=$R/easydarwin_amd/csrc
mkdir -p $R/easydarwin_amd/ab /tmp/ingestab
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I$R/include -I$S"
for a in "$@"; do
  tag=${a%%=*}; flags=${a#*=}
  /opt/rocm/bin/hipcc $F $flags -c $S/edgpu_kernels.hip -o /tmp/ingestab/kernels_$tag.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/easydarwin_amd/ab/libedgpu_$tag.so \
      /tmp/ingestab/kernels_$tag.o $S/edgpu_deframe.o $S/edgpu_egress.o $S/edgpu_engine.o $S/reflector_adapter.o -pthread
done
