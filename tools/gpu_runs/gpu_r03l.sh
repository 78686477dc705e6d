# round 3, run l: device->host readback calibration (hipMemcpyAsync into pinned memory, split over
# streams, vs a kernel storing straight into the pinned buffer) and the module bench at 16 write threads
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03l
mkdir -p $O
timeout -k 10 60 ./tools/pcie_d2h > $O/pcie_d2h.json && cat $O/pcie_d2h.json && \
timeout -k 10 60 ./tools/pcie_d2h 8388608 > $O/pcie_d2h_8m.json && cat $O/pcie_d2h_8m.json && \
timeout -k 10 200 python tools/bench_module.py --no-reference > $O/module_w16.json 2> $O/module_w16.err && \
python -c "import json;d=json.load(open('$O/module_w16.json'))['module'];print(d['relayed_per_s'], d['per_tick_ms'])"
