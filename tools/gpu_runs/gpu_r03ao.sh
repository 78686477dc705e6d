# round 3, run ao: the module's prestaging, instrumented (bytes copied ahead per tick): module
# bench alternating pushes, EDGPU_PRESTAGE_BYTES=0 vs default, two pairs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03ao
mkdir -p $O
for k in 1 2; do
  for p in 0 def; do
    if [ $p = 0 ]; then export EDGPU_PRESTAGE_BYTES=0; else unset EDGPU_PRESTAGE_BYTES; fi
    timeout -k 10 300 python tools/bench_module.py --no-reference --seconds 4 > $O/m_${p}_$k.json 2> $O/m_${p}_$k.err; r=$?
    echo "prestage=$p /$k rc=$r $(python -c "import json;d=json.load(open('$O/m_${p}_$k.json'))['module'];print(round(d['relayed_per_s']/1e6,1), d['per_tick_ms'], d['per_tick_bytes'])" 2>/dev/null)"
    [ $r -ne 0 ] && exit $r
  done
done
exit 0
