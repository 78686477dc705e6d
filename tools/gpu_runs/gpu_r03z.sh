# round 3, run z: candidate-window prefetch in the walk (EDGPU_TCP_CAND_PREFETCH=1: every round's
# block of a window loaded before the scan) vs the shipped build: interleave parity under it, then
# the --ingest tcp line three times each, alternating, in one call
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03z
mkdir -p $O
EDGPU_LIB=easydarwin_amd/ab/libedgpu_candpf.so timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_interleave.py > $O/tests_pf.log 2>&1; r=$?
echo "pf tests rc=$r $(tail -1 $O/tests_pf.log)"
[ $r -ne 0 ] && exit $r
for k in 1 2 3; do
  for v in default candpf; do
    EDGPU_LIB=easydarwin_amd/ab/libedgpu_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --ingest tcp > $O/tcp_${v}_$k.json 2> $O/tcp_${v}_$k.err; r=$?
    echo "$v/$k rc=$r $(python -c "import json;d=json.load(open('$O/tcp_${v}_$k.json'));print(d['kernel_ms']['ingest'])")"
    [ $r -ne 0 ] && exit $r
  done
done
exit 0
