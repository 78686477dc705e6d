# round 3, run t: walk shapes (tools/build_tcp_walk4_ab.sh CHUNK:CPW): interleave parity under each,
# then the --ingest tcp line twice per build, in one call; and the shipped default build's
# interleave + random parity (its walk now takes each chunk's setup from LDS)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03t
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_interleave.py \
  tests/test_gpu_random.py > $O/tests_default.log 2>&1; rc=$?
echo "default tests rc=$rc $(tail -1 $O/tests_default.log)"
[ $rc -ne 0 ] && exit $rc
for v in w32768x2_8 w16384x4_8 w24576x4_8 w32768x4_8 w16384x2_8; do
  L=easydarwin_amd/ab/libedgpu_$v.so
  EDGPU_LIB=$L timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_interleave.py > $O/tests_$v.log 2>&1; r=$?
  echo "$v tests rc=$r $(tail -1 $O/tests_$v.log)"
  [ $r -ne 0 ] && exit $r
done
for k in 1 2; do
  for v in w32768x2_8 w16384x4_8 w24576x4_8 w32768x4_8 w16384x2_8; do
    EDGPU_LIB=easydarwin_amd/ab/libedgpu_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --ingest tcp > $O/tcp_${v}_$k.json 2> $O/tcp_${v}_$k.err; r=$?
    echo "$v/$k rc=$r $(python -c "import json;d=json.load(open('$O/tcp_${v}_$k.json'));print(d['kernel_ms']['ingest'], d['value'])")"
    [ $r -ne 0 ] && exit $r
  done
done
exit 0
