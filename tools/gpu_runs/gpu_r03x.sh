# round 3, run x: where k_ingest's time goes today -- timing ablations in the measurement build
# (EDGPU_ABLATE 32: no slot copy, 64: no per-sender scans, 96: neither), descriptor ingest, C2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03x
mkdir -p $O
export EDGPU_LIB=easydarwin_amd/ab/libedgpu_ab.so
for k in 1 2; do
  for a in 0 32 64 96; do
    if [ $a = 0 ]; then unset EDGPU_ABLATE; else export EDGPU_ABLATE=$a; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --ablation-study > $O/abl_${a}_$k.json 2> $O/abl_${a}_$k.err; r=$?
    echo "ablate=$a/$k rc=$r $(python -c "import json;d=json.load(open('$O/abl_${a}_$k.json'));print(d['kernel_ms'])")"
    [ $r -ne 0 ] && exit $r
  done
done
exit 0
