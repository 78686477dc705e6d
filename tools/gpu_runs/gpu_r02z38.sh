# round 2, run z38: walk chunk size again now that a wave walks two chunks (k_tcp_walk<2>):
# 32 KiB (default) vs 16 / 24 KiB (EDGPU_TCP_CHUNK builds from tools/build_tcp_chunk_ab.sh,
# swapped into this scratch tree); --ingest tcp x2 each, interleave parity under each
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02z38
mkdir -p $O
cp easydarwin_amd/libedgpu.so $O/../libedgpu_default.so.bak
for c in default 16384 24576; do
  if [ $c = default ]; then cp $O/../libedgpu_default.so.bak easydarwin_amd/libedgpu.so; else cp easydarwin_amd/ab/libedgpu_chunk$c.so easydarwin_amd/libedgpu.so; fi
  if [ $c != default ]; then
    timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "interleave" > $O/gputest_$c.log 2>&1; rc=$?
    echo "chunk $c tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest_$c.log | tail -3; [ $rc -ne 0 ] && exit $rc
  fi
  for r in 1 2; do
    timeout -k 10 300 python3 bench.py --ingest tcp --no-cpu-baseline > $O/tcp_${c}_$r.json 2> $O/tcp_${c}_$r.err || { echo FAIL; tail -5 $O/tcp_${c}_$r.err; exit 1; }
  done
done
rm -f $O/../libedgpu_default.so.bak
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['kernel_ms']['ingest'])"; done
echo ALL_OK
