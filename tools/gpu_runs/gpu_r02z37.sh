# round 2, run z37 (the change it measured was reverted): k_plan_final launched with a wave per sender (512 blocks on C2) instead of
# a block per 256 sub-streams (64 blocks: 8 senders' dependent-load chains per wave in a row), vs
# the r02z36 library (head); full GPU suite under the new default; C2 bench x3 each, alternating;
# kernel trace of each; --subs 64 (C3 shape) once each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02z37
mkdir -p $O
cp easydarwin_amd/libedgpu.so $O/../libedgpu_default.so.bak
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/gputest_default.log 2>&1; rc=$?
echo "default tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest_default.log | tail -3; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  for c in default head; do
    if [ $c = default ]; then cp $O/../libedgpu_default.so.bak easydarwin_amd/libedgpu.so; else cp easydarwin_amd/ab/libedgpu_$c.so easydarwin_amd/libedgpu.so; fi
    timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/c2_${c}_$r.json 2> $O/c2_${c}_$r.err || { echo FAIL; tail -5 $O/c2_${c}_$r.err; exit 1; }
  done
done
for c in default head; do
  if [ $c = default ]; then cp $O/../libedgpu_default.so.bak easydarwin_amd/libedgpu.so; else cp easydarwin_amd/ab/libedgpu_$c.so easydarwin_amd/libedgpu.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/kt_$c -o kt -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/kt_$c.json 2> $O/kt_$c.err || { echo PROF_FAIL; exit 1; }
done
cp $O/../libedgpu_default.so.bak easydarwin_amd/libedgpu.so
for c in default head; do
  if [ $c = default ]; then cp $O/../libedgpu_default.so.bak easydarwin_amd/libedgpu.so; else cp easydarwin_amd/ab/libedgpu_$c.so easydarwin_amd/libedgpu.so; fi
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --subs 64 > $O/c3_$c.json 2> $O/c3_$c.err || { echo C3_FAIL; tail -5 $O/c3_$c.err; exit 1; }
done
cp $O/../libedgpu_default.so.bak easydarwin_amd/libedgpu.so
rm -f $O/../libedgpu_default.so.bak
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); k=d['kernel_ms']; print('$f', d['value'], d['ms_per_step'], round(k['tick_plan_plus_fanout']-k['fanout'],4), k['ingest'])"; done
for c in default head; do python3 - $O/kt_$c <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/kt_kernel_stats.csv', recursive=True)[0]
print(sys.argv[1], {r['Name'][:16]: round(float(r['AverageNs']) / 1e3, 1) for r in csv.DictReader(open(f)) if r['Name'].startswith('k_')})
PY
done
echo ALL_OK
