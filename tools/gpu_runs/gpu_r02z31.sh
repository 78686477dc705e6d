# round 2, run z31: why k_tcp_walk takes ~100 us whether or not its header chain is guessed
# ahead (r02z30): SQ counters and fetched bytes of the walk, sequential (spec0) vs default (8)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02z31
mkdir -p $O
cp easydarwin_amd/libedgpu.so $O/../libedgpu_default.so.bak
C=SQ_WAVES,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VMEM_RD,SQ_INSTS_VALU,SQ_INSTS_SALU
for c in default spec0; do
  if [ $c = default ]; then cp $O/../libedgpu_default.so.bak easydarwin_amd/libedgpu.so; else cp easydarwin_amd/ab/libedgpu_$c.so easydarwin_amd/libedgpu.so; fi
  timeout -s KILL 150 rocprofv3 --pmc $(echo $C | tr , ' ') -T --output-format csv --kernel-include-regex 'k_tcp' -d $O/sq_$c -o pmc -- python3 bench.py --ingest tcp --steps 3 --warmup 1 --no-cpu-baseline > $O/sq_$c.json 2> $O/sq_$c.err || { echo "SQ_FAIL $c"; tail -5 $O/sq_$c.err; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -T --output-format csv --kernel-include-regex 'k_tcp' -d $O/fetch_$c -o pmc -- python3 bench.py --ingest tcp --steps 3 --warmup 1 --no-cpu-baseline > $O/fetch_$c.json 2> $O/fetch_$c.err || { echo "FETCH_FAIL $c"; tail -5 $O/fetch_$c.err; exit 1; }
done
cp $O/../libedgpu_default.so.bak easydarwin_amd/libedgpu.so
rm -f $O/../libedgpu_default.so.bak
python3 - <<'PY'
import csv, glob, collections
for d in sorted(glob.glob('gpurun_out/r02z31/*_*/')):
    f = glob.glob(d + '**/pmc_counter_collection.csv', recursive=True)
    if not f: print(d, 'no csv'); continue
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f[0])):
        acc[r['Kernel_Name'][:14]][r['Counter_Name']].append(float(r['Counter_Value']))
    for k, cs in sorted(acc.items()):
        print(d, k, {n: round(sum(v) / len(v), 1) for n, v in sorted(cs.items())})
PY
echo ALL_OK
