# round 2, run z12: SQ counters of the fan-out on identity and rewriting windows, 16- vs
# 32-packet chunks (variants 46 / 31): where does the 16-packet patch path lose its time?
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02z12
mkdir -p $O
C=SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_VALU,SQ_INSTS_LDS,GRBM_GUI_ACTIVE
for cfg in "46 id" "46 rw" "31 id" "31 rw"; do
  set -- $cfg; v=$1; m=$2; X=""; [ $m = rw ] && X=--rewrite
  EDGPU_FANOUT=$v timeout -s KILL 150 rocprofv3 --pmc $(echo $C | tr , ' ') -T --output-format csv --kernel-include-regex 'k_fanout' -d $O/v${v}_$m -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline $X > $O/v${v}_$m.json 2> $O/v${v}_$m.err || { echo "PMC_FAIL $v $m"; tail -5 $O/v${v}_$m.err; exit 1; }
done
python3 - <<'PY'
import csv, glob, os, collections
for d in sorted(glob.glob('gpurun_out/r02z12/v*_*/')):
    f = glob.glob(d + '**/pmc_counter_collection.csv', recursive=True)
    if not f: print(d, 'no csv'); continue
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        acc[r['Counter_Name']].append(float(r['Counter_Value']))
    print(d, {k: round(sum(v) / len(v) / 1e6, 3) for k, v in sorted(acc.items())})
PY
echo ALL_OK
