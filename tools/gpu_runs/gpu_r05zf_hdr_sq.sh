# round 5: SQ counters of k_ingest with the slot copy skipped (measurement build, EDGPU_ABLATE=32)
# and in full, descriptor line: where the header phase's 81 us go.  Logs under gpurun_out/$1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05zf}
O=gpurun_out/$TAG
mkdir -p $O
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
EDGPU_LIB=$GRAFT_REPO_ROOT/easydarwin_amd/ab/libedgpu_ab.so EDGPU_ABLATE=32 timeout -s KILL 120 rocprofv3 --pmc $C -T --output-format csv --kernel-include-regex 'k_ingest' -d $O/hdr -o hdr -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --ablation-study > $O/hdr.json 2> $O/hdr.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc $C -T --output-format csv --kernel-include-regex 'k_ingest' -d $O/full -o full -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/full.json 2> $O/full.err || exit $?
C2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_FLAT"
EDGPU_LIB=$GRAFT_REPO_ROOT/easydarwin_amd/ab/libedgpu_ab.so EDGPU_ABLATE=32 timeout -s KILL 120 rocprofv3 --pmc $C2 -T --output-format csv --kernel-include-regex 'k_ingest' -d $O/hdr2 -o hdr2 -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --ablation-study > $O/hdr2.json 2> $O/hdr2.err || exit $?
python3 - <<PY
import csv, glob, collections
for tag in ("hdr", "full", "hdr2"):
    f = glob.glob("$O/%s/**/*counter_collection.csv" % tag, recursive=True)
    if not f: print(tag, "no csv"); continue
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(tag, {k: round(sum(v) / len(v)) for k, v in sorted(acc.items())})
PY
