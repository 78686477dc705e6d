# round 2, run s: k_ingest ablation (copy vs the rest)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02s
mkdir -p $O
for a in 0 32 64 96 0; do EDGPU_ABLATE=$a timeout -k 10 300 python bench.py --no-cpu-baseline --ablation-study --steps 8 --warmup 2 > $O/a$a.json 2> $O/a$a.err || { echo FAIL; tail -5 $O/a$a.err; exit 1; }; python -c "import json; d=json.load(open('$O/a$a.json')); print('ablate=$a', d['ms_per_step'], d['kernel_ms'])"; done
echo ALL_OK
