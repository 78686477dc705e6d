set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02d
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "qtss_module or pinned or engine_api or egress" > gpurun_out/r02d/newtests.log 2>&1; echo "new tests rc=$?"; tail -15 gpurun_out/r02d/newtests.log
for m in 0 2 1; do timeout -k 10 120 ./tools/repro_fpi 20000 $m || { echo REPRO_FAIL; exit 1; }; done | tee gpurun_out/r02d/repro_fpi.jsonl
bash tools/ab_fanout.sh r02d_ab 10 27 28 || { echo AB_FAIL; exit 1; }
BENCH_EXTRA=--rewrite TAGSUF=_rw bash tools/ab_fanout.sh r02d_ab 10 27 28 || { echo AB_FAIL; exit 1; }
for f in gpurun_out/r02d_ab/*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['roofline']['kernel'], d['roofline']['avg_kernel_ms'], d['roofline']['frac'], d['ms_per_step'], d['config']['rewrite'][:8])"; done
timeout -k 10 300 python bench.py --ingest host --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/r02d/bench_host.json 2> gpurun_out/r02d/bench_host.err || { echo HOST_FAIL; tail -20 gpurun_out/r02d/bench_host.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r02d/bench_host.json')); print('host', d['ms_per_step'], d['value'], d.get('pcie_H2D_GBps'), d['kernel_ms'])"
echo ALL_OK
