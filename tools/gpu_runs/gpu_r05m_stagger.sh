# round 5: k_ingest phase-stagger A/B (measurement build): odd session workgroups sleep k x ~3.4 us
# first (EDGPU_ABLATE bits 8-11) or take a half first round (bit 12); two passes over the variants,
# descriptor and RTSP-interleaved ingest.  Timing only.  Logs under gpurun_out/$1.
set -o pipefail
R=$GRAFT_REPO_ROOT
export EDGPU_LIB=$R/easydarwin_amd/ab/libedgpu_ab.so
TAG=${1:-r05m}
O=$R/gpurun_out/$TAG
mkdir -p $O
for rep in 1 2; do
  for ing in desc tcp; do
    for a in 0 256 768 1280 4096; do
      EDGPU_ABLATE=$a timeout -k 10 120 python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --ablation-study --ingest $ing > $O/${ing}_a${a}_r$rep.json 2> $O/${ing}_a${a}_r$rep.err || exit 1
      python3 -c "import json,sys; d=json.load(open('$O/${ing}_a${a}_r$rep.json')); print('$ing a=$a r$rep', d['ms_per_step'], d['kernel_ms'])"
    done
  done
done
