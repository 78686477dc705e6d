# round 2, run z2: store-pacing A/B on the default (31: dyn; 35: every window through the patch
# path; 36: s_sleep after each store row), identity x3
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_fanout.sh r02z2_ab 31 35 36 31 35 36 31 35 36 || { echo AB_FAIL; exit 1; }
for f in gpurun_out/r02z2_ab/*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['roofline']['kernel'], d['roofline']['avg_kernel_ms'], d['roofline']['frac'], d['ms_per_step'])"; done
echo ALL_OK
