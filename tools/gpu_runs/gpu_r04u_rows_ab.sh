# round 4: A/B of the module's readback -- the previous tree's per-descriptor readback (ab_old/, built
# from the commit before edgpu_fanout_rows) against the rows, read in place or copied to cacheable
# memory first (EDGPU_ROWS_COPY=1: a switch of that A/B build, removed after it).  Logs under gpurun_out/$1.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r04u_rows_ab}; mkdir -p $O
for k in 1 2; do
  for v in old new copy; do
    M=easydarwin_amd/libQTSSReflectorModule.so; [ $v = old ] && M=ab_old/libQTSSReflectorModule.so
    C=0; [ $v = copy ] && C=1
    for t in 100 20; do
      EDGPU_ROWS_COPY=$C EDGPU_QTSS_TICK_MSEC=$t timeout -k 10 200 python tools/bench_module.py --no-reference --tick-ms $t \
          --module $M > $O/${v}_t${t}_$k.json 2> $O/${v}_t${t}_$k.err || exit $?
      python3 -c "import json,sys; d=json.load(open('$O/${v}_t${t}_$k.json'))['module']; print('$v t$t run $k', round(d['relayed_per_s']/1e6,1), d['per_tick_ms'])"
    done
  done
done
