# round 5: egress workers taking plain UDP rows in blocks (the tree) against one worker per
# subscriber modulo the thread count (easydarwin_amd/ab/libedgpu_prev.so, the previous commit
# built by hand), alternating, one datagram per send and GSO; the egress tests first.  Logs under
# gpurun_out/$1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05zo}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 150 --timeout-method thread -p no:cacheprovider -m gpu -x tests/test_gpu_egress.py > $O/gputests.log 2>&1; rc=$?
tail -2 $O/gputests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in new prev; do
    for g in 0 1; do
      n=${v}_gso${g}_$rep
      if [ $v = prev ]; then export EDGPU_LIB=$GRAFT_REPO_ROOT/easydarwin_amd/ab/libedgpu_prev.so; else unset EDGPU_LIB; fi
      timeout -k 10 200 python tools/bench_egress.py --gso $g > $O/$n.json 2> $O/$n.err || exit $?
      python -c "
import json; d=json.load(open('$O/$n.json')); print('$n', round(d['egress_datagrams_per_s']/1e6,2), 'M/s', d['per_tick_mean']['send_ms'], 'ms send')"
    done
  done
done
unset EDGPU_LIB
timeout -k 10 300 python tools/bench_egress.py --gso 0 --reference > $O/new_ref.json 2> $O/new_ref.err || exit $?
python -c "
import json; d=json.load(open('$O/new_ref.json')); print('new vs reference', d['egress_datagrams_per_s']/1e6, d['reference']['sendto_datagrams_per_s']/1e6, d['egress_vs_reference_sendto'])"
