# round 2, run m: egress with UDP GSO -- parity tests, then datagrams/s with and without
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02m
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "egress" > $O/gputest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest.log | tail -5; [ $rc -ne 0 ] && exit 1
for g in 0 1; do timeout -k 10 300 python tools/bench_egress.py --gso $g > $O/egress_gso$g.json 2> $O/egress_gso$g.err || { echo EGRESS_FAIL; tail -5 $O/egress_gso$g.err; exit 1; }; cat $O/egress_gso$g.json; done
echo ALL_OK
