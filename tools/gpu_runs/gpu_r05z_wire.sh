# round 5: the wire path in reference-exact mode (one datagram per message) beside the reference's
# own sendto() write path on the same host, and the GSO mode.  Logs under gpurun_out/$1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05z_wire}
O=gpurun_out/$TAG
mkdir -p $O
run() {   # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err; local r=$?
  echo "$n rc=$r"; tail -c 900 $O/$n.json; echo
  return $r
}
run egress_nogso 300 python tools/bench_egress.py --gso 0 --reference && \
run egress_gso 300 python tools/bench_egress.py --gso 1 && \
run egress_nogso_rx16 300 python tools/bench_egress.py --gso 0 --receivers 16
exit $?
