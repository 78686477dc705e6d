# round 3, run n: kernel + memory-copy trace of the egress bench and the module bench (where the
# readback time goes after the gather-into-pinned change)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03n
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -T --output-format csv -d $O/egress -o eg -- python3 tools/bench_egress.py > $O/egress.json 2> $O/egress.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -T --output-format csv -d $O/module -o md -- python3 tools/bench_module.py --no-reference > $O/module.json 2> $O/module.err
r=$?; find $O -name "*stats.csv" | head; exit $r
