# round 5: the last tree's smoke(), the driver's default bench command and the interleaved line.
# Logs under gpurun_out/$1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05zk}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --ingest tcp > $O/bench_tcp.json 2> $O/bench_tcp.err || exit $?
python - <<PY
import json
for n in ("bench_default", "bench_tcp"):
    d = json.loads(open("$O/%s.json" % n).read().strip().splitlines()[-1])
    print(n, round(d["value"] / 1e9, 3), d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["frac"], d["ingest"]["frac"],
          (d.get("cpu_baseline") or {}).get("value"))
PY
