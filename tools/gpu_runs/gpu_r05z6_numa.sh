# round 5: the box's CPU / NUMA topology beside the GPU, and the module's C2 line with its host
# threads on the GPU's NUMA node vs the other one (the push phase varies 1.7-5.8 ms per tick from
# box to box).  Logs under gpurun_out/$1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05z6}
O=gpurun_out/$TAG
mkdir -p $O
{ lscpu; echo; numactl -H 2>&1; echo; grep Cpus_allowed_list /proc/self/status; echo OMP=$OMP_NUM_THREADS;
  for d in /sys/bus/pci/devices/*; do
    if [ "$(cat $d/vendor)" = 0x1002 ] && grep -qE "0x(1200|0380)" $d/class; then echo "$d node=$(cat $d/numa_node) cpus=$(cat $d/local_cpulist)"; fi
  done; rocm-smi --showbus 2>&1 | head -20; } > $O/topo.txt 2>&1
python - <<'PY' >> $O/topo.txt 2>&1
import torch
p = torch.cuda.get_device_properties(0)
print("torch pci", getattr(p, "pci_bus_id", None), getattr(p, "pci_domain_id", None), getattr(p, "pci_device_id", None))
PY
cat $O/topo.txt | tail -30
exit 0
