# round 6: where the GPU sits relative to the host CPUs (PCI address, NUMA node, local CPU list) and the
# CPU topology the drop-in threads are pinned over
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_n
mkdir -p $O
{
  timeout -k 5 60 python3 -c "
import torch
p = torch.cuda.get_device_properties(0)
print('gpu', p.name, 'pci', p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
"
  for d in /sys/bus/pci/devices/*; do
    if [ "$(cat $d/vendor 2>/dev/null)" = "0x1002" ] && [ "$(cat $d/class 2>/dev/null | cut -c1-6)" = "0x1200" ]; then
      echo "$d numa_node=$(cat $d/numa_node) local_cpulist=$(cat $d/local_cpulist)"
    fi
  done
  grep -c processor /proc/cpuinfo
  lscpu | grep -E "^(CPU\(s\)|On-line|Thread|Core|Socket|NUMA|L3|Model name)"
  python3 -c "import os; print('affinity', sorted(os.sched_getaffinity(0))[:40], len(os.sched_getaffinity(0)))"
  cat /sys/fs/cgroup/cpu.max 2>/dev/null
  cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null
  for c in 0 1 2 8 16 32 64 128; do echo "cpu$c core=$(cat /sys/devices/system/cpu/cpu$c/topology/core_id) pkg=$(cat /sys/devices/system/cpu/cpu$c/topology/physical_package_id) siblings=$(cat /sys/devices/system/cpu/cpu$c/topology/thread_siblings_list) l3=$(cat /sys/devices/system/cpu/cpu$c/cache/index3/shared_cpu_list 2>/dev/null)"; done
} > $O/topo.txt 2>&1
echo "rc=$?" >> $O/done.txt
