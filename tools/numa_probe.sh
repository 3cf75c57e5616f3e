#!/bin/bash
# Host topology of the GPU box (profiling only): the visible GPU's PCI address, its NUMA node and
# local CPUs, the CPU quota and affinity.
O=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/numa.txt
{
  echo "env: ROCR=$ROCR_VISIBLE_DEVICES HIP=$HIP_VISIBLE_DEVICES CUDA=$CUDA_VISIBLE_DEVICES"
  cat /sys/fs/cgroup/cpu.max
  python3 -c "import os; a=sorted(os.sched_getaffinity(0)); print('affinity', len(a), a[:4], a[-4:])"
  lscpu | grep -E "NUMA|Socket|Model name|Thread|Core"
  timeout 60 python3 -c "import torch; p=torch.cuda.get_device_properties(0); print('bus', p.pci_bus_id, p.pci_device_id, p.pci_domain_id)"
  for d in /sys/class/drm/card*/device; do echo "$d $(cat $d/numa_node 2>/dev/null) $(cat $d/local_cpulist 2>/dev/null) $(basename $(readlink -f $d))"; done
} > "$O" 2>&1
