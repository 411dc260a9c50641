#!/bin/bash
# the box's host settings that shape page faults and CPU shares (read only)
for f in /proc/sys/kernel/numa_balancing /sys/kernel/mm/transparent_hugepage/enabled /sys/fs/cgroup/cpu.max; do
  echo "$f: $(cat $f 2>/dev/null)"
done
lscpu | grep -E "NUMA|Model name|Socket|Thread" 
python3 -c "import os;print('affinity', len(os.sched_getaffinity(0)))"
