# host topology of the GPU box as this process sees it (pool placement), and A/B of pinning
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/topo
mkdir -p $O
{
nproc; taskset -p $$; cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null
lscpu | head -30
for d in /sys/bus/pci/devices/*; do v=$(cat $d/vendor); c=$(cat $d/class); if [ "$v" = "0x1002" ]; then case $c in 0x0380*|0x1200*) echo "$d $c $(cat $d/local_cpulist) numa $(cat $d/numa_node)";; esac; fi; done
for i in 0 8 16 24 32 48 64; do echo "cpu$i l3: $(cat /sys/devices/system/cpu/cpu$i/cache/index3/shared_cpu_list 2>/dev/null) sib: $(cat /sys/devices/system/cpu/cpu$i/topology/thread_siblings_list 2>/dev/null)"; done
uptime
} > $O/topo.txt 2>&1
timeout -k 10 120 python -u -c "
import os, ctypes, json
import torch
print('visible', torch.cuda.device_count())
print(torch.cuda.get_device_properties(0).pci_bus_id if hasattr(torch.cuda.get_device_properties(0),'pci_bus_id') else '')
" >> $O/topo.txt 2>&1
HDPM_BENCH_TIMELINE=1 timeout -k 10 120 python -u bench.py --steps 300 --warmup 20 --no-cpu-baseline > $O/c5_tl300_pin.jsonl 2> $O/c5_tl300_pin.err
HDPM_PIN_THREADS=0 HDPM_BENCH_TIMELINE=1 timeout -k 10 120 python -u bench.py --steps 300 --warmup 20 --no-cpu-baseline > $O/c5_tl300_nopin.jsonl 2> $O/c5_tl300_nopin.err
exit 0
