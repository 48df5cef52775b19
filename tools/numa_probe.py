"""Where the bench's host thread runs relative to its GPU (diagnostic): the
GPU's PCI address and NUMA node from sysfs, the CPUs local to it, and the
CPUs this process may use."""
import glob
import os

import torch

torch.cuda.set_device(0)
p = torch.cuda.get_device_properties(0)
print("props:", {k: getattr(p, k) for k in dir(p) if "pci" in k.lower()})
allowed = sorted(os.sched_getaffinity(0))
print("allowed cpus:", len(allowed), allowed[:8], "...", allowed[-4:])
dom = getattr(p, "pci_domain_id", 0)
bus = getattr(p, "pci_bus_id", None)
dev = getattr(p, "pci_device_id", None)
if bus is not None:
    for path in glob.glob(f"/sys/bus/pci/devices/{dom:04x}:{bus:02x}:{dev:02x}.*"):
        for f in ("numa_node", "local_cpulist"):
            try:
                print(path, f, open(os.path.join(path, f)).read().strip())
            except OSError as e:
                print(path, f, e)
print("numa nodes:", sorted(glob.glob("/sys/devices/system/node/node*")))
for n in sorted(glob.glob("/sys/devices/system/node/node*"))[:16]:
    try:
        print(n, open(n + "/cpulist").read().strip())
    except OSError:
        pass
print("current cpu:", os.sched_getaffinity(0) and open("/proc/self/stat").read().split()[38])
