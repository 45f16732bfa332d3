#!/usr/bin/env python3
"""Where does pinned host memory land?  Allocates a 512 MiB pinned stage the
way the engine does (hipHostMalloc, default flags) and prints, from
/proc/self/numa_maps, how many of its pages sit on each NUMA node, next to
the NUMA node of the GPU's PCI function (DESIGN.md §6.1 "Readers on the
GPU's NUMA node").  Diagnostic only."""
import ctypes
import json
import os
import sys

import torch

torch.cuda.init()
hip = ctypes.CDLL("libamdhip64.so.7")
ptr = ctypes.c_void_p()
size = 512 << 20
rc = hip.hipHostMalloc(ctypes.byref(ptr), ctypes.c_size_t(size), ctypes.c_uint(0))
if rc != 0:
    print(json.dumps({"error": f"hipHostMalloc rc={rc}"}))
    sys.exit(1)
start = ptr.value
pages = {}
with open("/proc/self/numa_maps") as f:
    for line in f:
        parts = line.split()
        addr = int(parts[0], 16)
        if addr <= start < addr + size * 2:
            for p in parts[1:]:
                if p.startswith("N") and "=" in p:
                    k, v = p.split("=")
                    pages[k] = pages.get(k, 0) + int(v)
pr = torch.cuda.get_device_properties(0)
bus = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
node = open(f"/sys/bus/pci/devices/{bus}/numa_node").read().strip()
print(json.dumps({"stage_pages_by_node": pages, "gpu_numa_node": node}))
hip.hipHostFree(ptr)
