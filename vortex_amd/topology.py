"""GPUs this process may use, counted without HIP and without torch.

bench.py decides whether a plain ``--gpus N`` run can get N ranks BEFORE it
starts them, in a parent process that must never initialise the GPU (the
ranks are its children; a parent holding a HIP runtime that then forks and
execs a launcher is the pattern this pool punishes).  ``torch.cuda.
device_count()`` cannot be trusted for that: without amdsmi it falls back to
``hipGetDeviceCount``, a HIP runtime init.  This module reads the kernel's
KFD topology instead (plain sysfs files, nothing mapped or opened on the
device):

* ``/sys/class/kfd/kfd/topology/nodes/<k>/properties`` — one node per CPU
  socket and per GPU; a GPU node has ``gfx_target_version != 0`` and names its
  DRM render node (``drm_render_minor``).  A node whose properties the device
  cgroup hides (EPERM) is not ours.
* ``/dev/dri/renderD<minor>`` — a container sees only the render nodes it was
  given, so a GPU counts only when its render node exists here.
* ``ROCR_VISIBLE_DEVICES`` / ``HIP_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES``
  (and ``GPU_DEVICE_ORDINAL``) narrow the set the runtime would expose; the
  count is capped by each one that is set (an empty value hides every GPU).

``visible_gpus()`` returns ``None`` when the topology cannot be read at all;
callers treat that as "unknown" and refuse, never fall back to HIP.
"""
from __future__ import annotations

import os
from typing import Optional

KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"
VISIBILITY_VARS = ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "GPU_DEVICE_ORDINAL")


def _properties(path: str) -> Optional[dict]:
    try:
        with open(path) as f:
            text = f.read()
    except OSError:  # EPERM: the device cgroup hides this node from us
        return None
    out = {}
    for line in text.splitlines():
        parts = line.split()
        if len(parts) == 2:
            try:
                out[parts[0]] = int(parts[1])
            except ValueError:
                pass
    return out


def kfd_gpus(nodes_dir: str = KFD_NODES, dev_dir: str = "/dev/dri") -> Optional[list]:
    """The KFD GPU nodes usable here, as dicts (node, gfx_target_version,
    drm_render_minor, location_id, unique_id); None if the topology is absent."""
    try:
        names = sorted(os.listdir(nodes_dir), key=lambda s: (not s.isdigit(), int(s) if s.isdigit() else 0, s))
    except OSError:
        return None
    gpus = []
    for name in names:
        p = _properties(os.path.join(nodes_dir, name, "properties"))
        if not p or p.get("gfx_target_version", 0) == 0:
            continue
        minor = p.get("drm_render_minor")
        if minor is None or not os.path.exists(os.path.join(dev_dir, f"renderD{minor}")):
            continue
        gpus.append({"node": name, "gfx_target_version": p["gfx_target_version"], "drm_render_minor": minor,
                     "location_id": p.get("location_id"), "unique_id": p.get("unique_id")})
    return gpus


def visibility_cap(environ=None) -> Optional[int]:
    """The smallest device count any *_VISIBLE_DEVICES variable allows, or
    None when none is set."""
    env = os.environ if environ is None else environ
    cap = None
    for var in VISIBILITY_VARS:
        if var not in env:
            continue
        val = env[var].strip()
        k = 0 if not val else len([x for x in val.split(",") if x.strip()])
        cap = k if cap is None else min(cap, k)
    return cap


def visible_gpus(nodes_dir: str = KFD_NODES, dev_dir: str = "/dev/dri", environ=None) -> Optional[int]:
    """GPUs a HIP process started with this environment would see, from
    sysfs only (no HIP, no torch); None when the KFD topology is unreadable."""
    gpus = kfd_gpus(nodes_dir, dev_dir)
    if gpus is None:
        return None
    n = len(gpus)
    cap = visibility_cap(environ)
    return n if cap is None else min(n, cap)


def hip_runtime_mapped(pid: str = "self") -> bool:
    """True if this process has the HIP runtime (libamdhip64) mapped: what a
    GPU-free parent must never have."""
    try:
        with open(f"/proc/{pid}/maps") as f:
            return any("libamdhip64" in line for line in f)
    except OSError:
        return False
