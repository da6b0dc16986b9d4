"""NUMA placement of the host side next to the GPU it feeds.

The host path (staging bodies into page-locked memory, the host packer, the H2D DMA) moves
several GB per fleet through host memory; on a two-socket host, threads and pages on the far
socket send every byte over the inter-socket link.  ``gpu_local_cpus(device)`` reads the GPU's
NUMA node from sysfs (its PCI address from the HIP runtime); ``bind_local(device)`` restricts
this process (and every thread it creates afterwards, the host runtime's worker pool included)
to that node's CPUs, within the CPUs the process may already use.  Pages are placed by first
touch, so bind before allocating the bodies and staging buffers."""
from __future__ import annotations

import os
from typing import Optional


def _parse_cpulist(text: str) -> set:
    cpus = set()
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            cpus.update(range(int(a), int(b) + 1))
        else:
            cpus.add(int(part))
    return cpus


def gpu_numa_node(device: int = 0) -> Optional[int]:
    """The NUMA node of HIP device ``device`` (None when sysfs does not say)."""
    import torch

    try:
        bus = torch.cuda.get_device_properties(device).pci_bus_id
        dom = getattr(torch.cuda.get_device_properties(device), "pci_domain_id", 0)
        dev = getattr(torch.cuda.get_device_properties(device), "pci_device_id", 0)
        addr = f"{dom:04x}:{bus:02x}:{dev:02x}.0"
        with open(f"/sys/bus/pci/devices/{addr}/numa_node") as fh:
            node = int(fh.read().strip())
        return node if node >= 0 else None
    except (OSError, ValueError, AttributeError, RuntimeError):
        return None


def _one_per_core(cpus: set) -> set:
    """The lowest-numbered hardware thread of each core in ``cpus`` (SMT siblings dropped)."""
    out = set()
    for c in sorted(cpus):
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as fh:
                sib = _parse_cpulist(fh.read())
        except OSError:
            sib = {c}
        if min(sib & cpus or {c}) == c:
            out.add(c)
    return out


def gpu_local_cpus(device: int = 0, one_per_core: bool = False) -> Optional[set]:
    """CPUs of the GPU's NUMA node that this process may use (one hardware thread per core
    with ``one_per_core``: two busy threads of ours never share a core), or None."""
    node = gpu_numa_node(device)
    if node is None:
        return None
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as fh:
            local = _parse_cpulist(fh.read())
    except OSError:
        return None
    mine = local & os.sched_getaffinity(0)
    if one_per_core and mine:
        mine = _one_per_core(mine)
    return mine or None


def bind_local(device: int = 0, one_per_core: bool = False) -> Optional[set]:
    """Restrict this process to the GPU-local CPUs (returns them), or leave it (None).

    sched_setaffinity(0, ...) moves the calling thread only (Linux affinity is per thread), so
    every thread the process already runs — HIP / torch runtime threads, worker-pool threads of
    an earlier parallel call — is moved too, through /proc/self/task; threads created later
    inherit the mask from their creator."""
    cpus = gpu_local_cpus(device, one_per_core)
    if cpus:
        os.sched_setaffinity(0, cpus)
        try:
            tids = [int(t) for t in os.listdir("/proc/self/task")]
        except OSError:
            tids = []
        for tid in tids:
            try:
                os.sched_setaffinity(tid, cpus)
            except OSError:  # the thread ended meanwhile
                pass
    return cpus


def page_nodes(addr: int, nbytes: int, samples: int = 64) -> Optional[dict]:
    """{NUMA node: pages} over ``samples`` pages spread across [addr, addr + nbytes) (the
    move_pages query form: no page moves), or None where the kernel does not say.  Where a
    page-locked staging buffer landed decides whether the H2D DMA and the staging threads
    cross the socket link."""
    import ctypes
    import platform

    if nbytes <= 0 or platform.machine() != "x86_64":
        return None
    page = os.sysconf("SC_PAGE_SIZE")
    first = addr // page * page
    n = max(1, min(samples, nbytes // page))
    step = max(page, (nbytes // n) // page * page)
    pages = (ctypes.c_void_p * n)(*[first + i * step for i in range(n)])
    status = (ctypes.c_int * n)()
    libc = ctypes.CDLL(None, use_errno=True)
    SYS_move_pages = 279
    if libc.syscall(SYS_move_pages, 0, ctypes.c_ulong(n), pages, None, status, 0) != 0:
        return None
    out: dict = {}
    for s in status:
        out[int(s)] = out.get(int(s), 0) + 1  # a negative entry: -errno (e.g. -14 not mapped)
    return out


def mapping_info(addr: int, nbytes: int = 1) -> Optional[dict]:
    """The /proc/self/smaps entries overlapping [addr, addr + nbytes), summed: Size, Rss and
    how much is backed by transparent huge pages (kB), and the mappings' count, or None.  A
    DMA source on 4-KiB pages costs the IOMMU one translation per 4 KiB; on 2-MiB pages, one per
    2 MiB."""
    keys = ("Size:", "Rss:", "AnonHugePages:", "Locked:")
    out: dict = {}
    try:
        with open("/proc/self/smaps") as fh:
            take = False
            for line in fh:
                head = line.split(None, 1)[0]
                if not head.endswith(":"):
                    lo, hi = (int(x, 16) for x in head.split("-"))
                    take = lo < addr + max(nbytes, 1) and hi > addr
                    if take:
                        out["mappings"] = out.get("mappings", 0) + 1
                elif take and head in keys:
                    out[head[:-1]] = out.get(head[:-1], 0) + int(line.split()[1])
    except (OSError, ValueError):
        return None
    return out or None


__all__ = ["bind_local", "gpu_local_cpus", "gpu_numa_node", "mapping_info", "page_nodes"]
