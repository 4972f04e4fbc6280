"""NUMA placement of the host lane's shared segments (Linux syscalls through ctypes, no libnuma).

A lane segment is written by the sender's D2H and read by the receiver's H2D. Its pages are
reserved by the sender (``posix_fallocate`` in hostlane.py), so without a policy they land on the
sender's current node; on a two-socket host some pairs' copies then cross the socket link. The
lane binds each segment to the NUMA node of its RECEIVING GPU while the pages are reserved
(``preferred``: the thread's policy, MPOL_PREFERRED, restored to the default right after), so
the receiver's H2D reads local memory and only a cross-socket pair's D2H crosses the link; and
reports where the pages are (``node_of``). Every call degrades to "no placement" where the kernel
or a sandbox refuses the syscall: placement is an optimisation, never a condition to run.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import platform
from typing import Optional

# x86_64 syscall numbers (the MI355X hosts are x86_64); other machines: no placement
_SYS = {"x86_64": {"mbind": 237, "set_mempolicy": 238, "get_mempolicy": 239}}.get(platform.machine(), {})
MPOL_DEFAULT, MPOL_PREFERRED = 0, 1
MPOL_F_NODE, MPOL_F_ADDR = 1 << 0, 1 << 1

_libc = None


def _syscall():
    global _libc
    if _libc is None:
        _libc = ctypes.CDLL(None, use_errno=True)
        _libc.syscall.restype = ctypes.c_long
    return _libc.syscall


def available() -> bool:
    return bool(_SYS)


def set_preferred(node: Optional[int]) -> Optional[str]:
    """The calling thread's memory policy: MPOL_PREFERRED on ``node`` (None or < 0: the default
    policy). Returns None on success, else the reason it was not applied."""
    if not _SYS:
        return f"no NUMA syscalls known for {platform.machine()}"
    sc = _syscall()
    if node is None or node < 0:
        rc = sc(_SYS["set_mempolicy"], ctypes.c_int(MPOL_DEFAULT), None, ctypes.c_ulong(0))
    else:
        nbits = max(64, (int(node) // 64 + 1) * 64)
        mask = (ctypes.c_ulong * (nbits // 64))()
        mask[node // 64] = 1 << (node % 64)
        rc = sc(_SYS["set_mempolicy"], ctypes.c_int(MPOL_PREFERRED), mask, ctypes.c_ulong(nbits + 1))
    if rc != 0:
        e = ctypes.get_errno()
        return f"set_mempolicy: {os.strerror(e)} (errno {e})"
    return None


@contextlib.contextmanager
def preferred(node: Optional[int]):
    """Within the block, this thread's page allocations prefer ``node``; yields None when the
    policy is in force, else why not (the block runs either way)."""
    if node is None or node < 0:
        yield "no NUMA node given"
        return
    why = set_preferred(node)
    try:
        yield why
    finally:
        if why is None:
            set_preferred(None)


def node_of(addr: int) -> Optional[int]:
    """The NUMA node of the page at host address ``addr`` (get_mempolicy MPOL_F_NODE |
    MPOL_F_ADDR; the page is faulted in as by a read), or None when the kernel will not say."""
    if not _SYS:
        return None
    mode = ctypes.c_int(-1)
    rc = _syscall()(_SYS["get_mempolicy"], ctypes.byref(mode), None, ctypes.c_ulong(0),
                    ctypes.c_void_p(addr), ctypes.c_ulong(MPOL_F_NODE | MPOL_F_ADDR))
    return int(mode.value) if rc == 0 and mode.value >= 0 else None


def gpu_numa_node(device: int) -> Optional[int]:
    """The NUMA node the kernel reports for GPU ``device``'s PCI function (None: unknown, or a
    single-node host reporting -1)."""
    try:
        import torch
        pr = torch.cuda.get_device_properties(device)
        bdf = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
        with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as fh:
            n = int(fh.read().strip())
    except (OSError, ValueError, AttributeError, RuntimeError):
        return None
    return n if n >= 0 else None
