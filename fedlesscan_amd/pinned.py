"""Page-locked host buffers (hipHostMalloc through the C-ABI) exposed as memoryviews.

A result store that writes each client document into page-locked memory
(store.InMemoryClientResultStore(pinned=True)) lets StreamingFold DMA every
layer straight from the document into the device chunk (fa_copy_h2d) instead
of packing it into staging first (fa_pack).  The memory is released when the
last view into it is gone.  Needs a GPU (the HIP runtime allocates it).
"""
from __future__ import annotations

import ctypes
import sys

from . import _lib


class _Pin:
    """Owns one hipHostMalloc block; freed when the last view drops it."""

    __slots__ = ("ptr", "__weakref__")

    def __init__(self, n: int):
        p = ctypes.c_void_p()
        _lib.call("fa_host_alloc", ctypes.addressof(p), n)
        self.ptr = p.value

    def __del__(self):
        if self.ptr and not sys.is_finalizing():
            _lib.load().fa_host_free(self.ptr)
        self.ptr = None


def pinned_bytes(n: int) -> memoryview:
    """A writable, page-locked byte buffer of n bytes (n >= 1)."""
    if n <= 0:
        raise ValueError("pinned_bytes needs n >= 1")
    pin = _Pin(n)
    arr = (ctypes.c_uint8 * n).from_address(pin.ptr)
    arr._pin = pin  # the array (and every memoryview of it) keeps the block alive
    return memoryview(arr).cast("B")


def is_pinned(ptr: int, nbytes: int) -> bool:
    """True if [ptr, ptr+nbytes) lies inside one page-locked allocation."""
    return bool(_lib.load().fa_host_is_pinned(ptr, nbytes))
