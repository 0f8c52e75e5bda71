"""Device buffers, streams and events of the HIP runtime libdwpa22000.so runs its kernels on.

The product path owns its runtime: a framework that bundles a second libamdhip64 (the torch ROCm wheel does)
must not hand its streams or events to the library.  Device pointers are plain addresses.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as L


class DeviceBuffer:
    def __init__(self, nbytes: int, device: int = 0):
        self.device, self.nbytes = device, int(nbytes)
        p = ctypes.c_void_p()
        L.check(L.load().dwpa_dev_alloc(device, self.nbytes, ctypes.byref(p)), "dev_alloc")
        self.ptr = p.value

    @classmethod
    def from_numpy(cls, arr: np.ndarray, device: int = 0, pad: int = 0):
        arr = np.ascontiguousarray(arr)
        b = cls(arr.nbytes + pad, device)
        L.check(L.load().dwpa_dev_upload(device, b.ptr, arr.ctypes.data, arr.nbytes), "dev_upload")
        return b

    def download(self, nbytes: int | None = None, offset: int = 0) -> bytes:
        n = self.nbytes - offset if nbytes is None else nbytes
        out = ctypes.create_string_buffer(max(1, n))
        L.check(L.load().dwpa_dev_download(self.device, out, self.ptr + offset, n), "dev_download")
        return out.raw[:n]

    def free(self):
        if self.ptr:
            L.load().dwpa_dev_free(self.device, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Stream:
    def __init__(self, device: int = 0):
        p = ctypes.c_void_p()
        L.check(L.load().dwpa_stream_create(device, ctypes.byref(p)), "stream_create")
        self.handle = p.value

    def synchronize(self):
        L.check(L.load().dwpa_stream_sync(self.handle), "stream_sync")

    def __del__(self):
        try:
            L.load().dwpa_stream_destroy(self.handle)
        except Exception:
            pass


class Event:
    def __init__(self, device: int = 0):
        p = ctypes.c_void_p()
        L.check(L.load().dwpa_event_create(device, ctypes.byref(p)), "event_create")
        self.handle = p.value

    def record(self, stream: Stream | None = None):
        L.check(L.load().dwpa_event_record(self.handle, stream.handle if stream else None), "event_record")

    def elapsed_ms(self, stop: "Event") -> float:
        ms = ctypes.c_float(0)
        L.check(L.load().dwpa_event_elapsed_ms(self.handle, stop.handle, ctypes.byref(ms)), "event_elapsed")
        return float(ms.value)

    def __del__(self):
        try:
            L.load().dwpa_event_destroy(self.handle)
        except Exception:
            pass


def dictionary_arrays(words):
    """list of bytes -> (uint64 offsets[n+1], uint8 bytes) host arrays in the HBM dictionary layout."""
    lens = np.fromiter((len(w) for w in words), dtype=np.int64, count=len(words))
    off = np.zeros(len(words) + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    data = np.frombuffer(b"".join(words) + b"\0" * 64, dtype=np.uint8)
    return off, data


class Dictionary:
    """An HBM-resident dictionary: uint64 offsets[n+1] + bytes (64 zero bytes of tail padding)."""

    def __init__(self, off: np.ndarray, data: np.ndarray, device: int = 0):
        self.n = len(off) - 1
        self.off = DeviceBuffer.from_numpy(off.astype(np.uint64), device)
        self.data = DeviceBuffer.from_numpy(data, device, pad=64)

    @classmethod
    def from_words(cls, words, device: int = 0):
        off, data = dictionary_arrays(words)
        return cls(off, data, device)
