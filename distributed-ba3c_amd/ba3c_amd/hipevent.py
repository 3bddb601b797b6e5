"""HIP events with explicit fence flags (torch.cuda.Event cannot pass them).

torch.cuda.Event records with HIP's default system-scope release, and on MI355X that release
writes back the eight XCDs' L2s and invalidates them: each recorded event left a 5-6 us gap in
the step's kernel timeline (rocprofv3, profiles/r06/).  Timing marks only need the timestamp,
so `timing_event()` records with hipEventDisableSystemFence.  Stream joins need ordering, not a
cache flush: every kernel of this path reads and writes device memory only, and HIP's kernel
dispatch packets already carry the agent-scope acquire / release that orders one kernel's
stores before a later kernel's loads on any queue, so `join_event()` records with
hipEventReleaseToDevice (a device-scope release, the scope those kernels need).

The library is the HIP runtime torch loaded (torch/lib/libamdhip64.so), the one libba3c.so and
RCCL resolve to as well, so these events live in the same runtime as torch's streams.
"""
import ctypes
import os

import torch

HIP_EVENT_DISABLE_TIMING = 0x2
HIP_EVENT_DISABLE_SYSTEM_FENCE = 0x20000000
HIP_EVENT_RELEASE_TO_DEVICE = 0x40000000

_HIP = None


def _hip():
    global _HIP
    if _HIP is None:
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
        lib = ctypes.CDLL(path if os.path.exists(path) else "libamdhip64.so")
        P = ctypes.c_void_p
        lib.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(P), ctypes.c_uint]
        lib.hipEventRecord.argtypes = [P, P]
        lib.hipEventSynchronize.argtypes = [P]
        lib.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), P, P]
        lib.hipEventDestroy.argtypes = [P]
        lib.hipStreamWaitEvent.argtypes = [P, P, ctypes.c_uint]
        lib.hipGetErrorString.restype = ctypes.c_char_p
        lib.hipGetErrorString.argtypes = [ctypes.c_int]
        _HIP = lib
    return _HIP


def _check(rc, what):
    if rc != 0:
        raise RuntimeError("%s failed: %s" % (what, _hip().hipGetErrorString(rc).decode()))


def _stream_ptr(stream):
    if stream is None:
        stream = torch.cuda.current_stream()
    return ctypes.c_void_p(stream.cuda_stream)


class HipEvent(object):
    """A HIP event created with explicit flags; API as torch.cuda.Event's (record, wait,
    elapsed_time, synchronize)."""

    def __init__(self, flags):
        self.flags = flags
        self._ev = ctypes.c_void_p()
        _check(_hip().hipEventCreateWithFlags(ctypes.byref(self._ev), flags),
               "hipEventCreateWithFlags")

    def record(self, stream=None):
        _check(_hip().hipEventRecord(self._ev, _stream_ptr(stream)), "hipEventRecord")

    def wait(self, stream=None):
        """Make `stream` (default: the current one) wait for this event."""
        _check(_hip().hipStreamWaitEvent(_stream_ptr(stream), self._ev, 0), "hipStreamWaitEvent")

    def synchronize(self):
        _check(_hip().hipEventSynchronize(self._ev), "hipEventSynchronize")

    def elapsed_time(self, end):
        """Milliseconds from this event to `end` (waits for `end`)."""
        end.synchronize()
        ms = ctypes.c_float()
        _check(_hip().hipEventElapsedTime(ctypes.byref(ms), self._ev, end._ev),
               "hipEventElapsedTime")
        return float(ms.value)

    def __del__(self):
        try:
            if self._ev:
                _hip().hipEventDestroy(self._ev)
                self._ev = ctypes.c_void_p()
        except Exception:
            pass


def event_mode():
    """BA3C_EVENTS: 'light' (default: timing marks without a system fence, joins with a device
    release) or 'torch' (torch.cuda.Event for both: the system-scope defaults, A/B)."""
    m = os.environ.get("BA3C_EVENTS", "light")
    if m not in ("light", "torch"):
        raise ValueError("BA3C_EVENTS must be 'light' or 'torch' (got %r)" % m)
    return m


def timing_event():
    """An event for timestamps only (no fence)."""
    if event_mode() == "torch":
        return torch.cuda.Event(enable_timing=True)
    return HipEvent(HIP_EVENT_DISABLE_SYSTEM_FENCE)


def join_event():
    """An event for ordering one stream after another's device work (device-scope release)."""
    if event_mode() == "torch":
        return torch.cuda.Event()
    return HipEvent(HIP_EVENT_DISABLE_TIMING | HIP_EVENT_RELEASE_TO_DEVICE)


def wait_stream(waiter, other, ev=None):
    """`waiter` waits for the work enqueued on `other` so far (torch.cuda.Stream.wait_stream
    with a device-scope event).  `ev`: a join_event() to reuse."""
    if event_mode() == "torch" and ev is None:
        waiter.wait_stream(other)
        return
    ev = ev or join_event()
    ev.record(other)
    if isinstance(ev, HipEvent):
        ev.wait(waiter)
    else:
        waiter.wait_event(ev)
