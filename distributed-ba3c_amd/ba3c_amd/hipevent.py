"""HIP events with explicit fence flags (torch.cuda.Event cannot pass them).

torch.cuda.Event records with HIP's default system-scope release.  Timing marks only need the
timestamp, so `timing_event()` records with hipEventDisableSystemFence.  Stream joins need
ordering, not a system-scope flush: every kernel of this path reads and writes device memory
only, and HIP's kernel dispatch packets already carry the agent-scope acquire / release that
orders one kernel's stores before a later kernel's loads on any queue, so `join_event()`
records with hipEventReleaseToDevice.  Measured (profiles/r06/, same box): the world-1 N>1 step
1.779 -> 1.761 ms with these events for its cross-stream joins; the N=1 step is unchanged.
What the flags do NOT remove: every event recorded on the learner stream between two of its
kernels still leaves a 5-6 us gap in the kernel timeline (rocprofv3 traces r06b-d, whatever
the flags), so the step records as few as it needs and the timing marks stay out of the timed
steps (bench.py).

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
        lib.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(P), ctypes.c_uint32,
                                                     ctypes.POINTER(ctypes.c_uint32)]
        lib.hipStreamDestroy.argtypes = [P]
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


class CuMaskedStream(object):
    """A HIP stream whose kernels may only use `n_cus` of the device's CUs
    (hipExtStreamCreateWithCUMask), spread evenly over the CU numbering, as a torch stream
    (`.stream`, torch.cuda.ExternalStream).  bench.py's configs[4] partition: the predictor's
    forward on a subset of the CUs beside the learner's step."""

    def __init__(self, n_cus, device=None):
        dev = torch.device(device or "cuda")
        total = torch.cuda.get_device_properties(dev).multi_processor_count
        if not 0 < n_cus <= total:
            raise ValueError("n_cus must be in [1, %d]" % total)
        words = (total + 31) // 32
        mask = (ctypes.c_uint32 * words)()
        for i in range(n_cus):
            cu = (i * total) // n_cus
            mask[cu // 32] |= 1 << (cu % 32)
        self.n_cus = n_cus
        self._s = ctypes.c_void_p()
        with torch.cuda.device(dev):
            _check(_hip().hipExtStreamCreateWithCUMask(ctypes.byref(self._s), words, mask),
                   "hipExtStreamCreateWithCUMask")
        self.stream = torch.cuda.ExternalStream(self._s.value, device=dev)

    def __del__(self):
        try:
            if self._s:
                _hip().hipStreamDestroy(self._s)
                self._s = ctypes.c_void_p()
        except Exception:
            pass
