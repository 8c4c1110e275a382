"""engine.serialized restores the calling thread's current HIP device (the session calls bind their
own device to the thread): a multi-device aggregation must not leave the caller's later work -- its
training, in simulate_experiment -- on the last GPU the engine drove.  CPU: a recording fake of the
two C-ABI calls (fedagg_device_get / fedagg_device_set)."""

import ctypes

import pytest

from substrafl_amd import _native, engine


class _Lib:
    def __init__(self, current=0, get_rc=0):
        self.current, self.get_rc, self.sets = current, get_rc, []

    def fedagg_device_get(self, out):
        out._obj.value = self.current
        return self.get_rc

    def fedagg_device_set(self, d):
        self.sets.append(d)
        self.current = d
        return 0


class _Engine:
    def __init__(self, lib, devices):
        self.lib, self.devices = lib, devices

    def lock_devices(self):
        return self.devices

    @engine.serialized
    def call(self, fail=False):
        self.lib.current = self.devices[-1]  # what the session calls do to the thread
        if fail:
            raise RuntimeError("boom")
        return "ok"


@pytest.mark.parametrize("fail", [False, True])
def test_serialized_restores_the_callers_device(monkeypatch, fail):
    lib = _Lib(current=2)
    monkeypatch.setattr(_native, "load", lambda: lib)
    e = _Engine(lib, [0, 5, 7])
    if fail:
        with pytest.raises(RuntimeError):
            e.call(fail=True)
    else:
        assert e.call() == "ok"
    assert lib.current == 2 and lib.sets == [2]


def test_no_device_to_restore_without_a_gpu(monkeypatch):
    lib = _Lib(current=0, get_rc=100)  # hipGetDevice fails (no GPU): nothing is set back
    monkeypatch.setattr(_native, "load", lambda: lib)
    assert _Engine(lib, [0]).call() == "ok" and lib.sets == []


def test_abi_exports_the_device_calls():
    lib = _native.load()
    assert callable(lib.fedagg_device_get) and callable(lib.fedagg_device_set)
    assert _native.SIGNATURES["fedagg_device_get"][1] == [ctypes.POINTER(ctypes.c_int)]


def test_locks_released_when_the_library_fails_to_load(monkeypatch):
    """a load failure (missing library, ABI mismatch) inside serialized raises to the
    caller and releases the device locks -- another thread's call then gets the same error
    instead of blocking forever."""
    import threading

    from substrafl_amd import runtime

    def boom():
        raise _native.NativeLibraryError("no library")

    monkeypatch.setattr(_native, "load", boom)
    e = _Engine(None, [0, 3])
    with pytest.raises(_native.NativeLibraryError):
        e.call()
    for d in (0, 3):
        lk = runtime.device_lock(d)
        assert lk.acquire(timeout=1)  # free
        lk.release()
    errs = []
    th = threading.Thread(target=lambda: errs.append(pytest.raises(_native.NativeLibraryError, e.call)))
    th.start()
    th.join(timeout=5)
    assert not th.is_alive() and errs
