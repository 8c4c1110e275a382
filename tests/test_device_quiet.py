"""bench.wait_device_quiet (the timed region starts after the driver has cleared the previous
process's freed device memory; DESIGN §5 "C5 per launch") against a stand-in amdsmi: it waits
while the firmware-averaged SOC clock is high, stops when it falls, gives up at its bound, and
labels the record when amdsmi is absent -- never raising into the bench line."""

import sys
import types

import pytest

import bench


class _FakeSmi(types.ModuleType):
    def __init__(self, socs, bdf="0000:a7:00.0"):
        super().__init__("amdsmi")
        self.socs, self.bdf, self.reads, self.shut = list(socs), bdf, 0, False

    def amdsmi_init(self):
        pass

    def amdsmi_shut_down(self):
        self.shut = True

    def amdsmi_get_processor_handles(self):
        return ["h0"]

    def amdsmi_get_gpu_device_bdf(self, h):
        return self.bdf

    def amdsmi_get_gpu_metrics_info(self, h):
        v = self.socs[min(self.reads, len(self.socs) - 1)]
        self.reads += 1
        return {"current_socclks": [v, v, "N/A", 65535]}


@pytest.fixture
def fake(monkeypatch):
    import substrafl_amd.runtime as rt

    monkeypatch.setattr(rt, "device_pci_bus_id", lambda d: "0000:a7:00.0")

    def install(socs, **kw):
        m = _FakeSmi(socs, **kw)
        monkeypatch.setitem(sys.modules, "amdsmi", m)
        return m

    return install


def test_waits_while_the_clear_runs(fake):
    m = fake([328.5, 328.5, 312.0, 180.0])
    rec = bench.wait_device_quiet(0)
    assert rec["soc_clock_mhz_at_check"] == 328.5 and rec["soc_clock_mhz_at_start"] == 180.0
    assert rec["waited_s"] >= 0.05 and rec["gave_up"] is False and m.shut


def test_no_wait_when_quiet(fake):
    fake([39.5])
    rec = bench.wait_device_quiet(0)
    assert rec["waited_s"] < 0.05 and rec["soc_clock_mhz_at_start"] == 39.5 and not rec["gave_up"]


def test_gives_up_at_its_bound(fake):
    fake([328.5])
    rec = bench.wait_device_quiet(0, limit_s=0.1)
    assert rec["gave_up"] is True and 0.1 <= rec["waited_s"] < 1.0


def test_other_device_or_no_amdsmi_is_labelled(fake, monkeypatch):
    fake([328.5], bdf="0000:05:00.0")
    assert "no amdsmi handle" in bench.wait_device_quiet(0)["skipped"]
    monkeypatch.setitem(sys.modules, "amdsmi", None)  # import amdsmi -> ImportError
    assert "skipped" in bench.wait_device_quiet(0)
