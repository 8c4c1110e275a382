"""The per-rank stream budget of the client-sharded executors (DESIGN.md §6 "Streams"): HIP maps a
process's streams onto GPU_MAX_HW_QUEUES (4 on the boxes) hardware queues, so the push executor's
aux streams are capped at what the queues leave after the caller's stream -- and after a live
native RCCL communicator's three (its own stream, RCCL's device and host streams)."""

import pytest

from substrafl_amd import push
from substrafl_amd.rccl import RcclTransport


def test_budget_alone_fills_the_queues():
    assert push.aux_stream_budget(4, rccl_live=False) == 3  # caller + 3 aux = 4 queues
    assert push.aux_stream_budget(8, rccl_live=False) == 3  # never more than a step's launches need
    assert push.aux_stream_budget(2, rccl_live=False) == 1
    assert push.aux_stream_budget(1, rccl_live=False) == 0


def test_budget_with_a_live_communicator():
    assert push.aux_stream_budget(4, rccl_live=True) == 0  # caller + comm + RCCL's two = 4
    assert push.aux_stream_budget(6, rccl_live=True) == 2
    for q in range(1, 33):
        for live in (False, True):
            n = push.aux_stream_budget(q, rccl_live=live)
            assert 0 <= n <= 3
            assert 1 + n + (push.RCCL_STREAMS if live else 0) <= max(q, 1 + (push.RCCL_STREAMS if live else 0))


def test_hw_queues_from_the_environment(monkeypatch):
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    assert push._hw_queues() == 4
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "2")
    assert push._hw_queues() == 2
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "bogus")
    assert push._hw_queues() == push.GPU_MAX_HW_QUEUES
    monkeypatch.delenv("GPU_MAX_HW_QUEUES")
    assert push._hw_queues() == push.GPU_MAX_HW_QUEUES


def test_execute_caps_aux_streams_while_a_communicator_lives(monkeypatch):
    """PushTransport.execute passes at most aux_stream_budget(queues, live communicators > 0) aux
    streams to fedagg_push_execute, whatever it created (no GPU: the native call is recorded)."""
    seen = {}

    class Lib:
        def fedagg_push_execute(self, *a):
            seen["naux"] = a[-2]
            seen["aux"] = a[-3]
            return 0

    class Prog:
        nruns = nwaits = ntags = 0
        runs = waits = tags = None
        nsteps = 3
        ncopies = 0
        copies = None
        stage_u = None

        class plan:
            root = 0

    tr = object.__new__(push.PushTransport)
    tr.lib, tr.world, tr.rank, tr.base, tr._timeout, tr._dev = Lib(), 2, 1, 0, 1, 0
    tr._page = __import__("numpy").zeros(8, "uint64")
    tr._aux = [object()] * 3
    tr._aux_ptrs = object()
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    monkeypatch.setattr(RcclTransport, "_live", 0)
    tr.execute(Prog(), 0)
    assert seen["naux"] == 3
    monkeypatch.setattr(RcclTransport, "_live", 1)
    tr.execute(Prog(), 0)
    assert seen["naux"] == 0 and seen["aux"] is None
    assert tr.base == 2 * (Prog.nsteps + 1)


@pytest.mark.parametrize("q", [4])
def test_design_table_counts(q):
    """The DESIGN.md table: native 4 streams, push alone 4, push beside a live communicator 4."""
    assert 1 + push.RCCL_STREAMS == q
    assert 1 + push.aux_stream_budget(q, False) == q
    assert 1 + push.aux_stream_budget(q, True) + push.RCCL_STREAMS == q
