"""CPU: failure handling of the direct-RCCL data-parallel step (rgbac/parallel.py).

* CommWatchdog against a stub communicator: an asynchronous RCCL error, or an armed step that
  overruns its deadline, aborts the communicator and ends the process with a non-zero status
  (the exit function is injected here, so nothing exits); a step whose completion query turns
  true is disarmed and never fires.
* GradBuckets refuses to finish a step whose gradient notifications differ from the learning
  step's (a non-tail bucket still pending at the end of backward would be launched late,
  after buckets other ranks already sent: mismatched collectives)."""
import threading

import pytest
import torch
import torch.distributed as dist

from rgbac.parallel import CommWatchdog, GradBuckets


class StubComm:
    def __init__(self):
        self.err = 0
        self.aborts = 0

    def async_error(self):
        return self.err

    def abort(self):
        self.aborts += 1


class Clock:
    def __init__(self):
        self.t = 100.0

    def __call__(self):
        return self.t


def _dog(comm, clock, exits, timeout=10.0):
    return CommWatchdog(comm, timeout_s=timeout, poll_s=0.01, exit_code=7,
                        exit_fn=exits.append, clock=clock, log=lambda m: None)


def test_deadline_aborts_and_exits_nonzero():
    comm, clock, exits = StubComm(), Clock(), []
    wd = _dog(comm, clock, exits)
    assert wd.check() is None                 # not armed: nothing to time
    wd.arm(done=lambda: False)
    clock.t += 9.0
    assert wd.check() is None and comm.aborts == 0 and exits == []
    clock.t += 2.0                            # 11 s > 10 s deadline
    reason = wd.check()
    assert reason is not None and "not complete" in reason
    assert comm.aborts == 1 and exits == [7]
    assert wd.check() == reason and comm.aborts == 1 and exits == [7]   # fires once


def test_async_error_fires_unarmed():
    comm, clock, exits = StubComm(), Clock(), []
    wd = _dog(comm, clock, exits)
    comm.err = 6                              # e.g. ncclRemoteError
    reason = wd.check()
    assert reason is not None and "asynchronous error 6" in reason
    assert comm.aborts == 1 and exits == [7]


def test_completed_step_disarms():
    comm, clock, exits = StubComm(), Clock(), []
    wd = _dog(comm, clock, exits)
    state = {"done": False}
    wd.arm(done=lambda: state["done"])
    clock.t += 5.0
    assert wd.check() is None
    state["done"] = True
    assert wd.check() is None                 # completion seen: disarmed
    clock.t += 100.0
    assert wd.check() is None and comm.aborts == 0 and exits == []
    wd.arm()                                  # explicit disarm path
    wd.disarm()
    clock.t += 100.0
    assert wd.check() is None and exits == []


def test_thread_fires_on_error():
    comm, exits = StubComm(), []
    fired = threading.Event()

    def ex(code):
        exits.append(code)
        fired.set()
    wd = CommWatchdog(comm, timeout_s=60.0, poll_s=0.005, exit_code=5, exit_fn=ex,
                      log=lambda m: None).start()
    try:
        comm.err = 3
        assert fired.wait(5.0)
    finally:
        wd.stop()
    assert exits == [5] and comm.aborts == 1


@pytest.fixture
def world1():
    dist.init_process_group("gloo", store=dist.HashStore(), rank=0, world_size=1)
    yield
    dist.destroy_process_group()


def test_buckets_refuse_changed_graph(world1):
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(6, 16), torch.nn.GELU(), torch.nn.Linear(16, 3))
    params = list(m.parameters())
    flat = torch.zeros(sum(p.numel() for p in params))
    off = 0
    for p in params:
        p.grad = flat[off:off + p.numel()].view_as(p)
        off += p.numel()
    gb = GradBuckets(params, flat, bucket_bytes=64)
    x = torch.randn((4, 6))
    for _ in range(2):                        # learning step, then a regular one
        gb.begin()
        m(x).pow(2).sum().backward()
        gb.finish()
    assert gb.learned
    # the first layer takes no part in this loss: its bucket never completes in backward
    gb.begin()
    h = m[1](m[0](x).detach())
    m[2](h).pow(2).sum().backward()
    with pytest.raises(RuntimeError, match="autograd graph changed"):
        gb.finish()
    gb.remove()


class ClosableComm(StubComm):
    """A stub with RcclComm's close protocol: ``comm`` is None once closed, and close()
    stops every attached watchdog first."""

    def __init__(self):
        super().__init__()
        self.comm = object()
        self.watchdogs = []
        self.polls = 0

    def async_error(self):
        assert self.comm is not None, "polled a closed communicator"
        self.polls += 1
        return 0

    def close(self):
        for wd in self.watchdogs:
            wd.stop()
        self.watchdogs = []
        self.comm = None


def test_close_stops_attached_watchdog():
    comm, clock, exits = ClosableComm(), Clock(), []
    wd = _dog(comm, clock, exits).start()
    assert comm.watchdogs == [wd]
    deadline = 200
    while comm.polls == 0 and deadline:
        threading.Event().wait(0.01)
        deadline -= 1
    comm.close()
    assert wd._thread is None
    assert wd.check() is None and exits == []        # a closed communicator is not polled


def _agree_worker(rank, world, port, out):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rgbac.parallel import group_all_ok
        out.put((rank, group_all_ok(True, torch.device("cpu")),
                 group_all_ok(rank != 1, torch.device("cpu"))))
    finally:
        dist.destroy_process_group()


def test_group_agrees_on_a_failure_gloo():
    """One rank failing (e.g. librccl.so missing there) makes every rank give the direct RCCL
    path up together (rgbac.parallel.group_all_ok, gloo world 2)."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_agree_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    assert res == [(0, True, False), (1, True, False)]
