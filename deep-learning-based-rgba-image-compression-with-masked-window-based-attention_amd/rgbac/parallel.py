"""Data-parallel training (trainRGB.py:178-198 across ranks).

One process per GPU (torchrun); every rank runs the full model on its shard of
the global batch.  The only exchange is the gradient all-reduce: the flat fp32
gradient buffer of rgbac.optim.AdamClamp is cut into ~25 MB buckets in REVERSE
parameter order (the order backward produces them), and each bucket's
all-reduce (backend "nccl" = RCCL over xGMI) is launched as soon as the last
gradient of its parameters has landed -- overlapped with the rest of backward
on RCCL's own stream.  ``finish()`` waits for all buckets and hands the 1/world
mean to the optimizer kernel, which applies it before the per-element clamp (the
reference clamps the global-batch gradient).

A bucket's gradients have landed when the post-accumulate-grad hooks of all its
parameters have fired.  That holds for both ways a gradient reaches the flat
buffer: autograd's own AccumulateGrad (GDN / EntropyBottleneck
reparametrisations, the relative-position tables, ...), and the weight-gradient
reduce kernel adding its sums straight into ``.grad`` (rgbac.autograd
DIRECT_GRAD: the conv's backward returns None for the weight, yet autograd still
runs the parameter's AccumulateGrad node -- and its hook -- once every use of the
parameter has been back-propagated, i.e. after the last add was enqueued).  So
the data-parallel step runs exactly the backward of the 1-GPU step.

The first step is a learning step: it counts the hook calls of each parameter (a
parameter that takes no part in the loss -- EntropyBottleneck.quantiles would be
one if its medians were not in the graph -- never fires) and launches every
bucket in ``finish()``.  The counts are
MAX-reduced over the ranks so every rank cuts the same buckets; from step 2 on
a bucket launches from the notification that completes its count, and
parameters that never notify sit in a tail bucket reduced in ``finish()``.
Steps from then on issue the same collectives in the same order on every rank,
so a step can be captured in a HIP graph (RCCL collectives are stream-ordered).
"""
import atexit
import contextlib
import ctypes
import os
import sys
import threading
import time

import torch
import torch.distributed as dist

from . import _lib


@contextlib.contextmanager
def _stdout_to_stderr():
    """Route file descriptor 1 to 2 while RCCL initialises: librccl prints its version banner
    to stdout, where it would land in front of bench.py's one JSON line."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        os.dup2(saved, 1)
        os.close(saved)


class RcclComm:
    """In-place sum all-reduce through RCCL called directly (csrc/comm.cpp: the librccl.so
    torch itself loaded, one ncclAllReduce per call), on a communication stream of its own:
    ``allreduce(t)`` makes that stream wait for the current (compute) stream, enqueues the
    collective there and returns an event; ``wait(ev)`` makes the current stream wait for it.
    Every step is stream-ordered, so a bucket all-reduce issued from a backward hook overlaps
    the rest of backward, and the whole step captures into a HIP graph -- no ProcessGroup
    work object or watchdog thread is involved.  torch.distributed only bootstraps it: rank
    0's 128-byte unique id is broadcast over ``group`` once.

    Communicators are cached per (group, device); the cache holds the group object itself, so
    a destroyed-and-recreated group can never be matched to a stale communicator by a recycled
    ``id``.  ``close()`` destroys one (``abort()`` aborts it), and every live one is destroyed
    at interpreter exit."""

    _cache = {}

    @classmethod
    def get(cls, device, group=None):
        gk = group if group is not None else dist.group.WORLD
        key = (id(gk), device.index, dist.get_world_size(group), dist.get_rank(group))
        ent = cls._cache.get(key)
        if ent is not None and ent[0] is gk and ent[1].comm is not None:
            return ent[1]
        if ent is not None:
            # a stale entry (the group was destroyed and re-created, or the communicator was
            # aborted): release its communicator before replacing it
            try:
                ent[1].close()
            except RuntimeError:
                pass
            del cls._cache[key]
        c = cls(device, group)
        cls._cache[key] = (gk, c)
        return c

    @classmethod
    def close_all(cls):
        for _, c in list(cls._cache.values()):
            c.close()
        cls._cache.clear()

    def __init__(self, device, group=None):
        self.comm = None
        self.watchdogs = []
        self.world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        # every rank loads and checks librccl.so BEFORE the unique id goes out, and the group
        # agrees on the outcome: one rank failing alone would otherwise fall back to
        # torch.distributed while its peers block in the broadcast or in ncclCommInitRank
        lib = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        err = None
        try:
            _lib.call("rgbac_comm_load", lib.encode())
        except (RuntimeError, OSError) as e:
            err = e
        if not group_all_ok(err is None, device, group):
            raise RuntimeError(f"direct RCCL unavailable on some rank "
                               f"({err if err is not None else 'a peer failed to load it'})")
        uid = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            with _stdout_to_stderr():
                _lib.call("rgbac_comm_unique_id", ctypes.c_void_p(uid.data_ptr()))
        if self.world > 1:
            src = dist.get_global_rank(group, 0) if group is not None else 0
            u = uid.to(device) if dist.get_backend(group) == "nccl" else uid
            dist.broadcast(u, src=src, group=group)
            uid = u.cpu()
        comm = ctypes.c_void_p()
        err = None
        try:
            with _stdout_to_stderr():
                _lib.call("rgbac_comm_init", ctypes.c_void_p(uid.data_ptr()), self.world, rank,
                          device.index, ctypes.byref(comm))
        except RuntimeError as e:
            err = e
        # an init that returned an error on one rank: every rank gives the path up together
        ok = group_all_ok(err is None, device, group)
        if not ok:
            if err is None and comm.value:
                _lib.call("rgbac_comm_destroy", comm)
            raise RuntimeError(f"RCCL communicator init failed on some rank "
                               f"({err if err is not None else 'a peer failed'})")
        self.comm = comm
        self.device = device
        self.stream = torch.cuda.Stream(device)

    def allreduce(self, t):
        cur = torch.cuda.current_stream(t.device)
        self.stream.wait_stream(cur)
        _lib.call("rgbac_comm_allreduce_sum", self.comm, _lib.dtype_code(t.dtype), t.data_ptr(),
                  t.numel(), self.stream.cuda_stream)
        ev = torch.cuda.Event()
        ev.record(self.stream)
        return ev

    def wait(self, ev):
        torch.cuda.current_stream(self.device).wait_event(ev)

    def count(self):
        """Ranks the communicator itself spans (ncclCommCount)."""
        n = ctypes.c_int(0)
        _lib.call("rgbac_comm_count", self.comm, ctypes.byref(n))
        return n.value

    def async_error(self):
        """0 while healthy, else RCCL's asynchronous error code (ncclCommGetAsyncError)."""
        e = ctypes.c_int(0)
        _lib.call("rgbac_comm_async_error", self.comm, ctypes.byref(e))
        return e.value

    def _stop_watchdogs(self):
        me = threading.current_thread()
        for wd in self.watchdogs:
            if wd._thread is not me:           # (a watchdog aborting from its own thread)
                wd.stop()
        self.watchdogs = []

    def abort(self):
        self._stop_watchdogs()
        if self.comm is not None and self.comm.value:
            _lib.call("rgbac_comm_abort", self.comm)
        self.comm = None

    def close(self):
        """Destroy the communicator; every watchdog attached to it is stopped first, so none
        polls a destroyed communicator."""
        self._stop_watchdogs()
        if self.comm is not None and self.comm.value:
            _lib.call("rgbac_comm_destroy", self.comm)
        self.comm = None


def group_all_ok(ok, device, group=None):
    """MIN-reduce a success flag over ``group`` (a CUDA tensor for an RCCL group, CPU for
    gloo): True only when every rank passed ``ok=True``."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return bool(ok)
    dev = device if dist.get_backend(group) == "nccl" else torch.device("cpu")
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()))


atexit.register(RcclComm.close_all)


class CommWatchdog:
    """Failure detection for the direct-RCCL step.  A collective whose peer died never
    completes: the surviving ranks would block inside a graph replay forever (there is no
    ProcessGroup watchdog on this path).  A host thread polls ``comm.async_error()`` every
    ``poll_s`` and, while a step is armed, its completion event; on an asynchronous error, or
    when an armed step has not completed ``timeout_s`` after ``arm()``, it aborts the
    communicator and ends the process with ``exit_code`` (``os._exit``: no Python teardown
    that could itself block on the GPU).  It never restarts or re-executes anything.

    ``comm`` needs ``async_error()`` and ``abort()``; ``exit_fn`` and ``clock`` are
    injectable (tests run it against a stub communicator on the CPU)."""

    def __init__(self, comm, timeout_s=300.0, poll_s=0.5, exit_code=3, exit_fn=None,
                 clock=None, log=None):
        self.comm, self.timeout_s, self.poll_s, self.exit_code = comm, timeout_s, poll_s, exit_code
        self.exit_fn = exit_fn if exit_fn is not None else os._exit
        self.clock = clock if clock is not None else time.monotonic
        self.log = log if log is not None else (lambda m: print(m, file=sys.stderr, flush=True))
        self._lock = threading.Lock()
        self._deadline = None
        self._done = None                  # callable -> True once the armed step completed
        self.fired = None                  # reason string once it fired
        self._stop = threading.Event()
        self._thread = None

    def start(self):
        ws = getattr(self.comm, "watchdogs", None)
        if ws is not None and self not in ws:
            ws.append(self)                # the communicator's close() / abort() stops it
        if self._thread is None:
            self._thread = threading.Thread(target=self._run, name="rgbac-comm-watchdog",
                                            daemon=True)
            self._thread.start()
        return self

    def stop(self):
        self._stop.set()
        if self._thread is not None and self._thread is not threading.current_thread():
            self._thread.join()
        self._thread = None

    def arm(self, done=None):
        """A step was enqueued; ``done()`` (e.g. a recorded event's ``query``) says when it has
        completed.  ``done=None``: the caller disarms explicitly."""
        with self._lock:
            self._deadline = self.clock() + self.timeout_s
            self._done = done

    def disarm(self):
        with self._lock:
            self._deadline = None
            self._done = None

    def check(self):
        """One poll (the thread's body; callable directly).  Returns the reason it fired, or
        None."""
        if self.fired is not None:
            return self.fired
        if getattr(self.comm, "comm", True) is None:
            return None                    # the communicator was closed: nothing to watch
        reason = None
        err = self.comm.async_error()
        if err:
            reason = f"RCCL asynchronous error {err}"
        else:
            with self._lock:
                dl, done = self._deadline, self._done
            if dl is not None:
                if done is not None and done():
                    self.disarm()
                elif self.clock() > dl:
                    reason = f"step not complete {self.timeout_s:.1f} s after it was enqueued"
        if reason is not None:
            self.fired = reason
            self.log(f"rgbac.parallel: {reason}; aborting the communicator and exiting "
                     f"with status {self.exit_code}")
            try:
                self.comm.abort()
            finally:
                self.exit_fn(self.exit_code)
        return reason

    def _run(self):
        while not self._stop.wait(self.poll_s):
            if getattr(self.comm, "comm", True) is None:
                return                     # closed: stop quietly
            if self.check() is not None:
                return


class GradBuckets:
    """Bucketed all-reduce of the flat gradient buffer, launched from the parameters'
    post-accumulate-grad hooks."""

    def __init__(self, params, flat_grad, bucket_bytes=25 << 20, group=None, comm=None):
        self.params = list(params)
        self.flat = flat_grad
        self.group = group
        self.comm = comm                   # RcclComm, or None: torch.distributed.all_reduce
        self.world = dist.get_world_size(group)
        # param i occupies [off_i, off_i + n_i) of the flat buffer (AdamClamp layout)
        self.offs, off = [], 0
        for p in self.params:
            self.offs.append((off, p.numel()))
            off += p.numel()
        assert off == flat_grad.numel()
        self.per = max(1, bucket_bytes // flat_grad.element_size())
        self.expect = None                 # notifications per parameter per step (learned)
        self.count = [0] * len(self.params)
        self._cut(list(range(len(self.params) - 1, -1, -1)), [])
        self.active = False
        # measurement only (bench.py's exposed all-reduce time): issue no collective at all
        self.skip = False
        self.hooks = [p.register_post_accumulate_grad_hook(self._hook(i))
                      for i, p in enumerate(self.params)]

    @property
    def learned(self):
        return self.expect is not None

    def _runs(self, idx):
        """Contiguous flat ranges covering params ``idx``."""
        rs = sorted(self.offs[i] for i in idx)
        out = []
        for lo, n in rs:
            if out and out[-1][1] == lo:
                out[-1][1] = lo + n
            else:
                out.append([lo, lo + n])
        return [tuple(r) for r in out]

    def _cut(self, order, tail):
        """Buckets of ~per elements over ``order`` (backward order), plus a tail bucket."""
        self.buckets = []                  # [ranges, [param idx]]
        cur, size = [], 0
        for i in order:
            cur.append(i)
            size += self.offs[i][1]
            if size >= self.per:
                self.buckets.append([self._runs(cur), cur])
                cur, size = [], 0
        if cur:
            self.buckets.append([self._runs(cur), cur])
        self.tail = None
        if tail:
            self.tail = len(self.buckets)
            self.buckets.append([self._runs(tail), list(tail)])
        self.owner = {}
        for b, (_, idx) in enumerate(self.buckets):
            for i in idx:
                self.owner[i] = b
        self.pending = [0] * len(self.buckets)
        self.works = [None] * len(self.buckets)

    def _hook(self, i):
        def fn(_p):
            self._note(i)
        return fn

    def _note(self, i):
        if not self.active:
            return
        self.count[i] += 1
        if not self.learned:
            return                         # learning step: every bucket goes out in finish()
        b = self.owner[i]
        if b == self.tail:
            return
        self.pending[b] -= 1
        if self.pending[b] == 0:
            self._launch(b)
        elif self.pending[b] < 0:
            raise RuntimeError(f"rgbac.parallel: parameter {i} notified more often than in "
                               "the learning step (the autograd graph changed between steps)")

    def _launch(self, b):
        # the weight-gradient reductions still queued by rgbac.autograd add into these
        # gradients: issue them first (stream order then puts them before the collective)
        from .autograd import flush_reductions
        flush_reductions()
        if self.skip:
            self.works[b] = []
            return
        if self.comm is not None:
            self.works[b] = [self.comm.allreduce(self.flat[lo:hi]) for lo, hi in self.buckets[b][0]]
            return
        self.works[b] = [dist.all_reduce(self.flat[lo:hi], op=dist.ReduceOp.SUM,
                                         group=self.group, async_op=True)
                         for lo, hi in self.buckets[b][0]]

    def _wait(self, w):
        if self.comm is not None:
            self.comm.wait(w)
        else:
            w.wait()

    def allreduce_all(self):
        """The whole flat buffer through the same collective path, outside any step (the
        bench's standalone all-reduce time)."""
        if self.comm is not None:
            self.comm.wait(self.comm.allreduce(self.flat))
        else:
            dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=self.group)

    def begin(self):
        """Call before loss.backward()."""
        for b, (_, idx) in enumerate(self.buckets):
            self.pending[b] = sum(self.expect[i] for i in idx) if self.learned else len(idx)
            self.works[b] = None
        self.count = [0] * len(self.params)
        self.active = True

    def launched_in_backward(self):
        """Buckets whose all-reduce went out before finish() in this step."""
        return sum(w is not None for w in self.works)

    def finish(self):
        """Call after loss.backward(): all-reduce what backward did not launch (the tail, or
        everything in the learning step), wait for every bucket (stream-ordered: the
        current stream waits for RCCL's); returns 1/world."""
        self.active = False
        if self.learned:
            # every rank must issue the same collectives in the same order: a non-tail bucket
            # that did not complete its learned count during backward would be launched here,
            # after buckets another rank may already have sent -- mismatched RCCL calls (a
            # silent hang or a sum over different ranges).  Refuse before launching anything.
            short = [b for b in range(len(self.buckets))
                     if b != self.tail and (self.works[b] is None or self.pending[b] != 0)]
            if short or self.count != self.expect:
                raise RuntimeError(
                    "rgbac.parallel: gradient notifications differ from the learning step "
                    f"(buckets {short} incomplete at the end of backward): the autograd graph "
                    "changed between steps")
        for b in range(len(self.buckets)):
            if self.works[b] is None:
                self._launch(b)
        for ws in self.works:
            for w in ws:
                self._wait(w)
        if not self.learned:
            # every rank must cut the same buckets (else ranks would issue all-reduces of
            # different ranges and counts): every rank takes part, whatever it counted
            cnt = torch.tensor(self.count, dtype=torch.int32, device=self.flat.device)
            dist.all_reduce(cnt, op=dist.ReduceOp.MAX, group=self.group)
            self.expect = [int(c) for c in cnt.tolist()]
            quiet = [i for i, c in enumerate(self.expect) if c == 0]
            order = [i for i in range(len(self.params) - 1, -1, -1) if self.expect[i]]
            self._cut(order, quiet)
        return 1.0 / self.world

    def remove(self):
        for h in self.hooks:
            h.remove()


class DataParallelTrainer:
    """net + AdamClamp + GradBuckets: ``step(loss)`` = backward with overlapped all-reduce,
    clamp, Adam (one launch).

    Buckets exist whenever a process group is up with more than one rank, or with
    ``force_buckets`` at any world size (world 1 then runs the real RCCL path: the hooks
    issue single-rank all-reduces, and the parameters stay bit-identical to the plain
    step).  With an RCCL ("nccl") group the buckets go through RcclComm (``rccl=False``:
    torch.distributed.all_reduce instead, as with gloo).  ``comm_events``: an optional list receiving, per step, a pair of timing events
    recorded on the compute stream at the end of backward and after the last bucket has been
    waited for -- the all-reduce time backward did not hide.  Pass ``external=True`` events
    (``make_comm_events``) when the step is captured in a HIP graph."""

    def __init__(self, net, optimizer, bucket_bytes=25 << 20, force_buckets=False, group=None,
                 rccl=None, watchdog_s=None):
        self.net, self.opt = net, optimizer
        self.buckets = None
        self.comm = None
        self.comm_events = None
        self.watchdog = None
        if dist.is_available() and dist.is_initialized() and \
                (force_buckets or dist.get_world_size(group) > 1):
            flat = optimizer.flat_grad
            if rccl is None:               # RCCL directly whenever the group is RCCL's
                rccl = flat.is_cuda and dist.get_backend(group) == "nccl"
            comm = None
            if rccl:
                try:
                    comm = RcclComm.get(flat.device, group)
                except (RuntimeError, OSError) as e:
                    # no usable librccl.so (or its init failed): torch.distributed's own
                    # all_reduce over the same group, bucketed the same way
                    print(f"rgbac.parallel: direct RCCL unavailable ({e}); using "
                          "torch.distributed.all_reduce", file=sys.stderr, flush=True)
            self.comm = comm
            self.buckets = GradBuckets(optimizer.params, flat, bucket_bytes, group=group,
                                       comm=comm)
            if comm is not None and watchdog_s:
                # opt-in failure detection for eager steps (the direct-RCCL path has no
                # ProcessGroup watchdog): each step arms it until the step's completion event
                # fires.  A caller replaying a captured step arms it around each replay.
                self.watchdog = CommWatchdog(comm, timeout_s=float(watchdog_s)).start()

    @staticmethod
    def make_comm_events(external=False):
        return (torch.cuda.Event(enable_timing=True, external=external),
                torch.cuda.Event(enable_timing=True, external=external))

    def step(self, loss):
        self.opt.zero_grad()
        if self.buckets is not None:
            self.buckets.begin()
        loss.backward()
        if self.buckets is not None:
            ev = None
            if self.comm_events is not None:
                ev = self.comm_events if isinstance(self.comm_events, tuple) else \
                    self.make_comm_events()
                ev[0].record()
            self.opt.grad_scale = self.buckets.finish()
            if ev is not None:
                ev[1].record()
                if isinstance(self.comm_events, list):
                    self.comm_events.append(ev)
        self.opt.step()
        if self.watchdog is not None and not torch.cuda.is_current_stream_capturing():
            done = torch.cuda.Event()
            done.record()
            self.watchdog.arm(done=done.query)
