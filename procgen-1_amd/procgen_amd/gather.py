"""Double-buffered observation all-gather across the GPUs of one node.

The north star concatenates every rank's ``uint8[E, 64, 64, 3]`` observation shard with an RCCL
all-gather over xGMI.  Done on the engine's stream after every step, the gather serialises with
the next step (805 MB in, 5.6 GB out per GPU per step at 65,536 envs x 8 GPUs).  Here step t
renders into local buffer ``t % 2`` (``procgen_set_obs_buffer``), its all-gather runs on a
separate communication stream, and step t+1 renders into the other buffer meanwhile:

    engine stream :  step t -> [rendered t] -> step t+1 -> [rendered t+1] -> wait(gathered t) -> step t+2
    comm stream   :          wait(rendered t) -> all_gather(out[t%2] <- local[t%2]) -> [gathered t] ...

Ordering rules (each an event):
  * the gather of step t starts after step t's render (``rendered``);
  * step t+2 renders into local[t % 2] only after the gather of step t has read it (``gathered``);
  * the gather of step t+2 overwrites out[t % 2] only after the consumer released step t's
    result (``release``), when the consumer asked for that.

On CPU tensors (gloo, tests) the streams and events are no-ops and the same bookkeeping runs
synchronously, which is what tests/test_dist_cpu.py checks against an unsharded run.
"""
import torch


class _NoStream:
    def wait_event(self, ev):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class ObsGather:
    """``step(act)`` enqueues one engine step whose observations land in a fresh local buffer and
    starts their all-gather; it returns a slot k.  ``result(k)`` makes the caller's current stream
    wait for that gather and returns the ``[world * E, 64, 64, 3]`` tensor (valid until the step
    two later is issued, or until ``release(k)`` when the consumer needs longer)."""

    def __init__(self, num_envs, world=1, dist=None, device="cuda", engine_stream=None, bind=None,
                 obs_shape=(64, 64, 3), alive=None):
        self.world = world
        self.dist = dist
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        shape = (num_envs,) + tuple(obs_shape)
        self.local = [torch.empty(shape, dtype=torch.uint8, device=self.device) for _ in range(2)]
        self.out = [torch.empty((world * num_envs,) + tuple(obs_shape), dtype=torch.uint8, device=self.device)
                    for _ in range(2)]
        self.bind = bind  # bind(tensor): the engine renders the following steps into `tensor`
        # alive(): False once the engine was closed (its streams are gone and it holds no pointer into
        # the local buffers any more), so close() must neither wait on its stream nor unbind
        self.alive = alive
        if self.cuda:
            self.engine = engine_stream
            self.comm = torch.cuda.Stream(device=self.device)
        else:
            self.engine = self.comm = _NoStream()
        self.gathered = [None, None]
        self.released = [None, None]
        self.t = 0

    def _event(self, stream):
        if not self.cuda:
            return None
        ev = torch.cuda.Event()
        ev.record(stream)
        return ev

    def step(self, act):
        k = self.t & 1
        if self.gathered[k] is not None:
            self.engine.wait_event(self.gathered[k])  # local[k] was read by the gather of step t - 2
        self.bind(self.local[k])
        act()
        rendered = self._event(self.engine)
        if rendered is not None:
            self.comm.wait_event(rendered)
        if self.released[k] is not None:
            self.comm.wait_event(self.released[k])
            self.released[k] = None
        ctx = torch.cuda.stream(self.comm) if self.cuda else self.comm
        with ctx:
            if self.dist is not None:
                self.dist.all_gather_into_tensor(self.out[k], self.local[k])
            else:
                self.out[k].copy_(self.local[k], non_blocking=True)
        self.gathered[k] = self._event(self.comm)
        self.t += 1
        return k

    def result(self, k):
        if self.cuda and self.gathered[k] is not None:
            torch.cuda.current_stream(self.device).wait_event(self.gathered[k])
        return self.out[k]

    def release(self, k):
        """The consumer is done with result(k) once the work enqueued so far on its current stream ran."""
        if self.cuda:
            self.released[k] = self._event(torch.cuda.current_stream(self.device))

    def local_obs(self, k):
        return self.local[k]

    def sync_engine(self):
        """Make the engine stream wait until both outstanding gathers have read their local buffer.
        Call before anything that renders outside ``step`` (``set_state``, ``set_latent_state``
        re-render every env into the bound buffer, which a gather may still be reading)."""
        for ev in self.gathered:
            if ev is not None:
                self.engine.wait_event(ev)

    def close(self):
        """Unbind: the engine renders into its own tensor again, after every gather has read the
        local buffers, which may then be freed (the engine keeps a raw pointer while bound)."""
        if self.bind is None:
            return
        engine_alive = self.alive is None or self.alive()
        if engine_alive:
            self.sync_engine()
        if self.cuda:  # the gathers (torch's comm stream, not the engine's) have read the local buffers
            for ev in self.gathered:
                if ev is not None:
                    ev.synchronize()
        if not engine_alive:
            self.bind = None
            return
        try:
            self.bind(None)
        finally:
            self.bind = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
