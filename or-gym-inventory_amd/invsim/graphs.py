"""HIP-graph capture of a step loop (SURVEY §7 layer 5).

The reference's hot loop is the caller's ``for t: action = agent(obs);
obs, reward, ... = env.step(action)`` (``benchmark_InvManagementBacklogEnv.py:389-440``,
``benchmark_NetInvMgmtBacklogEnv.py:221-262``).  With a torch policy in that
loop every iteration costs a few host-side launches (the policy's ops plus the
``invsim_step`` call, ~5-12 us of Python each), which at 32 768-65 536 envs is
as long as the step kernel itself.  :class:`StepGraph` records ``fn()`` --
any mix of torch ops and ``env.step`` / ``env.rollout`` / ``env.rollout_policy``
/ ``env.reset`` calls on one env -- into one HIP graph (``torch.cuda.CUDAGraph``
over the env's device) and replays it with one host call.

The env's host side keeps a *position* (lock-step period, demand-lookahead
slot) that selects each launch's kernel and parameters; those are baked into
the graph.  ``invsim_capture_begin`` / ``invsim_capture_end`` bracket the
capture: nothing runs while capturing, so the position is put back, and the
capture is accepted only if ``fn`` brings the env back to the position it
started from (a whole number of episode cycles: ``periods + 1`` steps with
the default ``next_step`` autoreset, ``periods`` with ``same_step``).  Every
replay then starts where the graph was recorded; :meth:`StepGraph.replay`
checks it.  The numpy (parity) demand stream only: the fast stream's
launch-step counter is a launch parameter and would repeat on replay.

Example::

    env = InvManagementBacklogEnv(65536, device="cuda:0")
    obs0, _ = env.reset(seed=0)
    obs = obs0.clone()                        # static input of the graph
    def loop():
        o, ret = obs, 0
        for _ in range(31):                   # periods + 1 (next_step autoreset)
            a = policy(o)
            o, r, te, tr, _ = env.step(a)
            ret = ret + r
        obs.copy_(o)                          # next replay starts from here
        return ret
    g = StepGraph(env, loop)                  # runs loop() once (warm-up), then records it
    for _ in range(100):
        ret = g.replay()                      # 31 env steps + the policy, one host call
"""
import torch

from . import _capi


class StepGraph:
    """Record ``fn()`` (torch ops + calls on ``env``) as one HIP graph.

    ``warmup`` eager runs of ``fn`` come first (they step the env for real, on
    a side stream, as ``torch.cuda.graph`` recommends; at least one is needed
    so that the demand lookahead is primed before the position is recorded).
    ``outputs`` is what ``fn`` returned during capture: static tensors the
    replays overwrite.  ``steps`` is the number of env steps one replay runs.
    """

    def __init__(self, env, fn, warmup=1, pool=None):
        self.env = env
        dev = env.device
        cur = torch.cuda.current_stream(dev)
        if warmup:
            side = torch.cuda.Stream(dev)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                for _ in range(int(warmup)):
                    fn()
            cur.wait_stream(side)
        torch.cuda.synchronize(dev)
        self.position = env.position()
        self.graph = torch.cuda.CUDAGraph()
        lib, h = env._lib, env._h
        _capi.check(lib.invsim_capture_begin(h), h, "capture_begin")
        steps = _capi.C.c_int64(0)
        ended = False
        try:
            with torch.cuda.device(dev), torch.cuda.graph(self.graph, pool=pool):
                out = fn()
            rc = lib.invsim_capture_end(h, _capi.C.byref(steps))
            ended = True
            _capi.check(rc, h, "capture_end")
        except BaseException:
            if not ended:
                lib.invsim_capture_end(h, None)   # put the position back; the graph is discarded
            self.graph = None
            raise
        self.outputs = out
        self.steps = int(steps.value)

    def replay(self):
        """Run the recorded loop once (on the current stream); returns ``outputs``."""
        if self.graph is None:
            raise RuntimeError("StepGraph: capture failed, nothing to replay")
        pos = self.env.position()
        if pos != self.position:
            raise RuntimeError(
                f"StepGraph.replay: the env is at position {pos:#x}, the graph was recorded at "
                f"{self.position:#x} (eager calls moved it by a part of an episode cycle)")
        self.graph.replay()
        return self.outputs
