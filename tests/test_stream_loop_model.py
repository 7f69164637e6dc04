"""Model check of the rollout kernels' flat stream loop (csrc/kernels.hpp
`stream_flat_loop`, used by im_roll3 / im_roll3o / net_roll / net_roll3o).

The device loop lets each lane of the demand wave run ahead through its own
draws into an LDS ring of RD chunks of CH launch steps, and passes workgroup
barrier b once every lane holds chunk b.  The consumer (dynamics) wave reads
chunk c between barriers c and c + 1.  This test restates the loop's control
flow step for step in Python, drives it with random PTRS acceptances (and
reset steps that draw nothing), and checks on every schedule that

  * the loop ends having passed exactly nb barriers (no deadlock, no extra
    barrier: every wave of the workgroup must execute the same count),
  * chunk c is complete before barrier c,
  * no slot is overwritten while the consumer may still read it, so the
    consumer of chunk c sees exactly the draws of chunk c's steps in stream
    order.
"""
import numpy as np
import pytest


def run_stream_loop(K, CH, RD, RL, nb, t0, T, accept, lanes=64):
    """Restatement of stream_flat_loop<CH, RD, RL>(K, nb, t0, T, draw, put).
    accept(lane) -> bool is one attempt.  Returns (ring writes, barrier log)."""
    j = np.zeros(lanes, int)
    r = np.zeros(lanes, int)
    t = np.full(lanes, t0)
    b = 0
    writes = []              # (barriers passed, lane, slot, draw r, launch step j, per-lane seq)
    seq = np.zeros(lanes, int)
    passed_at = []           # per barrier: min j over lanes when it was passed
    guard = 0
    while True:
        while b < nb and np.all(j >= min((b + 1) * CH, K)):
            passed_at.append(int(j.min()))
            b += 1
        if b == nb:
            break
        for ln in range(lanes):
            if j[ln] < K and j[ln] // CH - RD + 2 <= b:
                if t[ln] >= T:                 # NEXT_STEP reset step: no draw
                    t[ln] = 0
                    j[ln] += 1
                elif accept(ln):
                    writes.append((b, ln, int(j[ln] % (RD * CH)), int(r[ln]), int(j[ln]), int(seq[ln])))
                    seq[ln] += 1
                    r[ln] += 1
                    if r[ln] == RL:
                        r[ln] = 0
                        j[ln] += 1
                        t[ln] += 1
        guard += 1
        assert guard < 100000, "stream loop does not terminate"
    return writes, passed_at


@pytest.mark.parametrize("K,CH,RD,RL,extra,t0,T", [
    (30, 2, 8, 1, 1, 0, 30),      # net_roll3o, default graph
    (75, 2, 8, 3, 1, 5, 30),      # net_roll3o, custom graph (3 draws per step)
    (30, 8, 4, 1, 0, 0, 30),      # im_roll3 / net_roll (2 roles: nch barriers)
    (61, 2, 8, 1, 1, 29, 30),     # im_roll3o, a reset early in the launch
    (61, 4, 4, 1, 1, 29, 30),     # im_roll3o (CH, RD) = (4, 4) A/B build
    (40, 2, 8, 1, 1, 0, 4),       # resets in most chunks
    (9, 8, 4, 1, 0, 3, 30),       # a partial last chunk
    (2, 2, 8, 3, 1, 30, 30),      # the first step is a reset
    (17, 4, 2, 1, 1, 0, 7),       # the smallest ring
])
@pytest.mark.parametrize("p_acc", [0.87, 0.3, 1.0])
def test_stream_flat_loop_schedule(K, CH, RD, RL, extra, t0, T, p_acc):
    rng = np.random.default_rng(K * 1000 + CH * 100 + RD * 10 + RL)
    nch = (K + CH - 1) // CH
    nb = nch + extra
    writes, passed = run_stream_loop(K, CH, RD, RL, nb, t0, T, lambda ln: rng.random() < p_acc)
    assert len(passed) == nb
    for c in range(nb):
        assert passed[c] >= min((c + 1) * CH, K)           # chunk c complete before barrier c
    # reference: the launch steps' periods and which of them draw
    draws_step = []
    t = t0
    for k in range(K):
        if t >= T:
            t = 0
            draws_step.append(False)
        else:
            t += 1
            draws_step.append(True)
    lanes = {w[1] for w in writes}
    for ln in lanes:
        lw = [w for w in writes if w[1] == ln]
        steps = [w[4] for w in lw]
        exp = [k for k in range(K) for _ in range(RL) if draws_step[k]]
        assert steps == exp                                 # each drawing step's RL draws, in stream order
    # slot safety: the consumer reads chunk c's slots while the stream wave has
    # passed c + 1 barriers; a write at that time must not hit one of them
    # (chunk c is complete before barrier c, so any such write would replace it)
    for (bw, ln, slot, r, jw, _) in writes:
        c = bw - 1
        if 0 <= c < nch:
            lo, hi = c * CH, min((c + 1) * CH, K)
            chunk_slots = {k % (RD * CH) for k in range(lo, hi)}
            assert slot not in chunk_slots or lo <= jw < hi, (bw, ln, slot, jw)
        assert jw // CH - RD + 2 <= bw                      # the slot's previous step was consumed
    # the values the consumer sees: the last write to (lane, slot, r) before it
    # reads chunk c (stream wave at <= c + 1 barriers) is chunk c's own step
    hist = {}
    for (bw, ln, slot, r, jw, _) in writes:
        hist.setdefault((ln, slot, r), []).append((bw, jw))
    for c in range(nch):
        for k in range(c * CH, min((c + 1) * CH, K)):
            if not draws_step[k]:
                continue
            for ln in lanes:
                for rr in range(RL):
                    cand = [jw for (bw, jw) in hist.get((ln, k % (RD * CH), rr), []) if bw <= c + 1]
                    assert cand and cand[-1] == k, (c, k, ln, rr)
