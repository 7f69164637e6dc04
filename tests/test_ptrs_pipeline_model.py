"""CPU model of the Newsvendor rollout's software-pipelined PTRS wave
(csrc/newsvendor.hip, NV_PTRS_PIPE): each trip draws the NEXT candidate's two
uniforms while it tests the pending one, the pending candidate survives chunk
boundaries inside an episode, and it is rewound before a reset's five uniforms
and before the final state store.

The model restates that control flow over an abstract stream (a position in
uniforms; a candidate at position p consumes uniforms p, p + 1, and whether it
is accepted is a fixed function of p and the episode's rate, as numpy's PTRS
candidate is of its two uniforms and lam) and checks it against the
sequential sampler (one candidate drawn and tested per trip, numpy's
random_poisson_ptrs loop, newsvendor.py:146): the same draws, the same stream
position at every reset and at the end of the launch.  Test infrastructure
only (no product code is imported).
"""
import random

import pytest


def accepted(p, ep, seed):
    """A candidate's fixed outcome: the stream position and the episode's rate."""
    return random.Random((seed * 1000003 + p) * 31 + ep).random() < 0.87


def chunks(K, T, t0, CH):
    """The launch's chunks as nv_chunk cuts them: (len, reset) with NEXT_STEP
    autoreset at t >= T (the reset step ends its chunk and draws nothing)."""
    out, t, k = [], t0, 0
    while k < K:
        n, rs = 0, False
        while n < CH and n < K - k:
            n += 1
            if t >= T:
                rs = True
                break
            t += 1
        if rs:
            t = 0
        out.append((n, rs))
        k += n
    return out


def sequential(K, T, t0, CH, seed):
    pos, ep, draws, marks = 0, 0, [], []
    for n, rs in chunks(K, T, t0, CH):
        nd = n - (1 if rs else 0)
        j = 0
        while j < nd:
            acc = accepted(pos, ep, seed)
            if acc:
                draws.append((ep, pos))
                j += 1
            pos += 2
        if rs:
            marks.append(pos)      # the reset's uniforms start here
            pos += 5
            ep += 1
    marks.append(pos)              # the stored state
    return draws, marks


def pipelined(K, T, t0, CH, seed):
    """The kernel's loop: st = position after the uniforms drawn so far,
    pend / pg / pending candidate position as in nv_roll_kernel."""
    st, ep, draws, marks = 0, 0, [], []
    pend, pg, pc = False, 0, 0
    for n, rs in chunks(K, T, t0, CH):
        nd = n - (1 if rs else 0)
        if not pend and nd > 0:
            pg, pc, st, pend = st, st, st + 2, True
        j = 0
        while j < nd:
            nh, nc = st, st        # the next candidate, drawn ahead
            st += 2
            if accepted(pc, ep, seed):
                draws.append((ep, pc))
                j += 1
            pc, pg = nc, nh
        if rs:
            if pend:
                st, pend = pg, False
            marks.append(st)
            st += 5
            ep += 1
    if pend:
        st = pg
    marks.append(st)
    return draws, marks


@pytest.mark.parametrize("seed", range(40))
def test_pipelined_ptrs_wave_consumes_the_stream_like_the_sequential_one(seed):
    rng = random.Random(seed)
    K = rng.choice([1, 2, 7, 8, 9, 30, 65])
    T = rng.choice([1, 3, 8, 40])
    t0 = rng.randrange(0, T + 1)
    CH = rng.choice([1, 2, 8])
    assert pipelined(K, T, t0, CH, seed) == sequential(K, T, t0, CH, seed)


def test_model_covers_resets_inside_and_at_chunk_ends():
    # a reset in the middle of the launch, one at its first step, none at all
    cs = {(K, T, t0) for K, T, t0 in [(30, 8, 0), (30, 8, 8), (9, 40, 3)]}
    for K, T, t0 in cs:
        for seed in range(5):
            assert pipelined(K, T, t0, 8, seed) == sequential(K, T, t0, 8, seed)
    assert any(rs for _, rs in chunks(30, 8, 0, 8)) and chunks(30, 8, 8, 8)[0] == (1, True)
