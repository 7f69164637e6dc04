"""Stand-in for gymnasium.utils.seeding.np_random."""
import numpy as np


def np_random(seed=None):
    seed_seq = np.random.SeedSequence(seed)
    rng = np.random.Generator(np.random.PCG64(seed_seq))
    return rng, seed_seq.entropy
