"""MI355X-native batched Coup environment (2-player Coup of
BStarcheus/open_spiel_coup, bit-exact), HIP kernels behind a C ABI.

    from open_spiel_coup_amd import BatchedCoupEnv
    env = BatchedCoupEnv(batch=1 << 20, seed=1)
    ts = env.step()          # uniform random policy, obs for both players
"""
from .env import BatchedCoupEnv, FIRST, MID, LAST, SKIPPED, NUM_ACTIONS, OBS_SIZE, INFO_STATE_SIZE  # noqa: F401
from . import packed  # noqa: F401

__all__ = ["BatchedCoupEnv", "FIRST", "MID", "LAST", "SKIPPED", "NUM_ACTIONS", "OBS_SIZE", "INFO_STATE_SIZE", "packed"]
