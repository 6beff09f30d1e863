"""`vector_env.SyncVectorEnv` (open_spiel/python/vector_env.py:17-78) with the
reference's semantics, over a list of rl_environment.Environment facades.

This is the compatibility surface.  The vectorised path the reference's
SyncVectorEnv stands in for is BatchedCoupEnv: one kernel steps every game,
and observations stay on the GPU as [B, 2, 98] / [B, 2, 2492] tensors.
"""


class SyncVectorEnv:
    def __init__(self, envs):
        if not isinstance(envs, list):
            raise ValueError("Need to call this with a list of rl_environment.Environment objects")
        self.envs = envs

    def __len__(self):
        return len(self.envs)

    def observation_spec(self):
        return self.envs[0].observation_spec()

    @property
    def num_players(self):
        return self.envs[0].num_players

    def step(self, step_outputs, reset_if_done=False):
        """vector_env.py:40-67: returns (time_steps, reward, done, unreset_time_steps)."""
        time_steps = [self.envs[i].step([step_outputs[i].action]) for i in range(len(self.envs))]
        reward = [step.rewards for step in time_steps]
        done = [step.last() for step in time_steps]
        unreset_time_steps = time_steps
        if reset_if_done:
            time_steps = self.reset(envs_to_reset=done)
        return time_steps, reward, done, unreset_time_steps

    def reset(self, envs_to_reset=None):
        """vector_env.py:69-78"""
        if envs_to_reset is None:
            envs_to_reset = [True for _ in range(len(self.envs))]
        return [self.envs[i].reset() if envs_to_reset[i] else self.envs[i].get_time_step()
                for i in range(len(self.envs))]
