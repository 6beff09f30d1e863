"""`vector_env.SyncVectorEnv` (open_spiel/python/vector_env.py:17-78) over
rl_environment.Environment facades, stepped as one batch.

The reference steps its envs one after another in a Python loop
(vector_env.py:54-57).  Here the vector env adopts its envs' games: their
lane records and histories move into lane i of one shared N-lane
BatchedCoupEnv, and each Environment keeps working on its lane (its own
step / reset / get_state / set_state still apply to that game).  A vector
step is then one reset launch for the envs that restart and one step launch
for the rest (lanes not stepped take action -1, which the kernel skips) that
writes every env's tensors, legal mask, player, rewards and step type
straight into mapped host memory (coup_step_host) -- instead of N round
trips.

Chance streams: env i draws its deals from global env id i under the first
env's seed; the envs' own seeds no longer apply once
adopted.  The reference's envs sample from independent RandomState(None)
streams (rl_environment.py:119-131), which no caller can replay either.

A vector env of at most LANE_OPS_UPTO envs steps them one lane op each
(Environment.step on its lane, through the op server): below that size the
lane ops' round trips cost less than a launch and a synchronisation.  Both
forms give the same games (tests/test_gpu_vector_env.py).

Host-resident envs (round 4: an Environment's game is a host state by
default) are not moved to the device (unless there are more than HOST_UPTO
of them; default: any number stays): the vector env keeps them on the host
and re-keys their chance streams as adoption would (env i: global env id i
under the first env's seed), so the games, deals and time steps are those of
the adopted form.  Each step is then the host build of the lane rules per
env (~0.5 us) and the time step's lists, which a launch cannot make cheaper:
measured from 1 to 1024 envs the kept form is as fast as the adopted one or
faster, except OBSERVATION at 256 envs.  Envs whose
games are on device lanes (COUP_STATE_DEVICE=1) are adopted as before.

Envs with a caller-supplied chance sampler (the State API path), envs of
different games / observation types / devices, or envs already adopted by
another vector env are stepped in the reference's loop instead.

Errors: an action outside 0..127 raises SpielError before anything is
applied.  Actions outside LegalActions() are applied as Environment.step
applies them (pyspiel's unchecked apply_action); one the reference's
DoApplyAction would raise on is rejected by its lane (the other envs' actions
are applied) and raises SpielError after the launch; with the games kept on
the host, as in the reference's loop, the envs before it are applied and the
ones after it are not.
"""
import numpy as np
import torch

from . import pyspiel
from .env import BatchedCoupEnv


LANE_OPS_UPTO = 2
HOST_UPTO = None  # host-resident envs stay on the host up to this many (None: any number, 0: never)


class SyncVectorEnv:
    def __init__(self, envs, batched=True):
        """batched=False keeps the reference's one-env-at-a-time loop."""
        if not isinstance(envs, list):
            raise ValueError("Need to call this with a list of rl_environment.Environment objects")
        self.envs = envs
        self._shared = None
        self._host = False  # host-resident games kept on the host (see the module doc)
        if batched and self._can_batch():
            if all(e._hq is not None for e in envs) and (HOST_UPTO is None or len(envs) <= HOST_UPTO):
                self._host = True
                self._rekey_host(self.envs[0]._seed)
            else:
                self._adopt(self.envs[0]._seed)

    def __len__(self):
        return len(self.envs)

    def observation_spec(self):
        return self.envs[0].observation_spec()

    @property
    def num_players(self):
        return self.envs[0].num_players

    @property
    def batched(self):
        """True when one shared env steps every game, or the host-resident
        games are stepped on the host under the shared stream (module doc)."""
        return self._shared is not None or self._host

    # ------------------------------------------------------------ adoption
    def _can_batch(self):
        from .rl_environment import Environment
        envs = self.envs
        if not envs or not all(isinstance(e, Environment) and e._batchable() for e in envs):
            return False
        if len({id(e) for e in envs}) != len(envs):
            return False
        e0 = envs[0]
        return all(e._use_observation == e0._use_observation and e._device == e0._device
                   and e.num_players == e0.num_players == 2
                   and str(e.game) == str(e0.game) for e in envs)

    def _adopt(self, seed):
        """Move every env's game into lane i of a new shared env keyed by
        `seed` (records, histories and each env's pending-reset flag carry
        over), and bind the envs to their lanes."""
        envs = self.envs
        lanes = [e._export_lane() for e in envs]  # host-resident games and device lanes alike
        records = torch.cat([r for r, _ in lanes])
        hist = torch.cat([h for _, h in lanes])
        shared = BatchedCoupEnv(len(envs), seed=seed, auto_reset=False, obs=False, info_state=False, history=True,
                                device=envs[0]._device, unchecked=True)  # as each env's own (rl_environment.py)
        shared.import_state(records)
        shared.import_history(hist)
        envs[0]._pool.attach(shared)  # an env stepping alone goes through the op server too
        self._shared = shared
        for i, e in enumerate(envs):
            e._bind_lane(shared, i, self)

    def _rekey_host(self, seed):
        for i, e in enumerate(self.envs):
            e._host_rekey(seed, i, self)

    def _rekey(self, seed):
        """Environment.seed() of an adopted env: the shared stream takes the
        new seed, every lane keeps its game."""
        if self._host:
            self._rekey_host(seed)
            return
        for e in self.envs:
            e._owner = None
        self._adopt(seed)

    # ------------------------------------------------------------ batched ops
    def _query(self):
        e0 = self.envs[0]
        return self._shared.query_host(obs=e0._use_observation, info_state=not e0._use_observation)

    def _time_steps(self, q, firsts, prev_q=None, prev=None):
        """Time steps from one query of every lane: FIRST where firsts[i] (a
        lane reset this call), else what Environment.get_time_step reports --
        from prev_q when given (lanes unchanged since that query), or prev[i]
        itself when that was already such a time step (MID or LAST)."""
        from .rl_environment import StepType
        out = []
        for i, (e, first) in enumerate(zip(self.envs, firsts)):
            if not first and prev is not None and not prev[i].first():
                out.append(prev[i])  # the tensors are host lists: reuse, do not rebuild
                continue
            src = q if first or prev_q is None else prev_q
            row = {k: v[i] for k, v in src.items()}
            if first:
                out.append(e._time_step(row, StepType.FIRST, None))
            else:
                st = StepType.LAST if int(row["terminal"]) else StepType.MID
                e._should_reset = st == StepType.LAST
                out.append(e._time_step(row, st, [float(x) for x in row["rewards"]]))
        return out

    def _reset_lanes(self, resets):
        mask = torch.tensor(np.asarray(resets, dtype=np.uint8))
        sh = self._shared
        sh._bind_stream()
        from . import _native
        _native.check(sh.lib.coup_reset(sh._h, sh._mask_ptr(mask)))
        for e, r in zip(self.envs, resets):
            if r:
                e._should_reset = False

    def _step_batched(self, step_outputs):
        envs = self.envs
        n = len(envs)
        resets = [bool(e._should_reset) for e in envs]
        acts = np.full(n, -1, dtype=np.int8)
        unknown = []  # envs whose action the last time step did not list as legal
        for i, e in enumerate(envs):
            if resets[i]:
                continue
            a = int(step_outputs[i].action)
            if e._enable_legality_check:
                legal = e._last["legal_actions"][e._last["current_player"]] if e._last else []
                if a not in legal:
                    raise RuntimeError(f"step() called on illegal action {a}")
            if not 0 <= a < 128:
                raise pyspiel.SpielError(f"illegal action {a}")  # not an int8 action id
            cur = e._last["current_player"] if e._last else -1
            if not (cur >= 0 and a in e._last["legal_actions"][cur]):
                unknown.append(i)
            acts[i] = a
        if any(resets):
            self._reset_lanes(resets)
        if not all(resets):
            # one launch whose outputs (skipped lanes: their current state) land
            # in mapped host memory: no separate query
            e0 = envs[0]
            self._q_step = self._shared.step_host(acts, obs=e0._use_observation, info_state=not e0._use_observation)
            if unknown and self._shared.error_count():
                # DoApplyAction raised in the reference for one of them (coup.cc:490-809)
                raise pyspiel.SpielError(f"apply_action failed among envs {unknown}")
        else:
            self._q_step = self._query()
        return self._time_steps(self._q_step, resets)

    # ------------------------------------------------------------ public API
    def step(self, step_outputs, reset_if_done=False):
        """vector_env.py:40-67: returns (time_steps, reward, done, unreset_time_steps)."""
        one_by_one = self._shared is None or len(self.envs) <= LANE_OPS_UPTO
        if one_by_one:
            time_steps = [self.envs[i].step([step_outputs[i].action]) for i in range(len(self.envs))]
        else:
            time_steps = self._step_batched(step_outputs)
        reward = [step.rewards for step in time_steps]
        done = [step.last() for step in time_steps]
        unreset_time_steps = time_steps
        if reset_if_done:
            if self._shared is None and not self._host:
                time_steps = self.reset(envs_to_reset=done)
            elif one_by_one:
                # lane ops or host games: an env that goes on keeps its time step, unless
                # that was a FIRST, which get_time_step reports as MID (as the
                # reference's reset(envs_to_reset) does)
                time_steps = [e.reset() if d else (e.get_time_step() if t.first() else t)
                              for e, d, t in zip(self.envs, done, time_steps)]
            elif any(done):
                # the envs that go on are unchanged since the step's query
                self._reset_lanes(done)
                time_steps = self._time_steps(self._query(), done, prev_q=self._q_step, prev=time_steps)
            else:
                time_steps = self._time_steps(self._q_step, done, prev=time_steps)
        return time_steps, reward, done, unreset_time_steps

    def reset(self, envs_to_reset=None):
        """vector_env.py:69-78"""
        if envs_to_reset is None:
            envs_to_reset = [True for _ in range(len(self.envs))]
        if self._shared is None or len(self.envs) <= LANE_OPS_UPTO:
            return [self.envs[i].reset() if envs_to_reset[i] else self.envs[i].get_time_step()
                    for i in range(len(self.envs))]
        resets = [bool(r) for r in envs_to_reset]
        if any(resets):
            self._reset_lanes(resets)
        return self._time_steps(self._query(), resets)
