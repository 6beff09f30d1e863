"""`rl_environment`-shaped facade (open_spiel/python/rl_environment.py) over
the GPU engine.

    from open_spiel_coup_amd import rl_environment
    env = rl_environment.Environment("coup")
    ts = env.reset()
    while not ts.last():
        ts = env.step([agent_action(ts)])

Semantics follow the reference line for line: observation type defaults to
INFORMATION_STATE (rl_environment.py:195-200), chance events are sampled
until a decision node (:369-382), every time step carries both players'
tensors and legal actions (:219-268), discounts are 0 at LAST (:252-254),
and step() after LAST resets (:310-311).  One Environment drives one lane of
a BatchedCoupEnv: its own one-lane env, or -- once a vector_env.SyncVectorEnv
adopts it -- lane i of the vector env's shared N-lane env, so that the
vector env steps all of its games with one launch.  Batched learners that do
not need per-game time steps should use BatchedCoupEnv directly.

Chance sampling: by default the deals come from the build's Philox contract
 inside the kernel, keyed by `seed` (None, the default:
64 bits of OS entropy, so independent environments deal independent games,
like the reference's RandomState(None) sampler).  Passing a
`chance_event_sampler` (an object called with the state, like the
reference's ChanceEventSampler, :119-131) switches to the State API path:
decisions and deals are applied one at a time and the sampler picks each
deal.
"""
import collections
import os
import enum
import struct

import numpy as np
import torch

from . import _native, pyspiel
from .env import BatchedCoupEnv, HISTORY_BYTES


class StepType(enum.Enum):
    """rl_environment.py:96-112"""
    FIRST = 0
    MID = 1
    LAST = 2

    def first(self):
        return self is StepType.FIRST

    def mid(self):
        return self is StepType.MID

    def last(self):
        return self is StepType.LAST


class TimeStep(collections.namedtuple("TimeStep", ["observations", "rewards", "discounts", "step_type"])):
    """rl_environment.py:47-93"""
    __slots__ = ()

    def first(self):
        return self.step_type == StepType.FIRST

    def mid(self):
        return self.step_type == StepType.MID

    def last(self):
        return self.step_type == StepType.LAST

    def is_simultaneous_move(self):
        return self.observations["current_player"] == pyspiel.PlayerId.SIMULTANEOUS

    def current_player(self):
        return self.observations["current_player"]


class ObservationType(enum.Enum):
    """rl_environment.py:134-137"""
    OBSERVATION = 0
    INFORMATION_STATE = 1


class ChanceEventSampler:
    """rl_environment.py:119-131: numpy-sampled chance events (used only when
    passed explicitly to Environment)."""

    def __init__(self, seed=None):
        self.seed(seed)

    def seed(self, seed=None):
        self._rng = np.random.RandomState(seed)

    def __call__(self, state):
        actions, probs = zip(*state.chance_outcomes())
        return self._rng.choice(actions, p=probs)


def registered_games():
    return pyspiel.registered_games()


_ext = None


def _float_lists(rows):
    """The per-player Python lists of a time step (rl_environment.py:243-248
    hands out fresh lists of floats) from a [P, n] float32 array, built in C
    by the library's CPython binding (_coup_host.float_lists): integral
    values -- every element of both tensors -- share a few float objects,
    and the lists are kept out of the cyclic collector, so a 256-env vector
    step costs per env what an 8-env one does.  Equal
    to numpy's tolist element by element; each list is the caller's own.
    Contract: these lists are not tracked by the cyclic collector (a list of
    floats cannot be in a cycle; CPython untracks tuples and dicts of atomic
    values the same way), so a caller that puts a container into one and
    closes a reference cycle through it must break that cycle itself."""
    global _ext
    if _ext is None:
        _native.load()
        from . import _coup_host
        _ext = _coup_host
    if not (type(rows) is np.ndarray and rows.dtype == np.float32 and rows.flags.c_contiguous):
        rows = np.ascontiguousarray(rows, dtype=np.float32)
    return _ext.float_lists(rows, rows.shape[0], rows.shape[1])


_LEGAL = {}  # 18-bit mask -> ascending action ids (copied per time step)
_REWARDS = struct.Struct("<bb")  # coup_slot_result.rewards, at byte 120


def _legal_list(mask):
    """LegalActions() of a mask as a fresh list (the reference's time step
    holds a new list per step)."""
    got = _LEGAL.get(mask)
    if got is None:
        got = _LEGAL[mask] = tuple(a for a in range(18) if (mask >> a) & 1)
    return list(got)


def _rewards(q):
    """Rewards() of a result as the time step's list of floats."""
    raw = getattr(q, "_raw", None)
    if raw is not None:
        r0, r1 = _REWARDS.unpack_from(raw, 120)
        return [float(r0), float(r1)]
    return [float(x) for x in q["rewards"]]


def _resolve_seed(seed):
    """The sampling-contract seed of an Environment.  None draws 64 bits of
    OS entropy, as the reference's default ChanceEventSampler does with
    np.random.RandomState(None) (rl_environment.py:119-131): two
    default-constructed environments deal different games."""
    if seed is None:
        return int.from_bytes(os.urandom(8), "little")
    return int(seed) & ((1 << 64) - 1)


class Environment:
    """rl_environment.Environment for Coup on the GPU (one lane)."""

    def __init__(self, game="coup", discount=1.0, chance_event_sampler=None, observation_type=None,
                 include_full_state=False, mfg_distribution=None, mfg_population=None,
                 enable_legality_check=False, seed=None, device=None, **kwargs):
        if isinstance(game, str):
            self._game = pyspiel.load_game(game, kwargs or None)
        else:
            self._game = game
        if mfg_distribution is not None or mfg_population is not None:
            raise ValueError("coup is not a mean-field game")
        self._sampler = chance_event_sampler
        self._include_full_state = include_full_state
        self._enable_legality_check = enable_legality_check
        self._num_players = self._game.num_players()
        self._discounts = [discount] * self._num_players
        if observation_type is None:
            observation_type = ObservationType.INFORMATION_STATE
        self._use_observation = observation_type == ObservationType.OBSERVATION
        self._device = device
        self._seed = _resolve_seed(seed)
        self._owner = None  # the SyncVectorEnv whose shared env holds this game, if any
        self._make_env()
        self._should_reset = True
        self._last = None

    # ------------------------------------------------------------ plumbing
    def _make_env(self):
        self._hq = None
        if self._sampler is None and not pyspiel.DEVICE_STATES:
            # host-resident (round 4): the env's game is a host state, and
            # reset / step are the library's host build of the device lane
            # ops (coup_host_state_step: same rules, same Philox deals of
            # stream (seed, env id 0)), ~1 us instead of a device round trip;
            # a SyncVectorEnv that adopts the env moves the game to a lane
            self._env, self._lane, self._owner, self._last = None, 0, None, None
            # the game's chance stream: (seed, global env id), a 1-lane env's
            # lane 0 under its own seed until a SyncVectorEnv re-keys it
            self._hseed, self._env_id = self._seed, 0
            self._pool = pyspiel._pool(self._device)  # the HIP device is required all the same
            self._hq = self._host_step(None, -1, _native.SLOT_INIT | _native.SLOT_DEAL)
            return
        # one lane of a 2-player history env, attached to the device's op
        # server (pyspiel's lane pool): reset and step are one coup_slot_op
        # each (COUP_SLOT_RESET / COUP_SLOT_DEAL) whose 128-byte result and
        # tensors come back in the same round trip
        # unchecked: step() applies its action as the reference's does,
        # through pyspiel's apply_action (rl_environment.py:296-298), which
        # has no legality check (pyspiel.cc:266); enable_legality_check
        # rejects an illegal one in Python first
        self._env = BatchedCoupEnv(1, seed=self._seed, auto_reset=False, obs=False, info_state=False,
                                   history=True, device=self._device, unchecked=True)
        self._pool = pyspiel._pool(self._device)
        self._pool.attach(self._env)
        self._lane = 0
        self._owner = None
        self._act = torch.empty(1, dtype=torch.int8, pin_memory=True)
        self._last = None

    def _bind_lane(self, env, lane, owner):
        """Play on lane `lane` of `env` (a SyncVectorEnv's shared env, which
        already holds this game's record and history) from now on."""
        self._env, self._lane, self._owner = env, int(lane), owner
        self._hq = None

    def _host_step(self, raw, action, mode):
        """coup_host_state_step on the env's host state; with the time
        step's tensor when the op succeeds."""
        q = pyspiel._host().step(raw, action, mode, self._hseed, self._env_id)
        return self._with_tensor(q) if q["ok"] else q

    def _with_tensor(self, q):
        """q (a host result) with the time step's tensor of both players."""
        if self._use_observation:
            q["obs"] = pyspiel._host().tensors(q._raw, True, False)[0]
        else:
            q["info_state"] = pyspiel._host().tensors(q._raw, False, True)[1]
        return q

    def _op(self, action, flags):
        """reset / step / query (action -1, flags 0) of the env's game: on
        its host state, or as one lane op on its device lane."""
        if self._hq is not None:
            if action < 0 and not flags:
                return self._hq
            q = self._host_step(self._hq._raw, action, flags)
            if q["ok"]:
                self._hq = q
            return q
        return self._lane_op(action, flags)

    def _key_stream(self, env_id):
        """Key this env's chance stream as global env id `env_id` under its
        seed and start over (tests: an env stepped alone that deals what lane
        `env_id` of a vector env deals)."""
        if self._hq is not None:
            self._hseed, self._env_id = self._seed, int(env_id)
            self._hq = self._host_step(None, -1, _native.SLOT_INIT | _native.SLOT_DEAL)
        else:
            self._env = BatchedCoupEnv(1, seed=self._seed, env_id_base=int(env_id), auto_reset=False, obs=False,
                                       info_state=False, history=True, device=self._device, unchecked=True)
            self._pool.attach(self._env)
            self._lane, self._owner = 0, None
        self._should_reset, self._last = True, None

    def _host_rekey(self, seed, env_id, owner):
        """A SyncVectorEnv keeping this host-resident game on the host: its
        later deals are global env id `env_id`'s under `seed` (what lane
        `env_id` of an adopting vector env would deal); the game itself is
        kept."""
        self._hseed, self._env_id, self._owner = seed, int(env_id), owner

    def _export_lane(self):
        """The game's record [1, 4] int32 and history [1, 96] uint8, on the
        device (SyncVectorEnv adoption)."""
        if self._hq is not None:
            raw = self._hq._raw
            dev = torch.device(self._device) if self._device is not None else torch.device("cuda")
            rec = torch.frombuffer(bytearray(raw[:16]), dtype=torch.int32).view(1, 4).to(dev)
            hist = torch.frombuffer(bytearray(raw[16:16 + HISTORY_BYTES]), dtype=torch.uint8).view(1, HISTORY_BYTES)
            return rec, hist.to(dev)
        j = self._lane
        return self._env.export_state()[j:j + 1], self._env.export_history()[j:j + 1]

    def _lane_op(self, action, flags):
        """reset / step of this env's lane as one coup_slot_op, with the time
        step's tensor."""
        return self._pool.lane_op(self._env, self._lane, action, flags, obs=self._use_observation,
                                  info=not self._use_observation)

    def _batchable(self):
        """Whether a SyncVectorEnv may adopt this env: in-kernel chance
        sampling (no caller sampler), on no other vector env."""
        return self._sampler is None and self._owner is None

    def _lane_actions(self, action):
        """[B] int8 actions: `action` on this env's lane, -1 (skip) elsewhere."""
        if self._env.batch == 1:
            self._act[0] = int(action)
            return self._act.to(self._env.device, non_blocking=True)
        a = torch.full((self._env.batch,), -1, dtype=torch.int8)
        a[self._lane] = int(action)
        return a.to(self._env.device)

    def _lane_actions_host(self, action):
        """[B] int8 host actions: `action` on this env's lane, -1 (skip) elsewhere."""
        a = np.full(self._env.batch, -1, dtype=np.int8)
        a[self._lane] = int(action)
        return a

    def _lane_mask(self):
        if self._env.batch == 1:
            return None
        m = torch.zeros(self._env.batch, dtype=torch.uint8)
        m[self._lane] = 1
        return m

    def _state_view(self):
        if self._hq is not None:
            raw = self._hq._raw
            return (np.frombuffer(raw, np.uint32, 4, 0).copy(),
                    np.frombuffer(raw, np.uint8, HISTORY_BYTES, 16).copy())
        j = self._lane
        words = self._env.export_state()[j].cpu().numpy().view(np.uint32).reshape(4).copy()
        hist = self._env.export_history()[j].cpu().numpy().reshape(HISTORY_BYTES).copy()
        return words, hist

    def _history_list(self, words, hist):
        from .packed import lane
        n = lane(words.reshape(1, 4))["move_number"]
        out = []
        for i in range(n):
            e = int(hist[i])
            out.append((-1 if e & 0x20 else (e >> 6) & 1, e & 0x1F))
        return out

    def _time_step(self, q, step_type, rewards):
        cur = int(q["current_player"])
        mask = int(q["legal_mask"]) & 0x3FFFF
        if cur >= 0 and not mask:
            # legal_actions(cur) raises at a decision node no legal play
            # reaches (coup.cc:886, 892, 936), as in the reference's
            # get_time_step (rl_environment.py:243-248)
            raise pyspiel.SpielError("Error in LegalActions(): Invalid action progression")
        legal_cur = _legal_list(mask) if cur >= 0 else []
        tensors = q["obs" if self._use_observation else "info_state"]
        if tensors.shape[0] != self._num_players:
            tensors = tensors[:self._num_players]
        if self._num_players == 2:
            legal = [legal_cur, []] if cur == 0 else ([[], legal_cur] if cur == 1 else [[], []])
        else:
            legal = [legal_cur if p == cur else [] for p in range(self._num_players)]
        obs = {"info_state": _float_lists(tensors), "legal_actions": legal, "current_player": cur,
               "serialized_state": []}
        if self._include_full_state:
            obs["serialized_state"] = pyspiel.serialize_game_and_state(self._game, self.get_state)
        discounts = None
        if step_type == StepType.MID:
            discounts = list(self._discounts)
        elif step_type == StepType.LAST:
            discounts = [0.0 for _ in self._discounts]
        self._last = obs
        return TimeStep(obs, rewards, discounts, step_type)

    def _query(self):
        q = self._env.query_host(obs=self._use_observation, info_state=not self._use_observation)
        return {k: v[self._lane] for k, v in q.items()}

    def _sample_external_events(self):
        """rl_environment.py:369-382 with a caller-supplied sampler."""
        while True:
            q = self._query()
            if int(q["current_player"]) != pyspiel.PlayerId.CHANCE:
                return q
            outcome = self._sampler(self.get_state)
            self._env.apply_action(torch.tensor([int(outcome)], dtype=torch.int8))

    # ------------------------------------------------------------ public API
    def seed(self, seed=None):
        """Re-key the env's chance stream (ChanceEventSampler.seed).  On an
        env a SyncVectorEnv has adopted this re-keys the vector env's shared
        stream (every lane keeps its game); this env restarts on its next step
        either way."""
        if self._sampler is not None:
            self._sampler.seed(seed)
            return
        self._seed = _resolve_seed(seed)
        if self._owner is not None:
            self._owner._rekey(self._seed)
        else:
            self._make_env()
        self._should_reset = True

    def get_time_step(self):
        # an answered query op on the lane (no action): one round trip to the
        # op server instead of a query launch
        q = self._query() if self._sampler is not None else self._op(-1, 0)
        step_type = StepType.LAST if int(q["terminal"]) else StepType.MID
        self._should_reset = step_type == StepType.LAST
        return self._time_step(q, step_type, _rewards(q))

    def step(self, actions):
        assert len(actions) == self.num_actions_per_step, (
            "Invalid number of actions! Expected {}".format(self.num_actions_per_step))
        if self._should_reset:
            return self.reset()
        if self._enable_legality_check:
            legal = self._last["legal_actions"][self._last["current_player"]] if self._last else []
            if actions[0] not in legal:
                raise RuntimeError(f"step() called on illegal action {actions[0]}")
        if not 0 <= int(actions[0]) < 128:
            raise pyspiel.SpielError(f"illegal action {actions[0]}")  # not an int8 action id
        if self._sampler is None:
            # the decision, then the chance deals that follow under the
            # sampling contract, and the time step's answers: one op on the
            # lane (the op server's wave when the pool has one)
            q = self._op(int(actions[0]), _native.SLOT_DEAL | _native.SLOT_UNCHECKED)
            if not q["ok"]:
                # DoApplyAction raised in the reference (coup.cc:490-809), or the
                # result leaves the packed record (a known gap); the lane is unchanged
                raise pyspiel._apply_failed(self._last["current_player"] if self._last else -1, int(actions[0]), q)
            step_type = StepType.LAST if q["terminal"] else StepType.MID
            self._should_reset = step_type == StepType.LAST
            return self._time_step(q, step_type, _rewards(q))
        # legal per the last time step's mask (which came from the GPU): the
        # kernel cannot reject it, so the error counter's synchronisation is
        # skipped
        cur = self._last["current_player"] if self._last else -1
        known_legal = cur >= 0 and int(actions[0]) in self._last["legal_actions"][cur]
        self._env.apply_action(self._lane_actions(actions[0]))
        self._sample_external_events()
        if not known_legal and self._env.error_count():
            raise pyspiel.SpielError(f"apply_action({actions[0]}) failed")
        return self.get_time_step()

    def reset(self):
        self._should_reset = False
        if self._sampler is None:
            q = self._op(-1, _native.SLOT_RESET | _native.SLOT_DEAL)
        else:
            self._env.new_initial_state()
            q = self._sample_external_events()
        return self._time_step(q, StepType.FIRST, None)

    def observation_spec(self):
        return dict(
            info_state=tuple([self._game.observation_tensor_size() if self._use_observation
                              else self._game.information_state_tensor_size()]),
            legal_actions=(self._game.num_distinct_actions(),),
            current_player=(),
            serialized_state=(),
        )

    def action_spec(self):
        return dict(num_actions=self._game.num_distinct_actions(), min=0,
                    max=self._game.num_distinct_actions() - 1, dtype=int)

    @property
    def use_observation(self):
        return self._use_observation

    @property
    def name(self):
        return self._game.get_type().short_name

    @property
    def num_players(self):
        return self._game.num_players()

    @property
    def num_actions_per_step(self):
        return 1

    @property
    def is_turn_based(self):
        return True

    @property
    def max_game_length(self):
        return self._game.max_game_length()

    @property
    def is_chance_node(self):
        q = self._query() if self._sampler is not None else self._op(-1, 0)
        return int(q["current_player"]) == pyspiel.PlayerId.CHANCE

    @property
    def game(self):
        return self._game

    @property
    def get_state(self):
        """A pyspiel-shaped CoupState snapshot of the env's lane."""
        words, hist = self._state_view()
        if self._hq is not None:
            return pyspiel.CoupState._from_host(self._game, self._hq, self._history_list(words, hist))
        return pyspiel.CoupState._from_env(self._game, self._env._h, self._lane, self._history_list(words, hist))

    def set_state(self, new_state):
        assert new_state.get_game() == self.game, "State must have been created by the same game."
        if self._hq is not None:
            q = new_state._q.copy()  # the state's record and history (its last answer)
            for k in ("obs", "info_state"):
                q.pop(k, None)
            self._hq = self._with_tensor(q)
            self._last = None
            return
        self._env._bind_stream()
        new_state._copy_to_env(self._env._h, self._lane)
        self._last = None  # the cached legal actions no longer describe the lane

    @property
    def mfg_distribution(self):
        return None
