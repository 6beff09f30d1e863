"""`pyspiel`-shaped per-game facade over the GPU engine.

The reference's callers (Deep CFR, MCCFR, agent_cmp, human_game) use
`pyspiel.load_game("coup")` and per-game `State` objects
(open_spiel/python/pybind11/pyspiel.cc:263-375).  This module gives them the
same surface with only an import swap:

    from open_spiel_coup_amd import pyspiel
    game = pyspiel.load_game("coup")
    state = game.new_initial_state()

A `CoupState` is, by default, host-resident: its 128-byte coup_slot_result
(record, history bytes, legal mask, player, rewards, returns) is the state,
and every op -- apply_action, child, tensors, strings -- runs the library's
host build of the same lane rules and decoders the kernels run
(coup_host_state_*, csrc/coup_host.cpp; ~1 us from Python, where any device
round trip is 7-10 us).  The library, and a HIP device, are still required:
there is no separate CPU rules engine and no build without the GPU library.
With COUP_STATE_DEVICE=1 (or game._device_states) a State instead owns one
lane of a device-resident lane pool and each op is a coup_slot_op on that
lane, served by the pool's resident op-server wave (COUP_SERVER=0: a launch
per op).  Strings are formatted by the library's host formatter
(coup_host_state_string; strings.py is the same in Python).
This is the compatibility path; batched learners use BatchedCoupEnv.
"""
import atexit
import ctypes
import enum
import os
import struct
import threading
import weakref

import numpy as np
import torch

from . import _native, packed, strings
from ._native import CoupError
from .env import BatchedCoupEnv, INFO_STATE_SIZE, OBS_SIZE

SpielError = CoupError


class UnrepresentableActionError(SpielError):
    """A SpielError for an action the reference's DoApplyAction ACCEPTS but
    whose result leaves the packed record's fields (a 16th coin, an unsorted
    3-4 card hand; only unchecked play reaches such states): a known parity
    gap of the packed representation, not an action the
    reference rejects.  The state is left unchanged."""


class PlayerId(enum.IntEnum):
    """open_spiel/spiel_globals.h:28-36"""
    DEFAULT = -1
    CHANCE = -1
    SIMULTANEOUS = -2
    INVALID = -3
    TERMINAL = -4
    MEAN_FIELD = -5


class GameType:
    """The fields of open_spiel::GameType (spiel.h:42-153) Coup defines
    (coup.cc:38-52)."""

    class Dynamics(enum.Enum):
        SIMULTANEOUS = 0
        SEQUENTIAL = 1
        MEAN_FIELD = 2

    class ChanceMode(enum.Enum):
        DETERMINISTIC = 0
        EXPLICIT_STOCHASTIC = 1
        SAMPLED_STOCHASTIC = 2

    class Information(enum.Enum):
        ONE_SHOT = 0
        PERFECT_INFORMATION = 1
        IMPERFECT_INFORMATION = 2

    class Utility(enum.Enum):
        ZERO_SUM = 0
        CONSTANT_SUM = 1
        GENERAL_SUM = 2
        IDENTICAL = 3

    class RewardModel(enum.Enum):
        REWARDS = 0
        TERMINAL = 1

    def __init__(self):
        self.short_name = "coup"
        self.long_name = "Coup"
        self.dynamics = GameType.Dynamics.SEQUENTIAL
        self.chance_mode = GameType.ChanceMode.EXPLICIT_STOCHASTIC
        self.information = GameType.Information.IMPERFECT_INFORMATION
        self.utility = GameType.Utility.ZERO_SUM
        self.reward_model = GameType.RewardModel.REWARDS
        self.max_num_players = 2
        self.min_num_players = 2
        self.provides_information_state_string = True
        self.provides_information_state_tensor = True
        self.provides_observation_string = True
        self.provides_observation_tensor = True
        self.provides_factored_observation_string = False
        self.parameter_specification = {}


# coup_slot_result (include/coup_mi355x.h), 128 bytes
_SLOT_RESULT = np.dtype([("record", "<u4", (4,)), ("history", "u1", (96,)), ("legal_mask", "<u4"),
                         ("cur_player", "i1"), ("terminal", "u1"), ("ok", "u1"), ("unrepresentable", "u1"),
                         ("rewards", "i1", (2,)), ("returns", "i1", (2,)), ("pad", "u1", (4,))])
assert _SLOT_RESULT.itemsize == 128
_RESULT_TAIL = struct.Struct("<IbBBBbbbb")  # legal_mask .. returns, at byte 112


class _Result(dict):
    """A coup_slot_result (128 bytes) as the facade's result dict.  The
    scalars a walk reads at every node (legal mask, player, terminal, ok)
    are unpacked at once; record, history, rewards and returns become numpy
    views of the raw bytes on first use."""
    __slots__ = ("_raw",)
    _LAZY = {"record": (np.uint32, 4, 0), "history": (np.uint8, 96, 16), "rewards": (np.int8, 2, 120),
             "returns": (np.int8, 2, 122)}

    def __missing__(self, key):
        dt, n, off = self._LAZY[key]
        v = np.frombuffer(self._raw, dt, n, off)
        self[key] = v
        return v

    def copy(self):
        c = _Result(self)
        c._raw = self._raw
        return c


def _parse_result(raw):
    """One coup_slot_result (128 bytes) -> the facade's result dict."""
    lm, cp, term, ok, unrep = _RESULT_TAIL.unpack_from(raw, 112)[:5]
    q = _Result(legal_mask=lm, current_player=cp, terminal=bool(term), ok=bool(ok), unrepresentable=bool(unrep))
    q._raw = raw
    return q


# mask (bits 0..17) -> ascending legal actions; masks repeat, so each is built once
_LEGAL = {}


def _legal_list(m):
    t = _LEGAL.get(m)
    if t is None:
        t = _LEGAL[m] = tuple(a for a in range(18) if (m >> a) & 1)
    return list(t)


def _action_id(action):
    """An action id for ApplyAction: outside 0..17 DoApplyAction raises at
    any node (coup.cc:493 chance, :806 decision; spiel.cc:327 for -1)."""
    a = int(action)
    if not 0 <= a < 18:
        raise SpielError(f"Invalid player action {a}")
    return a


def _action_string(player, action):
    try:
        return strings.action_to_string(player, action)
    except Exception:
        return str(action)


def _apply_failed(player, action, q=None):
    """The SpielError of an action the lane rejected: DoApplyAction raises
    there in the reference (a SPIEL_CHECK or SpielFatalError of coup.cc:
    490-809) or the state is terminal -- or, UnrepresentableActionError, the
    reference accepts it but the result leaves the packed record's fields
    (coup_slot_result.unrepresentable)."""
    if q is not None and q.get("unrepresentable"):
        return UnrepresentableActionError(
            f"ApplyAction({action}) by player {player}: the reference accepts this action, but its result "
            f"leaves the packed record's fields (known parity gap, DESIGN.md section 8); state unchanged")
    return SpielError(f"ApplyAction({action}) by player {player} rejected: DoApplyAction raises here "
                      f"(or the state is terminal)")


class _Pool:
    """Device-resident lane pool: every live CoupState owns one lane of a
    2-player history env (segments of SEG lanes, grown on demand).  Each
    State op is one coup_slot_op launch on its lane, and only ops that need
    an answer copy a 128-byte result back (one synchronisation); a clone is
    a device-to-device lane copy with no round trip.

    Thread-safe: one lock serialises alloc / release / op, because every op
    answers through the pool's one pinned result buffer (and each segment's
    one scratch), and ctypes releases the GIL inside coup_slot_op.  States
    of one pool may therefore be used from several threads, as the
    reference's independent State objects can."""

    SEG = 4096

    def __init__(self, device):
        self.device = torch.device(device)
        self.lock = threading.RLock()
        self.lib = _native.load()
        self._slot_op = self.lib.coup_slot_op
        self.segs = []
        self.free = []
        nbytes = _native.SLOT_RESULT_BYTES + 2 * OBS_SIZE * 4 + 2 * INFO_STATE_SIZE * 4
        self.host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        self.buf = self.host.numpy()
        self.host_ptr = ctypes.c_void_p(self.host.data_ptr())
        # the device-resident op server (coup_server_*): single ops on the
        # pool's lanes run on one resident wave instead of a launch each.
        # COUP_SERVER=0 keeps the launch path (A/B); COUP_SERVER_IDLE_US sets
        # how long the wave waits for the next op before it leaves.
        self.srv = None
        self._attached = []  # weak references to other envs attached to the server (rl_environment)
        if os.environ.get("COUP_SERVER", "1") != "0":
            h = ctypes.c_void_p()
            with torch.cuda.device(self.device):
                _native.check(self.lib.coup_server_create(int(os.environ.get("COUP_SERVER_IDLE_US", "2000")),
                                                          ctypes.byref(h)))
            self.srv = h
        atexit.register(_close_pool, weakref.ref(self))

    def attach(self, env):
        """Route `env`'s single-lane ops (coup_slot_op) through this pool's op
        server too (the per-game rl_environment envs); no-op without one."""
        with self.lock:
            if self.srv is not None:
                _native.check(self.lib.coup_attach_server(env._h, self.srv))
                env._served = True
                self._attached.append(weakref.ref(env))

    def close(self):
        """Stop the op server (its wave leaves) and detach the envs it serves."""
        with self.lock:
            if self.srv is None:
                return
            others = [r() for r in self._attached]
            for env in self.segs + [e for e in others if e is not None]:
                if env._h:
                    _native.check(self.lib.coup_attach_server(env._h, None))
                env._served = False
            _native.check(self.lib.coup_server_destroy(self.srv))
            self.srv = None

    def server_stats(self):
        """(requests, wave launches, running, idle_us) of the op server, or None."""
        if self.srv is None:
            return None
        out = (ctypes.c_uint64 * 4)()
        _native.check(self.lib.coup_server_stats(self.srv, out))
        return tuple(int(x) for x in out)

    def alloc(self):
        with self.lock:
            return self._alloc()

    def _alloc(self):
        if not self.free:
            env = BatchedCoupEnv(self.SEG, seed=0, auto_reset=False, obs=False, history=True, device=self.device)
            if self.srv is not None:
                _native.check(self.lib.coup_attach_server(env._h, self.srv))
                env._served = True
            k = len(self.segs)
            self.segs.append(env)
            self.free.extend((k, i) for i in range(self.SEG - 1, -1, -1))
        return self.free.pop()

    def release(self, slot):
        with self.lock:
            self.free.append(slot)

    def handle(self, slot):
        return self.segs[slot[0]]._h

    def apply_op(self, slot, src_slot, action):
        """The answered unchecked ApplyAction of apply_action (slot) and
        child (slot None: a new one, a copy of src_slot first) as one C call
        under one lock acquisition -- the per-node ops of a tree walk
        (deep_cfr.py:440-447, outcome_sampling_mccfr.py:61-100) without the
        general op's bookkeeping.  Returns (slot, result)."""
        with self.lock:
            new = slot is None
            if new:
                slot = self._alloc()
            env = self.segs[slot[0]]
            if not env._served:
                env._bind_stream()
            if src_slot is None:
                rc = self._slot_op(env._h, slot[1], None, 0, action, _native.SLOT_UNCHECKED, self.host_ptr)
            else:
                rc = self._slot_op(env._h, slot[1], self.segs[src_slot[0]]._h, src_slot[1], action,
                                   _native.SLOT_UNCHECKED, self.host_ptr)
            if rc:
                if new:
                    self.free.append(slot)
                _native.check(rc)
            return slot, _parse_result(self.buf[:_native.SLOT_RESULT_BYTES].tobytes())

    def op(self, slot, src=None, action=-1, init=False, obs=False, info=False, result=True, unchecked=False):
        """coup_slot_op on `slot`; src = (coup_env handle, lane) or None;
        unchecked: the action as pyspiel's apply_action applies it
        (COUP_SLOT_UNCHECKED)."""
        with self.lock:
            return self._op(slot, src, action, init, obs, info, result, unchecked)

    def ops(self, seg, reqs, src_seg=None, obs=False, info=False, unchecked=False):
        """coup_slot_ops: the (lane, src_lane, action) requests on segment
        `seg` (copies from segment `src_seg`) in one launch; returns one
        result dict per request, like op()."""
        with self.lock:
            n = len(reqs)
            rf = _native.SLOT_UNCHECKED if unchecked else 0
            arr = (_native.SlotReq * n)(*[_native.SlotReq(lane, src, action, rf) for lane, src, action in reqs])
            per = _native.SLOT_RESULT_BYTES
            nbytes = n * (per + (2 * OBS_SIZE * 4 if obs else 0) + (2 * INFO_STATE_SIZE * 4 if info else 0))
            if getattr(self, "_batch_host", None) is None or self._batch_host.numel() < nbytes:
                self._batch_host = torch.empty(max(nbytes, 1 << 16), dtype=torch.uint8, pin_memory=True)
            env = self.segs[seg]
            env._bind_stream()
            flags = (_native.SLOT_OBS if obs else 0) | (_native.SLOT_INFO if info else 0)
            src_h = self.segs[src_seg]._h if src_seg is not None else None
            _native.check(self.lib.coup_slot_ops(env._h, n, arr, src_h, flags,
                                                 ctypes.c_void_p(self._batch_host.data_ptr())))
            buf = self._batch_host.numpy()[:nbytes]
            raw = buf[:n * per].tobytes()
            off = n * per
            obs_t = info_t = None
            if obs:
                obs_t = buf[off:off + n * 2 * OBS_SIZE * 4].view(np.float32).reshape(n, 2, OBS_SIZE).copy()
                off += n * 2 * OBS_SIZE * 4
            if info:
                info_t = buf[off:off + n * 2 * INFO_STATE_SIZE * 4].view(np.float32).reshape(
                    n, 2, INFO_STATE_SIZE).copy()
            out = []
            for k in range(n):
                q = _parse_result(raw[k * per:(k + 1) * per])
                if obs:
                    q["obs"] = obs_t[k]
                if info:
                    q["info_state"] = info_t[k]
                out.append(q)
            return out

    def _op(self, slot, src, action, init, obs, info, result, unchecked=False):
        flags = ((_native.SLOT_INIT if init else 0) | (_native.SLOT_OBS if obs else 0)
                 | (_native.SLOT_INFO if info else 0) | (0 if result else _native.SLOT_NO_RESULT)
                 | (_native.SLOT_UNCHECKED if unchecked else 0))
        src_h, src_lane = src if src is not None else (None, 0)
        return self._lane_op(self.segs[slot[0]], slot[1], src_h, src_lane, action, flags, obs, info, result)

    def lane_op(self, env, lane, action=-1, flags=0, obs=False, info=False):
        """One answered coup_slot_op on lane `lane` of `env` (any 2-player
        history env, e.g. an rl_environment env attached with attach());
        flags: extra COUP_SLOT_* (RESET / DEAL)."""
        flags |= (_native.SLOT_OBS if obs else 0) | (_native.SLOT_INFO if info else 0)
        with self.lock:
            return self._lane_op(env, lane, None, 0, action, flags, obs, info, True)

    def _lane_op(self, env, lane, src_h, src_lane, action, flags, obs, info, result):
        if not getattr(env, "_served", False):
            env._bind_stream()  # a served env's ops launch nothing
        _native.check(self.lib.coup_slot_op(env._h, lane, src_h, src_lane, int(action), flags,
                                            self.host_ptr if result else None))
        if not result:
            return None
        b = self.buf
        q = _parse_result(b[:_native.SLOT_RESULT_BYTES].tobytes())
        off = _native.SLOT_RESULT_BYTES
        if obs:
            q["obs"] = b[off:off + 2 * OBS_SIZE * 4].view(np.float32).reshape(2, OBS_SIZE).copy()
            off += 2 * OBS_SIZE * 4
        if info:
            q["info_state"] = b[off:off + 2 * INFO_STATE_SIZE * 4].view(np.float32).reshape(2, INFO_STATE_SIZE).copy()
        return q


_pools = {}

# Per-game States are host-resident by default: the library's host build of
# the lane rules (coup_host_state_*, csrc/coup_host.cpp) applies each op on
# the calling thread, ~1 us from Python, against ~7-10 us for any device
# round trip.  COUP_STATE_DEVICE=1 keeps them on the
# device lane pool (every op a coup_slot_op on the op server), as before
# round 4; a game can also choose per instance (CoupGame._device_states).
DEVICE_STATES = os.environ.get("COUP_STATE_DEVICE", "0") == "1"


class _Host:
    """The host-resident State ops of libcoup_mi355x.so (coup_host_state_*),
    through their CPython binding _coup_host (csrc/host_ext.c, linked to the
    library; ctypes would add ~0.7 us per call).  A host state is its
    128-byte coup_slot_result (record, history bytes, answers), kept as an
    immutable bytes object inside its _Result: clones share it."""

    def __init__(self):
        _native.load()  # torch's HIP runtime, then the library the binding links
        from . import _coup_host
        _coup_host.bind(_Result)  # init / apply return _Result objects, built in C
        self._ext = _coup_host
        self.apply = _coup_host.apply  # (raw, action, flags) -> _Result
        self.step = _coup_host.step    # (raw or None, action, mode, seed, env_id) -> _Result

    def init(self):
        return self._ext.init()

    def string(self, raw, kind, player):
        """0 ObservationString, 1 InformationStateString, 2 ToString."""
        try:
            return self._ext.string(raw, kind, player)
        except ValueError:
            raise SpielError(f"invalid player {player}") from None

    def tensors(self, raw, obs, info):
        """[2][98] and / or [2][2492] float32 arrays (None where not asked)."""
        o = np.empty((2, OBS_SIZE), np.float32) if obs else None
        i = np.empty((2, INFO_STATE_SIZE), np.float32) if info else None
        self._ext.tensors(raw, o, i)
        return o, i


_host_ops = None


def _tensor_list(row):
    """One tensor row as the fresh list of floats pyspiel returns
    (pyspiel.cc's vector<float> cast), built by the library's binding from
    shared small floats.  An ordinary list: it stays tracked by the cyclic
    GC (only rl_environment's time-step lists are untracked, the contract
    documented on rl_environment.Environment)."""
    row = np.ascontiguousarray(row, dtype=np.float32)
    return _host()._ext.float_lists(row, 1, row.size, 0)[0]


def _host():
    global _host_ops
    if _host_ops is None:
        _host_ops = _Host()
    return _host_ops


def _close_pool(ref):
    pool = ref()
    if pool is not None:
        try:
            pool.close()
        except Exception:
            pass


def _pool(device=None):
    dev = torch.device(device if device is not None else "cuda")
    if dev.index is None:
        dev = torch.device(dev.type, torch.cuda.current_device())
    key = (dev.type, dev.index)
    if key not in _pools:
        _pools[key] = _Pool(dev)
    return _pools[key]


class CoupGame:
    """open_spiel::coup::CoupGame (coup.h:199-231)."""

    def __init__(self, params=None, device=None):
        if params:
            raise SpielError("coup takes no parameters (coup.cc:51-52)")
        self._type = GameType()
        self._device = device
        self._pool = None  # the lane pool of `device`, bound on first use
        self._device_states = DEVICE_STATES  # States on device lanes instead of the host (module doc)

    def _bind_pool(self):
        self._pool = _pool(self._device)
        return self._pool

    # --- metadata (coup.h:203-220, spiel.h:888-890)
    def get_type(self):
        return self._type

    def num_distinct_actions(self):
        return 18

    def max_chance_outcomes(self):
        return 5

    def num_players(self):
        return 2

    def min_utility(self):
        return -2.0

    def max_utility(self):
        return 2.0

    def utility_sum(self):
        return 0.0

    def max_game_length(self):
        return 90

    def max_chance_nodes_in_history(self):
        return 45

    def max_move_number(self):
        return 135

    def max_history_length(self):
        return 135

    def information_state_tensor_shape(self):
        return [INFO_STATE_SIZE]

    def information_state_tensor_size(self):
        return INFO_STATE_SIZE

    def observation_tensor_shape(self):
        return [OBS_SIZE]

    def observation_tensor_size(self):
        return OBS_SIZE

    def policy_tensor_shape(self):
        return [18]

    def get_parameters(self):
        return {}

    def action_to_string(self, player, action):
        return strings.action_to_string(player, action)

    def __str__(self):
        return "coup()"

    def serialize(self):
        return "coup()"

    def __eq__(self, other):
        return isinstance(other, CoupGame)

    def __hash__(self):
        return hash("coup()")

    def new_initial_state(self):
        return CoupState(self)

    def deserialize_state(self, text):
        """Game::DeserializeState (spiel.cc:393-425): replay the history."""
        st = self.new_initial_state()
        for line in text.split("\n"):
            if line:
                st.apply_action(int(line))
        return st


class CoupState:
    """open_spiel::coup::CoupState (coup.h:111-197) over the MI355X engine.

    Host-resident (the default, _slot None): the state is the 128-byte
    coup_slot_result in self._q and every op runs the library's host build
    of the lane rules.  Device-resident (game._device_states): the state
    owns a lane of the device pool and every op is a coup_slot_op.  Both
    give the same results (tests/test_gpu_facade.py runs both)."""

    def __init__(self, game, _src=None, _history=None, _q=None, _slot=None, _host_q=None):
        self._game = game
        # the device pool is bound for host states too: the facade needs the
        # HIP device (snapshots, batched ops with tensors), and says so at once
        self._pool = game._pool if game._pool is not None else game._bind_pool()
        if _host_q is not None:  # a host state
            self._slot, self._q, self._history = None, _host_q, _history
            return
        if _slot is not None:  # filled by a batched op (children / apply_actions)
            self._slot, self._q, self._history = _slot, _q, _history
            return
        if not game._device_states:
            self._slot = None
            if _src is None:
                self._q, self._history = _host().init(), []
            else:  # snapshot of a device lane (rl_environment.get_state): one answered read
                h, lane = _src
                with self._pool.lock:
                    _native.check(self._pool.lib.coup_slot_op(h, lane, None, 0, -1, 0, self._pool.host_ptr))
                    self._q = _parse_result(self._pool.buf[:_native.SLOT_RESULT_BYTES].tobytes())
                self._history = _history
            return
        self._slot = self._pool.alloc()
        if _src is None:
            self._q = self._pool.op(self._slot, init=True)
            self._history = []
        else:  # Clone / snapshot: a device-side lane copy
            self._q = self._pool.op(self._slot, src=_src, result=_q is None)
            if _q is not None:
                self._q = _q.copy()
            self._history = _history

    def __del__(self):
        try:
            if self._slot is not None:
                self._pool.release(self._slot)
        except Exception:
            pass

    @classmethod
    def _from_host(cls, game, q, history):
        """Snapshot of a host-resident game (rl_environment.get_state): a host
        State, or -- for a game whose States live on device lanes -- the
        record and history written into a new pool lane."""
        q = q.copy()
        for k in ("obs", "info_state"):
            q.pop(k, None)
        if not game._device_states:
            return cls(game, _history=history, _host_q=q)
        pool = game._pool if game._pool is not None else game._bind_pool()
        slot = pool.alloc()
        with pool.lock:
            _native.check(pool.lib.coup_write_lane(pool.handle(slot), slot[1], q._raw))
        return cls(game, _slot=slot, _q=q, _history=history)

    @classmethod
    def _from_env(cls, game, env_handle, lane, history):
        """Snapshot lane `lane` of a 2-player history env (rl_environment)."""
        return cls(game, _src=(env_handle, lane), _history=history)

    def _copy_to_env(self, env_handle, lane):
        """Write this state into lane `lane` of a 2-player history env."""
        if self._slot is None:
            with self._pool.lock:
                _native.check(self._pool.lib.coup_write_lane(env_handle, lane, self._q._raw))
            return
        env = self._pool.segs[self._slot[0]]
        with self._pool.lock:
            env._bind_stream()
            _native.check(env.lib.coup_slot_op(env_handle, lane, env._h, self._slot[1], -1,
                                               _native.SLOT_NO_RESULT, None))

    # ------------------------------------------------------------- internals
    def _query(self, obs=False, info=False):
        need_obs = obs and "obs" not in self._q
        need_info = info and "info_state" not in self._q
        if (need_obs or need_info) and self._slot is None:
            o, i = _host().tensors(self._q._raw, need_obs, need_info)
            if need_obs:
                self._q["obs"] = o
            if need_info:
                self._q["info_state"] = i
            return self._q
        if need_obs or need_info:
            q = self._pool.op(self._slot, obs=obs, info=info)
            for k in ("obs", "info_state"):
                if k not in q and k in self._q:
                    q[k] = self._q[k]
            self._q = q
        return self._q

    def _words(self):
        return self._q["record"].reshape(1, 4)

    @property
    def _rec(self):
        return self._q["record"]

    @property
    def _hist(self):
        return self._q["history"]

    # ------------------------------------------------------------- State API
    def get_game(self):
        return self._game

    def num_players(self):
        return 2

    def num_distinct_actions(self):
        return 18

    def current_player(self):
        return self._q["current_player"]

    def is_terminal(self):
        return self._q["terminal"]

    def is_chance_node(self):
        return self.current_player() == PlayerId.CHANCE

    def is_player_node(self):
        return self.current_player() >= 0

    def is_simultaneous_node(self):
        return False

    def is_mean_field_node(self):
        return False

    def _mask(self):
        return self._q["legal_mask"] & 0xFFFFFFFF

    def legal_actions(self, player=None):
        """LegalActions() / LegalActions(player) (spiel.h:255-261)."""
        q = self._q
        cur = q["current_player"]
        if (player is not None and player != cur) or cur == -4:  # PlayerId.TERMINAL
            return []
        mask = q["legal_mask"] & 0x3FFFF
        if not mask and cur >= 0:
            # a decision node no legal play reaches (unchecked actions):
            # LegalActions() raises (coup.cc:886, 892, 936)
            raise SpielError("Error in LegalActions(): Invalid action progression")
        return _legal_list(mask)

    def legal_actions_mask(self, player=None):
        """LegalActionsMask (spiel.cc:371-377): length 5 at chance nodes."""
        cur = self.current_player()
        p = cur if player is None else player
        length = 5 if p == PlayerId.CHANCE else 18
        mask = [0] * length
        for a in self.legal_actions(p):
            mask[a] = 1
        return mask

    def chance_outcomes(self):
        """ChanceOutcomes (coup.cc:1062-1077): exact count/total doubles."""
        if not self.is_chance_node():
            raise SpielError("chance_outcomes() at a non-chance node")
        w1 = struct.unpack_from("<I", self._q._raw, 4)[0]
        deck = [(w1 >> (4 * t)) & 0xF for t in range(5)]  # w1 [19:0], type t at 4t
        total = float(sum(deck))
        return [(t, deck[t] / total) for t in range(5) if deck[t] > 0]

    def legal_chance_outcomes(self):
        return [a for a, _ in self.chance_outcomes()]

    def _legal(self, a):
        return 0 <= a < 18 and (self._mask() >> a) & 1 and self.current_player() != PlayerId.TERMINAL

    def apply_action(self, action):
        """State::ApplyAction (spiel.cc:322-331) on the GPU, bound as pyspiel
        binds it (pyspiel.cc:266): no legality check -- DoApplyAction's own
        checks decide (COUP_SLOT_UNCHECKED), for legal
        actions too (LegalActions can offer one DoApplyAction refuses once
        unchecked play has left legal play's states).  Raises SpielError, the
        state unchanged, where the reference raises."""
        player = self._q["current_player"]
        a = _action_id(action)
        if self._slot is None:
            q = _host().apply(self._q._raw, a, _native.SLOT_UNCHECKED)
        else:
            _, q = self._pool.apply_op(self._slot, None, a)
        if not q["ok"]:
            raise _apply_failed(player, a, q)
        self._q = q
        self._history = self._history + [(player, a)]

    def apply_action_with_legality_check(self, action):
        """State::ApplyActionWithLegalityCheck (spiel.cc:334-344)."""
        a = _action_id(action)
        if not self._legal(a):
            p = self.current_player()
            raise SpielError(f"Current player {p} calling ApplyAction with illegal action ({a}): "
                             f"{_action_string(p, a)}")
        self.apply_action(a)

    def child(self, action):
        """clone() + apply_action(action) (State::Child, spiel.h) as ONE op:
        the new state's lane is a copy of this one with the action applied."""
        player = self._q["current_player"]
        a = _action_id(action)
        if self._slot is None:
            q = _host().apply(self._q._raw, a, _native.SLOT_UNCHECKED)
            if not q["ok"]:
                raise _apply_failed(player, a, q)
            return CoupState(self._game, _history=self._history + [(player, a)], _host_q=q)
        slot, q = self._pool.apply_op(None, self._slot, a)
        if not q["ok"]:
            self._pool.release(slot)
            raise _apply_failed(player, a, q)
        return CoupState(self._game, _slot=slot, _q=q, _history=self._history + [(player, a)])

    def children(self, actions, obs=False, info_state=False):
        """[self.child(a) for a in actions] in one launch per pool segment
        (coup_slot_ops: each child is a device-side copy of this lane plus
        ApplyAction).  Deep CFR expands every legal action of a traverser
        node this way (deep_cfr.py:440-471).  With obs / info_state the
        children's tensors come back with the same round trip."""
        actions = [_action_id(a) for a in actions]
        player = self.current_player()
        if not actions:
            return []
        if self._slot is None:
            out = []
            for a in actions:
                c = self.child(a)
                if obs or info_state:
                    c._query(obs=obs, info=info_state)
                out.append(c)
            return out
        pool = self._pool
        if len(actions) == 1 and pool.srv is not None and not (obs or info_state):
            return [self.child(actions[0])]  # one op server request beats a launch
        slots = [pool.alloc() for _ in actions]
        out = [None] * len(actions)
        try:
            by_seg = {}
            for k, s in enumerate(slots):
                by_seg.setdefault(s[0], []).append(k)
            for seg, ks in by_seg.items():
                res = pool.ops(seg, [(slots[k][1], self._slot[1], actions[k]) for k in ks], src_seg=self._slot[0],
                               obs=obs, info=info_state, unchecked=True)
                for k, q in zip(ks, res):
                    if not q["ok"]:
                        raise _apply_failed(player, actions[k], q)
                    out[k] = CoupState(self._game, _slot=slots[k], _q=q,
                                       _history=self._history + [(player, actions[k])])
        except Exception:
            for k, s in enumerate(slots):
                if out[k] is None:
                    pool.release(s)
            raise
        return out

    def legal_children(self, obs=False, info_state=False):
        """[(a, self.child(a)) for a in self.legal_actions()] in one launch:
        the frontier of a traverser node (deep_cfr.py:440-471) or of a chance
        node (the chance outcomes, in ascending order)."""
        acts = self.legal_actions()
        return list(zip(acts, self.children(acts, obs=obs, info_state=info_state)))

    def clone(self):
        if self._slot is None:  # the result bytes are immutable: shared
            return CoupState(self._game, _history=list(self._history), _host_q=self._q)
        return CoupState(self._game, _src=(self._pool.handle(self._slot), self._slot[1]),
                         _history=list(self._history), _q=self._q)

    def __copy__(self):
        return self.clone()

    def __deepcopy__(self, memo):
        return self.clone()

    def rewards(self):
        return [float(x) for x in self._query()["rewards"]]

    def returns(self):
        return [float(x) for x in self._query()["returns"]]

    def player_reward(self, player):
        return self.rewards()[player]

    def player_return(self, player):
        return self.returns()[player]

    def observation_tensor(self, player=None):
        p = self.current_player() if player is None else player
        return _tensor_list(self._query(obs=True)["obs"][p])

    def information_state_tensor(self, player=None):
        p = self.current_player() if player is None else player
        return _tensor_list(self._query(info=True)["info_state"][p])

    def observation_string(self, player=None):
        p = self.current_player() if player is None else player
        return _host().string(self._q._raw, 0, p)

    def information_state_string(self, player=None):
        """InformationStateString (coup.cc:290-373), the MCCFR info-set key
        (outcome_sampling_mccfr.py:81-87): the library's host formatter."""
        p = self.current_player() if player is None else player
        return _host().string(self._q._raw, 1, p)

    def action_to_string(self, player, action=None):
        if action is None:  # action_to_string(action) for the current player
            player, action = self.current_player(), player
        return strings.action_to_string(player, action)

    def history(self):
        return [a for _, a in self._history]

    def full_history(self):
        return list(self._history)

    def history_str(self):
        return ", ".join(str(a) for a in self.history())

    def move_number(self):
        return (struct.unpack_from("<I", self._q._raw, 8)[0] >> 22) & 0x7F  # w2 [28:22]

    def serialize(self):
        """State::Serialize (spiel.cc:297-311)."""
        return "".join(f"{a}\n" for a in self.history())

    def __str__(self):
        return _host().string(self._q._raw, 2, 0)

    def to_string(self):
        return str(self)

    # packed access for callers that batch states themselves
    def packed_record(self):
        return self._rec.copy()

    def history_bytes(self):
        return self._hist.copy()


def apply_actions(states, actions):
    """states[k].apply_action(actions[k]) for every k, one launch per pool
    segment (coup_slot_ops): a frontier of independent games advanced
    together (MCCFR walkers, many rl_environment-style games).  The states
    must be distinct objects.  Actions apply as apply_action applies them
    (no legality check); where the reference would raise, that state stays
    unchanged, every other one advances, and SpielError names the first."""
    states, actions = list(states), [_action_id(a) for a in actions]
    if len(states) != len(actions):
        raise ValueError("one action per state")
    if len({id(s) for s in states}) != len(states):
        raise ValueError("apply_actions needs distinct states")
    players = [st.current_player() for st in states]
    by_pool = {}
    failed = None
    for k, st in enumerate(states):
        if st._slot is None:  # host states: the host op each
            q = _host().apply(st._q._raw, actions[k], _native.SLOT_UNCHECKED)
            if not q["ok"]:
                if failed is None or k < failed:
                    failed, failed_q = k, q
                continue
            st._q = q
            st._history = st._history + [(players[k], actions[k])]
            continue
        by_pool.setdefault((id(st._pool), st._slot[0]), []).append(k)
    for (_, seg), ks in by_pool.items():
        pool = states[ks[0]]._pool
        res = pool.ops(seg, [(states[k]._slot[1], -1, actions[k]) for k in ks], unchecked=True)
        # every state of the launch has advanced (or not) on the device:
        # bring each host view up to date before reporting a failure
        for k, q in zip(ks, res):
            if not q["ok"]:
                states[k]._q = pool.op(states[k]._slot)
                if failed is None or k < failed:
                    failed, failed_q = k, q
                continue
            states[k]._q = q
            states[k]._history = states[k]._history + [(players[k], actions[k])]
    if failed is not None:
        raise _apply_failed(players[failed], actions[failed], failed_q)


def load_game(name, params=None):
    """LoadGame (spiel.h:1081-1090) for the one game this build provides."""
    short = name.split("(")[0] if isinstance(name, str) else name
    if short != "coup":
        raise SpielError(f"unknown game '{name}': this build provides only 'coup'")
    return CoupGame(params or None)


def registered_names():
    return ["coup"]


def registered_games():
    """RegisteredGames (pyspiel.cc): the GameType of every game this build
    registers (rl_environment.registered_games, rl_environment.py:115-116)."""
    return [GameType()]


# the pybind class names callers annotate with or test against (pyspiel.Game,
# pyspiel.State: rl_environment.py:156, 184; best_response.py:217)
Game = CoupGame
State = CoupState


def serialize_game_and_state(game, state):
    """SerializeGameAndState (spiel.cc:428-448)."""
    return ("# Automatically generated by OpenSpiel SerializeGameAndState\n[Meta]\nVersion: 1\n\n"
            f"[Game]\n{game.serialize()}\n[State]\n{state.serialize()}\n")


def deserialize_game_and_state(text):
    """DeserializeGameAndState (spiel.cc:450-493)."""
    section, game_s, state_lines = None, "", []
    for line in text.split("\n"):
        if line.startswith("#"):
            continue
        if line in ("[Meta]", "[Game]", "[State]"):
            section = line
            continue
        if section == "[Game]" and line:
            game_s = line
        elif section == "[State]":
            state_lines.append(line)
    game = load_game(game_s)
    return game, game.deserialize_state("\n".join(state_lines))
