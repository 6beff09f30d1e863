"""ctypes wrapper of the CPU parity oracle (oracle/coup_oracle.c).

TEST INFRASTRUCTURE ONLY.  Importable from tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg; the product package never imports it.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")

OBS_SIZE = 98
INFO_SIZE = 2492
MAX_HIST = 136


class _OcCard(ctypes.Structure):
    _fields_ = [("value", ctypes.c_int), ("state", ctypes.c_int)]


class _OcPlayer(ctypes.Structure):
    _fields_ = [("cards", _OcCard * 4), ("ncards", ctypes.c_int),
                ("coins", ctypes.c_int), ("last_action", ctypes.c_int),
                ("lost_challenge", ctypes.c_int)]


class _OcState(ctypes.Structure):
    _fields_ = [("deck", ctypes.c_int * 5), ("pl", _OcPlayer * 2),
                ("queue", ctypes.c_int * 8), ("qlen", ctypes.c_int),
                ("turn_player", ctypes.c_int), ("move_player", ctypes.c_int),
                ("opp_player", ctypes.c_int), ("turn_begin", ctypes.c_int),
                ("turn_number", ctypes.c_int), ("is_chance", ctypes.c_int),
                ("rewards", ctypes.c_int * 2), ("move_number", ctypes.c_int),
                ("hist_len", ctypes.c_int),
                ("hist_player", ctypes.c_int * MAX_HIST),
                ("hist_action", ctypes.c_int * MAX_HIST),
                ("hist_deal_to", ctypes.c_int * MAX_HIST),
                ("error", ctypes.c_int)]


class _RolloutArgs(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64), ("env_id_base", ctypes.c_uint32),
                ("n", ctypes.c_int64), ("steps", ctypes.c_int64),
                ("auto_reset", ctypes.c_int), ("obs_overwrite", ctypes.c_int),
                ("actions", ctypes.c_void_p), ("rewards", ctypes.c_void_p),
                ("step_type", ctypes.c_void_p), ("legal", ctypes.c_void_p),
                ("obs", ctypes.c_void_p), ("info", ctypes.c_void_p),
                ("final_state", ctypes.c_void_p), ("final_hist", ctypes.c_void_p),
                ("decisions", ctypes.c_void_p), ("episodes_done", ctypes.c_void_p),
                ("return_sum_p0", ctypes.c_void_p), ("lane_episodes", ctypes.c_void_p),
                ("lane_return_sum", ctypes.c_void_p)]


class _NpPlayer(ctypes.Structure):
    _fields_ = [("cards", _OcCard * 4), ("ncards", ctypes.c_int), ("coins", ctypes.c_int),
                ("last_action", ctypes.c_int), ("lost_challenge", ctypes.c_int)]


class _NpState(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("deck", ctypes.c_int * 5), ("pl", _NpPlayer * 6),
                ("queue", ctypes.c_int * 8), ("qlen", ctypes.c_int), ("init_left", ctypes.c_int),
                ("T", ctypes.c_int), ("M", ctypes.c_int), ("O", ctypes.c_int), ("begin", ctypes.c_int),
                ("turn", ctypes.c_int), ("move", ctypes.c_int), ("rewards", ctypes.c_int * 6),
                ("error", ctypes.c_int)]


class _NpRolloutArgs(ctypes.Structure):
    _fields_ = [("n_players", ctypes.c_int), ("seed", ctypes.c_uint64), ("env_id_base", ctypes.c_uint32),
                ("n", ctypes.c_int64), ("steps", ctypes.c_int64), ("auto_reset", ctypes.c_int),
                ("actions", ctypes.c_void_p), ("rewards", ctypes.c_void_p), ("step_type", ctypes.c_void_p),
                ("legal", ctypes.c_void_p), ("obs", ctypes.c_void_p), ("final_state", ctypes.c_void_p),
                ("episodes_done", ctypes.c_void_p), ("return_sum_p0", ctypes.c_void_p),
                ("lane_episodes", ctypes.c_void_p), ("lane_return_sum", ctypes.c_void_p),
                ("cur_player", ctypes.c_void_p)]


class _WindowArgs(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64), ("env_id_base", ctypes.c_uint32), ("players", ctypes.c_int),
                ("n", ctypes.c_int64), ("steps", ctypes.c_int64), ("from_", ctypes.c_int64), ("stride", ctypes.c_int64),
                ("auto_reset", ctypes.c_int),
                ("actions", ctypes.c_void_p), ("rewards", ctypes.c_void_p), ("step_type", ctypes.c_void_p),
                ("legal", ctypes.c_void_p), ("cur_player", ctypes.c_void_p),
                ("obs_w", ctypes.c_void_p), ("obs_hash", ctypes.c_void_p),
                ("info_w", ctypes.c_void_p), ("info_hash", ctypes.c_void_p),
                ("stats_from", ctypes.c_int64), ("nsnap", ctypes.c_int),
                ("snap_at", ctypes.c_int64 * 4), ("snap_state", ctypes.c_void_p * 4),
                ("snap_eps", ctypes.c_void_p * 4), ("snap_ret", ctypes.c_void_p * 4)]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        srcs = ["coup_oracle.c", "coup_oracle.h", "coup_nplayer.c", "coup_nplayer.h"]
        if not os.path.exists(_LIB_PATH) or any(
                os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, f)) for f in srcs):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.POINTER(_OcState)
        L.oc_init.argtypes = [P]
        L.oc_is_terminal.argtypes = [P]
        L.oc_current_player.argtypes = [P]
        L.oc_legal_actions.argtypes = [P, ctypes.POINTER(ctypes.c_int)]
        L.oc_legal_mask.argtypes = [P]
        L.oc_legal_mask.restype = ctypes.c_uint32
        L.oc_apply_action.argtypes = [P, ctypes.c_int]
        L.oc_apply_action_unchecked.argtypes = [P, ctypes.c_int]
        L.oc_returns.argtypes = [P, ctypes.POINTER(ctypes.c_int)]
        L.oc_rewards.argtypes = [P, ctypes.POINTER(ctypes.c_int)]
        L.oc_chance_outcomes.argtypes = [P, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_double)]
        L.oc_observation_tensor.argtypes = [P, ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
        L.oc_info_state_tensor.argtypes = [P, ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
        for f in (L.oc_observation_string, L.oc_info_state_string):
            f.argtypes = [P, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        L.oc_to_string.argtypes = [P, ctypes.c_char_p, ctypes.c_int]
        L.oc_pack.argtypes = [P, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
        L.oc_history_bytes.argtypes = [P, ctypes.POINTER(ctypes.c_uint8)]
        L.oc_draw.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
        L.oc_draw.restype = ctypes.c_uint32
        L.oc_philox4x32_10.argtypes = [ctypes.POINTER(ctypes.c_uint32)] * 2 + [ctypes.POINTER(ctypes.c_uint32)]
        L.oc_rollout.argtypes = [ctypes.POINTER(_RolloutArgs)]
        NP = ctypes.POINTER(_NpState)
        L.np_init.argtypes = [NP, ctypes.c_int]
        L.np_is_terminal.argtypes = [NP]
        L.np_current_player.argtypes = [NP]
        L.np_legal_mask.argtypes = [NP]
        L.np_legal_mask.restype = ctypes.c_uint32
        L.np_apply_action.argtypes = [NP, ctypes.c_int]
        L.np_returns.argtypes = [NP, ctypes.POINTER(ctypes.c_int)]
        L.np_observation_tensor.argtypes = [NP, ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
        L.np_pack.argtypes = [NP, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
        L.np_rollout.argtypes = [ctypes.POINTER(_NpRolloutArgs)]
        L.oc_rollout_window.argtypes = [ctypes.POINTER(_WindowArgs)]
        L.np_rollout_window.argtypes = [ctypes.POINTER(_WindowArgs)]
        _lib = L
    return _lib


class OracleState:
    """One reference-semantics Coup game (pyspiel.State-like surface)."""

    def __init__(self):
        self._s = _OcState()
        lib().oc_init(ctypes.byref(self._s))

    def clone(self):
        c = OracleState.__new__(OracleState)
        c._s = _OcState()
        ctypes.memmove(ctypes.byref(c._s), ctypes.byref(self._s), ctypes.sizeof(_OcState))
        return c

    @property
    def raw(self):
        return self._s

    def is_terminal(self):
        return bool(lib().oc_is_terminal(ctypes.byref(self._s)))

    def current_player(self):
        return lib().oc_current_player(ctypes.byref(self._s))

    def is_chance_node(self):
        return self.current_player() == -1

    def legal_actions(self):
        buf = (ctypes.c_int * 18)()
        n = lib().oc_legal_actions(ctypes.byref(self._s), buf)
        return list(buf[:n])

    def legal_mask(self):
        return lib().oc_legal_mask(ctypes.byref(self._s))

    def apply_action(self, a):
        err = lib().oc_apply_action(ctypes.byref(self._s), int(a))
        if err:
            raise RuntimeError(f"oracle apply_action({a}) failed with code {err}")

    def apply_action_unchecked(self, a):
        """pyspiel's apply_action (pyspiel.cc:266, spiel.cc:322-331): no
        legality check; raises RuntimeError, the state unchanged, where the
        reference raises (or where the result leaves the packed record:
        code 4)."""
        err = lib().oc_apply_action_unchecked(ctypes.byref(self._s), int(a))
        if err:
            raise RuntimeError(f"oracle apply_action_unchecked({a}) failed with code {err}")

    def returns(self):
        buf = (ctypes.c_int * 2)()
        lib().oc_returns(ctypes.byref(self._s), buf)
        return list(buf)

    def rewards(self):
        buf = (ctypes.c_int * 2)()
        lib().oc_rewards(ctypes.byref(self._s), buf)
        return list(buf)

    def chance_outcomes(self):
        acts = (ctypes.c_int * 5)()
        probs = (ctypes.c_double * 5)()
        n = lib().oc_chance_outcomes(ctypes.byref(self._s), acts, probs)
        return [(acts[i], probs[i]) for i in range(n)]

    def observation_tensor(self, player):
        out = np.zeros(OBS_SIZE, np.float32)
        lib().oc_observation_tensor(ctypes.byref(self._s), player,
                                    out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        return out

    def information_state_tensor(self, player):
        out = np.zeros(INFO_SIZE, np.float32)
        lib().oc_info_state_tensor(ctypes.byref(self._s), player,
                                   out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        return out

    def _string(self, fn, *args):
        buf = ctypes.create_string_buffer(8192)
        n = fn(ctypes.byref(self._s), *args, buf, 8192)
        assert n < 8192
        return buf.value.decode()

    def observation_string(self, player):
        return self._string(lib().oc_observation_string, player)

    def information_state_string(self, player):
        return self._string(lib().oc_info_state_string, player)

    def to_string(self):
        return self._string(lib().oc_to_string)

    def pack(self, episode=0, err=0):
        out = (ctypes.c_uint32 * 4)()
        lib().oc_pack(ctypes.byref(self._s), episode, err, out)
        return list(out)

    def history(self):
        return list(self._s.hist_action[:self._s.hist_len])

    def history_bytes(self):
        out = (ctypes.c_uint8 * 96)()
        lib().oc_history_bytes(ctypes.byref(self._s), out)
        return bytes(out)

    def coins(self, p):
        return self._s.pl[p].coins

    def cards(self, p):
        pl = self._s.pl[p]
        return [(pl.cards[i].value, pl.cards[i].state) for i in range(pl.ncards)]

    def deck(self):
        return list(self._s.deck)

    def last_action(self, p):
        return self._s.pl[p].last_action


def draw(seed, env_id, episode, draw_idx):
    return lib().oc_draw(seed, env_id, episode, draw_idx)


def philox(ctr, key):
    c = (ctypes.c_uint32 * 4)(*ctr)
    k = (ctypes.c_uint32 * 2)(*key)
    o = (ctypes.c_uint32 * 4)()
    lib().oc_philox4x32_10(c, k, o)
    return list(o)


def rollout(seed, n, steps, env_id_base=0, auto_reset=True, want_obs=False,
            obs_overwrite=False, want_trajectory=True, want_info=False):
    """Uniform-random batched rollout under the sampling contract.

    Returns a dict of numpy arrays (step-major: [steps][n]...)."""
    out = {}
    a = _RolloutArgs()
    a.seed, a.env_id_base, a.n, a.steps = seed, env_id_base, n, steps
    a.auto_reset, a.obs_overwrite = int(auto_reset), int(obs_overwrite)

    def buf(name, shape, dtype):
        arr = np.zeros(shape, dtype)
        out[name] = arr
        return arr.ctypes.data

    if want_trajectory:
        a.actions = buf("actions", (steps, n), np.int8)
        a.rewards = buf("rewards", (steps, n, 2), np.int8)
        a.step_type = buf("step_type", (steps, n), np.uint8)
        a.legal = buf("legal", (steps, n), np.uint32)
    if want_obs:
        shape = (n, 2, OBS_SIZE) if obs_overwrite else (steps, n, 2, OBS_SIZE)
        a.obs = buf("obs", shape, np.float32)
    if want_info:
        a.info = buf("info", (steps, n, 2, INFO_SIZE), np.float32)
    a.final_state = buf("final_state", (n, 4), np.uint32)
    a.final_hist = buf("final_hist", (n, 96), np.uint8)
    a.decisions = buf("decisions", (1,), np.int64)
    a.episodes_done = buf("episodes_done", (1,), np.int64)
    a.return_sum_p0 = buf("return_sum_p0", (1,), np.int64)
    a.lane_episodes = buf("lane_episodes", (n,), np.int32)
    a.lane_return_sum = buf("lane_return_sum", (n,), np.int32)
    lib().oc_rollout(ctypes.byref(a))
    return out


class NpState:
    """One game of the N-player extension (coup_nplayer.h)."""

    def __init__(self, n):
        self.n = n
        self._s = _NpState()
        lib().np_init(ctypes.byref(self._s), n)

    def is_terminal(self):
        return bool(lib().np_is_terminal(ctypes.byref(self._s)))

    def current_player(self):
        return lib().np_current_player(ctypes.byref(self._s))

    def is_chance_node(self):
        return self.current_player() == -1

    def legal_mask(self):
        return lib().np_legal_mask(ctypes.byref(self._s))

    def legal_actions(self):
        m = self.legal_mask()
        k = 5 if m & (1 << 31) else 18
        return [a for a in range(k) if (m >> a) & 1]

    def apply_action(self, a):
        err = lib().np_apply_action(ctypes.byref(self._s), int(a))
        if err:
            raise RuntimeError(f"np_apply_action({a}) failed with code {err}")

    def returns(self):
        buf = (ctypes.c_int * 6)()
        lib().np_returns(ctypes.byref(self._s), buf)
        return list(buf[:self.n])

    def rewards(self):
        return list(self._s.rewards[:self.n])

    def observation_tensor(self, player):
        out = np.zeros(49 * self.n, np.float32)
        lib().np_observation_tensor(ctypes.byref(self._s), player,
                                    out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        return out

    def pack(self, episode=0):
        out = (ctypes.c_uint32 * 8)()
        lib().np_pack(ctypes.byref(self._s), episode, out)
        return list(out)

    def coins(self, p):
        return self._s.pl[p].coins

    def cards(self, p):
        pl = self._s.pl[p]
        return [(pl.cards[i].value, pl.cards[i].state) for i in range(pl.ncards)]


def np_rollout(n_players, seed, n, steps, env_id_base=0, auto_reset=True, want_obs=False):
    """Uniform-random rollout of the N-player extension (step-major arrays)."""
    out = {}
    a = _NpRolloutArgs()
    a.n_players, a.seed, a.env_id_base, a.n, a.steps, a.auto_reset = (
        n_players, seed, env_id_base, n, steps, int(auto_reset))

    def buf(name, shape, dtype):
        arr = np.zeros(shape, dtype)
        out[name] = arr
        return arr.ctypes.data

    a.actions = buf("actions", (steps, n), np.int8)
    a.rewards = buf("rewards", (steps, n, n_players), np.int8)
    a.step_type = buf("step_type", (steps, n), np.uint8)
    a.legal = buf("legal", (steps, n), np.uint32)
    if want_obs:
        a.obs = buf("obs", (steps, n, n_players, 49 * n_players), np.float32)
    a.final_state = buf("final_state", (n, 8), np.uint32)
    a.episodes_done = buf("episodes_done", (1,), np.int64)
    a.return_sum_p0 = buf("return_sum_p0", (1,), np.int64)
    a.lane_episodes = buf("lane_episodes", (n,), np.int32)
    a.lane_return_sum = buf("lane_return_sum", (n,), np.int32)
    a.cur_player = buf("cur_player", (steps, n), np.int8)
    lib().np_rollout(ctypes.byref(a))
    return out


def hash_weights(length):
    """The two rows of linear-hash weights (uint32 in [1, 2^18)) for tensors
    of `length` floats per lane (oc_window_args): fixed, so the GPU side
    (tests/lane_digest.py) hashes with the same ones."""
    rng = np.random.default_rng(0x436F7570 + length)
    return np.ascontiguousarray(rng.integers(1, 1 << 18, size=(2, length), dtype=np.uint32))


def window_threads():
    """Host threads for the window driver: the job's CPU share (OMP_NUM_THREADS
    on the GPU box), at most the affinity set."""
    avail = len(os.sched_getaffinity(0))
    want = int(os.environ.get("OMP_NUM_THREADS", avail) or avail)
    return max(1, min(avail, want))


def window(players, seed, n, steps, from_, env_id_base=0, auto_reset=True, obs_hash=False, info_hash=False,
           snaps=(), stats_from=0, threads=None, chunk=None):
    """Every lane of a uniform rollout of `n` lanes, outputs of steps
    [from_, steps) only ([steps - from_][n] step-major arrays: actions,
    rewards, step_type, legal, cur_player, and with obs_hash / info_hash the
    [.., n, 2] uint64 hashes of the ObservationTensor / InformationStateTensor
    pair, hash_weights), plus per snapshot step s in `snaps` the records
    snap_state[s] ([n, 4] / [n, 8]) and the per-lane episode counts / player-0
    return sums counted from step stats_from (snap_eps[s], snap_ret[s]).  The
    lanes are split over `threads` host threads (ctypes releases the GIL)."""
    import concurrent.futures
    assert len(snaps) <= 4 and all(0 < x <= steps for x in snaps)
    R, P = steps - from_, players
    W = 4 if players == 2 else 8
    out = {"actions": np.zeros((R, n), np.int8), "rewards": np.zeros((R, n, P), np.int8),
           "step_type": np.zeros((R, n), np.uint8), "legal": np.zeros((R, n), np.uint32),
           "cur_player": np.zeros((R, n), np.int8),
           "snap_state": {x: np.zeros((n, W), np.uint32) for x in snaps},
           "snap_eps": {x: np.zeros(n, np.int32) for x in snaps},
           "snap_ret": {x: np.zeros(n, np.int32) for x in snaps}}
    ow = iw = None
    if obs_hash:
        ow = hash_weights(2 * OBS_SIZE)
        out["obs_hash"] = np.zeros((R, n, 2), np.uint64)
    if info_hash:
        iw = hash_weights(2 * INFO_SIZE)
        out["info_hash"] = np.zeros((R, n, 2), np.uint64)
    threads = threads or window_threads()
    chunk = chunk or max(256, -(-n // (4 * threads)))
    fn = lib().oc_rollout_window if players == 2 else lib().np_rollout_window

    def run(lo):
        m = min(chunk, n - lo)
        a = _WindowArgs()
        a.seed, a.env_id_base, a.players = seed, env_id_base + lo, players
        a.n, a.steps, a.from_, a.stride, a.auto_reset = m, steps, from_, n, int(auto_reset)
        a.actions = out["actions"].ctypes.data + lo
        a.rewards = out["rewards"].ctypes.data + lo * P
        a.step_type = out["step_type"].ctypes.data + lo
        a.legal = out["legal"].ctypes.data + 4 * lo
        a.cur_player = out["cur_player"].ctypes.data + lo
        if ow is not None:
            a.obs_w, a.obs_hash = ow.ctypes.data, out["obs_hash"].ctypes.data + 16 * lo
        if iw is not None:
            a.info_w, a.info_hash = iw.ctypes.data, out["info_hash"].ctypes.data + 16 * lo
        a.stats_from, a.nsnap = stats_from, len(snaps)
        for k, x in enumerate(snaps):
            a.snap_at[k] = x
            a.snap_state[k] = out["snap_state"][x].ctypes.data + 4 * W * lo
            a.snap_eps[k] = out["snap_eps"][x].ctypes.data + 4 * lo
            a.snap_ret[k] = out["snap_ret"][x].ctypes.data + 4 * lo
        rc = fn(ctypes.byref(a))
        if rc:
            raise RuntimeError(f"oracle window driver failed ({rc})")

    with concurrent.futures.ThreadPoolExecutor(threads) as ex:
        list(ex.map(run, range(0, n, chunk)))
    return out
