"""Batched Coup environment on one MI355X: torch tensors over the C ABI.

`BatchedCoupEnv` is the vectorised replacement of the reference's per-game
Python loop (rl_environment.Environment + SyncVectorEnv,
open_spiel/python/rl_environment.py:143-470, vector_env.py:17-78): one call
steps every lane on the GPU.  Buffers are caller-visible torch tensors on
the env's device; kernels run on torch's current stream.
"""
import ctypes

import numpy as np
import torch

from . import _native

FIRST, MID, LAST = 0, 1, 2
SKIPPED = 3  # coup_step with a negative action: the lane was left untouched
NUM_ACTIONS = 18
OBS_SIZE = 98
INFO_STATE_SIZE = 2492
HISTORY_BYTES = _native.HISTORY_BYTES
CHANCE_FLAG = 1 << 31


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _addr(t):
    return t.data_ptr() if t is not None else None


def obs_size(num_players):
    """ObservationTensor size per player: 98 for the 2-player game
    (coup.cc:1118-1130), 49 N for the N-player extension."""
    return 49 * num_players


class BatchedCoupEnv:
    """B independent Coup games stepped together (2 players: the reference
    game; 3..6: the N-player extension).

    Args:
      batch: number of lanes B.
      seed: 64-bit seed of the sampling contract.
      env_id_base: global id of lane 0 (lane i uses env_id_base + i); ranks
        of a multi-GPU job pass disjoint ranges.
      auto_reset: SyncVectorEnv(reset_if_done=True) semantics if True,
        rl_environment semantics (LAST, then reset on the next step) if False.
      obs: write ObservationTensor of both players on every step.
      info_state: write InformationStateTensor of both players on every step
        (implies history).
      history: keep per-lane histories (InformationStateTensor, strings).
      device: CUDA (HIP) device.
      num_players: 2 (the reference game) .. 6.  N > 2 has no history /
        info_state; rewards / returns are [B, N], obs [B, N, 49 N].
      generic: run the N-player engine also at N = 2 (cross-checks).
      episode_stats: keep per-lane accumulators of the episodes that end and
        player 0's Returns() of each (coup.cc:1016-1032), updated by every
        step at the lanes that reach LAST.  True: int32 tensors `episodes`
        and `return_sum`; 2 or 4: ONE packed word per lane of that many bytes,
        `return_sum << (4 * bytes) | episodes` (`episode_word`,
        csrc/coup_episodes.h), the multi-GPU collective's payload as it
        stands (episode_payload()).  A packed word holds
        episode_capacity() steps; eager steps past that fold it into int32
        totals first (graph replays are not seen: clear or fold between
        them).  episode_stats() returns the unpacked int32 pair either way.
      unchecked: caller actions outside LegalActions() (step, apply_action)
        are applied as pyspiel's apply_action does -- no legality check,
        DoApplyAction's own checks decide (COUP_FLAG_UNCHECKED, DESIGN.md
        section 8); 2 players.  Otherwise such a lane is left unchanged and
        counts in error_count().
    """

    _served = False  # attached to an op server (pyspiel's lane pool sets it)

    def __init__(self, batch, seed=0, env_id_base=0, auto_reset=True, obs=True, info_state=False,
                 history=False, device=None, num_players=2, generic=False, episode_stats=False, unchecked=False):
        if not (0 <= int(env_id_base) and int(env_id_base) + int(batch) <= 1 << 32):
            raise ValueError("env ids are 32-bit: need 0 <= env_id_base and env_id_base + batch <= 2^32")
        self.lib = _native.load()
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise ValueError("BatchedCoupEnv runs on a HIP device only")
        self._dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.batch = int(batch)
        self.seed = int(seed)
        self.env_id_base = int(env_id_base)
        self.auto_reset = bool(auto_reset)
        self.history = bool(history or info_state)
        self.num_players = int(num_players)
        self.obs_size = obs_size(self.num_players)
        flags = ((_native.FLAG_AUTO_RESET if self.auto_reset else 0) | (_native.FLAG_HISTORY if self.history else 0)
                 | (_native.FLAG_GENERIC if generic else 0) | (_native.FLAG_UNCHECKED if unchecked else 0))
        self._h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _native.check(self.lib.coup_create_ex(self.batch, self.seed, self.env_id_base, flags, self.num_players,
                                                  ctypes.byref(self._h)))
        self.state_words = self.lib.coup_state_bytes(self._h) // 4
        B, dev, P = self.batch, self.device, self.num_players
        self.actions = torch.empty(B, dtype=torch.int8, device=dev)
        self.rewards = torch.zeros(B, P, dtype=torch.int8, device=dev)
        self.step_type = torch.zeros(B, dtype=torch.uint8, device=dev)
        self.legal_mask = torch.zeros(B, dtype=torch.int32, device=dev)
        self.cur_player = torch.zeros(B, dtype=torch.int8, device=dev)
        self.obs = torch.zeros(B, P, self.obs_size, dtype=torch.float32, device=dev) if obs else None
        self.info_state = (torch.zeros(B, 2, INFO_STATE_SIZE, dtype=torch.float32, device=dev)
                           if info_state else None)
        packed = episode_stats is not True and episode_stats in (2, 4)
        if episode_stats and not packed and episode_stats is not True and episode_stats != 1:
            raise ValueError("episode_stats: False, True (int32 pair) or 2 / 4 (packed word bytes)")
        self.episode_word_bytes = int(episode_stats) if packed else 0
        self.episode_word = (torch.zeros(B, dtype=torch.int16 if episode_stats == 2 else torch.int32, device=dev)
                             if packed else None)
        self._ep_fold = None  # int32 (episodes, return sums) folded out of the packed word
        self._ep_steps = 0    # steps accumulated in the packed word since its last fold / clear
        self.episodes = torch.zeros(B, dtype=torch.int32, device=dev) if episode_stats and not packed else None
        self.return_sum = torch.zeros(B, dtype=torch.int32, device=dev) if episode_stats and not packed else None
        self._out = _native.StepOutputs(
            _addr(self.actions), _addr(self.rewards), _addr(self.step_type), _addr(self.legal_mask),
            _addr(self.cur_player), _addr(self.obs), _addr(self.info_state), *self._ep_fields())

    # ------------------------------------------------------------ plumbing
    def _ep_fields(self):
        """The accumulator fields of a coup_step_outputs (episodes,
        return_sum, episode_word, episode_word_bytes)."""
        return (_addr(self.episodes), _addr(self.return_sum), _addr(self.episode_word), self.episode_word_bytes)

    def _ep_reserve(self, steps):
        """Account for `steps` eager steps about to accumulate into the
        packed word: fold it first if they would overflow its fields."""
        if self.episode_word is None:
            return
        cap = self.episode_capacity()
        if steps > cap:
            raise ValueError(f"{steps} steps in one launch overflow the {self.episode_word_bytes}-byte episode word "
                             f"(capacity {cap}); use episode_stats=4 or True")
        if self._ep_steps + steps > cap:
            self.fold_episode_stats()
        self._ep_steps += steps

    def _bind_stream(self):
        # the raw handle of torch's current stream (no Stream object: this runs
        # before every launch of the per-game facades)
        s = torch._C._cuda_getCurrentRawStream(self._dev_index)
        if s != getattr(self, "_bound_stream", None):
            _native.check(self.lib.coup_set_stream(self._h, ctypes.c_void_p(s)))
            self._bound_stream = s

    def reload_knobs(self):
        """Re-read the dispatch knobs (COUP_OBS_SPLIT, COUP_REGROUP, ...) from
        the environment: coup_create reads them once, launches never do
        (tests and A/B runs switching this env between forms)."""
        _native.check(self.lib.coup_reload_knobs(self._h))

    def close(self):
        if self._h:
            self.lib.coup_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _mask_ptr(self, mask):
        if mask is None:
            return None
        mask = mask.to(device=self.device, dtype=torch.uint8).contiguous()
        self._keep = mask
        return _ptr(mask)

    def set_output(self, name, tensor):
        """Point one step output (e.g. 'obs') at a caller-owned tensor."""
        setattr(self, name, tensor)
        setattr(self._out, name, _addr(tensor))

    # ------------------------------------------------------------ batched API
    def reset(self, mask=None):
        """rl_environment.reset for all lanes (or lanes where mask != 0)."""
        self._bind_stream()
        _native.check(self.lib.coup_reset(self._h, self._mask_ptr(mask)))
        return self.query(obs=self.obs is not None, info_state=self.info_state is not None)

    def step(self, actions=None):
        """One batched env step.  actions: int8/long tensor [B] of decision
        actions, or None for the in-kernel uniform random policy; a negative
        action skips its lane (left untouched, step type SKIPPED, no error).
        Returns a dict of tensors (views of the env's output buffers)."""
        self._bind_stream()
        a = None
        if actions is not None:
            actions = actions.to(device=self.device, dtype=torch.int8).contiguous()
            if actions.numel() != self.batch:
                raise ValueError("actions must have one entry per lane")
            self._keep_actions = actions
            a = _ptr(actions)
        self._ep_reserve(1)
        _native.check(self.lib.coup_step(self._h, a, ctypes.byref(self._out)))
        out = {"actions": self.actions, "rewards": self.rewards, "step_type": self.step_type,
               "legal_mask": self.legal_mask, "current_player": self.cur_player}
        if self.obs is not None:
            out["obs"] = self.obs
        if self.info_state is not None:
            out["info_state"] = self.info_state
        return out

    def step_host(self, actions=None, obs=False, info_state=False, active_only=False):
        """`step` for small batches that want the answers on the host
        (coup_step_host: the kernel writes into mapped pinned memory, one
        launch and one synchronisation).  actions: host int8-convertible [B]
        (negative entries skip lanes) or None for the uniform policy.
        Returns numpy arrays: legal_mask, current_player, step_type, rewards,
        actions, terminal (step type LAST), and obs / info_state if asked --
        [B, ...], or with active_only (COUP_HOST_ACTIVE) only the rows of the
        lanes whose action is >= 0, in lane order."""
        self._bind_stream()
        B, P = self.batch, self.num_players
        want = (_native.HOST_OBS if obs else 0) | (_native.HOST_INFO if info_state else 0)
        if active_only:
            if actions is None:
                raise ValueError("active_only needs actions")
            want |= _native.HOST_ACTIVE
        key = (want,)
        if getattr(self, "_sh_key", None) != key:
            off = (ctypes.c_size_t * 6)()
            total = self.lib.coup_step_host_layout(B, P, want, off)
            self._sh_off = list(off)
            self._sh_buf = np.empty(max(total, 1), dtype=np.uint8)
            self._sh_key = key
        a = None
        if actions is not None:
            acts = np.ascontiguousarray(np.asarray(actions, dtype=np.int8).reshape(B))
            self._sh_acts = acts
            a = ctypes.c_void_p(acts.ctypes.data)
        _native.check(self.lib.coup_step_host(self._h, a, want, ctypes.c_void_p(self._sh_buf.ctypes.data)))
        h, off = self._sh_buf, self._sh_off
        out = {"legal_mask": h[off[0]:off[0] + 4 * B].view(np.int32).copy(),
               "current_player": h[off[1]:off[1] + B].view(np.int8).copy(),
               "step_type": h[off[2]:off[2] + B].copy(),
               "rewards": h[off[3]:off[3] + B * P].view(np.int8).reshape(B, P).copy(),
               "actions": h[off[4]:off[4] + B].view(np.int8).copy()}
        out["terminal"] = (out["step_type"] == LAST).astype(np.uint8)
        o = off[5]
        rows = int((self._sh_acts >= 0).sum()) if active_only else B
        if obs:
            n = rows * P * self.obs_size * 4
            out["obs"] = h[o:o + n].view(np.float32).reshape(rows, P, self.obs_size).copy()
            o += (n + 15) // 16 * 16
        if info_state:
            n = rows * 2 * INFO_STATE_SIZE * 4
            out["info_state"] = h[o:o + n].view(np.float32).reshape(rows, 2, INFO_STATE_SIZE).copy()
        return out

    def episode_capacity(self):
        """Steps the packed episode word holds between folds: every field
        must stay in range with one episode per step and |Returns()[0]| <=
        2 (N - 1) (None for the int32 pair)."""
        if self.episode_word is None:
            return None
        lim = 127 if self.episode_word_bytes == 2 else 32767
        return min(2 * lim + 1, lim // (2 * (self.num_players - 1)))

    def _unpack_word(self):
        w = self.episode_word
        if self.episode_word_bytes == 2:
            return (w & 0xFF).to(torch.int32), (w >> 8).to(torch.int32)  # arithmetic shift: signed sums
        return w & 0xFFFF, w >> 16

    def fold_episode_stats(self):
        """Move the packed word's counts into int32 totals and zero it."""
        if self.episode_word is None:
            return
        eps, ret = self._unpack_word()
        if self._ep_fold is None:
            self._ep_fold = (eps.clone(), ret.clone())
        else:
            self._ep_fold[0].add_(eps)
            self._ep_fold[1].add_(ret)
        self.episode_word.zero_()
        self._ep_steps = 0

    def episode_stats(self):
        """(episodes, return_sum) per lane since the last clear_episode_stats
        (int32 [B] device tensors; needs episode_stats).  The pair form
        returns the env's own tensors, the packed form an unpacked copy."""
        if self.episodes is not None:
            return self.episodes, self.return_sum
        if self.episode_word is None:
            raise ValueError("env created without episode_stats")
        eps, ret = self._unpack_word()
        if self._ep_fold is not None:
            eps, ret = eps + self._ep_fold[0], ret + self._ep_fold[1]
        return eps, ret

    def episode_payload(self):
        """The per-lane accumulators as the collective's payload: the packed
        word itself, viewed as int32 (an int16 word's lane pairs; RCCL has no
        int16 type; needs an even batch), or [B, 2] int32 (episodes,
        return_sum) for the pair form.  The packed payload is exact only
        while nothing was folded out of it (clear_episode_stats before the
        window it covers)."""
        if self.episode_word is not None:
            if self._ep_fold is not None:
                raise ValueError("the packed word was folded: clear_episode_stats before collecting a payload")
            if self.episode_word_bytes == 2:
                if self.batch % 2:
                    raise ValueError("an int16 payload needs an even batch")
                return self.episode_word.view(torch.int32)
            return self.episode_word
        eps, ret = self.episode_stats()
        return torch.stack((eps, ret), 1)

    def clear_episode_stats(self):
        if self.episodes is not None:
            self.episodes.zero_()
            self.return_sum.zero_()
        if self.episode_word is not None:
            self.episode_word.zero_()
            self._ep_fold = None
            self._ep_steps = 0

    def step_many(self, steps):
        """`steps` uniform-policy env steps as one call (coup_step_many): the
        same results as `steps` step() calls -- the output buffers hold the
        last step's outputs.  From 2^20 lanes with observations the rules of
        up to 8 steps run as one regrouped trajectory launch storing every
        step's records, then the observation writer once per step (DESIGN.md
        section 5)."""
        self._bind_stream()
        self._ep_reserve(int(steps))
        _native.check(self.lib.coup_step_many(self._h, int(steps), ctypes.byref(self._out)))

    def capture_steps(self, steps, actions=None):
        """Record `steps` batched env steps (uniform policy, or the fixed
        `actions` tensor every step) as one HIP graph; `graph.replay()` then
        runs them with a single launch, writing the usual output buffers.
        Removes the per-step host overhead where a step's kernel is short
        (small B).  Uniform steps are recorded through coup_step_many (the
        rules-trajectory split step where it applies).  The env must outlive the
        graph."""
        a = None
        if actions is not None:
            actions = actions.to(device=self.device, dtype=torch.int8).contiguous()
            self._graph_actions = actions
            a = _ptr(actions)
        self._ep_reserve(int(steps))  # the first replay's steps (later replays: the caller clears or folds)
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.graph(g, stream=side):
            self._bind_stream()
            if a is None:
                _native.check(self.lib.coup_step_many(self._h, int(steps), ctypes.byref(self._out)))
            else:
                for _ in range(int(steps)):
                    _native.check(self.lib.coup_step(self._h, a, ctypes.byref(self._out)))
        torch.cuda.current_stream(self.device).wait_stream(side)
        self._bind_stream()
        return g

    def trajectory_buffers(self, steps):
        """Device buffers for `steps` recorded env steps: [T, B, ...] versions of
        the step outputs this env writes (the learner-side replay data of
        rl_environment time steps, rl_environment.py:282-322)."""
        T, B, P, dev = int(steps), self.batch, self.num_players, self.device
        buf = {"actions": torch.empty(T, B, dtype=torch.int8, device=dev),
               "rewards": torch.empty(T, B, P, dtype=torch.int8, device=dev),
               "step_type": torch.empty(T, B, dtype=torch.uint8, device=dev),
               "legal_mask": torch.empty(T, B, dtype=torch.int32, device=dev),
               "current_player": torch.empty(T, B, dtype=torch.int8, device=dev)}
        if self.obs is not None:
            buf["obs"] = torch.empty(T, B, P, self.obs_size, dtype=torch.float32, device=dev)
        if self.info_state is not None:
            buf["info_state"] = torch.empty(T, B, 2, INFO_STATE_SIZE, dtype=torch.float32, device=dev)
        return buf

    def _slice_outputs(self, buf, t):
        return _native.StepOutputs(*[_addr(buf[k][t]) if k in buf else None for k in
                                     ("actions", "rewards", "step_type", "legal_mask", "current_player", "obs",
                                      "info_state")], *self._ep_fields())

    def _fused_trajectory(self, buf):
        """Whether coup_step_trajectory takes `buf` in one call: always with
        tensors (the library's rules-trajectory split observation step from
        2^20 lanes, else one coup_step per slice); without them only on an
        env without history (its one-launch kernels keep none)."""
        return "obs" in buf or "info_state" in buf or not self.history

    def _trajectory_outputs(self, buf):
        return _native.StepOutputs(*[_addr(buf[k]) if k in buf else None for k in
                                     ("actions", "rewards", "step_type", "legal_mask", "current_player", "obs",
                                      "info_state")], *self._ep_fields())

    def collect_trajectory(self, steps, buf=None):
        """`steps` uniform-policy env steps whose outputs land in slice t of
        [T, B, ...] device buffers (trajectory_buffers); returns them.  One
        coup_step_trajectory call: without tensors or history ONE launch
        (state in registers); with observations the rules-trajectory split
        step from 2^20 lanes, else one coup_step per slice inside the library.  A
        history env without tensors takes one coup_step per slice here.  Same
        results either way."""
        buf = buf if buf is not None else self.trajectory_buffers(steps)
        self._bind_stream()
        self._ep_reserve(int(steps))
        if self._fused_trajectory(buf):
            out = self._trajectory_outputs(buf)
            _native.check(self.lib.coup_step_trajectory(self._h, int(steps), ctypes.byref(out)))
            return buf
        for t in range(int(steps)):
            out = self._slice_outputs(buf, t)
            _native.check(self.lib.coup_step(self._h, None, ctypes.byref(out)))
        return buf

    def step_trajectory_launcher(self, steps, buf):
        """collect_trajectory(steps, buf) as a zero-argument callable that only
        enqueues the one coup_step_trajectory launch (timing loops)."""
        if not self._fused_trajectory(buf):
            raise ValueError("coup_step_trajectory without tensors needs an env without history")
        self._bind_stream()
        out = self._trajectory_outputs(buf)
        fn, h, k, ref = self.lib.coup_step_trajectory, self._h, int(steps), ctypes.byref(out)
        reserve = self._ep_reserve

        def launch():
            reserve(k)
            _native.check(fn(h, k, ref))
        launch.out = out  # keeps the struct alive with the callable
        launch.buf = buf
        return launch

    def capture_trajectory(self, steps, buf=None):
        """collect_trajectory recorded as one HIP graph: `graph.replay()`
        steps the env `steps` times and refills the same [T, B, ...] buffers.
        Returns (graph, buffers).  The env must outlive the graph."""
        buf = buf if buf is not None else self.trajectory_buffers(steps)
        self._ep_reserve(int(steps))  # the first replay's steps (later replays: the caller clears or folds)
        fused = self._fused_trajectory(buf)
        self._traj_outs = ([self._trajectory_outputs(buf)] if fused else
                           [self._slice_outputs(buf, t) for t in range(int(steps))])
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.graph(g, stream=side):
            self._bind_stream()
            if fused:
                _native.check(self.lib.coup_step_trajectory(self._h, int(steps), ctypes.byref(self._traj_outs[0])))
            for out in ([] if fused else self._traj_outs):
                _native.check(self.lib.coup_step(self._h, None, ctypes.byref(out)))
        torch.cuda.current_stream(self.device).wait_stream(side)
        self._bind_stream()
        return g, buf

    def rollout(self, steps, stats=None):
        """`steps` uniform-random steps per lane in one launch.  stats: optional
        dict with int32 [B] tensors 'episodes', 'return_sum', 'length_sum'
        (accumulated), or {'episode_word': int16 / int32 [B]} for the packed
        form (new_stats(packed_bytes))."""
        self.rollout_launcher(steps, stats)()

    def rollout_launcher(self, steps, stats=None):
        """rollout(steps, stats) with its arguments bound up front: a
        zero-argument callable that only enqueues the launch (on the stream
        current when it was made), for timing loops."""
        self._bind_stream()
        s = None
        if stats is not None:
            w = stats.get("episode_word")
            s = _native.RolloutStats(_addr(stats.get("episodes")), _addr(stats.get("return_sum")),
                                     _addr(stats.get("length_sum")), _addr(w),
                                     0 if w is None else w.element_size())
        fn, h, k, ref = self.lib.coup_rollout, self._h, int(steps), ctypes.byref(s) if s else None

        def launch():
            _native.check(fn(h, k, ref))
        launch.stats = s  # keeps the struct alive with the callable
        launch.steps = k
        return launch

    def new_stats(self, packed_bytes=None):
        """Zeroed rollout statistics: int32 'episodes', 'return_sum' and
        'length_sum', or with packed_bytes = 2 / 4 one packed 'episode_word'
        (csrc/coup_episodes.h; no lengths)."""
        if packed_bytes is not None:
            if packed_bytes not in (2, 4):
                raise ValueError("packed_bytes: 2 or 4")
            dt = torch.int16 if packed_bytes == 2 else torch.int32
            return {"episode_word": torch.zeros(self.batch, dtype=dt, device=self.device)}
        z = lambda: torch.zeros(self.batch, dtype=torch.int32, device=self.device)  # noqa: E731
        return {"episodes": z(), "return_sum": z(), "length_sum": z()}

    # ------------------------------------------------- State surface per lane
    def new_initial_state(self, mask=None):
        self._bind_stream()
        _native.check(self.lib.coup_new_initial_state(self._h, self._mask_ptr(mask)))

    def apply_action(self, actions):
        """State::ApplyAction per lane (decision or chance outcome; <0 = skip)."""
        self._bind_stream()
        actions = actions.to(device=self.device, dtype=torch.int8).contiguous()
        self._keep_actions = actions
        _native.check(self.lib.coup_apply_action(self._h, _ptr(actions)))

    def query(self, obs=True, info_state=False):
        self._bind_stream()
        B, dev, P = self.batch, self.device, self.num_players
        q = {"legal_mask": torch.empty(B, dtype=torch.int32, device=dev),
             "current_player": torch.empty(B, dtype=torch.int8, device=dev),
             "terminal": torch.empty(B, dtype=torch.uint8, device=dev),
             "rewards": torch.empty(B, P, dtype=torch.int8, device=dev),
             "returns": torch.empty(B, P, dtype=torch.int8, device=dev)}
        if obs:
            q["obs"] = torch.empty(B, P, self.obs_size, dtype=torch.float32, device=dev)
        if info_state:
            q["info_state"] = torch.empty(B, 2, INFO_STATE_SIZE, dtype=torch.float32, device=dev)
        qo = _native.QueryOutputs(*[_addr(q.get(k)) for k in
                                    ("legal_mask", "current_player", "terminal", "rewards", "returns", "obs",
                                     "info_state")])
        _native.check(self.lib.coup_query(self._h, ctypes.byref(qo)))
        return q

    def query_host(self, obs=True, info_state=False):
        """`query` for small batches that want the answers on the host: one
        device buffer holds every output (lane-major sections), and one copy
        into pinned memory brings it back (a single synchronisation).
        Returns numpy arrays keyed like `query`."""
        self._bind_stream()
        B, P = self.batch, self.num_players
        sizes = [("legal_mask", 4 * B), ("current_player", B), ("terminal", B), ("rewards", B * P),
                 ("returns", B * P)]
        if obs:
            sizes.append(("obs", 4 * B * P * self.obs_size))
        if info_state:
            sizes.append(("info_state", 4 * B * 2 * INFO_STATE_SIZE))
        offs, total = {}, 0
        for k, n in sizes:
            offs[k] = total
            total += (n + 15) // 16 * 16
        if getattr(self, "_qh_total", None) != total:
            self._qh_dev = torch.empty(total, dtype=torch.uint8, device=self.device)
            self._qh_host = torch.empty(total, dtype=torch.uint8, pin_memory=True)
            self._qh_total = total
        base = self._qh_dev.data_ptr()
        qo = _native.QueryOutputs(*[(base + offs[k]) if k in offs else None for k in
                                    ("legal_mask", "current_player", "terminal", "rewards", "returns", "obs",
                                     "info_state")])
        _native.check(self.lib.coup_query(self._h, ctypes.byref(qo)))
        self._qh_host.copy_(self._qh_dev, non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        h = self._qh_host.numpy()
        shapes = {"legal_mask": (np.int32, (B,)), "current_player": (np.int8, (B,)), "terminal": (np.uint8, (B,)),
                  "rewards": (np.int8, (B, P)), "returns": (np.int8, (B, P)),
                  "obs": (np.float32, (B, P, self.obs_size)), "info_state": (np.float32, (B, 2, INFO_STATE_SIZE))}
        out = {}
        for k, n in sizes:
            dt, shape = shapes[k]
            out[k] = h[offs[k]:offs[k] + n].view(dt).reshape(shape).copy()
        return out

    def export_state(self):
        self._bind_stream()
        out = torch.empty(self.batch, self.state_words, dtype=torch.int32, device=self.device)
        _native.check(self.lib.coup_export_state(self._h, _ptr(out)))
        return out

    def import_state(self, packed):
        self._bind_stream()
        packed = packed.to(device=self.device, dtype=torch.int32).contiguous()
        if packed.shape != (self.batch, self.state_words):
            raise ValueError(f"packed state must be [B, {self.state_words}] int32")
        self._keep_state = packed
        _native.check(self.lib.coup_import_state(self._h, _ptr(packed)))

    def export_history(self):
        self._bind_stream()
        out = torch.empty(self.batch, HISTORY_BYTES, dtype=torch.uint8, device=self.device)
        _native.check(self.lib.coup_export_history(self._h, _ptr(out)))
        return out

    def import_history(self, hist):
        self._bind_stream()
        hist = hist.to(device=self.device, dtype=torch.uint8).contiguous()
        if hist.shape != (self.batch, HISTORY_BYTES):
            raise ValueError(f"history must be [B, {HISTORY_BYTES}] uint8")
        self._keep_hist = hist
        _native.check(self.lib.coup_import_history(self._h, _ptr(hist)))

    def error_count(self):
        """Lanes that rejected an action since the last call (synchronises)."""
        self._bind_stream()
        n = ctypes.c_int64()
        _native.check(self.lib.coup_error_count(self._h, ctypes.byref(n)))
        return n.value
