"""Per-op latency of the per-game facades, as interleaved repeats in one
process (measurement tool only).

Rows:
  - the State facade with host-resident States (the default), and on the
    lane pool, with the device-resident op server
    (default) and with one launch per op (a second pool built under
    COUP_SERVER=0): child(a) + legal_actions(), clone(), the tensors;
  - batched ops (coup_slot_ops): n children of one node, one action on each
    of n states;
  - rl_environment.Environment.step (INFORMATION_STATE, the reference's
    default, and OBSERVATION) and 1-lane queries;
  - SyncVectorEnv.step per env step, batched over one shared env against
    the reference's loop over the envs.

Every row is measured once per round, rounds interleaved (`--rounds`, default
5), and reported as {median, min, max} microseconds per op: the spread
between rounds shows run-to-run noise (host-core contention, clocks) next
to the differences between rows.
"""
import argparse
import json
import os
import random
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from open_spiel_coup_amd import pyspiel  # noqa: E402


class _Out:
    def __init__(self, a):
        self.action = a


def _pool_game(server):
    """A game bound to a pool of its own, with or without the op server."""
    prev = os.environ.get("COUP_SERVER")
    os.environ["COUP_SERVER"] = "1" if server else "0"
    try:
        pool = pyspiel._Pool(torch.device("cuda", torch.cuda.current_device()))
    finally:
        if prev is None:
            os.environ.pop("COUP_SERVER", None)
        else:
            os.environ["COUP_SERVER"] = prev
    game = pyspiel.load_game("coup")
    game._pool = pool
    game._device_states = True  # States on this pool's lanes
    return game, pool


def _host_game():
    """A game whose States are host-resident (the default since round 4)."""
    game = pyspiel.load_game("coup")
    game._device_states = False
    return game


def _opening(game):
    st = game.new_initial_state()
    for a in (0, 1, 2, 3):
        st.apply_action(a)
    return st


def _timed(fn, n):
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return 1e6 * (time.perf_counter() - t0) / n


def state_rows(tag, game, n):
    st = _opening(game)
    rows = {}
    rows[f"{tag}_child_plus_legal_us"] = _timed(lambda: st.child(0).legal_actions(), n)
    rows[f"{tag}_clone_us"] = _timed(st.clone, n)

    def obs():
        st.observation_tensor(0)
        st._q.pop("obs", None)

    def info():
        st.information_state_tensor(0)
        st._q.pop("info_state", None)
    rows[f"{tag}_observation_tensor_us"] = _timed(obs, n)
    rows[f"{tag}_information_state_tensor_us"] = _timed(info, max(n // 4, 50))
    s2 = _opening(game)

    def apply_one():
        nonlocal s2
        if s2.is_terminal():
            s2 = _opening(game)
        s2.apply_action(s2.legal_actions()[0])
    rows[f"{tag}_apply_action_us"] = _timed(apply_one, n)
    rng = random.Random(0)
    s3 = _opening(game)

    def mccfr_node():
        # outcome_sampling_mccfr.py:81-87 per node: legal_actions,
        # information_state_string (the info-set key), apply_action
        nonlocal s3
        if s3.is_terminal():
            s3 = _opening(game)
        legal = s3.legal_actions()
        if not s3.is_chance_node():
            s3.information_state_string(s3.current_player())
        s3.apply_action(rng.choice(legal))
    rows[f"{tag}_mccfr_node_us"] = _timed(mccfr_node, n)
    rows[f"{tag}_information_state_string_us"] = _timed(lambda: s3.information_state_string(0), n)
    return rows


def raw_rows(tag, game, n):
    """coup_slot_op itself from a tight ctypes loop (no facade code): an
    answered query (no action), an answered apply of the lane's first legal
    action to a copy (child), an unanswered copy (clone)."""
    import ctypes
    from open_spiel_coup_amd import _native
    st = _opening(game)
    pool = st._pool
    env = pool.segs[st._slot[0]]
    env._bind_stream()
    dst = pool.alloc()
    h, lane, dh, dl, host = env._h, st._slot[1], pool.segs[dst[0]]._h, dst[1], pool.host_ptr
    f = pool.lib.coup_slot_op
    rows = {}
    rows[f"raw_{tag}_query_us"] = _timed(lambda: f(h, lane, None, 0, -1, 0, host), n)
    rows[f"raw_{tag}_child_us"] = _timed(lambda: f(dh, dl, h, lane, 0, 0, host), n)
    rows[f"raw_{tag}_clone_us"] = _timed(lambda: f(dh, dl, h, lane, -1, _native.SLOT_NO_RESULT, None), n)
    f(h, lane, None, 0, -1, 0, host)  # drain the clones
    pool.release(dst)
    return rows


def batched_rows(tag, game, n):
    st = _opening(game)
    rows = {}
    for k in (1, 7, 64, 1024):
        acts = [0] * k
        reps = max(10, n // k)
        rows[f"{tag}_children_n{k}_us_per_child"] = _timed(lambda: st.children(acts), reps) / k
        rows[f"{tag}_children_n{k}_with_info_state_us_per_child"] = _timed(
            lambda: st.children(acts, info_state=True), max(5, reps // 4)) / k
    frontier = [st.clone() for _ in range(1024)]
    t0 = time.perf_counter()
    pyspiel.apply_actions(frontier, [0] * 1024)
    rows[f"{tag}_apply_actions_n1024_us_per_state"] = 1e6 * (time.perf_counter() - t0) / 1024
    return rows


def rl_rows(n):
    from open_spiel_coup_amd import pyspiel, rl_environment
    rows = {}
    rng = random.Random(0)  # the caller's pick: ~0.5 us (numpy's choice over a list is ~10x that)
    for otype, tag in ((rl_environment.ObservationType.INFORMATION_STATE, "info"),
                       (rl_environment.ObservationType.OBSERVATION, "obs")):
        for suffix, device in (("", False), ("_device_lane", True)):
            # default: the host-resident game (round 4); _device_lane: the
            # game on a device lane (COUP_STATE_DEVICE=1), a round trip per op
            saved, pyspiel.DEVICE_STATES = pyspiel.DEVICE_STATES, device
            try:
                env = rl_environment.Environment("coup", seed=3, observation_type=otype)
            finally:
                pyspiel.DEVICE_STATES = saved
            ts = [env.reset()]

            def step():
                t = ts[0]
                p = t.observations["current_player"]
                ts[0] = env.step([rng.choice(t.observations["legal_actions"][p])]) if not t.last() else env.reset()
            rows[f"rl_environment_step_{tag}{suffix}_us"] = _timed(step, n)
            if device:
                e1 = env._env
                rows[f"query_host_{tag}_us"] = _timed(
                    lambda: e1.query_host(obs=tag == "obs", info_state=tag == "info"), n)
    return rows


def vector_env_rows(steps=40):
    """SyncVectorEnv.step(reset_if_done=True) per env step: the default
    (host-resident games kept on the host under the shared stream up to
    vector_env.HOST_UPTO envs, adopted beyond), the games adopted into one
    shared device env (HOST_UPTO = 0: one launch per step), kept on the host
    at any size (HOST_UPTO = None; beyond a finite default cut only), and the
    reference's loop over the envs (batched=False)."""
    from open_spiel_coup_amd import rl_environment, vector_env
    rows = {}
    rng = random.Random(1)
    for otype, tag in ((rl_environment.ObservationType.INFORMATION_STATE, "info"),
                       (rl_environment.ObservationType.OBSERVATION, "obs")):
        for k in (1, 8, 64, 256, 1024):
            for form in ("batched", "device", "host", "loop"):
                if form == "loop" and k > 64 or form == "host" and (vector_env.HOST_UPTO is None or
                                                                      k <= vector_env.HOST_UPTO):
                    continue
                envs = [rl_environment.Environment("coup", seed=k, observation_type=otype) for _ in range(k)]
                upto = {"device": 0, "host": None}.get(form, vector_env.HOST_UPTO)
                saved, vector_env.HOST_UPTO = vector_env.HOST_UPTO, upto
                try:
                    venv = vector_env.SyncVectorEnv(envs, batched=form != "loop")
                finally:
                    vector_env.HOST_UPTO = saved
                ts = venv.reset()

                def run(m, ts):
                    for _ in range(m):
                        outs = [_Out(rng.choice(t.observations["legal_actions"][t.current_player()]))
                                for t in ts]
                        ts, _, _, _ = venv.step(outs, reset_if_done=True)
                    return ts
                ts = run(3, ts)
                t0 = time.perf_counter()
                run(steps, ts)
                us = 1e6 * (time.perf_counter() - t0) / (steps * k)
                rows[f"vector_env_{tag}_n{k}_{form}_us_per_env_step"] = us
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", type=int, default=1000, help="ops per row per round")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--no-vector", action="store_true")
    a = ap.parse_args()
    g_srv, p_srv = _pool_game(True)
    g_launch, p_launch = _pool_game(False)
    g_host = _host_game()
    # warm the paths (segments allocated, code paths and the wave started)
    state_rows("warm_server", g_srv, 50)
    state_rows("warm_launch", g_launch, 50)
    state_rows("warm_host", g_host, 50)
    samples = {}
    for _ in range(a.rounds):
        rows = {}
        rows.update(state_rows("host", g_host, a.ops))
        rows.update(state_rows("server", g_srv, a.ops))
        rows.update(state_rows("launch", g_launch, a.ops))
        rows.update(raw_rows("server", g_srv, a.ops))
        rows.update(raw_rows("launch", g_launch, a.ops))
        rows.update(batched_rows("server", g_srv, a.ops))
        rows.update(batched_rows("host", g_host, a.ops))
        rows.update(rl_rows(a.ops // 2))
        if not a.no_vector:
            rows.update(vector_env_rows())
        for k, v in rows.items():
            samples.setdefault(k, []).append(v)
    out = {"tool": "facade_latency", "ops_per_round": a.ops, "rounds": a.rounds,
           "server_stats": dict(zip(("requests", "launches", "running", "idle_us"), p_srv.server_stats())),
           "rows_us": {k: {"median": round(statistics.median(v), 2), "min": round(min(v), 2), "max": round(max(v), 2)}
                       for k, v in samples.items()}}
    p_srv.close()
    p_launch.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
