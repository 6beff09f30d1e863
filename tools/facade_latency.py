"""Per-op latency of the per-game State facade: the lane pool (coup_slot_op,
one launch + one 128-byte read-back per answered op) against the previous
design (one-lane scratch env: import record + history, apply, error count,
export record + history), and the batched ops (coup_slot_ops: n children of
one node, or one action on each of n states, per launch), timed in one
process.  Measurement tool only."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from open_spiel_coup_amd import pyspiel  # noqa: E402
from open_spiel_coup_amd.env import BatchedCoupEnv, HISTORY_BYTES  # noqa: E402


def scratch_apply(env, rec, hist, action):
    env.import_state(torch.from_numpy(rec.view(np.int32).reshape(1, 4)))
    env.import_history(torch.from_numpy(hist.reshape(1, HISTORY_BYTES)))
    env.apply_action(torch.tensor([int(action)], dtype=torch.int8))
    assert env.error_count() == 0
    return (env.export_state().cpu().numpy().view(np.uint32).reshape(4).copy(),
            env.export_history().cpu().numpy().reshape(HISTORY_BYTES).copy())


def scratch_query(env, rec, hist):
    env.import_state(torch.from_numpy(rec.view(np.int32).reshape(1, 4)))
    env.import_history(torch.from_numpy(hist.reshape(1, HISTORY_BYTES)))
    q = env.query(obs=False, info_state=False)
    return {k: v.cpu().numpy()[0] for k, v in q.items()}


class _Out:
    def __init__(self, a):
        self.action = a


def vector_env_rows(steps=40):
    """SyncVectorEnv.step(reset_if_done=True) per env step: one shared env
    (batched) against the reference's loop over the envs, for both
    observation types."""
    from open_spiel_coup_amd import rl_environment, vector_env
    rows = {}
    rng = np.random.default_rng(1)
    for otype, tag in ((rl_environment.ObservationType.INFORMATION_STATE, "info"),
                       (rl_environment.ObservationType.OBSERVATION, "obs")):
        for k in (1, 8, 64, 256):
            for batched in (True, False):
                if not batched and k > 64:
                    continue
                envs = [rl_environment.Environment("coup", seed=k, observation_type=otype) for _ in range(k)]
                venv = vector_env.SyncVectorEnv(envs, batched=batched)
                ts = venv.reset()

                def run(m, ts):
                    for _ in range(m):
                        outs = [_Out(int(rng.choice(t.observations["legal_actions"][t.current_player()])))
                                for t in ts]
                        ts, _, _, _ = venv.step(outs, reset_if_done=True)
                    return ts
                ts = run(3, ts)
                t0 = time.perf_counter()
                run(steps, ts)
                us = 1e6 * (time.perf_counter() - t0) / (steps * k)
                rows[f"vector_env_{tag}_n{k}_{'batched' if batched else 'loop'}_us_per_env_step"] = round(us, 1)
    return rows


def main(n=2000):
    game = pyspiel.load_game("coup")
    st = game.new_initial_state()
    for a in (0, 1, 2, 3):
        st.apply_action(a)
    for _ in range(50):
        st.child(0).legal_actions()
    t0 = time.perf_counter()
    for _ in range(n):
        st.child(0).legal_actions()
    pool_child = (time.perf_counter() - t0) / n
    t0 = time.perf_counter()
    for _ in range(n):
        st.clone()
    pool_clone = (time.perf_counter() - t0) / n
    t0 = time.perf_counter()
    for _ in range(n):
        st.observation_tensor(0)
        st._q.pop("obs", None)
    pool_obs = (time.perf_counter() - t0) / n
    env = BatchedCoupEnv(1, seed=0, auto_reset=False, obs=False, history=True)
    rec, hist = st.packed_record(), st.history_bytes()
    for _ in range(50):
        scratch_apply(env, rec, hist, 0)
    t0 = time.perf_counter()
    for _ in range(n):
        r2, h2 = scratch_apply(env, rec, hist, 0)
        scratch_query(env, r2, h2)
    scratch_child = (time.perf_counter() - t0) / n
    # batched: all children of one node in one call, per child
    batched = {}
    for k in (1, 7, 64, 1024):
        acts = [0] * k
        for _ in range(5):
            st.children(acts)
        reps = max(20, n // k)
        t0 = time.perf_counter()
        for _ in range(reps):
            st.children(acts)
        batched[f"children_n{k}_us_per_child"] = round(1e6 * (time.perf_counter() - t0) / (reps * k), 2)
        t0 = time.perf_counter()
        for _ in range(max(5, reps // 4)):
            st.children(acts, info_state=True)
        batched[f"children_n{k}_with_info_state_us_per_child"] = round(
            1e6 * (time.perf_counter() - t0) / (max(5, reps // 4) * k), 2)
    frontier = [st.clone() for _ in range(1024)]
    for _ in range(3):
        pyspiel.apply_actions(frontier, [0] * 1024)
        frontier = [st.clone() for _ in range(1024)]
    t0 = time.perf_counter()
    pyspiel.apply_actions(frontier, [0] * 1024)
    batched["apply_actions_n1024_us_per_state"] = round(1e6 * (time.perf_counter() - t0) / 1024, 2)
    from open_spiel_coup_amd import rl_environment
    renv = rl_environment.Environment("coup", seed=3)
    ts = renv.reset()
    rng = np.random.default_rng(0)
    t0 = time.perf_counter()
    for _ in range(n):
        p = ts.observations["current_player"]
        ts = renv.step([int(rng.choice(ts.observations["legal_actions"][p]))]) if p >= 0 else renv.reset()
    rl_step = (time.perf_counter() - t0) / n
    e1 = renv._env
    t0 = time.perf_counter()
    for _ in range(n):
        {k: v.cpu().numpy()[0] for k, v in e1.query(obs=False, info_state=True).items()}
    query_per_tensor = (time.perf_counter() - t0) / n
    t0 = time.perf_counter()
    for _ in range(n):
        e1.query_host(obs=False, info_state=True)
    query_one_copy = (time.perf_counter() - t0) / n
    vector = vector_env_rows()
    print(json.dumps({"tool": "facade_latency", "ops": n,
                      "rl_environment_step_us": round(1e6 * rl_step, 1),
                      "query_info_per_tensor_copies_us": round(1e6 * query_per_tensor, 1),
                      "query_info_one_copy_us": round(1e6 * query_one_copy, 1),
                      "pool_child_plus_legal_us": round(1e6 * pool_child, 1),
                      "pool_clone_us": round(1e6 * pool_clone, 1),
                      "pool_observation_tensor_us": round(1e6 * pool_obs, 1),
                      "scratch_env_child_plus_legal_us": round(1e6 * scratch_child, 1), **batched, **vector}))


if __name__ == "__main__":
    main()
