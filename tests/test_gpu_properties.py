"""Product-path properties and parity at the bench batch (2^20 lanes):
illegal actions refused, env-id shard invariance, per-lane invariants and
determinism at full size, graph replay == eager steps, sampled lanes of a
regrouped rollout == the oracle, the query's InformationStateTensor == the
step's, [T, B] trajectory buffers == single steps and the oracle, and the
episode-counter wrap flag.  Reference semantics: coup.cc:522-808 (the
transition), :248-287 (ObservationTensor), rl_environment.py:243-248."""
import numpy as np
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu

from open_spiel_coup_amd import BatchedCoupEnv, packed  # noqa: E402


def _np(t):
    return t.detach().cpu().numpy()


def test_illegal_action_rejected():
    env = BatchedCoupEnv(4, seed=0, obs=False)
    before = _np(env.export_state()).copy()
    # at the first decision P1 may not Pass / Block / LoseCard
    env.step(torch.tensor([9, 10, 7, 18], dtype=torch.int8))
    assert env.error_count() == 4
    np.testing.assert_array_equal(_np(env.export_state()), before)


def test_shard_invariance():
    """Lanes [k, k+m) of one env == an env of m lanes with env_id_base=k:
    the basis of id-range sharding over GPUs."""
    seed, steps = 99, 64
    big = BatchedCoupEnv(1024, seed=seed, obs=False)
    part = BatchedCoupEnv(256, seed=seed, env_id_base=512, obs=False)
    big.rollout(steps)
    part.rollout(steps)
    np.testing.assert_array_equal(_np(big.export_state())[512:768], _np(part.export_state()))


# ------------------------------------------------------ full-size properties

def test_full_batch_properties():
    """At the benchmark batch (2^20 lanes): per-lane invariants after many
    steps.  Deck + hands always hold 15 cards, at most one face-up card per
    live player's 2-card hand, legal masks non-empty and well-formed, obs
    one-hots valid and coins mirrored, rewards zero-sum."""
    B = 1 << 20
    env = BatchedCoupEnv(B, seed=1, obs=True)
    for _ in range(40):
        o = env.step()
    d = packed.decode(_np(env.export_state()))
    cards = np.zeros(B, np.int64)
    for p in (0, 1):
        h = d["hand"][:, p]
        for i in range(4):
            cards += ((h >> (4 * i)) & 0xF) != 0xF
    assert np.all(d["deck"].sum(1) + cards == 15)
    assert np.all(d["queue_len"] == 0) and np.all(d["error"] == 0)
    legal = _np(o["legal_mask"]).astype(np.uint32)
    assert np.all(legal != 0) and np.all(legal < (1 << 18))
    obs = _np(o["obs"])
    assert np.all(obs[:, 0, 0] == 1) and np.all(obs[:, 1, 1] == 1)
    assert np.all(obs[:, :, 42:44].sum(-1) == 1)
    assert np.all(obs[:, 0, 60:62] == d["coins"]) and np.all(obs[:, 1, 60:62] == d["coins"])
    rw = _np(o["rewards"]).astype(np.int32)
    assert np.all(rw[:, 0] == -rw[:, 1]) and np.all(np.abs(rw) <= 2)
    assert env.error_count() == 0


def test_determinism_full_batch():
    B = 1 << 20
    a = BatchedCoupEnv(B, seed=3, obs=False)
    b = BatchedCoupEnv(B, seed=3, obs=False)
    a.rollout(50)
    for _ in range(50):
        b.step()
    assert torch.equal(a.export_state(), b.export_state())


def test_graph_replay_matches_eager():
    """K steps captured in one HIP graph (BatchedCoupEnv.capture_steps, used
    by bench.py for short kernels) == K eager coup_step calls."""
    a = BatchedCoupEnv(4096, seed=5, obs=True)
    b = BatchedCoupEnv(4096, seed=5, obs=True)
    g = b.capture_steps(10)
    for _ in range(3):
        for _ in range(10):
            oa = a.step()
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(a.export_state(), b.export_state())
    for k in ("actions", "rewards", "step_type", "legal_mask", "obs"):
        assert torch.equal(oa[k], getattr(b, "cur_player" if k == "current_player" else k)), k
    assert a.error_count() == 0 and b.error_count() == 0


def test_full_batch_sampled_lanes_match_oracle():
    """At the benchmark batch, where the fused rollout regroups lanes by
    decision (coup_regroup.h): three 256-lane slices of a 2^20-lane env
    after 120 rollout steps == the oracle run on those env ids alone."""
    B, steps, seed = 1 << 20, 120, 13
    env = BatchedCoupEnv(B, seed=seed, obs=False)
    env.rollout(steps)
    words = _np(env.export_state()).astype(np.uint32)
    for k in (0, 524_288 + 77, B - 256):
        ref = oracle.rollout(seed=seed, n=256, steps=steps, env_id_base=k, auto_reset=True, want_trajectory=False)
        np.testing.assert_array_equal(words[k:k + 256], ref["final_state"], err_msg=f"slice {k}")
    assert env.error_count() == 0


@pytest.mark.parametrize("n", [1, 300, 1100])
def test_query_info_state_equals_step_output(n):
    """coup_query's InformationStateTensor (one thread per float4 up to 1024
    lanes, the wave writer above) == the step kernel's, after 30 steps."""
    env = BatchedCoupEnv(n, seed=77, auto_reset=True, obs=False, info_state=True)
    for _ in range(30):
        o = env.step()
    q = env.query(obs=False, info_state=True)
    np.testing.assert_array_equal(_np(q["info_state"]), _np(o["info_state"]))


@pytest.mark.parametrize("graph", [False, True])
def test_trajectory_collection_matches_stepwise(graph):
    """[T, B, ...] trajectory buffers (eager collect_trajectory, or one HIP
    graph replay) == T single steps of an identical env, and the oracle."""
    n, T, seed = 300, 12, 5
    ref = oracle.rollout(seed=seed, n=n, steps=T, want_obs=True)
    env = BatchedCoupEnv(n, seed=seed, obs=True)
    if graph:
        g, buf = env.capture_trajectory(T)
        g.replay()
        torch.cuda.synchronize()
    else:
        buf = env.collect_trajectory(T)
    twin = BatchedCoupEnv(n, seed=seed, obs=True)
    for t in range(T):
        o = twin.step()
        for k in ("actions", "rewards", "step_type", "legal_mask", "current_player", "obs"):
            np.testing.assert_array_equal(_np(buf[k][t]), _np(o[k]), err_msg=f"{k} step {t}")
        np.testing.assert_array_equal(_np(buf["actions"][t]), ref["actions"][t])
        np.testing.assert_array_equal(_np(buf["obs"][t]), ref["obs"][t])
    np.testing.assert_array_equal(_np(env.export_state()), _np(twin.export_state()))


@pytest.mark.parametrize("players", [2, 6])
def test_episode_counter_wrap_is_flagged(players):
    """Each lane's episode number keys its Philox counter (DESIGN.md section
    4).  Near the top of the counter (2^28 for 2 players, 2^30 for N) the
    lanes keep stepping; the episode that wraps to 0 -- whose stream would
    repeat the lane's first game -- carries the record's error flag, and
    the episodes before and after it do not."""
    n = 512
    env = BatchedCoupEnv(n, seed=9, obs=False, num_players=players, episode_stats=True)
    w = env.export_state().cpu().numpy().view(np.uint32).copy()
    top = (1 << 28) - 2 if players == 2 else (1 << 30) - 2
    if players == 2:  # w3 [31:7] bits 24..0, w2 [31:29] bits 27..25
        w[:, 3] = (w[:, 3] & 0x7F) | ((top & 0x1FFFFFF) << 7)
        w[:, 2] = (w[:, 2] & 0x1FFFFFFF) | (((top >> 25) & 7) << 29)
    else:  # w7 bits 24..0, w6 [31:27] bits 29..25
        w[:, 7] = top & 0x1FFFFFF
        w[:, 6] = (w[:, 6] & 0x07FFFFFF) | (((top >> 25) & 31) << 27)
    env.import_state(torch.from_numpy(w.view(np.int32)))

    def episode_and_err(words):
        if players == 2:
            d = packed.decode(words)
            return d["episode"], d["error"]
        ww = words.astype(np.int64)
        return (ww[:, 7] & 0x1FFFFFF) | ((ww[:, 6] >> 27) << 25), (ww[:, 3] >> 31) & 1

    seen_zero = np.zeros(n, bool)
    for _ in range(80 if players == 2 else 700):  # 6-player games run ~10x longer
        env.step()
        ep, err = episode_and_err(env.export_state().cpu().numpy().view(np.uint32))
        assert np.all(err[ep == 0] == 1)
        assert np.all(err[ep != 0] == 0)
        seen_zero |= ep == 0
    assert seen_zero.sum() > n // 2
