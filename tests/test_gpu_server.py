"""The device-resident op server (coup_server_*):
single State ops of the lane pool run on one resident wave that polls a
request ring in mapped host memory.  Every other GPU test of the per-game
facade (tests/test_gpu_slot_pool.py, test_gpu_facade.py, test_rust_abi.py,
test_gpu_cpp_api.py) already runs through it, since the pool starts one by
default; these tests aim at the protocol itself: results against the launch
path and the oracle, ordering with stream work on the same lanes, the ring
wrapping, the idle exit and relaunch, and no wave outliving its process."""
import os
import subprocess
import sys
import time

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

from open_spiel_coup_amd import pyspiel, rl_environment  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _same(st, ref):
    assert st.packed_record().tolist() == [int(x) for x in ref.pack(0)]
    assert st.history() == ref.history()
    assert st.current_player() == ref.current_player()
    if not ref.is_terminal():
        assert st.legal_actions() == ref.legal_actions()
    assert st.returns() == [float(x) for x in ref.returns()]


def _fresh_pool(monkeypatch, **env):
    """A pool of its own (with its own server), built under `env`."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    import torch
    pool = pyspiel._Pool(torch.device("cuda", torch.cuda.current_device()))
    game = pyspiel.load_game("coup")
    game._pool = pool
    game._device_states = True  # these tests are about the device path
    return game, pool


def test_server_is_on_by_default_and_serves_the_facade():
    game = pyspiel.load_game("coup")
    game._device_states = True
    st = game.new_initial_state()
    pool = st._pool
    assert pool.srv is not None, "the pool should start an op server (COUP_SERVER unset)"
    before = pool.server_stats()[0]
    for a in (0, 1, 2, 3):
        st = st.child(a)
    st.information_state_tensor(0)
    assert pool.server_stats()[0] >= before + 5


def test_server_results_equal_launch_path_and_oracle(monkeypatch):
    """Random playouts with clones, children, both tensors and illegal
    actions, once through the server and once through per-op launches
    (COUP_SERVER=0): identical results, and equal to the oracle."""
    outs = []
    for server in ("1", "0"):
        game, pool = _fresh_pool(monkeypatch, COUP_SERVER=server)
        assert (pool.srv is not None) == (server == "1")
        rng = np.random.default_rng(21)
        log = []
        for g in range(12):
            st, ref = game.new_initial_state(), oracle.OracleState()
            for k in range(60):
                if ref.is_terminal():
                    break
                a = int(rng.choice(ref.legal_actions()))
                if k % 3 == 0:
                    st = st.child(a)
                elif k % 3 == 1:
                    c = st.clone()
                    c.apply_action(a)
                    st = c
                else:
                    st.apply_action(a)
                ref.apply_action(a)
                _same(st, ref)
                if k % 7 == 0:
                    for p in (0, 1):
                        o, i = st.observation_tensor(p), st.information_state_tensor(p)
                        assert o == list(ref.observation_tensor(p))
                        assert i == list(ref.information_state_tensor(p))
                        log.append((tuple(o), tuple(i)))
                if k % 11 == 5 and not ref.is_terminal():
                    # an action outside LegalActions: applied as the reference
                    # applies it (no legality check), or refused where
                    # DoApplyAction raises -- either way equal to the oracle
                    bad = next(x for x in range(18) if x not in ref.legal_actions())
                    r2 = ref.clone()
                    try:
                        r2.apply_action_unchecked(bad)
                    except RuntimeError:
                        with pytest.raises(pyspiel.SpielError):
                            st.apply_action(bad)
                        _same(st, ref)
                    else:
                        while r2.is_chance_node():
                            r2.apply_action(r2.legal_actions()[0])
                        if r2.current_player() >= 0 and not r2.legal_actions():
                            continue  # a node no legal play reaches: not for this walk
                        st.apply_action(bad)
                        ref.apply_action_unchecked(bad)
                        log.append(("unchecked", bad))
                        _same(st, ref)
            log.append(tuple(st.packed_record().tolist()))
        outs.append(log)
        pool.close()
    assert outs[0] == outs[1]


def test_server_ordered_with_stream_work_on_the_same_lanes(monkeypatch):
    """Server ops interleaved with batched children (coup_slot_ops, on the
    stream) and rl_environment snapshots (launch path across envs): every
    state against the oracle after each mix."""
    game, pool = _fresh_pool(monkeypatch)
    rng = np.random.default_rng(4)
    st, ref = game.new_initial_state(), oracle.OracleState()
    for step in range(40):
        if ref.is_terminal():
            st, ref = game.new_initial_state(), oracle.OracleState()
        acts = ref.legal_actions()
        kids = st.children(acts)  # stream path, reading the lane the server just wrote
        k = int(rng.integers(len(acts)))
        st = kids[k]
        ref.apply_action(acts[k])
        _same(st, ref)
        if ref.is_terminal():
            continue
        a = int(rng.choice(ref.legal_actions()))
        st.apply_action(a)  # server, on a lane coup_slot_ops wrote
        ref.apply_action(a)
        _same(st, ref)
    env = rl_environment.Environment("coup", seed=9)
    env._game._device_states = True  # its snapshots on pool lanes too
    env.reset()
    for _ in range(5):
        ts = env.get_time_step()
        if ts.last():
            env.reset()
            continue
        p = ts.observations["current_player"]
        env.step([ts.observations["legal_actions"][p][0]])
    snap = env.get_state  # pool lane written by a launch from the rl env's lane
    r2 = oracle.OracleState()
    for a in snap.history():
        r2.apply_action(a)
    c = snap.clone()  # server op reading that lane
    c._q = c._pool.op(c._slot)  # answered, through the server
    # the env's lane carries its episode counter (bits of word 3): the same
    # record as the snapshot, and the oracle's game otherwise
    assert c.packed_record().tolist() == snap.packed_record().tolist()
    ep = int(snap.packed_record()[3]) >> 7
    assert c.packed_record().tolist() == [int(x) for x in r2.pack(ep)]
    assert c.history() == r2.history() and c.legal_actions() == r2.legal_actions()
    pool.close()


def test_server_ring_wraps_under_many_asynchronous_ops(monkeypatch):
    """Hundreds of unanswered ops (clones) posted back to back -- more than
    the 64-slot ring -- then answered ones: every clone holds its source."""
    game, pool = _fresh_pool(monkeypatch)
    root = game.new_initial_state()
    for a in (0, 1, 2, 3, 0):
        root.apply_action(a)
    clones = [root.clone() for _ in range(300)]
    for c in clones[::37] + clones[-3:]:
        assert c.packed_record().tolist() == root.packed_record().tolist()
        assert c.legal_actions() == root.legal_actions()
    # answered ops on the clones themselves
    for c in clones[:5]:
        c._q = pool.op(c._slot)
        assert c.packed_record().tolist() == root.packed_record().tolist()
    assert pool.server_stats()[0] >= 300
    pool.close()


def test_server_idle_exit_and_relaunch(monkeypatch):
    """A short idle time: the wave leaves between ops and the next op starts
    a new one; results stay exact."""
    game, pool = _fresh_pool(monkeypatch, COUP_SERVER_IDLE_US="500")
    rng = np.random.default_rng(2)
    st, ref = game.new_initial_state(), oracle.OracleState()
    for k in range(30):
        if ref.is_terminal():
            break
        a = int(rng.choice(ref.legal_actions()))
        st = st.child(a)
        ref.apply_action(a)
        _same(st, ref)
        if k % 4 == 0:
            time.sleep(0.003)  # > idle: the wave has left
    req, launches, running, idle = pool.server_stats()
    assert idle == 500 and launches >= 5, (req, launches)
    pool.close()
    assert pool.server_stats() is None


def test_destroy_does_not_wait_out_an_idle_wave(monkeypatch):
    """coup_destroy frees memory, which synchronises the device: it stops the
    resident waves first instead of waiting out their idle time (here 2 s),
    and the next op starts a new wave."""
    import torch
    from open_spiel_coup_amd import BatchedCoupEnv
    game, pool = _fresh_pool(monkeypatch, COUP_SERVER_IDLE_US="2000000")
    st = game.new_initial_state()
    for a in (0, 1, 2, 3):
        st = st.child(a)  # the wave is up and idling
    other = BatchedCoupEnv(64, seed=3, device="cuda")
    torch.cuda.synchronize()
    launches = pool.server_stats()[1]
    st = st.child(st.legal_actions()[0])
    t0 = time.perf_counter()
    other.close()
    dt = time.perf_counter() - t0
    assert dt < 0.5, f"coup_destroy took {dt:.3f} s: it waited for the idle wave"
    assert pool.server_stats()[2] == 0  # the destroy stopped the wave
    ref = oracle.OracleState()
    for a in st.history():
        ref.apply_action(a)
    st = st.child(ref.legal_actions()[0])
    ref.apply_action(ref.legal_actions()[0])
    _same(st, ref)
    assert pool.server_stats()[1] > launches  # the ops after it started a new wave
    pool.close()


def test_server_ops_alongside_env_create_destroy_in_threads():
    """Pool ops in one thread while another creates, steps and destroys
    rl_environment envs attached to the same server (coup_destroy, stream ops
    and drains from a second thread): every state of the first
    thread equals the oracle's, and every env's games are legal play."""
    import gc
    import threading
    game = pyspiel.load_game("coup")
    errors = []

    def playouts():
        try:
            rng = np.random.default_rng(5)
            for g in range(20):
                st, ref = game.new_initial_state(), oracle.OracleState()
                while not ref.is_terminal():
                    a = int(rng.choice(ref.legal_actions()))
                    st = st.child(a) if rng.integers(2) else st
                    if st.history() != ref.history() + [a]:
                        st.apply_action(a)
                    ref.apply_action(a)
                    _same(st, ref)
        except Exception as e:  # noqa: BLE001 - reported by the main thread
            errors.append(e)

    def envs():
        try:
            for k in range(25):
                env = rl_environment.Environment("coup", seed=k)
                ts = env.reset()
                for _ in range(6):
                    if ts.last():
                        ts = env.reset()
                    p = ts.observations["current_player"]
                    ts = env.step([ts.observations["legal_actions"][p][0]])
                del env
                gc.collect()
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    ts = [threading.Thread(target=playouts), threading.Thread(target=envs)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in ts), "a thread hung"
    assert not errors, errors


def test_no_wave_outlives_its_process():
    """A process that uses the server and exits without closing the pool
    leaves nothing running: it exits promptly and a second process finds
    the GPU usable."""
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from open_spiel_coup_amd import pyspiel\n"
            "s = pyspiel.load_game('coup').new_initial_state()\n"
            "for a in (0, 1, 2, 3): s = s.child(a)\n"
            "print(s.legal_actions())\n" % ROOT)
    for _ in range(2):
        t0 = time.perf_counter()
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        assert r.stdout.strip() == "[0, 1, 3, 5, 6]"
        assert time.perf_counter() - t0 < 60


@pytest.mark.parametrize("otype", ["info", "obs"])
def test_environment_lane_ops_equal_batched_steps(otype, monkeypatch):
    """rl_environment.Environment's reset and step are single lane ops
    (COUP_SLOT_RESET | COUP_SLOT_DEAL, COUP_SLOT_DEAL; through the op
    server): they deal exactly what coup_reset / coup_step deal on the same
    stream.  A 1-lane BatchedCoupEnv with the same seed, driven by the same
    actions, matches record and history for record, and every time step's
    tensors equal its query."""
    import torch
    from open_spiel_coup_amd import BatchedCoupEnv
    obs_type = (rl_environment.ObservationType.OBSERVATION if otype == "obs"
                else rl_environment.ObservationType.INFORMATION_STATE)
    monkeypatch.setattr(pyspiel, "DEVICE_STATES", True)  # the env's game on a device lane (lane ops)
    env = rl_environment.Environment("coup", seed=123, observation_type=obs_type)
    twin = BatchedCoupEnv(1, seed=123, auto_reset=False, obs=False, history=True)
    assert env._pool.srv is not None
    rng = np.random.default_rng(6)
    ts = env.reset()
    twin.reset()
    episodes = 0
    for k in range(300):
        q = twin.query(obs=otype == "obs", info_state=otype == "info")
        assert torch.equal(env._env.export_state(), twin.export_state()), k
        mv = int(env.get_state.move_number())
        assert torch.equal(env._env.export_history()[:, :mv], twin.export_history()[:, :mv]), k
        t = q["obs" if otype == "obs" else "info_state"][0].cpu().numpy()
        for p in (0, 1):
            assert ts.observations["info_state"][p] == t[p].tolist(), k
        cur = int(q["current_player"][0])
        assert ts.observations["current_player"] == cur
        if ts.last():
            episodes += 1
            ts = env.reset()
            twin.reset()
            continue
        a = int(rng.choice(ts.observations["legal_actions"][cur]))
        ts = env.step([a])
        o = twin.step(torch.tensor([a], dtype=torch.int8))
        assert ts.rewards == [float(x) for x in o["rewards"][0].cpu().tolist()]
        assert ts.last() == (int(o["step_type"][0]) == 2)
    assert episodes >= 3
    assert twin.error_count() == 0
