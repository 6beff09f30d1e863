"""Coup env-steps/sec on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c3i|c2|c2r|c2t|c4|c4r|c4t]

--gpus N: N ranks, one process per GPU.  Under torchrun (WORLD_SIZE set) N
must equal WORLD_SIZE; run directly with N > 1, this process starts the N
rank processes itself (before it touches the GPU) with the torchrun
environment, relays rank 0's line and fails if any rank fails.

Workload (default c3 = configs[2] of BASELINE.json, the batch-2^20 config the
metric is quoted on): 2-player Coup, B = 2^20 lanes per GPU, uniform-random
policy drawn in-kernel, one env step per lane per launch, with the
ObservationTensor of both players written out (fp32 [B][2][98]) every step
plus actions, rewards, step types and legal masks -- the batched
rl_environment/SyncVectorEnv step.  Synthetic data: the games themselves.

Other configs (secondary lines, not the headline):
  c3i  as c3 but InformationStateTensor x2 (fp32 [B][2][2492]) instead, B = 2^18
  c2   configs[1]: B = 65,536, no observations, one launch per step
  c2r  configs[1] fused: B = 65,536, `steps` env steps in ONE launch (coup_rollout)
  c4   configs[3]: 6-player extension, B = 2^20, no observations (parity
       unpinned w.r.t. the 2-player reference; pinned to oracle/coup_nplayer.c)
  c4r  c4 fused: `steps` 6-player env steps in ONE launch
  c2t, c4t  c2 / c4 as ONE coup_step_trajectory launch of `steps` env steps
       with every step's outputs (actions, rewards, step types, legal masks,
       players) stored to [K][B] trajectory buffers

A "step" is one batched env step over all B lanes; value = env-steps/s of
the whole job (N x B x K / max-over-ranks wall time).  Before the W warmup
steps, --settle (default 256) untimed steps run through the fused rollout so
the lanes are spread over game phases as in a long run (a freshly reset batch
is in lock-step, and its first steps diverge less); after them, untimed
repeats of the timed K steps for --power-warm-ms (default 40 ms of GPU time)
bring the GPU from its idle power state to the one sustained load runs in
(tools/dpm_probe.py; reported as power_warm).  Multi-GPU: one
process per GPU (torchrun), global env ids sharded by rank, no collective
inside the step loop; every step accumulates, per lane, the episodes that
end and player 0's Returns() of each (coup.cc:1016-1032), and the timed
region ends with one RCCL all-gather of those per-lane episode counts and
return sums (the collation of SURVEY.md 8(e)).

roofline: algorithmic bytes per launch over the step
kernel's average duration from HIP events on the launch stream; traffic:
HBM bytes per launch from the rocprofv3 PMC passes recorded in profiles/
(null if absent).  From 2^20 lanes the observation step is split
(coup_obs_split_variant: the rules step without tensors, then an
address-order observation writer) and its K timed steps run as coup_step_many's
rules-trajectory form (chunks of up to 8 steps as one regrouped rules launch
that keeps the records in registers and stores every step's records, then
the writer once per step); c3i's InformationStateTensor step is split from
2^18 lanes.  The same process then times a store-only sweep on this box: for
the split steps coup_measure_store_sweep -- the same address-order grid over
the same tensor buffer, stores only -- and for the fused step
coup_measure_step_traffic (its loads and stores with no rules);
roofline.store_sweep_ms is that time and sweep_over_kernel = sweep / kernel
time, store_sweep_form says which.  It is NOT a bound: the sweep runs slower
than the split writers themselves; the bound is the
spec figure in `peak`.  roofline.valu_issue_frac: VALU instructions per
launch (profiles/traffic.json, from the SQ_INSTS_VALU pass of the same form)
x 4 cycles / (1024 SIMDs x the box's gfx clock x the launch's time) -- the
share of the chip's VALU issue slots the timed launch used; `bound` names
whichever of the two fractions is higher.
`box` names the GPU box (boxes differ in HBM store rate).
cpu_baseline: the C oracle (a scalar port of the reference rules, ~14x
faster than the reference's own C++ on the survey host) on one
host core, same per-lane workload.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# configs whose K timed steps replay from one HIP graph: c2 and c4, whose
# step kernels (9 us, 60 us) are shorter than the host's per-step launch
# cost, and c3, where the graph removes the ~6 us gap per step that eager
# launches leave between kernels
# configs whose K timed steps are one HIP graph of coup_step_many (c3: 23
# launches per 20 steps; c2 / c4: ONE trajectory launch, which the graph
# submits with less host time than an eager Python call -- the wall clock
# counts that host time -- at the price of ~6-13 us of graph-launch packets
# inside the event window: c2's kernel_ms is 87 us of kernel plus that,
# profiles/r05/c2/)
GRAPH_AUTO = ("c2", "c3", "c4")


def bare_many_active(with_obs, with_info, fused):
    """Whether the timed steps are coup_step_many's tensor-free form: ONE
    trajectory launch for the K steps (every step's outputs over the [B]
    buffers; mirrors coup_kernels.hip `many_bare`, COUP_PIPE=0 turns it
    off: then K coup_step launches)."""
    return (not fused and not with_obs and not with_info and
            os.environ.get("COUP_PIPE", "1").strip() != "0")
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "traffic.json")

# config -> (default batch, obs, info_state, fused, algorithmic bytes per lane-step, workload name, players);
# fused: False (one coup_step per step), "rollout" (coup_rollout: statistics
# only) or "traj" (coup_step_trajectory: every step's outputs)
CONFIGS = {
    "c3": (1 << 20, True, False, False, 824, "coup-2p-uniform-b2^20-obs", 2),
    "c3i": (1 << 18, False, True, False, 40 + 2 * 2492 * 4 + 96 + 96, "coup-2p-uniform-b2^18-infostate", 2),
    "c2": (65536, False, False, False, 40, "coup-2p-uniform-b65536", 2),
    "c2r": (65536, False, False, "rollout", 32, "coup-2p-uniform-b65536-fused-rollout", 2),
    "c2t": (65536, False, False, "traj", 40, "coup-2p-uniform-b65536-fused-trajectory", 2),
    # 2 x 48 B state + mask 4 + action 1 + rewards 6 + 1
    "c4": (1 << 20, False, False, False, 108, "coup-6p-uniform-b2^20", 6),
    "c4r": (1 << 20, False, False, "rollout", 96, "coup-6p-uniform-b2^20-fused-rollout", 6),
    "c4t": (1 << 20, False, False, "traj", 108, "coup-6p-uniform-b2^20-fused-trajectory", 6),
}


def payload_width(players, steps, batch):
    """Bytes per lane of the collective's payload: per lane, the finished-
    episode count and the player-0 return sum of `steps` steps (at most
    `steps` episodes, |return| <= 2(N-1) per episode).  While both fit 8 bits
    (2(N-1) K <= 127: K <= 63 steps for 2 players, the driver's K = 20 among
    them) one int16 per lane; while they fit 16 bits (K <= 1000) one int32;
    else two int32."""
    if 2 * (players - 1) * steps <= 127 and batch % 2 == 0:
        return 2
    return 4 if steps <= 1000 else 8


def episode_stats_mode(width):
    """BatchedCoupEnv(episode_stats=...) for a payload width: the packed word
    the step kernels accumulate in place (2 / 4 bytes, csrc/coup_episodes.h),
    so the payload needs no packing inside the timed window; the int32 pair
    beyond 1000 steps."""
    return width if width in (2, 4) else True


def pack_episodes(eps, ret, width):
    """[B] int32 episode counts and return sums -> the payload format, as a
    torch computation: what the kernels' packed word holds (int16 return << 8
    | episodes with lane pairs viewed as int32, RCCL having no int16 type;
    int32 return << 16 | episodes), or [B, 2] int32.  Tests compare the
    kernels' words with it; the timed path does not run it."""
    import torch
    if width == 2:
        return ((ret.to(torch.int16) << 8) | eps.to(torch.int16)).view(torch.int32)
    if width == 4:
        return (ret << 16) | eps
    return torch.stack((eps, ret), 1)


def unpack_episodes(g, width):
    """The gathered payload (the packed words as int32, or [world * B, 2]
    int32 pairs) -> (episodes, return sums) as int32 [world * B]."""
    import torch
    if width == 2:
        h = g.view(torch.int16)
        return (h & 0xFF).to(torch.int32), (h >> 8).to(torch.int32)  # arithmetic shift: signed sums
    if width == 4:
        return g & 0xFFFF, g >> 16
    return g[:, 0], g[:, 1]


def _regrouped(batch):
    """Does the library regroup lanes by decision for a launch of `batch`
    lanes (the *_sorted step / rollout kernels)?  Mirrors
    coup::regroup_lanes (csrc/coup_regroup.h): COUP_REGROUP forces it,
    else batches of 2^18 lanes and more."""
    e = os.environ.get("COUP_REGROUP")
    if e is not None:
        return int(e) != 0
    return batch >= (1 << 18)


def _np_step_lanes(players):
    """Lanes per regrouping block of the N-player step kernel coup_step
    launches (coup_nplayer.hip step_sort_lanes; COUP_NP_SORT_THREADS A/B)."""
    e = os.environ.get("COUP_NP_SORT_THREADS")
    if e in ("256", "512", "1024"):
        return int(e)
    return 1024 if players >= 6 else 512


_SPLIT_WRITERS = {1: "coup::k_obs_sweep<1>", 2: "coup::k_obs_sweep<0>", 3: "coup::k_obs_sweep_rows<256, 1>",
                  4: "coup::k_obs_sweep_rows<256, 2>", 5: "coup::k_obs_sweep_rows<128, 1>",
                  6: "coup::k_obs_sweep_rows<64, 1>", 7: "coup::k_obs_sweep_rows<512, 1>",
                  9: "coup::k_obs_sweep_rows<256, 3>",
                  10: "coup::k_obs_sweep_rows<256, 4>", 11: "coup::k_obs_sweep_rows<512, 2>",
                  12: "coup::k_obs_sweep_rows<128, 4>", 13: "coup::k_obs_sweep_rows<128, 2>",
                  14: "coup::k_obs_sweep_rows<1024, 2>", 15: "coup::k_obs_sweep_rows<1024, 1>",
                  16: "coup::k_obs_sweep_rows<512, 3>", 17: "coup::k_obs_sweep_rows<512, 4>"}


def obs_split_active(batch):
    """The split observation step's writer variant coup_step uses for this
    batch (0: the fused step kernel; COUP_OBS_SPLIT overrides)."""
    from open_spiel_coup_amd import _native
    return int(_native.load().coup_obs_split_variant(int(batch)))


TRAJ_CHUNK_DEFAULT, TRAJ_CHUNK_MAX = 10, 32  # coup::kTrajChunkDefault, kTrajChunkMax


def step_many_form(batch, players, graph):
    """The form coup_step_many gives the timed steps (uniform steps recorded
    through it: the graph path) on a 2-player env whose split step uses the
    shipped writer (variant 11) -- "rules-trajectory" (COUP_PIPE=1, the
    default: chunks of COUP_TRAJ_CHUNK steps as one regrouped rules launch
    plus a writer launch per step; needs the regrouped rules), "pipelined"
    (COUP_PIPE=2, measurement builds: rules(t + 1) beside writer(t) in one
    launch), "fused-trajectory" (COUP_PIPE=4: one launch for the K steps
    writing the observations itself) -- or None (per-step launches).  Mirrors coup_kernels.hip
    `many_form`."""
    if not (graph and players == 2 and obs_split_active(batch) == 11):
        return None
    v = os.environ.get("COUP_PIPE", "1").strip()
    if v == "0":
        return None
    if v == "2":
        from open_spiel_coup_amd import _native
        if _native.load().coup_build_flags() & _native.BUILD_AB_VARIANTS:
            return "pipelined"
    if not _regrouped(batch):
        return None
    return "fused-trajectory" if v == "4" else "rules-trajectory"


def traj_stage():
    """The library's rules-trajectory output staging (coup_build_flags bits
    3:1; the STAGE template argument the launch log spells)."""
    from open_spiel_coup_amd import _native
    return (_native.load().coup_build_flags() >> _native.BUILD_TRAJ_STAGE_SHIFT) & _native.BUILD_TRAJ_STAGE_MASK


def traj_chunk():
    """COUP_TRAJ_CHUNK as coup::read_knobs clamps it."""
    try:
        c = int(os.environ.get("COUP_TRAJ_CHUNK", TRAJ_CHUNK_DEFAULT))
    except ValueError:
        c = TRAJ_CHUNK_DEFAULT
    return c if 1 <= c <= TRAJ_CHUNK_MAX else TRAJ_CHUNK_DEFAULT


_INFO_WRITERS = {1: "coup::k_info_sweep<512, 2>", 2: "coup::k_info_sweep<256, 2>", 3: "coup::k_info_sweep<1024, 2>",
                 4: "coup::k_info_sweep<512, 4>", 5: "coup::k_info_sweep<256, 4>"}


def info_split_active(batch):
    """The split InformationStateTensor step's writer variant (0: fused)."""
    from open_spiel_coup_amd import _native
    return int(_native.load().coup_info_split_variant(int(batch)))


def _writer(mode_env):
    """(ObsMode template value, block size) of the step kernel that
    coup_step launches for COUP_OBS_MODE (default 9; csrc/coup_kernels.hip)."""
    m = int(mode_env) if mode_env and mode_env.isdigit() and 1 <= int(mode_env) <= 9 else 9
    return {1: (1, 256), 2: (2, 256), 3: (3, 256), 4: (4, 256), 5: (5, 256), 6: (5, 1024), 7: (7, 1024),
            8: (8, 256), 9: (9, 256)}[m]


def expected_kernel(cfg, batch, graph):
    """The kernels the timed steps of config `cfg` at `batch` lanes launch
    (graph: recorded through capture_steps), spelled as the library's launch
    log spells them (coup_launch_log; rocprofv3 writes defaulted template
    arguments out): the mirror of coup_kernels.hip / coup_nplayer.hip's
    dispatch that the bench line's roofline.kernel reports.  The bench-size
    parity tests (tests/test_gpu_every_lane.py) assert that the library's log
    of their own calls equals it."""
    B = batch
    _, with_obs, with_info, fused, _, _, players = CONFIGS[cfg]
    bare = bare_many_active(with_obs, with_info, fused)
    sorted_ = _regrouped(B)
    if players != 2:
        ahead = os.environ.get("COUP_AHEAD", "1") != "0"
        if fused == "traj" or bare:
            return ("coup::np::k_trajectory_sorted<%d, 1024>" % players if sorted_ else
                    "coup::np::k_step_trajectory<%d>" % players)
        if fused:
            return ("coup::np::k_rollout_sorted<%d, 1024>" % players if sorted_ else "coup::np::k_rollout<%d>" % players)
        if sorted_:
            return "coup::np::k_step_sorted<%d, true, %s, %d>" % (players, "true" if ahead else "false",
                                                                 _np_step_lanes(players))
        return "coup::np::k_step<%d, true>" % players
    if fused == "traj" or bare:
        return ("coup::k_trajectory_sorted<1024, false, false, 8, %d>" % traj_stage() if sorted_ else
                "coup::k_step_trajectory")
    if fused:
        return "coup::k_rollout_sorted<1024>" if sorted_ else "coup::k_rollout"
    if with_info:
        isplit = info_split_active(B)
        return ("coup::k_step<true, 0, 256, 1, false> + " + _INFO_WRITERS.get(isplit, "coup::k_info_sweep")
                if isplit else "coup::k_step<true, 0, 256, 2, false>")
    if with_obs:
        split = obs_split_active(B)
        form = step_many_form(B, players, graph)
        if form == "pipelined":
            # one launch per step: the rules of step t + 1 beside the writer of step t
            return "coup::k_step_obs_pipe<512, 2>"
        if form:
            # one rules-trajectory launch per chunk of steps + the writer per step
            stage = os.environ.get("COUP_MANY_STAGE", "0").strip() not in ("0", "")
            return ("coup::k_trajectory_sorted<1024, false, true, 4, 0>" if form == "fused-trajectory" else
                    ("coup::k_trajectory_sorted<1024, true, false, 8, 1> + " if stage else
                     "coup::k_trajectory_sorted<1024, true, false, 8, %d, true> + " % traj_stage()) +
                    _SPLIT_WRITERS.get(split, "coup::k_obs_sweep"))
        if split:
            # the rules step without tensors (regrouped from 2^18 lanes) + the writer
            return "coup::k_step_sorted<true, 512> + " + _SPLIT_WRITERS.get(split, "coup::k_obs_sweep")
        return "coup::k_step<true, %d, %d, 0, false>" % _writer(os.environ.get("COUP_OBS_MODE"))
    tpl = os.environ.get("COUP_STEP_TPL", "1")
    if sorted_:
        return "coup::k_step_sorted<true, 512>"
    return "coup::k_step_group<%s, true>" % tpl if tpl in ("1", "2", "4") else "coup::k_step<true, 0, 256, 0, false>"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one process per GPU); default WORLD_SIZE, or 1.  Without torchrun, N > 1 starts the "
                         "N rank processes here")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--settle", type=int, default=256,
                    help="untimed env steps run first through the fused rollout (same trajectories as "
                         "coup_step), so the timed steps see the steady-state mix of game phases rather "
                         "than 2^20 lanes that all started together (not for info-state configs)")
    ap.add_argument("--power-warm-ms", type=float, default=40.0,
                    help="after the warm-up, untimed repeats of the timed K steps (the same graph replay, "
                         "fused launch or eager steps) until about this much GPU time has passed: the GPU "
                         "leaves its idle power state only under sustained load (tools/dpm_probe.py: the "
                         "c3 graph 151 us per step after idle gaps, 135.7 under sustained load; DESIGN.md "
                         "section 5); 0 turns it off")
    ap.add_argument("--gate-steps", type=int, default=-1,
                    help="untimed rollout steps enqueued right before the timed region (the gate; -1: "
                         "calibrated to the host's launch latency, 0: none -- tests comparing games across runs)")
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target duration of the bounded CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                    help="collectives of a multi-process run: nccl (RCCL over xGMI, one GPU per rank) or gloo "
                         "(a rehearsal of the multi-GPU path with several ranks sharing a GPU)")
    ap.add_argument("--force-collective", action="store_true",
                    help="run the collectives (all-gather, barrier, max over ranks) even at one rank, over a "
                         "one-rank communicator of --dist-backend (MASTER_ADDR / MASTER_PORT must be set)")
    ap.add_argument("--dump-episodes", default=None,
                    help="rank 0 saves the gathered per-lane episode counts and return sums (.npz; tests)")
    ap.add_argument("--graph", choices=("auto", "on", "off"), default="auto",
                    help="replay the K timed steps from one HIP graph (auto: on for c2, c3 and c4, "
                         "where it removes the per-step launch gaps)")
    return ap.parse_args()


def _cpu_threads():
    """Host threads for the all-cores sample: the job's CPU share (the GPU
    box exports OMP_NUM_THREADS = its share), at most the affinity set."""
    avail = len(os.sched_getaffinity(0))
    want = int(os.environ.get("OMP_NUM_THREADS", avail) or avail)
    return max(1, min(avail, want))


def _oracle_sample(players, with_obs, with_info, n, steps, env_id_base=0):
    from oracle import oracle
    if players != 2:
        oracle.np_rollout(players, seed=7, n=n, steps=steps, env_id_base=env_id_base)
    else:
        oracle.rollout(seed=7, n=n, steps=steps, env_id_base=env_id_base, want_obs=with_obs, obs_overwrite=True,
                       want_trajectory=False, want_info=with_info)


def cpu_baseline(target_s, with_obs, with_info, players=2):
    """Bounded sample of the same per-lane workload on the C oracle: one core
    (the reference's single-threaded path), then the same sample split over
    all of the job's host cores (ctypes releases the GIL, so Python threads
    run the C rollouts in parallel, one lane range per thread)."""
    import threading
    n = 1024 if players != 2 else (4096 if not with_info else 256)
    _oracle_sample(players, with_obs, with_info, n, 2)  # load / build the oracle
    steps, dt = 4, 0.0
    while dt < target_s / 16 and not (with_info and steps >= 64):
        steps *= 2
        t0 = time.perf_counter()
        _oracle_sample(players, with_obs, with_info, n, steps)
        dt = time.perf_counter() - t0
    steps = max(steps, int(steps * target_s / max(dt, 1e-9)))
    if with_info:
        steps = min(steps, 64)  # the oracle keeps every step's tensors
    t0 = time.perf_counter()
    _oracle_sample(players, with_obs, with_info, n, steps)
    dt = time.perf_counter() - t0
    what = " with ObservationTensor x2 written per step" if with_obs else ""
    what += " with InformationStateTensor x2 written per step" if with_info else ""
    src = "oracle/coup_nplayer.c" if players != 2 else "oracle/coup_oracle.c"
    out = {"value": n * steps / dt, "unit": "env-steps/s", "cores": 1, "kind": "port",
           "sample": f"{n} lanes x {steps} uniform-random {players}-player steps{what}, {dt:.1f} s, {src} -O2"}
    if players == 2:
        # the port runs the rules on the packed record; the reference C++ is slower
        # (it cannot be built here: coup.cc needs abseil)
        out["note"] = ("bit-exact scalar C port of the reference rules on the packed 16-B record; SURVEY.md section 6 "
                       "timed the reference C++ at 3.43e6 (bare) / 0.89e6 (obs x2) env-steps/s on 1 core of the "
                       "survey host, so this baseline overstates the reference's CPU speed by roughly 5-14x")
    k = _cpu_threads()
    if k > 1:
        # same total work per thread as the 1-core sample, k lane ranges
        th = [threading.Thread(target=_oracle_sample, args=(players, with_obs, with_info, n, steps, i * n))
              for i in range(k)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        dk = time.perf_counter() - t0
        out["all_cores"] = {"value": k * n * steps / dk, "cores": k,
                            "sample": f"{k} threads x ({n} lanes x {steps} steps), {dk:.1f} s"}
    return out


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _box_identity(dev):
    """Which GPU box ran this line (tools/boxinfo.sh fields, best effort).
    Read from sysfs, with no child process: a process that has initialised
    the GPU must not exec another program (rocm-smi is one)."""
    import glob
    import socket
    import torch
    p = torch.cuda.get_device_properties(dev)
    box = {"host": socket.gethostname(), "gpu": p.name, "arch": getattr(p, "gcnArchName", None),
           "cus": p.multi_processor_count, "uuid": str(getattr(p, "uuid", "")) or None}
    bus = getattr(p, "pci_bus_id", None)
    dom = getattr(p, "pci_domain_id", 0) or 0
    devno = getattr(p, "pci_device_id", 0) or 0
    cands = glob.glob("/sys/bus/pci/devices/%04x:%02x:%02x.*" % (dom, bus, devno)) if bus is not None else []
    if not cands:
        return box
    d = cands[0]
    box["pci"] = os.path.basename(d)
    for key, fname in (("serial", "serial_number"), ("compute_partition", "current_compute_partition"),
                       ("mem_partition", "current_memory_partition")):
        v = _read(os.path.join(d, fname))
        if v:
            box[key] = v
    for key, fname in (("sclk", "pp_dpm_sclk"), ("mclk", "pp_dpm_mclk"), ("fclk", "pp_dpm_fclk")):
        v = _read(os.path.join(d, fname))
        if v:
            cur = [ln for ln in v.splitlines() if ln.rstrip().endswith("*")]
            box[key] = (cur[0] if cur else v.splitlines()[0]).rstrip(" *")
    return box


def _time_traffic_ceiling(env, steps, stream):
    """Average duration of coup_measure_step_traffic over the env's own
    buffers (K launches replayed from one HIP graph, like the step)."""
    import ctypes
    import torch
    from open_spiel_coup_amd import _native
    rec = env.export_state()
    out = _native.StepOutputs(*[t.data_ptr() if t is not None else None for t in
                                (env.actions, env.rewards, env.step_type, env.legal_mask, env.cur_player,
                                 env.obs)])

    def launch(s):
        _native.check(env.lib.coup_measure_step_traffic(env.batch, ctypes.c_void_p(rec.data_ptr()),
                                                         ctypes.byref(out), ctypes.c_void_p(s)))

    for _ in range(3):
        launch(stream.cuda_stream)
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream(env.device)
    side.wait_stream(stream)
    with torch.cuda.graph(g, stream=side):
        for _ in range(steps):
            launch(side.cuda_stream)
    stream.wait_stream(side)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    g.replay()
    b.record(stream)
    b.synchronize()
    return a.elapsed_time(b) / steps


def _time_sweep_ceiling(buf, nf4, threads, passes, steps, stream):
    """Average duration of coup_measure_store_sweep -- the split writers'
    address-order store grid with no decode -- over the tensor buffer `buf`
    (nf4 float4), K launches replayed from one HIP graph like the steps."""
    import ctypes
    import torch
    from open_spiel_coup_amd import _native
    lib = _native.load()

    def launch(s):
        _native.check(lib.coup_measure_store_sweep(ctypes.c_void_p(buf.data_ptr()), int(nf4), threads, passes, 0,
                                                   ctypes.c_void_p(s)))

    for _ in range(3):
        launch(stream.cuda_stream)
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream(buf.device)
    side.wait_stream(stream)
    with torch.cuda.graph(g, stream=side):
        for _ in range(steps):
            launch(side.cuda_stream)
    stream.wait_stream(side)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    g.replay()
    b.record(stream)
    b.synchronize()
    return a.elapsed_time(b) / steps


VALU_CLOCK_GHZ = 2.4  # MI355X peak gfx clock (MI355X_MICROARCH.md)
SIMDS = 1024          # 256 CUs x 4 SIMDs


def valu_issue_frac(valu_insts, launch_ms, box=None):
    """Share of the chip's VALU issue slots a launch used: VALU instructions
    (summed over its waves; one wave64 VALU instruction takes 4 SIMD cycles)
    x 4 / (1024 SIMDs x 2.4 GHz x the launch's time).  The peak gfx clock,
    not the box's: sysfs shows the clock at the moment it is read (2252 MHz
    after a run that sustained ~2370, call r06a), so the peak figure gives
    the conservative (lower) fraction.  None without a profile of the same
    form."""
    if not valu_insts or not launch_ms:
        return None
    return valu_insts * 4.0 / (SIMDS * VALU_CLOCK_GHZ * 1e9 * launch_ms * 1e-3)


def roofline_fields(kernel, launched, achieved, traffic, valu_insts, launch_ms, bytes_per_launch, box, sweep_ms,
                    sweep_form, step_form, tensors=False):
    """The line's roofline object.  frac: algorithmic bytes / time against the
    HBM spec peak (the contract's roofline); valu_issue_frac: the VALU issue
    slots used (valu_issue_frac()).  bound: for the tensor-free forms
    (tensors False) whichever fraction is higher (the
    trajectory forms keep their state in registers and move far fewer bytes
    than their algorithmic count, so their HBM fraction bounds nothing); for
    the tensor-writing steps "hbm": their writers issue VALU on ~90% of the
    slots, but cutting the writer's VALU per float4 in half made the c3 step
    SLOWER (the nibble + table writer, 154.3 against 136.5 us, call r06d;
    DESIGN.md section 5), so VALU issue does not bound them.
    store_sweep_ms is a measurement, not a bound, and no field is called a
    ceiling."""
    hbm_frac = achieved / HBM_PEAK_GBS
    valu_frac = valu_issue_frac(valu_insts, launch_ms, box)
    valu_bound = not tensors and valu_frac is not None and valu_frac > hbm_frac
    return {"bound": "valu" if valu_bound else "hbm",
            "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": hbm_frac, "traffic": traffic,
            "kernel": kernel, "kernel_launched": launched, "kernel_ms": launch_ms,
            "bytes_per_launch": bytes_per_launch,
            "valu_issue_frac": valu_frac, "valu_insts_per_launch": valu_insts,
            "store_sweep_ms": sweep_ms, "sweep_over_kernel": (sweep_ms / launch_ms) if sweep_ms else None,
            "store_sweep_form": sweep_form,
            "store_sweep_note": "a store-only sweep timed beside the step, not a bound" if sweep_ms else None,
            "step_form": step_form}


def _calibrate_gate(env, stream, launch=None, factor=3.0):
    """Steps of an untimed rollout (the gate) that keep the GPU busy for
    `factor` times the host's enqueue latency of the timed launch (event record
    + `launch`: one fused rollout by default, or a HIP graph's replay), so the
    timed launch's start event fires with it already queued behind it and the
    GPU never idles between them.  Each step's duration is measured behind
    such a gate too."""
    import math
    import time
    import torch
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    one = launch or env.rollout_launcher(1)
    lat = []
    for _ in range(7):
        torch.cuda.synchronize()
        t = time.perf_counter()
        a.record(stream)
        one()
        lat.append(time.perf_counter() - t)
    torch.cuda.synchronize()
    probe = 64
    env.rollout(probe)  # busy while the measured launch is enqueued
    a.record(stream)
    env.rollout(probe)
    b.record(stream)
    b.synchronize()
    step_s = a.elapsed_time(b) * 1e-3 / probe
    # 3x the median by default: a launch right after a barrier is slower than
    # a warm one
    return max(1, math.ceil(factor * sorted(lat)[len(lat) // 2] / max(step_s, 1e-9)))


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def visible_gpus(sysfs="/sys/class/kfd/kfd/topology/nodes", env=None):
    """GPUs this process may use, counted without touching the GPU or
    importing torch (torch.cuda.device_count() falls back
    to hipGetDeviceCount, which initialises HIP, when amdsmi fails): the KFD
    topology nodes with a non-zero simd_count (CPU nodes have none),
    narrowed by ROCR_VISIBLE_DEVICES, then HIP_VISIBLE_DEVICES /
    CUDA_VISIBLE_DEVICES (comma-separated lists; an empty list hides every
    GPU; entries past the physical count are dropped, as the runtime does)."""
    import glob
    env = os.environ if env is None else env
    n = 0
    for prop in glob.glob(os.path.join(sysfs, "*", "properties")):
        try:
            with open(prop) as f:
                for ln in f:
                    k, _, v = ln.partition(" ")
                    if k == "simd_count" and int(v) > 0:
                        n += 1
                        break
        except (OSError, ValueError):
            continue
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is None:
            continue
        ids = [x for x in v.split(",") if x.strip()]
        n = min(n, len(ids))
        if var != "ROCR_VISIBLE_DEVICES":
            break  # HIP_VISIBLE_DEVICES, if set, wins over CUDA_VISIBLE_DEVICES
    return n


def launch_ranks(n, argv, backend="nccl", script=None):
    """--gpus N > 1 without torchrun: start N rank processes of `script`
    (this file) with `argv` and the torchrun environment (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR / MASTER_PORT on 127.0.0.1), one GPU each.  This
    process never initialises the GPU -- it counts GPUs from the KFD
    topology (visible_gpus) and does not import torch -- and execs nothing:
    the ranks are child processes.  Relays rank 0's JSON line; returns
    non-zero if any rank fails (the others are then stopped) or rank 0
    prints no line."""
    script = script or os.path.abspath(__file__)
    if backend == "nccl":
        vis = visible_gpus()
        if n > vis:
            print(f"bench.py: --gpus {n} with nccl needs {n} visible GPUs, found {vis}", file=sys.stderr)
            return 2
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr, text=True))
    lines = []
    reader = threading.Thread(target=lambda: lines.extend(procs[0].stdout), daemon=True)
    reader.start()
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 1
                print(f"bench.py: rank {procs.index(p)} exited with {c}; stopping the other ranks", file=sys.stderr)
                for q in live:
                    q.terminate()
                deadline = time.time() + 30
                for q in live:
                    try:
                        q.wait(max(0.1, deadline - time.time()))
                    except subprocess.TimeoutExpired:
                        q.kill()
                        q.wait()
                live = []
        time.sleep(0.05)
    reader.join(timeout=30)
    for ln in lines:
        if not ln.lstrip().startswith("{"):
            sys.stderr.write(ln)
    out = [ln for ln in lines if ln.lstrip().startswith("{")]
    if rc == 0 and not out:
        print("bench.py: rank 0 printed no line", file=sys.stderr)
        rc = 1
    if rc == 0:
        print(out[-1].rstrip("\n"), flush=True)
    return rc


def main():
    args = parse()
    if "WORLD_SIZE" in os.environ:
        ws = int(os.environ["WORLD_SIZE"])
        if args.gpus is not None and args.gpus != ws:
            print(f"bench.py: --gpus {args.gpus} disagrees with WORLD_SIZE={ws}", file=sys.stderr)
            sys.exit(2)
    elif args.gpus is not None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], args.dist_backend))
    elif args.gpus is not None and args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        sys.exit(2)
    import torch
    import torch.distributed as dist

    from open_spiel_coup_amd import BatchedCoupEnv
    from open_spiel_coup_amd import _native
    from open_spiel_coup_amd import distributed as D

    rank, world, _ = D.world_info()
    force = args.force_collective
    dev = D.init(args.dist_backend, gpu=True, force=force)  # RCCL over xGMI when world > 1
    grouped = world > 1 or force

    cfg = args.config
    B0, with_obs, with_info, fused, bytes_per_lane, workload, players = CONFIGS[cfg]
    B = args.batch or B0
    width = payload_width(players, args.steps, B)
    # per-lane finished-episode counts and player-0 return sums of the timed
    # steps, accumulated by the kernels in the collective's own format: one
    # packed word per lane (int16 return << 8 | episodes at the driver's K;
    # coup_step_outputs.episode_word, coup_rollout_stats for the fused rollout)
    env = BatchedCoupEnv(B, seed=args.seed, env_id_base=D.env_id_base(rank, B), auto_reset=True, obs=with_obs,
                         info_state=with_info, device=dev, num_players=players,
                         episode_stats=episode_stats_mode(width) if fused != "rollout" else False)
    stats = None
    if fused == "rollout":
        stats = env.new_stats(width) if width in (2, 4) else env.new_stats()

    def barrier():
        if grouped:
            dist.barrier()
        torch.cuda.synchronize()

    stream = torch.cuda.current_stream(dev)

    def make_gate(calibrate):
        n = calibrate() if args.gate_steps < 0 else args.gate_steps
        if n <= 0:
            g = lambda: None  # noqa: E731
            g.steps = 0
            return g
        return env.rollout_launcher(n)

    if args.settle > 0 and not with_info:
        env.rollout(args.settle)
    graph = None
    timed = None
    launched = None  # the library's launch log of the timed steps (coup_launch_log)
    if not fused and (args.graph == "on" or (args.graph == "auto" and cfg in GRAPH_AUTO)):
        for _ in range(args.warmup):
            env.step()
        # the warm-up's episodes out of the packed word before the capture
        # reserves the timed steps' room in it (warm-up + K > 63
        # folded an int16 word and the collate below refused it)
        env.clear_episode_stats()
        # uniform steps are recorded through coup_step_many: from 2^20 lanes
        # with observations its rules-trajectory split step
        _native.launch_log()  # clear: the log of the capture is the timed region's kernels
        graph = env.capture_steps(args.steps)
        launched = _native.launch_log()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))]
        # no gate ahead of a graph replay: its host submission takes a few
        # us, and a gate's remainder would count in the wall time (c2's
        # value 1.4e10 without, 0.9e10 with a 1.5x gate, calls r05q / r05t)
        gate = make_gate(lambda: 0)
    elif fused:
        env.rollout(args.warmup)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))]
        gate = make_gate(lambda: _calibrate_gate(env, stream))
        if fused == "traj":
            timed = env.step_trajectory_launcher(args.steps, env.trajectory_buffers(args.steps))
        else:
            timed = env.rollout_launcher(args.steps, stats)
    else:
        for _ in range(args.warmup):
            env.step()
        env.clear_episode_stats()  # as above: the warm-up never folds the timed steps' word
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))]
        if bare_many_active(with_obs, with_info, fused):
            # the K steps as one coup_step_many call (one trajectory launch)
            timed = lambda: env.step_many(args.steps)  # noqa: E731
            gate = make_gate(lambda: _calibrate_gate(env, stream, timed, factor=1.5))
            env.clear_episode_stats()  # the calibration's steps out of the packed word
        elif with_info:  # no rollout on a history env; a c3i step is ~1 ms, its launch latency noise
            gate = lambda: None  # noqa: E731
            gate.steps = 0
        else:
            gate = make_gate(lambda: _calibrate_gate(env, stream))
    def episode_payload():
        # the accumulators themselves (no kernel runs to build the payload)
        if stats is None:
            return env.episode_payload()
        if "episode_word" in stats:
            return stats["episode_word"].view(torch.int32) if width == 2 else stats["episode_word"]
        return torch.stack((stats["episodes"], stats["return_sum"]), 1)

    def unpack_payload(g):
        return unpack_episodes(g, width)

    # one collation outside the timed region: RCCL sets up its all-gather
    # channels lazily, and HIP loads torch's stack kernel on first use
    D.collate(episode_payload(), force=force)

    def unit():  # the timed region's K steps, untimed
        if graph is not None:
            graph.replay()
        elif timed is not None:
            timed()
        else:
            for _ in range(args.steps):
                env.step()

    # power warm-up: sustained load right before the timed region, so it
    # starts in the power state it runs in (the accumulators are cleared
    # below; the env advances, as in the warm-up)
    power_warm_steps, power_warm_ms = 0, 0.0
    if args.power_warm_ms > 0:
        tw = time.perf_counter()
        if graph is None:
            _native.launch_log()  # clear; the first repeat's launches are the timed region's
        unit()
        if graph is None:
            launched = _native.launch_log()
        torch.cuda.synchronize()
        one_ms = (time.perf_counter() - tw) * 1e3
        reps = min(int(args.power_warm_ms / max(one_ms, 1e-3)), 1000)
        for _ in range(reps):
            unit()
        torch.cuda.synchronize()
        power_warm_steps = (reps + 1) * args.steps
        power_warm_ms = (time.perf_counter() - tw) * 1e3
    if stats is not None:
        for t in stats.values():
            t.zero_()
    else:
        env.clear_episode_stats()
    barrier()
    # an untimed rollout ahead of the start event keeps the GPU busy while
    # the host enqueues the timed launch(es) or graph replay, so the event
    # pair brackets the kernels and not the host's launch latency and an idle
    # GPU's wake-up (~60 us: half of a 20-step c2r launch); enqueued before
    # t0, it overlaps that latency in the wall time too
    gate()
    t0 = time.perf_counter()
    if graph is not None:
        ev[0][0].record(stream)
        graph.replay()
        ev[0][1].record(stream)
    elif timed is not None:  # one fused launch, or coup_step_many's one trajectory launch
        ev[0][0].record(stream)
        timed()
        ev[0][1].record(stream)
    else:
        # K eager launches back to back: the span / K, like the graph replay
        ev[0][0].record(stream)
        for k in range(args.steps):
            env.step()
        ev[0][1].record(stream)
    # collate every lane's finished-episode count and player-0 return sum over
    # xGMI (RCCL all-gather, [world * B, 2] int32; identity at one rank)
    gathered = D.collate(episode_payload(), force=force)
    barrier()
    elapsed = time.perf_counter() - t0
    g_eps, g_ret = unpack_payload(gathered)
    ep_total = int(g_eps.sum())
    ret_total = int(g_ret.sum())
    if args.dump_episodes and rank == 0:
        import numpy as np
        np.savez(args.dump_episodes, episodes=g_eps.cpu().numpy(), return_sum=g_ret.cpu().numpy())

    # per env step: the span of the K steps (one replay, one fused launch or K
    # eager launches) / K, launch gaps included
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    elapsed = D.max_over_ranks(elapsed, dev, force=force)
    # the collective tail of the timed region (payload + all-gather + barrier)
    # and the max over ranks after it, timed again on their own with the GPU
    # idle: the share of a K-step window that does not scale with the lanes
    barrier()
    tc = time.perf_counter()
    D.collate(episode_payload(), force=force)
    barrier()
    D.max_over_ranks(0.0, dev, force=force)
    collective_ms = (time.perf_counter() - tc) * 1e3
    # every rank's tail (rank 0 prints them; one value at one rank)
    collective_ms_ranks = [float(x) for x in
                           D.collate(torch.tensor([collective_ms], dtype=torch.float64, device=dev), force=force)]
    errors = env.error_count()
    # the store ceiling of the step's writer, timed in this process on this
    # box: the split / pipelined steps' address-order writers against a
    # store-only sweep of their tensor buffer with the same grid; the fused
    # step against its own loads and stores with no rules
    ceiling_ms, ceiling_form = None, None  # the store-only sweep (not a bound, see the docstring)
    if players == 2 and not fused:
        if with_obs and obs_split_active(B):
            ceiling_ms = _time_sweep_ceiling(env.obs, B * 49, 512, 2, args.steps, stream)
            ceiling_form = "sweep: [B][2][98] fp32 stores in address order, 512 x 2 grid, no decode, tensor-like data"
        elif with_info and info_split_active(B):
            ceiling_ms = _time_sweep_ceiling(env.info_state, B * 1246, 1024, 2, args.steps, stream)
            ceiling_form = ("sweep: [B][2][2492] fp32 stores in address order, 1024 x 2 grid, no decode, "
                            "tensor-like data")
        elif not with_info and not bare_many_active(with_obs, with_info, fused):
            ceiling_ms = _time_traffic_ceiling(env, args.steps, stream)
            ceiling_form = "fused: the fused step's loads and stores, no rules"

    if rank == 0:
        bare = bare_many_active(with_obs, with_info, fused)
        per_launch = args.steps if (fused or bare) else 1  # env steps per launch of the timed kernel
        bytes_per_launch = bytes_per_lane * B * per_launch
        launch_ms = kern_ms * per_launch
        achieved = bytes_per_launch / (launch_ms * 1e-3) / 1e9
        traffic, valu_insts = None, None
        if os.path.exists(TRAFFIC_FILE):
            with open(TRAFFIC_FILE) as f:
                tr = json.load(f)
            ent = tr.get(cfg)
            # the profile of the same form: batch and env steps per launch
            if ent and ent.get("batch") == B and ent.get("steps_per_launch", 1) == per_launch:
                traffic = ent.get("hbm_bytes_per_launch")
                valu_insts = ent.get("valu_insts_per_launch")
        box = _box_identity(dev)
        kernel = expected_kernel(cfg, B, graph is not None)
        if launched is not None and launched != kernel:
            print(f"bench.py: the library launched {launched!r}, not the expected {kernel!r}", file=sys.stderr)
        outputs = ("ObservationTensor fp32 [B][2][98] per step" if with_obs else
                   "InformationStateTensor fp32 [B][2][2492] per step" if with_info else
                   "per-episode statistics only" if fused == "rollout" else
                   "actions, rewards, step types, legal masks, players: [K][B] trajectory buffers" if fused else
                   "actions, rewards, step types, legal masks, players per step, as ONE coup_step_many trajectory "
                   "launch for the K steps (state in registers, each step's outputs over the [B] buffers; not "
                   "comparable with per-step launches: COUP_PIPE=0)" if bare_many_active(with_obs, with_info, fused)
                   else "actions, rewards, step types, legal masks, players per step")
        line = {
            "metric": "Coup env-steps/sec at batch 2^20, 1/2/4/8 MI355X; HBM GB/s vs peak",
            "value": world * B * args.steps / elapsed,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_steps": args.settle if not with_info else 0,
            "power_warm": {"steps": power_warm_steps, "ms": power_warm_ms},
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (uniform-random self-play games)",
            "config": {"workload": workload, "batch_per_gpu": B, "global_batch": world * B, "players": players,
                       "outputs": outputs, "auto_reset": True, "fused_steps_per_launch": per_launch,
                       "hip_graph": graph is not None,
                       "gate_steps": gate.steps,
                       "parallelism": f"dp{world} (env-id sharding)" + ("" if args.dist_backend == "nccl" else
                                                                   " [gloo rehearsal, ranks share GPUs]")},
            "roofline": roofline_fields(
                kernel=kernel, launched=launched, achieved=achieved, traffic=traffic, valu_insts=valu_insts,
                launch_ms=launch_ms, bytes_per_launch=bytes_per_launch, box=box, sweep_ms=ceiling_ms,
                sweep_form=ceiling_form, tensors=bool(with_obs or with_info),
                step_form=("trajectory (coup_step_many)" if bare else
                           (with_obs and step_many_form(B, players, graph is not None))
                           or "split" if (with_obs and players == 2 and obs_split_active(B)) or
                           (with_info and info_split_active(B)) else "fused")),
            "episodes": {"finished": ep_total, "mean_return_p0": ret_total / max(ep_total, 1),
                         "collective": ("all_gather [world*B] int16 (return sum << 8 | episodes per lane)"
                                        if width == 2 else
                                        "all_gather [world*B] int32 (return sum << 16 | episodes per lane)"
                                        if width == 4 else
                                        "all_gather [world*B, 2] int32 (episodes, return sum per lane)")
                         if grouped else None,
                         "collective_ms": collective_ms,
                         "collective_ms_ranks": collective_ms_ranks,
                         "collective_backend": (args.dist_backend + (" (one-rank communicator)" if world == 1 else ""))
                         if grouped else None},
            "lane_errors": errors,
            "box": box,
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.cpu_seconds, with_obs, with_info, players)
        print(json.dumps(line), flush=True)
    if grouped:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
