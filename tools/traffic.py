"""Condense rocprofv3 output (tools/profile_gpu.sh) into committed evidence.

    python tools/traffic.py gpurun_out/prof/<tag>/<config> --config <config> [bench.py args]

Writes profiles/<tag>/<config>/kernel_stats.csv (the --stats summary as
produced), profiles/<tag>/<config>/summary.json, and the config's entry of
profiles/traffic.json, which bench.py reads for roofline.traffic.

HBM bytes per launch follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced streaming read (16 B/lane), so it is doubled; WRITE_SIZE is exact
for 16-B-per-lane streaming stores.
"""
import csv
import glob
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(pattern):
    out = []
    for path in sorted(glob.glob(pattern, recursive=True)):
        with open(path, newline="") as f:
            out.extend(csv.DictReader(f))
    return out


def col(row, *needles):
    for k in row:
        lk = k.lower()
        if all(n in lk for n in needles):
            return k
    raise KeyError(needles)


def main():
    src = sys.argv[1]
    args = sys.argv[2:]
    tag = os.path.basename(os.path.dirname(os.path.normpath(src)))
    cfg = "c3"
    batch = None
    steps = 20
    for i, a in enumerate(args):
        if a == "--config":
            cfg = args[i + 1]
        if a == "--batch":
            batch = int(args[i + 1])
        if a == "--steps":
            steps = int(args[i + 1])
    sys.path.insert(0, ROOT)
    from bench import CONFIGS
    batch = batch or CONFIGS[cfg][0]
    want_obs, want_info, fused, players = CONFIGS[cfg][1], CONFIGS[cfg][2], CONFIGS[cfg][3], CONFIGS[cfg][6]
    from bench import info_split_active, obs_split_active, step_many_form, traj_chunk
    split = obs_split_active(batch)
    isplit = info_split_active(batch)
    graph_on = "--graph" not in args or "off" not in args
    many = (step_many_form(batch, players, graph_on)
            if want_obs and not want_info and not fused and players == 2 else None)
    from bench import bare_many_active
    # coup_step_many's tensor-free form: ONE trajectory launch per K steps,
    # profiled like the fused trajectory configs (the timed launch is the last)
    bare = bool(bare_many_active(want_obs, want_info, fused))
    # coup_step_many recorded in the bench's graph.  The merged pipelined
    # step: K + 1 dispatches of ONE kernel per K steps -- the rules of step 1
    # alone, K - 1 launches of rules(t + 1) beside writer(t), the writer of
    # step K alone.  The rules-trajectory step: ceil(K / chunk) rules
    # launches of up to `chunk` steps each and K writer launches.
    pipe = many == "pipelined"
    chunks = -(-steps // traj_chunk()) if many == "rules-trajectory" else 1 if many == "fused-trajectory" else None
    dispatches_per_window = (steps + 1 if pipe else 1 if many == "fused-trajectory" else steps + chunks if chunks
                             else None)

    dst = os.path.join(ROOT, "profiles", tag, cfg)
    os.makedirs(dst, exist_ok=True)
    summary = {"tag": tag, "config": cfg, "batch": batch}

    def timed_kernel(kn):
        """Is `kn` the kernel bench.py times for this config?"""
        if fused == "traj" or bare:
            if players != 2:
                return bool(re.search(r"np::k_(step_trajectory|trajectory_sorted)<%d(, \w+)*>|"
                                      r"2np(17k_step_trajectory|19k_trajectory_sorted)ILi%dE" % (players, players), kn))
            return (("k_step_trajectory" in kn or "k_trajectory_sorted" in kn or "19k_trajectory_sorted" in kn)
                    and "np::" not in kn and "2np" not in kn)
        if players != 2:
            if fused:
                return bool(re.search(r"np::k_rollout(_sorted)?<%d(, \w+)*>|2np(9k_rollout|16k_rollout_sorted)ILi%dE"
                                      % (players, players), kn))
            return bool(re.search(r"np::k_step(_sorted)?<%d, true(, \w+)*>|"
                                  r"2np(6k_step|13k_step_sorted)ILi%dELb1E" % (players, players), kn))
        if "np::" in kn or "2np" in kn:
            return False
        if fused:
            return "k_rollout" in kn
        if want_info and not want_obs and isplit:
            # the split InformationStateTensor step: the history-keeping
            # rules step and k_info_sweep
            m = re.search(r"k_step<true, 0, \d+, 1(?:, false)?>", kn) or re.search(r"k_stepILb1ELi0ELi\d+ELi1E", kn)
            return bool("k_info_sweep" in kn or m)
        if pipe:
            return "k_step_obs_pipe" in kn or "15k_step_obs_pipe" in kn
        if many == "fused-trajectory":
            return bool(re.search(r"k_trajectory_sorted<\d+, false, true", kn) or
                        re.search(r"19k_trajectory_sortedILi\d+ELb0ELb1E", kn))
        if chunks:
            return bool("k_obs_sweep" in kn or re.search(r"k_trajectory_sorted<\d+, true", kn) or
                        re.search(r"19k_trajectory_sortedILi\d+ELb1E", kn))
        if want_obs and not want_info and split:
            # the split observation step: the rules step without tensors and
            # the observation writer, two kernels per env step
            return bool("k_obs_sweep" in kn or "k_step_sorted<true" in kn or "13k_step_sortedILb1E" in kn)
        if not want_obs and not want_info and ("k_step_group<" in kn or "12k_step_group" in kn):
            return True  # the rules-bound step (COUP_STEP_TPL, default 1: k_step_group<1, true>)
        m = (re.search(r"k_step<true, (\d+), \d+, (\d+)(?:, false)?>", kn) or
             re.search(r"k_stepILb1ELi(\d+)ELi\d+ELi(\d+)E", kn))
        return bool(m) and (m.group(1) != "0") == want_obs and (m.group(2) == "2") == want_info

    def kernel_bytes_per_lane(kn, role=None):
        """Algorithmic bytes per lane of one dispatch of timed kernel kn
        (40 B of rules traffic per lane-step, 784 B of
        ObservationTensor, 19,936 B of InformationStateTensor plus 2 x 96 B
        of history for the history-keeping rules step)."""
        total = CONFIGS[cfg][4]
        if pipe:
            return {"rules": 40, "writer": total - 40}.get(role, total)
        if many == "fused-trajectory":
            return total * steps  # every step's rules and observations in one launch
        if chunks and "trajectory_sorted" in kn:
            return 40 * steps / chunks  # the rules of the chunk's steps (mean steps per launch)
        if want_obs and split:
            return total - 40 if "k_obs_sweep" in kn else 40
        if want_info and isplit:
            return 2 * 2492 * 4 if "k_info_sweep" in kn else total - 2 * 2492 * 4
        return total

    stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(dst, "kernel_stats.csv"))
        for r in rows(stats[0]):
            name = r[col(r, "name")]
            if timed_kernel(name):
                summary.setdefault("timed_kernels", []).append(name)
                summary["timed_kernel"] = " + ".join(summary["timed_kernels"])
            if "k_step" in name or "k_rollout" in name or "k_obs" in name or "k_info" in name:
                # rocprof's --stats over EVERY dispatch of the process (settle,
                # warm-up and the cold first call included): not the steady
                # state -- per_kernel below is
                summary.setdefault("kernels_all_dispatches", {})[name] = {
                    "calls": int(r[col(r, "calls")]),
                    "avg_ns_all_dispatches": float(r[col(r, "average")]),
                }

    # the bench line printed by the traced command itself (trace.log): its
    # live HIP-event kernel time must agree with the trace's average
    trace_log = os.path.join(src, "trace.log")
    if os.path.exists(trace_log):
        with open(trace_log) as f:
            for line in f:
                if line.startswith("{") and '"metric"' in line:
                    bench = json.loads(line)
                    summary["bench_line_of_traced_command"] = {
                        "value": bench["value"], "ms_per_step": bench["ms_per_step"],
                        "kernel_ms": bench["roofline"]["kernel_ms"], "frac": bench["roofline"]["frac"],
                        "store_sweep_ms": bench["roofline"].get("store_sweep_ms"),
                        "sweep_over_kernel": bench["roofline"].get("sweep_over_kernel"),
                        "box": bench.get("box")}
                    tk = summary.get("timed_kernel")
                    if fused or bare:
                        # a fused config launches the same kernel for the settle,
                        # warm-up and timed rollouts (different step counts): compare
                        # the timed launch, the last dispatch in the kernel trace
                        last = [r for r in rows(os.path.join(src, "trace", "**", "*kernel_trace.csv"))
                                if timed_kernel(r[col(r, "kernel", "name")])]
                        if last:
                            r = max(last, key=lambda r: int(r[col(r, "dispatch")]))
                            rp = (int(r[col(r, "end", "timestamp")]) - int(r[col(r, "start", "timestamp")])) * 1e-6
                            summary["bench_vs_rocprof_kernel_ms"] = [bench["roofline"]["kernel_ms"], rp]
                            summary["rocprof_compared_dispatch"] = "the timed (last) rollout launch"
                    elif summary.get("timed_kernels"):
                        # the timed window: the last `steps` env steps' dispatches
                        # of the timed kernel(s) (after the warm-up launches,
                        # which include the first, cold one)
                        tks = set(summary["timed_kernels"])
                        per_step = len(tks)
                        disp = sorted((r for r in rows(os.path.join(src, "trace", "**", "*kernel_trace.csv"))
                                       if r[col(r, "kernel", "name")] in tks),
                                      key=lambda r: int(r[col(r, "start", "timestamp")]))
                        window = disp[-(dispatches_per_window or steps * per_step):]
                        dur = lambda r: int(r[col(r, "end", "timestamp")]) - int(r[col(r, "start", "timestamp")])  # noqa: E731
                        if window:
                            mean = sum(dur(r) for r in window) / steps * 1e-6
                            # the bench times the span of the K steps' launches / K
                            # (launch gaps included: eager launches, or a graph
                            # replay); the trace's first start to last end of the
                            # same dispatches is that span, their summed durations
                            # per step the kernels alone
                            span = (int(window[-1][col(window[-1], "end", "timestamp")]) -
                                    int(window[0][col(window[0], "start", "timestamp")])) / steps * 1e-6
                            rp = span
                            summary["rocprof_kernel_time_per_step_ms"] = mean
                            summary["rocprof_launch_gap_ms"] = span - mean
                            summary["rocprof_compared_dispatch"] = (f"span of the last {len(window)} dispatches (the "
                                                                    f"{steps} timed steps) / {steps}, as the bench times "
                                                                    "them")
                            # every timed kernel's steady-state
                            # mean over the timed dispatches only, its own
                            # algorithmic bytes and roofline fraction, and a check
                            # that the means sum to the span
                            groups = {}
                            for j, r in enumerate(window):
                                kn = r[col(r, "kernel", "name")]
                                if pipe:
                                    role = ("rules" if j == 0 else "writer" if j == len(window) - 1 else
                                            "rules+writer")
                                    key = f"{kn} [{role}]"
                                else:
                                    role, key = None, kn
                                groups.setdefault(key, (kn, role, []))[2].append(dur(r))
                            per_kernel, step_sum = {}, 0.0
                            for key, (kn, role, ds) in groups.items():
                                m_ns = sum(ds) / len(ds)
                                b = kernel_bytes_per_lane(kn, role if role != "rules+writer" else None) * batch
                                per_kernel[key] = {"dispatches": len(ds), "mean_us": m_ns * 1e-3,
                                                   "min_us": min(ds) * 1e-3, "max_us": max(ds) * 1e-3,
                                                   "bytes": b, "achieved_gbs": b / m_ns,
                                                   "frac": b / m_ns / 8000.0}
                                step_sum += sum(ds)
                            summary["per_kernel"] = per_kernel
                            summary["per_kernel_sum_check"] = {
                                "sum_of_means_per_step_us": step_sum / steps * 1e-3, "span_per_step_us": span * 1e3,
                                "pct": 100.0 * (step_sum / steps * 1e-6 - span) / span,
                                "ok_within_2pct": abs(step_sum / steps * 1e-6 - span) <= 0.02 * span}
                        else:
                            rp = sum(summary["kernels_all_dispatches"][k]["avg_ns_all_dispatches"] for k in tks) * 1e-6
                        summary["bench_vs_rocprof_kernel_ms"] = [bench["roofline"]["kernel_ms"], rp]

    # plain bench lines of the same lease, before and after the profiler passes
    for which in ("before", "after"):
        path = os.path.join(src, f"bench_{which}.json")
        if os.path.exists(path):
            with open(path) as f:
                for line in f:
                    if line.startswith("{") and '"metric"' in line:
                        b = json.loads(line)
                        summary[f"bench_line_{which}"] = {
                            "value": b["value"], "kernel_ms": b["roofline"]["kernel_ms"],
                            "frac": b["roofline"]["frac"], "store_sweep_ms": b["roofline"].get("store_sweep_ms"),
                            "sweep_over_kernel": b["roofline"].get("sweep_over_kernel")}
                        shutil.copy(path, os.path.join(dst, f"bench_{which}.json"))
    if summary.get("bench_vs_rocprof_kernel_ms"):
        a, b = summary["bench_vs_rocprof_kernel_ms"]
        summary["rocprof_minus_bench_pct"] = 100.0 * (b - a) / a
    if os.path.exists(os.path.join(src, "box.txt")):
        shutil.copy(os.path.join(src, "box.txt"), os.path.join(dst, "box.txt"))

    def counter(kind, cname):
        vals = {}
        for r in rows(os.path.join(src, kind, "**", "*counter_collection.csv")):
            kn = r[col(r, "kernel", "name")]
            if not timed_kernel(kn):
                continue
            if r[col(r, "counter", "name")] != cname:
                continue
            vals.setdefault(kn, []).append((int(r[col(r, "dispatch")]), float(r[col(r, "counter", "value")])))
        if not vals:
            return None
        if fused or bare:  # the timed launch only (see above)
            return sum(max(v)[1] for v in vals.values())
        # per env step: the timed steps' dispatches (the last K per kernel, or
        # the pipeline's last K + 1), summed, / K
        allv = sorted(x for v in vals.values() for x in v)
        n = dispatches_per_window or steps * len(vals)
        return sum(x for _, x in allv[-n:]) / steps

    fetch_kb = counter("fetch", "FETCH_SIZE")
    write_kb = counter("write", "WRITE_SIZE")
    summary["fetch_size_kb_avg"] = fetch_kb
    summary["write_size_kb_avg"] = write_kb
    traffic = None
    if fetch_kb is not None and write_kb is not None:
        traffic = (2.0 * fetch_kb + write_kb) * 1024.0
    if traffic is None:
        sys.exit(f"no FETCH_SIZE / WRITE_SIZE records for the step kernel under {src}; nothing written")
    summary["hbm_bytes_per_launch"] = traffic
    summary["correction"] = "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE halving)"
    # issue mix of the timed kernel.  SQ counters count quad-cycles, summed
    # over all waves; GRBM_GUI_ACTIVE is summed over the 8 XCDs (per XCD it
    # equals the kernel duration x ~2.4 GHz, checked below).  VALU busy =
    # SIMD-cycles issuing VALU / SIMD-cycles available, 1024 SIMDs.
    sq = {c: counter("sq", c) for c in ("SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_ACTIVE_INST_ANY",
                                         "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU", "SQ_WAIT_ANY", "GRBM_GUI_ACTIVE")}
    if all(v is not None for v in sq.values()) and sq["SQ_WAVE_CYCLES"] and sq["GRBM_GUI_ACTIVE"]:
        summary["issue"] = {
            "counters": sq,
            "valu_busy_pct": 100.0 * sq["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / (sq["GRBM_GUI_ACTIVE"] / 8),
            "gui_active_per_xcd_us_at_2.4GHz": sq["GRBM_GUI_ACTIVE"] / 8 / 2400.0,
            "wave_active_inst_frac": sq["SQ_ACTIVE_INST_ANY"] / sq["SQ_WAVE_CYCLES"],
            "wave_wait_frac": sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"],
            "valu_insts_per_wave": sq["SQ_INSTS_VALU"] / max(sq["SQ_WAVES"], 1.0),
        }
    with open(os.path.join(dst, "summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    path = os.path.join(ROOT, "profiles", "traffic.json")
    table = {}
    if os.path.exists(path):
        with open(path) as f:
            table = json.load(f)
    table[cfg] = {"batch": batch, "hbm_bytes_per_launch": traffic, "source": f"profiles/{tag}/{cfg}/summary.json",
                  "steps_per_launch": steps if (fused or bare) else 1}
    if summary.get("issue"):
        # VALU instructions (summed over waves) per launch as bench.py counts
        # launches: bench.py's roofline.valu_issue_frac
        table[cfg]["valu_insts_per_launch"] = summary["issue"]["counters"]["SQ_INSTS_VALU"]
        table[cfg]["valu_source"] = f"profiles/{tag}/{cfg}/summary.json"
    with open(path, "w") as f:
        json.dump(table, f, indent=1, sort_keys=True)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
