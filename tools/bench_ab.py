"""Alternating-process A/B of library builds through bench.py itself: for each
round, one bench.py process per library (COUP_LIB_PATH), in turn, so the
box's drift cancels.  Prints one JSON line per run and a summary line per
library (median / min of ms_per_step and kernel_ms).  Measurement tool only.

    python tools/bench_ab.py --rounds 5 LIB1.so LIB2.so[:VAR=VAL,...] [...] -- --config c3 --steps 20 --warmup 5

A library may carry environment settings after a colon (knobs read at
coup_create, e.g. COUP_REGROUP=1), so one library can run in two forms.
"""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    argv = sys.argv[1:]
    rounds = 5
    if argv[:1] == ["--rounds"]:
        rounds, argv = int(argv[1]), argv[2:]
    libs, args = (argv[:argv.index("--")], argv[argv.index("--") + 1:]) if "--" in argv else (argv, [])
    res = {lib: [] for lib in libs}
    for r in range(rounds):
        for lib in libs:
            path, _, kvs = lib.partition(":")
            env = dict(os.environ, COUP_LIB_PATH=os.path.abspath(path))
            for kv in filter(None, kvs.split(",")):
                k, v = kv.split("=", 1)
                env[k] = v
            p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline"] + args, env=env,
                               capture_output=True, text=True, timeout=240)
            if p.returncode != 0:
                sys.stderr.write(p.stderr[-3000:])
                raise SystemExit(f"bench.py failed with {lib} (rc {p.returncode})")
            line = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
            res[lib].append(line)
            print(json.dumps({"round": r, "lib": lib, "ms_per_step": line["ms_per_step"],
                              "kernel_ms": line.get("roofline", {}).get("kernel_ms"),
                              "frac": line.get("roofline", {}).get("frac"), "value": line["value"]}), flush=True)
    for lib, lines in res.items():
        ms = [l["ms_per_step"] * 1e3 for l in lines]
        print(json.dumps({"lib": lib, "median_us": statistics.median(ms), "min_us": min(ms), "n": len(ms)}), flush=True)


if __name__ == "__main__":
    main()
