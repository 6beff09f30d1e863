"""A stand-in rank for tests/test_bench_launcher.py: what bench.py's rank
processes do around the GPU work, on the CPU.  It reads the torchrun
environment that bench.launch_ranks sets, joins a gloo group, all-gathers
per-lane values of its env-id shard (lane i of rank r = global id r*B + i),
and rank 0 prints one JSON line.  `--fail-rank R` makes rank R exit with 3
before the collective (the others then block in it until stopped)."""
import argparse
import json
import os

import torch
import torch.distributed as dist

ap = argparse.ArgumentParser()
ap.add_argument("--gpus", type=int)
ap.add_argument("--batch", type=int, default=1000)
ap.add_argument("--fail-rank", type=int, default=-1)
args = ap.parse_args()
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
assert args.gpus == world and int(os.environ["LOCAL_RANK"]) == rank
assert os.environ["MASTER_ADDR"] == "127.0.0.1"
if rank == args.fail_rank:
    raise SystemExit(3)
dist.init_process_group("gloo")
ids = torch.arange(rank * args.batch, (rank + 1) * args.batch, dtype=torch.int64)
parts = [torch.empty_like(ids) for _ in range(world)]
dist.all_gather(parts, ids * 3 + 1)
g = torch.cat(parts)
if rank == 0:
    print("rank 0 log line on stdout, not JSON")
    print(json.dumps({"n_gpus": world, "lanes": int(g.numel()), "sum": int(g.sum())}), flush=True)
dist.destroy_process_group()
