"""One-rank RCCL worker for tests/test_gpu_dist.py (run in a fresh process
with RANK=0, WORLD_SIZE=1, MASTER_ADDR/PORT set).

It initialises the process group with the nccl backend (RCCL) exactly as
bench.py does for a multi-GPU job -- init_process_group("nccl",
device_id=...) -- but forces the collectives that a single process would
skip: the all_gather_into_tensor of bench.py's per-lane episode payloads
(int16 pairs viewed as int32, int32, and [B, 2] int32), their unpacking,
a records gather and the max-over-ranks all_reduce.  The payloads are the
envs' own accumulators (packed words for widths 2 and 4, as bench.py's),
which must equal bench.pack_episodes of the int32 pair; every gathered
tensor must equal its source (a one-rank gather is a copy), and the
unpacked episodes / return sums must equal env.episode_stats().

    python tests/dist_nccl_worker.py OUT_JSON BATCH STEPS
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
from open_spiel_coup_amd import BatchedCoupEnv  # noqa: E402
from open_spiel_coup_amd import distributed as D  # noqa: E402


def main():
    out_path, B, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    rank, world, _ = D.world_info()
    assert world == 1 and rank == 0
    dev = D.init("nccl", gpu=True, force=True)
    assert dist.is_initialized() and dist.get_backend() == "nccl" and dist.get_world_size() == 1
    # the int32 pair, and the packed words the kernels accumulate for the
    # bench's payload widths 2 and 4 (twin envs, same games)
    envs = {w: BatchedCoupEnv(B, seed=5, env_id_base=D.env_id_base(rank, B), obs=False,
                              episode_stats=bench.episode_stats_mode(w), device=dev) for w in (2, 4, 8)}
    for e in envs.values():
        e.rollout(64)
        e.clear_episode_stats()
        for _ in range(K):
            e.step()
    env = envs[8]
    eps, ret = env.episode_stats()
    res = {"backend": dist.get_backend(), "world": dist.get_world_size(), "episodes": int(eps.sum()),
           "widths": {}}
    for width in (2, 4, 8):
        payload = envs[width].episode_payload()
        assert torch.equal(payload, bench.pack_episodes(eps, ret, width)), width
        g = D.collate(payload, force=True)
        assert g.data_ptr() != payload.data_ptr(), "the collective must not be short-circuited"
        assert torch.equal(g, payload), width
        e2, r2 = bench.unpack_episodes(g, width)
        assert torch.equal(e2, eps) and torch.equal(r2, ret), width
        # the bench's collective tail on its own: all-gather + barrier
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        reps = 20
        for _ in range(reps):
            D.collate(envs[width].episode_payload(), force=True)
        dist.barrier()
        torch.cuda.synchronize()
        res["widths"][str(width)] = {"payload_bytes": payload.numel() * payload.element_size(),
                                     "all_gather_ms": (time.perf_counter() - t0) * 1e3 / reps}
    rec = env.export_state()
    assert torch.equal(D.collate(rec, force=True), rec)
    assert D.max_over_ranks(3.25, dev, force=True) == 3.25
    res["width_at_k"] = bench.payload_width(2, K, B)
    dist.destroy_process_group()
    with open(out_path, "w") as f:
        json.dump(res, f)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
