"""One rank of the 2-process HIP-engine test (tests/test_gpu_dist.py).

Started as a fresh child process (it initialises the GPU itself; nothing is
exec'd from a process that touched the GPU).  Rank r runs the libcoup_mi355x
engine on its env-id shard [r*B, (r+1)*B), then
all-gathers the per-lane results with open_spiel_coup_amd.distributed.collate
over gloo (both ranks share the box's one GPU; RCCL refuses two ranks on one
GPU).  Rank 0 writes the gathered tensors to OUT_DIR.

    RANK=r WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=p \
        python tests/dist_hip_worker.py OUT_DIR LANES_PER_RANK SEED FUSED_STEPS STEPS
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out_dir, B, seed, k_fused, k_step = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(
        sys.argv[5])
    import numpy as np
    import torch
    import torch.distributed as dist

    from open_spiel_coup_amd import BatchedCoupEnv
    from open_spiel_coup_amd import distributed as D

    rank, world, _ = D.world_info()
    dev = D.init("gloo", gpu=True)
    base = D.env_id_base(rank, B)
    # fused rollout (coup_rollout): per-lane episodes / return sums / lengths
    fused = BatchedCoupEnv(B, seed=seed, env_id_base=base, obs=False, device=dev)
    stats = fused.new_stats()
    fused.rollout(k_fused, stats)
    g_stats = D.collate(torch.stack([stats["episodes"], stats["return_sum"], stats["length_sum"]], 1))
    g_fused_rec = D.collate(fused.export_state())
    # the bench's step path: coup_step with the per-episode accumulators
    stepped = BatchedCoupEnv(B, seed=seed, env_id_base=base, obs=False, device=dev, episode_stats=True)
    for _ in range(k_step):
        stepped.step()
    eps, ret = stepped.episode_stats()
    g_step_stats = D.collate(torch.stack([eps, ret], 1))
    g_step_rec = D.collate(stepped.export_state())
    errors = torch.tensor([fused.error_count() + stepped.error_count()], dtype=torch.int64)
    dist.all_reduce(errors)
    if rank == 0:
        np.save(os.path.join(out_dir, "fused_stats.npy"), g_stats.cpu().numpy())
        np.save(os.path.join(out_dir, "fused_rec.npy"), g_fused_rec.cpu().numpy())
        np.save(os.path.join(out_dir, "step_stats.npy"), g_step_stats.cpu().numpy())
        np.save(os.path.join(out_dir, "step_rec.npy"), g_step_rec.cpu().numpy())
        np.save(os.path.join(out_dir, "errors.npy"), errors.numpy())
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
