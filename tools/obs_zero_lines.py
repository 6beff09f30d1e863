"""Share of all-zero 64 / 128 / 256 / 512-B segments in the tensors the
split writers store (c3's ObservationTensor [2^20][2][98], c3i's
InformationStateTensor [2^18][2][2492]) after a few uniform-random steps:
the data the store-sweep density shapes (tools/sweep_ab.py DENS) stand in
for.  Measurement tool only.

    python tools/obs_zero_lines.py [--steps 30]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def zero_shares(t):
    flat = t.reshape(-1)
    out = {}
    for seg in (64, 128, 256, 512):
        f = seg // 4
        n = flat.numel() // f
        nz = (flat[: n * f].view(n, f) != 0).any(dim=1)
        out[str(seg)] = round(1.0 - nz.float().mean().item(), 4)
    out["nonzero_float_share"] = round((flat != 0).float().mean().item(), 4)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    import torch
    from open_spiel_coup_amd.env import BatchedCoupEnv
    for name, batch, kw, field in (("c3_obs", 1 << 20, dict(obs=True), "obs"),
                                   ("c3i_info", 1 << 18, dict(obs=False, info_state=True), "info_state")):
        env = BatchedCoupEnv(batch, seed=7, **kw)
        rows = []
        for k in range(a.steps):
            env.step()
            if k in (0, 4, a.steps - 1):
                torch.cuda.synchronize()
                rows.append({"step": k + 1, **zero_shares(getattr(env, field))})
        print(json.dumps({"buffer": name, "zero_segment_share": rows}), flush=True)
        env.close()
        del env
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
