"""Where do the split and fused InformationStateTensor writers differ?
B lanes, one uniform step each way, both against the oracle's rollout.
Measurement / debugging tool only."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle  # noqa: E402
from open_spiel_coup_amd import BatchedCoupEnv  # noqa: E402


def run(split, B, seed, steps):
    os.environ["COUP_INFO_SPLIT"] = str(split)
    env = BatchedCoupEnv(B, seed=seed, auto_reset=True, obs=False, info_state=True, history=True, device="cuda")
    outs = [env.step()["info_state"].cpu().numpy().copy() for _ in range(steps)]
    env.close()
    return outs


def main():
    B, seed, steps = int(sys.argv[1]), 7, int(sys.argv[2]) if len(sys.argv) > 2 else 1
    fused, split = run(0, B, seed, steps), run(1, B, seed, steps)
    ref = oracle.rollout(seed=seed, n=B, steps=steps, want_info=True)["info"]
    for t in range(steps):
        bad = np.argwhere(fused[t] != split[t])
        print(f"step {t}: {len(bad)} differing floats; fused vs oracle {int((fused[t] != ref[t]).sum())}, "
              f"split vs oracle {int((split[t] != ref[t]).sum())}")
        for lane, p, f in bad[:12]:
            print(f"  lane {lane} player {p} float {f} (float4 {(p * 2492 + f) // 4} of the lane): fused "
                  f"{fused[t][lane, p, f]} split {split[t][lane, p, f]} oracle {ref[t][lane, p, f]}")


if __name__ == "__main__":
    main()
