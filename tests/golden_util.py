"""Shared helpers: load the golden fixtures and check a pyspiel.State-like
object against them.  Used for the oracle (CPU) and for the HIP path (GPU)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_playthrough():
    with open(os.path.join(GOLDEN, "playthrough_coup.json")) as f:
        return json.load(f)


def load_kats():
    with open(os.path.join(GOLDEN, "kat_coup_test.json")) as f:
        return json.load(f)["scenarios"]


def rstrip_lines(text):
    return "\n".join(line.rstrip() for line in text.split("\n"))


def dense(sparse, size):
    out = np.zeros(size, np.float32)
    for k, v in sparse:
        out[k] = v
    return out


def check_kat(check, cards, coins, last_action, current_player, legal, terminal,
              rewards, returns):
    """check: one entry of a KAT scenario.  The remaining arguments are
    callables returning the observed value (so absent keys cost nothing)."""
    for key, want in check.items():
        if key == "after":
            continue
        if key == "current_player":
            got = current_player()
        elif key == "legal":
            got = list(legal())
        elif key == "terminal":
            got = bool(terminal())
        elif key == "rewards":
            got = [float(x) for x in rewards()]
            want = [float(x) for x in want]
        elif key == "returns":
            got = [float(x) for x in returns()]
            want = [float(x) for x in want]
        elif key == "coins":
            got = [coins(0), coins(1)]
        elif key in ("coins0", "coins1"):
            got = coins(int(key[-1]))
        elif key == "last_action":
            got = [last_action(0), last_action(1)]
        elif key == "num_cards":
            got = [len(cards(0)), len(cards(1))]
        elif key == "num_cards0":
            got = len(cards(0))
        elif key == "all_face_down":
            got = all(st == 0 for p in (0, 1) for _, st in cards(p))
        elif key.startswith("card_state"):
            p, i = int(key[10]), int(key[12])
            got = cards(p)[i][1]
        elif key == "cards0_min_value":
            got = min(v for v, _ in cards(0))
        elif key == "cards0_face_down":
            got = all(st == 0 for _, st in cards(0))
        else:
            raise KeyError(key)
        assert got == want, f"{key}: got {got}, want {want}"
