"""Generate the golden fixtures under tests/golden/ from the reference's own
test data.  Run in the build container (it reads /root/reference); the
resulting JSON files are committed and travel to the GPU box.

  playthrough_coup.json  parsed from
      open_spiel/integration_tests/playthroughs/coup.txt  (the reference's
      golden transcript, replayed by integration_tests/playthrough_test.py)
  kat_coup_test.json     the 14 known-answer scenarios of
      open_spiel/games/coup_test.cc:41-539, transcribed as data (action
      sequence + the values each scenario checks).

Usage:  python tests/golden/make_golden.py [--reference /root/reference]
"""
import argparse
import ast
import json
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))

OBS_FIELDS = [("player", 2), ("p1_cards", 20), ("p2_cards", 20),
              ("cur_move_player", 2), ("cards_state", 16), ("coins", 2),
              ("last_action", 36)]
INFO_FIELDS = [("player", 2), ("p1_cards", 20), ("p2_cards", 20),
               ("cur_move_player", 2), ("cards_state", 16), ("coins", 2),
               ("history", 135 * 18)]


def _bits(s):
    return [1.0 if ch == "◉" else 0.0 for ch in s if ch in "◉◯"]


def _parse_tensor_block(lines, i, name):
    """Parse one field printed by generate_playthrough._format_tensor.

    Returns (values in row-major order of the field's shape, next line)."""
    line = lines[i]
    head, _, rest = line.partition(name)
    rest = rest.lstrip()
    if rest.startswith("= ["):
        vals = [float(v) for v in rest[3:-1].split(",")]
        return vals, i + 1
    if rest.startswith(":") and rest[1:].strip():
        # 1-D or 2-D: first row on this line, further rows indented
        rows = [_bits(rest[1:])]
        j = i + 1
        while j < len(lines) and lines[j].startswith(" ") and set(lines[j].strip()) <= set("◉◯"):
            rows.append(_bits(lines[j]))
            j += 1
        return [v for r in rows for v in r], j
    # 3-D (cards_state [2][4][2]): one text row per slot, players side by side
    j = i + 1
    rows = []
    while j < len(lines) and lines[j] and set(lines[j].replace(" ", "")) <= set("◉◯"):
        rows.append([_bits(part) for part in lines[j].split("  ")])
        j += 1
    nplayers = len(rows[0])
    vals = []
    for p in range(nplayers):
        for r in rows:
            vals.extend(r[p])
    return vals, j


def parse_playthrough(path):
    with open(path, encoding="utf-8") as f:
        lines = f.read().split("\n")
    states = []
    cur = None
    i = 0
    while i < len(lines):
        line = lines[i]
        m = re.match(r"^# State (\d+)$", line)
        if m:
            cur = {"index": int(m.group(1)), "to_string_lines": []}
            states.append(cur)
            i += 1
            while i < len(lines) and lines[i].startswith("#"):
                cur["to_string_lines"].append(lines[i][2:] if lines[i].startswith("# ") else "")
                i += 1
            continue
        if cur is None:
            i += 1
            continue
        if line.startswith("action: "):
            cur["action"] = int(line.split(":")[1])
        elif line.startswith("IsTerminal() = "):
            cur["is_terminal"] = line.endswith("True")
        elif line.startswith("History() = "):
            cur["history"] = ast.literal_eval(line.split(" = ", 1)[1])
        elif line.startswith("IsChanceNode() = "):
            cur["is_chance"] = line.endswith("True")
        elif line.startswith("CurrentPlayer() = "):
            cur["current_player"] = int(line.split(" = ")[1])
        elif line.startswith("LegalActions() = "):
            cur["legal_actions"] = ast.literal_eval(line.split(" = ", 1)[1])
        elif line.startswith("ChanceOutcomes() = "):
            cur["chance_outcomes"] = ast.literal_eval(line.split(" = ", 1)[1])
        elif line.startswith("Rewards() = "):
            cur["rewards"] = ast.literal_eval(line.split(" = ", 1)[1])
        elif line.startswith("Returns() = "):
            cur["returns"] = ast.literal_eval(line.split(" = ", 1)[1])
        else:
            for kind in ("InformationStateString", "ObservationString"):
                m = re.match(r"^%s\((\d)\) = (.*)$" % kind, line)
                if m:
                    cur.setdefault(kind, {})[m.group(1)] = json.loads(m.group(2))
            for kind, fields in (("InformationStateTensor", INFO_FIELDS),
                                 ("ObservationTensor", OBS_FIELDS)):
                m = re.match(r"^%s\((\d)\)\.(\w+)" % kind, line)
                if m:
                    p, field = m.group(1), m.group(2)
                    vals, j = _parse_tensor_block(lines, i, f"{kind}({p}).{field}")
                    size = dict(fields)[field]
                    assert len(vals) == size, (kind, field, len(vals), size)
                    cur.setdefault(kind, {}).setdefault(p, {})[field] = vals
                    i = j
                    break
            else:
                i += 1
                continue
            continue
        i += 1

    out = []
    for st in states:
        rec = {k: v for k, v in st.items() if k not in ("InformationStateTensor", "ObservationTensor")}
        tl = st["to_string_lines"]
        if tl and not tl[0].startswith("Apply action"):
            rec["to_string"] = "\n".join(tl) + "\n"
        del rec["to_string_lines"]
        for kind, fields, size in (("InformationStateTensor", INFO_FIELDS, 2492),
                                   ("ObservationTensor", OBS_FIELDS, 98)):
            if kind in st:
                rec[kind] = {}
                for p, fd in st[kind].items():
                    flat = []
                    for name, n in fields:
                        flat.extend(fd[name])
                    assert len(flat) == size
                    # sparse form: [[index, value], ...]
                    rec[kind][p] = [[k, v] for k, v in enumerate(flat) if v != 0.0]
        out.append(rec)
    # fill history of abbreviated states from the action chain
    hist = []
    for rec in out:
        if "history" not in rec:
            rec["history"] = list(hist)
        assert rec["history"] == hist, (rec["index"], rec["history"], hist)
        if "action" in rec:
            hist = hist + [rec["action"]]
    return out


# coup_test.cc known-answer scenarios, transcribed as data.  Each check is
# applied after the listed number of actions have been applied.
# Action ids: card deals 0..4 (Assassin, Ambassador, Captain, Contessa, Duke);
# Income 0, ForeignAid 1, Coup 2, Tax 3, Assassinate 4, Exchange 5, Steal 6,
# LoseCard1 7, LoseCard2 8, Pass 9, Block 10, Challenge 11, ExchangeReturnXY 12..17.
def kat_scenarios():
    S = []

    def sc(name, cite, actions, checks):
        S.append({"name": name, "cite": cite, "actions": actions, "checks": checks})

    deal_std = [1, 0, 3, 4]  # Ambassador, Assassin, Contessa, Duke
    sc("GameStart", "coup_test.cc:41-73", deal_std,
       [{"after": 0, "current_player": -1},
        {"after": 4, "num_cards": [2, 2], "all_face_down": True, "coins": [1, 2],
         "last_action": [-1, -1], "current_player": 0}])
    sc("Income", "coup_test.cc:75-97", deal_std + [0],
       [{"after": 5, "coins0": 2, "current_player": 1, "terminal": False,
         "rewards": [0, 0], "returns": [0, 0]}])
    sc("PassForeignAid", "coup_test.cc:99-126", deal_std + [1, 9],
       [{"after": 5, "current_player": 1, "legal": [9, 10]},
        {"after": 6, "coins0": 3, "terminal": False, "rewards": [0, 0], "returns": [0, 0]}])
    sc("BlockForeignAid", "coup_test.cc:128-156", deal_std + [1, 10, 9],
       [{"after": 6, "current_player": 0, "legal": [9, 11]},
        {"after": 7, "coins0": 1, "terminal": False, "rewards": [0, 0], "returns": [0, 0]}])
    sc("ChallengeForeignAid", "coup_test.cc:158-188", [4, 0, 3, 1, 1, 10, 11],
       [{"after": 7, "current_player": 1, "legal": [7, 8], "coins0": 3, "terminal": False,
         "rewards": [0, 0], "returns": [0, 0]}])
    sc("LoseCard", "coup_test.cc:190-223", deal_std + [0] * 11 + [2, 7],
       [{"after": 15, "current_player": 1, "coins1": 7},
        {"after": 16, "legal": [7, 8]},
        {"after": 17, "coins1": 0, "card_state0_0": 1, "terminal": False,
         "rewards": [-1, 1], "returns": [-1, 1]}])
    sc("Assassinate", "coup_test.cc:226-262", [0, 0, 3, 4, 1, 9, 0, 4, 7],
       [{"after": 7, "current_player": 0, "coins0": 3},
        {"after": 8, "legal": [7, 8, 10, 11]},
        {"after": 9, "coins0": 0, "card_state1_0": 1, "terminal": False,
         "rewards": [1, -1], "returns": [1, -1]}])
    sc("DoubleAssassinate", "coup_test.cc:264-291", [0, 0, 3, 4, 1, 9, 0, 4, 11],
       [{"after": 9, "coins0": 0, "terminal": True, "rewards": [2, -2], "returns": [2, -2]}])
    sc("Exchange", "coup_test.cc:294-345", deal_std + [5, 9, 4, 4, 12],
       [{"after": 5, "current_player": 1, "legal": [9, 11]},
        {"after": 6, "current_player": -1},
        {"after": 8, "current_player": 0, "num_cards0": 4, "legal": [12, 13, 14, 15, 16, 17]},
        {"after": 9, "num_cards0": 2, "cards0_min_value": 4, "cards0_face_down": True,
         "terminal": False, "rewards": [0, 0], "returns": [0, 0]}])
    sc("Steal", "coup_test.cc:348-379", [2, 0, 3, 4, 6, 9],
       [{"after": 5, "current_player": 1, "legal": [9, 10, 11]},
        {"after": 6, "coins0": 3, "coins1": 0, "current_player": 1, "terminal": False,
         "rewards": [0, 0], "returns": [0, 0]}])
    sc("BlockSteal", "coup_test.cc:381-422", [2, 2, 3, 4, 6, 10, 11, 2, 7],
       [{"after": 6, "current_player": 0, "legal": [9, 11]},
        {"after": 7, "current_player": -1},
        {"after": 8, "current_player": 0, "legal": [7, 8]},
        {"after": 9, "coins0": 1, "coins1": 2, "current_player": 1, "card_state0_0": 1,
         "terminal": False, "rewards": [-1, 1], "returns": [-1, 1]}])
    sc("BlockAssassinate", "coup_test.cc:425-467", [0, 3, 0, 3, 1, 9, 0, 4, 10, 11, 3],
       [{"after": 7, "current_player": 0},
        {"after": 9, "current_player": 0, "legal": [9, 11]},
        {"after": 10, "current_player": -1},
        {"after": 11, "coins0": 0, "current_player": 0, "legal": [7, 8], "terminal": False,
         "rewards": [0, 0], "returns": [0, 0]}])
    sc("Tax", "coup_test.cc:470-499", [1, 0, 4, 4, 3, 9],
       [{"after": 5, "current_player": 1, "legal": [9, 11]},
        {"after": 6, "coins0": 4, "current_player": 1, "terminal": False,
         "rewards": [0, 0], "returns": [0, 0]}])
    sc("ChallengeBlockForeignAid", "coup_test.cc:501-539", [1, 0, 4, 4, 1, 10, 11, 4],
       [{"after": 6, "current_player": 0, "legal": [9, 11]},
        {"after": 7, "current_player": -1},
        {"after": 8, "coins0": 1, "current_player": 0, "legal": [7, 8], "terminal": False,
         "rewards": [0, 0], "returns": [0, 0]}])
    return S


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    pt = os.path.join(args.reference, "open_spiel/integration_tests/playthroughs/coup.txt")
    states = parse_playthrough(pt)
    with open(os.path.join(HERE, "playthrough_coup.json"), "w") as f:
        json.dump({"source": "open_spiel/integration_tests/playthroughs/coup.txt",
                   "obs_size": 98, "info_size": 2492, "states": states}, f, separators=(",", ":"))
    with open(os.path.join(HERE, "kat_coup_test.json"), "w") as f:
        json.dump({"source": "open_spiel/games/coup_test.cc", "scenarios": kat_scenarios()}, f, indent=1)
    print(f"wrote {len(states)} playthrough states, {len(kat_scenarios())} KAT scenarios")


if __name__ == "__main__":
    main()
