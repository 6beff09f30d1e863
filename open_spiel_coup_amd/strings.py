"""Human-readable forms of a lane, formatted on the host from the packed
record and the history bytes.

Verbatim with the reference (pinned by integration_tests/playthroughs/
coup.txt):
  ObservationString / InformationStateString  CoupObserver::StringFrom (coup.cc:290-373)
  ToString                                     CoupState::ToString (coup.cc:945-987)
  ActionToString                               CoupGame::ActionToString (coup.cc:1143-1149)
String building is host work: the GPU keeps
only what the strings are made from.
"""
from . import packed

CARD_NAMES = ("Assassin", "Ambassador", "Captain", "Contessa", "Duke")
ACTION_NAMES = (
    "Income", "ForeignAid", "Coup", "Tax", "Assassinate", "Exchange", "Steal", "LoseCard1", "LoseCard2",
    "Pass", "Block", "Challenge", "ExchangeReturn12", "ExchangeReturn13", "ExchangeReturn14",
    "ExchangeReturn23", "ExchangeReturn24", "ExchangeReturn34")
FACE_NAMES = ("FaceDown", "FaceUp")
CHANCE_PLAYER = -1


def action_to_string(player, action):
    """CoupGame::ActionToString (coup.cc:1143-1149)."""
    if player == CHANCE_PLAYER:
        return "Chance drawn card:" + CARD_NAMES[action]
    return ACTION_NAMES[action]


def decode_history(hist_bytes, length):
    """History bytes -> [(player, action, deal_to)]; player -1 for deals."""
    out = []
    for i in range(length):
        e = hist_bytes[i]
        if e & 0x20:
            out.append((CHANCE_PLAYER, e & 0x1F, (e >> 6) & 1))
        else:
            out.append(((e >> 6) & 1, e & 0x1F, -1))
    return out


def _card_row(slot, value, face):
    return f"Card {slot + 1}: {value:<11}| {face}\n"


def _last_action(a):
    return "None" if a < 0 else ACTION_NAMES[a]


def _observer_string(lane, hist, player, perfect_recall):
    s = [f"Observer: P{player + 1}\n", f"Turn: {lane['turn_number']}\n", f"Move: P{lane['move_player'] + 1}\n"]
    for p in (0, 1):
        s.append(f"P{p + 1}\n        Card         State\n")
        for i, (t, face) in enumerate(lane["cards"][p]):
            shown = face == 1 or p == player
            s.append(_card_row(i, CARD_NAMES[t] if shown else "-", FACE_NAMES[face]))
        s.append(f"Coins: {lane['coins'][p]}\n")
        if perfect_recall:
            s.append("\n")
        else:
            s.append(f"Last Action: {_last_action(lane['last_action'][p])}\n\n")
    if perfect_recall:
        s.append("Action Sequence: ")
        n = len(hist)
        for i, (who, a, to) in enumerate(hist):
            # coup.cc:351-371: deals are shown to their receiver only, but the
            # ", " separator depends on the position in the full history
            if who == CHANCE_PLAYER:
                if to == player:
                    s.append("PC-" + CARD_NAMES[a] + (", " if i < n - 1 else ""))
            else:
                s.append(f"P{who + 1}-" + ACTION_NAMES[a] + (", " if i < n - 1 else ""))
        s.append("\n")
    return "".join(s)


def observation_string(words, hist_bytes, player, lane=0):
    """ObservationString(player) (kDefaultObsType)."""
    ln = packed.lane(words, lane)
    return _observer_string(ln, decode_history(hist_bytes, ln["move_number"]), player, False)


def information_state_string(words, hist_bytes, player, lane=0):
    """InformationStateString(player) (kInfoStateObsType, perfect recall)."""
    ln = packed.lane(words, lane)
    return _observer_string(ln, decode_history(hist_bytes, ln["move_number"]), player, True)


def to_string(words, hist_bytes, lane=0):
    """CoupState::ToString (coup.cc:945-987): every card shown."""
    ln = packed.lane(words, lane)
    hist = decode_history(hist_bytes, ln["move_number"])
    s = [f"Turn: {ln['turn_number']}\n", f"Move: P{ln['move_player'] + 1}\n"]
    for p in (0, 1):
        s.append(f"P{p + 1}\n        Card         State\n")
        for i, (t, face) in enumerate(ln["cards"][p]):
            s.append(_card_row(i, CARD_NAMES[t], FACE_NAMES[face]))
        s.append(f"Coins: {ln['coins'][p]}\n")
        s.append(f"Last Action: {_last_action(ln['last_action'][p])}\n\n")
    parts = []
    for who, a, _ in hist:
        parts.append(("PC-" + CARD_NAMES[a]) if who == CHANCE_PLAYER else (f"P{who + 1}-" + ACTION_NAMES[a]))
    s.append("Action Sequence: " + ", ".join(parts) + "\n")
    return "".join(s)
