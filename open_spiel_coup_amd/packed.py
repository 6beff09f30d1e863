"""Host-side view of the packed 16-byte lane record.

Pure format conversion (bit fields -> named fields); all game logic runs in
the HIP kernels.

  w0  [15:0] P1 hand, [31:16] P2 hand: nibble i = slot i, kind = 2*type+face
      (face 0 = down, 1 = up), 0xF = empty; slots sorted ascending.
  w1  [19:0] deck counts (type t at 4t), [23:20] P1 coins, [27:24] P2 coins,
      [30:28] P1 reward + 2, [31] error flag
  w2  [4:0] P1 last action (31 = None), [9:5] P2 last action, [10] P1 lost
      challenge, [11] P2 lost challenge, [14:12] deal-queue length,
      [18:15] deal-queue players (entry j = bit 15+j, front first),
      [19] turn player, [20] move player, [21] turn begin, [28:22] move number,
      [31:29] episode bits 27..25
  w3  [6:0] turn number, [31:7] episode bits 24..0 (28-bit episode counter)
"""
import numpy as np

NONE = 31


def _u32(words):
    w = np.asarray(words)
    if w.dtype != np.uint32:
        w = w.astype(np.int64).astype(np.uint32) if w.dtype.kind == "i" else w.astype(np.uint32)
    return w.reshape(-1, 4)


def decode(words):
    """[N,4] (any int dtype, e.g. a torch int32 export moved to numpy) ->
    dict of numpy arrays, one entry per field."""
    w = _u32(words)
    x, y, z, v = (w[:, k].astype(np.int64) for k in range(4))
    d = {
        "hand": np.stack([x & 0xFFFF, x >> 16], axis=1),
        "deck": np.stack([(y >> (4 * t)) & 0xF for t in range(5)], axis=1),
        "coins": np.stack([(y >> 20) & 0xF, (y >> 24) & 0xF], axis=1),
        "reward0": ((y >> 28) & 0x7) - 2,
        "error": (y >> 31) & 1,
        "last_action": np.stack([z & 0x1F, (z >> 5) & 0x1F], axis=1),
        "lost_challenge": np.stack([(z >> 10) & 1, (z >> 11) & 1], axis=1),
        "queue_len": (z >> 12) & 0x7,
        "queue_bits": (z >> 15) & 0xF,
        "turn_player": (z >> 19) & 1,
        "move_player": (z >> 20) & 1,
        "turn_begin": (z >> 21) & 1,
        "move_number": (z >> 22) & 0x7F,
        "turn_number": v & 0x7F,
        "episode": (v >> 7) | ((z >> 29) << 25),
    }
    return d


def hand_cards(hand16):
    """16-bit hand word -> [(type, face), ...] in slot order."""
    out = []
    for i in range(4):
        k = (int(hand16) >> (4 * i)) & 0xF
        if k == 0xF:
            break
        out.append((k >> 1, k & 1))
    return out


def lane(words, i=0):
    """Decoded fields of lane i as Python scalars, with hands as card lists."""
    d = decode(words)
    r = {k: (v[i].tolist() if hasattr(v[i], "tolist") else v[i]) for k, v in d.items()}
    r["cards"] = [hand_cards(d["hand"][i, 0]), hand_cards(d["hand"][i, 1])]
    r["last_action"] = [(-1 if a == NONE else a) for a in r["last_action"]]
    r["queue"] = [(int(d["queue_bits"][i]) >> j) & 1 for j in range(int(d["queue_len"][i]))]
    return r
