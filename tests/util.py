"""Helpers turning packed batch outputs into the reference's per-row shapes."""
import numpy as np

LABEL = {0: "other", 1: "devanagari", 2: "roman", 255: None}


def rows_u8(out, offs):
    out = np.asarray(out)
    offs = np.asarray(offs)
    raw = out.tobytes()
    return [raw[offs[i]:offs[i + 1]].decode("utf-8", "surrogatepass") for i in range(len(offs) - 1)]


def rows_ints(out, offs):
    out = np.asarray(out)
    offs = np.asarray(offs)
    return [[int(x) for x in out[offs[i]:offs[i + 1]]] for i in range(len(offs) - 1)]


def ends_to_lens(ends):
    return [b - a for a, b in zip([0] + ends[:-1], ends)]


def rows_runs(ends, labels, offs):
    ends = np.asarray(ends)
    labels = np.asarray(labels)
    offs = np.asarray(offs)
    res = []
    for i in range(len(offs) - 1):
        e = [int(x) for x in ends[offs[i]:offs[i + 1]]]
        lab = [LABEL[int(x)] for x in labels[offs[i]:offs[i + 1]]]
        res.append([[ln, lb] for ln, lb in zip(ends_to_lens(e), lab)])
    return res


NORM_KEYS = ((3, "norm"), (2, "norm_nolower"), (1, "norm_noclean"), (0, "norm_nfc"))
SEG_KEYS = ((3, False, "ak"), (3, True, "ak_m"), (-1, False, "ak_raw"), (-1, True, "ak_raw_m"))
SW_KEYS = ((3, "sw"), (-1, "sw_raw"))
