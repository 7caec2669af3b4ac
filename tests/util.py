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


def tiny_bpe_model(path):
    """A 43-token BPE model where two vocab strings are NOT their own merge_all result:
    "abc" (merges b c -> bc before a b -> ab, and no a bc merge: [a, bc]) and "cab" ([c, ab])."""
    import json
    letters = "abcdefghijklmnopqrstuvwxyz"
    specials = ["<pad>", "<unk>", "<s>", "</s>", "<mask>"]
    vocab = {t: i for i, t in enumerate(specials)}
    for ch in letters:
        vocab[ch] = len(vocab)
    merges = [("b", "c"), ("a", "b"), ("ab", "c"), ("d", "e"), ("de", "f"), ("x", "y"), ("y", "z"), ("xy", "z"),
              ("c", "a"), ("bc", "a"), ("ab", "ab"), ("ca", "b")]
    for a, b in merges:
        vocab.setdefault(a + b, len(vocab))
    tmpl = [{"SpecialToken": {"id": "<s>", "type_id": 0}}, {"Sequence": {"id": "A", "type_id": 0}},
            {"SpecialToken": {"id": "</s>", "type_id": 0}}]
    j = {"version": "1.0", "truncation": None, "padding": None,
         "added_tokens": [{"id": i, "content": t, "single_word": False, "lstrip": False, "rstrip": False,
                           "normalized": False, "special": True} for i, t in enumerate(specials)],
         "normalizer": {"type": "NFKC"}, "pre_tokenizer": {"type": "Whitespace"},
         "post_processor": {"type": "TemplateProcessing", "single": tmpl, "pair": tmpl + tmpl,
                            "special_tokens": {"<s>": {"id": "<s>", "ids": [2], "tokens": ["<s>"]},
                                               "</s>": {"id": "</s>", "ids": [3], "tokens": ["</s>"]}}},
         "decoder": None,
         "model": {"type": "BPE", "dropout": None, "unk_token": None, "continuing_subword_prefix": None,
                   "end_of_word_suffix": None, "fuse_unk": False, "byte_fallback": False, "ignore_merges": False,
                   "vocab": vocab, "merges": [[a, b] for a, b in merges]}}
    path.write_text(json.dumps(j))
    return str(path)
