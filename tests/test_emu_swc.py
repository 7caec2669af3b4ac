"""The SentencePiece word cache (akshar_amd/csrc/ak_swc.h, ak_model_build.h build_spm_wcache,
ak_tile_spm.h pass V) on the emulated tile kernel: every stored solution against the oracle's
encode of that word, and the encode against the oracle with the cache on, off and forced into tiny
tables (every probe colliding, most words dropped), with words past the cached length, and with
models whose cached words hold exact ties (margin 0: the row must redo from its carried base) or
cross the rebase bound."""
import copy

import numpy as np
import pytest

from oracle import oracle as O
from tests.emu import emu

SWC_MAXN = 16


@pytest.fixture(scope="module")
def em(spm_model):
    m = emu.Model(spm=spm_model)
    m.set_wc(-1)
    yield m


def _pieces(spm_model):
    return [p.decode("utf-8", "surrogatepass") for p in spm_model.pieces]


def _alphabet(spm_model):
    """Dense code -> char, as build_spm assigns them (sorted chars of NORMAL / USER_DEFINED / UNUSED
    pieces), rebuilt here independently of the C++ build."""
    chars = set()
    for p, t in zip(_pieces(spm_model), spm_model.types.tolist()):
        if t in (1, 4, 5):
            chars.update(p)
    return [None] + sorted(chars)


def _ws_words(spm_model):
    return [p for p, t in zip(_pieces(spm_model), spm_model.types.tolist())
            if t in (1, 4, 5) and p.startswith("▁") and 2 <= len(p) <= SWC_MAXN]


def test_table_matches_oracle(em, spm_model):
    """Each stored word's pieces are the oracle's encode of that word; every "▁" piece string of
    2..16 chars is a word of the build, and (almost) all are stored."""
    info = em.set_wc(-1)
    tab = em.wc_table().reshape(-1, 16)
    alpha = _alphabet(spm_model)
    words = _ws_words(spm_model)
    assert info["slots"] == len(tab) and info["words"] == len(words)
    assert info["stored"] + info["skipped"] >= 0.99 * info["words"]
    stored = []
    for e in tab:
        n = (int(e[0]) >> 12) & 31
        if n == 0:
            continue
        npc = (int(e[0]) >> 17) & 7
        codes = []
        for k in range(8):
            codes += [int(e[8 + k]) & 0xFFFF, int(e[8 + k]) >> 16]
        assert all(c == 0 for c in codes[n:]) and all(c & 0x8000 for c in codes[:n])
        word = "".join(alpha[c & 0x7FFF] for c in codes[:n])
        assert word.startswith("▁") and word in words
        pieces = [int(x) for x in e[2:2 + npc]]
        assert sum(p & 0xFF for p in pieces) == n
        stored.append((word[1:], [p >> 8 for p in pieces]))
    assert len(stored) == info["stored"]
    texts = [w for w, _ in stored]
    buf, offs = O.pack(texts)
    ref, ro = O.OracleSPM(spm_model).encode_batch(buf, offs)
    for i, (w, ids) in enumerate(stored):
        assert ref[ro[i]:ro[i + 1]].tolist() == ids, w


def _texts(spm_model, n=300, seed=7):
    """Rows mixing cached words, words past the cached length and random Hinglish."""
    from akshar_amd import synth
    cached = [w[1:] for w in _ws_words(spm_model)]
    rng = np.random.default_rng(seed)
    longw = ["abcdefghijklmnop", "abcdefghijklmnopq", "namastenamastenamaste", "कर्मण्येवाधिकारस्ते"]
    buf, offs = synth.generate(1, n // 2, seed=seed)
    base = [bytes(buf[offs[i]:offs[i + 1]]).decode() for i in range(n // 2)]
    texts = []
    for i in range(n):
        words = list(rng.choice(cached, size=8)) + [str(rng.choice(longw))]
        rng.shuffle(words)
        texts.append(" ".join(words) if i % 2 else base[i // 2] + " " + " ".join(words[:4]))
    return texts


@pytest.mark.parametrize("bits", [-1, None, 0, 1, 4])
def test_encode_vs_oracle(em, spm_model, bits):
    """bits -1: the product table; None: no cache; 0 / 1 / 4: 1 / 2 / 16 slots."""
    info = em.set_wc(bits)
    if bits is not None and bits >= 0:
        assert info["slots"] == 1 << bits and info["stored"] <= 1 << bits
    buf, offs = O.pack(_texts(spm_model))
    ids, oo, _ = emu.spm_tiles(em, buf, offs, rows=4)
    probes, hits = emu.last_counters()
    ref, ro = O.OracleSPM(spm_model).encode_batch(buf, offs)
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)
    if bits is None:
        assert probes == 0
    elif bits == -1:
        assert hits > 0.5 * probes, (probes, hits)
    em.set_wc(-1)


def test_hit_rate_on_bench_rows(em, spm_model):
    """The bench corpus (synthetic Hinglish, seed 1234): the words that are "▁" pieces hit."""
    from akshar_amd import synth
    em.set_wc(-1)
    buf, offs = synth.generate(1, 300, seed=1234)
    ids, oo, _ = emu.spm_tiles(em, buf, offs, rows=4)
    probes, hits = emu.last_counters()
    ref, ro = O.OracleSPM(spm_model).encode_batch(buf, offs)
    assert np.array_equal(ids, ref)
    assert 0.35 < hits / probes < 0.6, (probes, hits)


def _tied_model(spm_model, count=300):
    """The model with the score of `count` single-piece cached words set to exactly the float sum of a
    two-piece split of them ("▁x" + "y"): their base-0 lattice has margin 0 at the word end, so a hit
    must send the row to the exact redo from its carried base (where rounding decides the winner)."""
    m = copy.copy(spm_model)
    sc = np.asarray(spm_model.scores, dtype=np.float32).copy()
    pieces = _pieces(spm_model)
    pid = {p: i for i, p in enumerate(pieces)}
    types = spm_model.types.tolist()
    tied = []
    for w in _ws_words(spm_model):
        if len(tied) >= count or len(w) < 4:
            continue
        for cut in range(2, len(w)):
            a, b = w[:cut], w[cut:]
            if a in pid and b in pid and types[pid[a]] == 1 and types[pid[b]] == 1 and types[pid[w]] == 1:
                sc[pid[w]] = np.float32(sc[pid[a]] + sc[pid[b]])
                tied.append(w[1:])
                break
    m.scores = sc
    return m, tied


def test_ties_on_cached_words_redo_from_the_carried_base(spm_model):
    m, tied = _tied_model(spm_model)
    assert len(tied) >= 100
    em = emu.Model(spm=m)
    em.set_wc(-1)
    rng = np.random.default_rng(5)
    texts = [" ".join(rng.choice(tied, size=rng.integers(1, 14))) for _ in range(300)]
    buf, offs = O.pack(texts)
    ids, oo, _ = emu.spm_tiles(em, buf, offs, rows=4)
    probes, hits = emu.last_counters()
    assert hits > 0.9 * probes
    ref, ro = O.OracleSPM(m).encode_batch(buf, offs)
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)


@pytest.mark.parametrize("scale", [500.0, 2000.0])
def test_cached_words_across_the_rebase_bound(spm_model, scale):
    """Scaled scores carry rows past [-1e5, 1e5]: hits and solved words side by side still rebase
    as the oracle."""
    m = copy.copy(spm_model)
    m.scores = (np.asarray(spm_model.scores, dtype=np.float32) * np.float32(scale)).astype(np.float32)
    em = emu.Model(spm=m)
    em.set_wc(-1)
    buf, offs = O.pack(_texts(m, n=200, seed=11))
    ids, oo, _ = emu.spm_tiles(em, buf, offs, rows=4)
    probes, hits = emu.last_counters()
    assert hits > 0
    ref, ro = O.OracleSPM(m).encode_batch(buf, offs)
    assert np.array_equal(oo, ro) and np.array_equal(ids, ref)
