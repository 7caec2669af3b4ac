"""f3: the CLI `tokenize` streaming a whole file as ONE row (reference cli.py:25-90) and the exact
long-row cuts behind it (akshar_amd/longrows.py), against the reference CLI's own outputs
(tests/golden/cli_golden.json.gz, tools/gen_cli_golden.py) and the oracle."""
import gzip
import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests.conftest import BPE_PATH, ROOT, SPM_PATH
from tests.util import rows_ints, rows_u8

CLI_GOLDEN = os.path.join(ROOT, "tests", "golden", "cli_golden.json.gz")


@pytest.fixture(scope="module")
def cli_golden():
    with gzip.open(CLI_GOLDEN, "rt", encoding="utf-8") as f:
        return json.load(f)


def long_text(g):
    from akshar_amd import synth
    lines = []
    for kind, n, seed in g["long_recipe"]:
        lines += synth.lines(kind, n, seed=seed)
    return "\n".join(lines) + "\n"


def long_text_as_read(g):
    """long_text as the CLI sees it: open(..., "r") translates '\r\n' and '\r' to '\n'."""
    return long_text(g).replace("\r\n", "\n").replace("\r", "\n")


def _case(g, inp, model_type, fmt, model=True):
    for c in g["cases"]:
        if c["input"] == inp and c["format"] == fmt and (c["model"] is not None) == model and \
                (not model or c["model_type"] == model_type):
            return c["output"]
    raise KeyError((inp, model_type, fmt, model))


# SentencePiece on one whole-file row: the lattice carries the best score across the whole row,
# and sentencepiece 0.2.2 rebases it whenever it leaves [-1e5, 1e5] (oracle/akshar_oracle.c
# spm_encode_cps; ak_dev.h SpmSink). The whole row is pinned to the reference CLI, every id.


# ------------------------------------------------------------------ CPU: the cuts are exact
def test_cut_points_are_whitespace_after_solid_chars(cli_golden):
    from akshar_amd import longrows
    raw = long_text(cli_golden).encode()
    cuts = longrows.cut_points(raw)
    assert len(cuts) > 1000
    b = np.frombuffer(raw, np.uint8)
    assert np.isin(b[cuts], [0x20, 0x0A]).all()
    gaps = np.diff(np.concatenate([[0], cuts]))
    assert gaps.min() >= longrows.PIECE_BYTES and (gaps >= 768).mean() < 0.02  # pieces fit the tiles


def test_oracle_whole_row_matches_reference_cli_and_cut_pieces(cli_golden, bpe_model, spm_model):
    """The oracle on the ~1.5 MB file as one row reproduces the reference CLI's BPE and
    SentencePiece ids, and the BPE / normalize / segment results of the cut pieces, stitched,
    equal the one-row results."""
    from akshar_amd import longrows
    raw = long_text_as_read(cli_golden).encode()
    one = (np.frombuffer(raw, np.uint8).copy(), np.asarray([0, len(raw)], np.uint64))
    ids, _ = O.OracleBPE(bpe_model).encode_batch(*one)
    assert " ".join(map(str, ids)) == _case(cli_golden, "long", "bpe", "id")
    sids, _ = O.OracleSPM(spm_model).encode_batch(*one)
    ref = [int(x) for x in _case(cli_golden, "long", "sentencepiece", "id").split()]
    assert list(map(int, sids)) == ref
    buf, offs = longrows.split_rows(raw)
    pieces = (buf, offs.astype(np.uint64))
    pids, poo = O.OracleBPE(bpe_model).encode_batch(*pieces)
    assert np.array_equal(longrows.stitch_bpe(pids, poo), ids)
    n1, _ = O.normalize_batch(*one)
    np_, noo = O.normalize_batch(*pieces)
    assert n1.tobytes() == np_.tobytes()
    norm = n1.tobytes().decode()
    e1, _ = O.segment_batch(*one)
    toks = [norm[a:b] for a, b in zip(np.concatenate([[0], e1[:-1]]), e1)]
    assert " ".join(toks) == _case(cli_golden, "long", None, "text", model=False)


# ------------------------------------------------------------------ GPU: the CLI itself
def _cli(tmp_path, argv):
    from akshar_amd import cli
    out = tmp_path / "out.txt"
    cli.main(argv + ["-o", str(out)])
    return out.read_text(encoding="utf-8")


@pytest.mark.gpu
@pytest.mark.parametrize("inp", ["corpus", "long"])
def test_cli_tokenize_matches_reference(tmp_path, cli_golden, inp):
    path = tmp_path / "in.txt"
    path.write_text(cli_golden["corpus_text"] if inp == "corpus" else long_text(cli_golden), encoding="utf-8")
    for c in cli_golden["cases"]:
        if c["input"] != inp:
            continue
        argv = ["tokenize", "-i", str(path), "--format", c["format"], "--model-type", c["model_type"]]
        if c["model"]:
            argv += ["-m", BPE_PATH if c["model"].endswith(".json") else SPM_PATH]
        got = _cli(tmp_path, argv)
        assert got == c["output"], (inp, c["model"], c["format"])


@pytest.mark.gpu
def test_cli_errors_and_preprocess(tmp_path, capsys):
    from akshar_amd import cli
    with pytest.raises(SystemExit) as e:
        cli.main(["tokenize", "abc", "--format", "id"])
    assert e.value.code == 1 and "--model required for ID output" in capsys.readouterr().err
    with pytest.raises(SystemExit) as e:
        cli.main(["tokenize", "abc", "-m", "/nonexistent.model"])
    assert e.value.code == 1 and "Model file not found" in capsys.readouterr().err
    src = tmp_path / "c.txt"
    src.write_text("Heyyy यार kya HAAL hai\n\n  aaj मौसम  \nbohoooot\n", encoding="utf-8")
    dst = tmp_path / "p.txt"
    cli.main(["preprocess", str(src), str(dst)])
    assert dst.read_text(encoding="utf-8") == "hey यार kya haal hai\naaj मौसम\nbohot\n"
