"""Command-line interface (reference: src/akshar/cli.py:25-190, :305-372) on the MI355X engine.

  python -m akshar_amd tokenize [TEXT] [-i FILE] [-o OUT] [-m MODEL] [--model-type T] [--format text|json|id]
  python -m akshar_amd detokenize [TOKENS] [-i FILE] [-o OUT] [-m MODEL] [--model-type T]
  python -m akshar_amd explain TEXT [-m MODEL] [--model-type T]
  python -m akshar_amd preprocess INPUT OUTPUT     (the trainer's corpus preprocessing, cli.py:165-190)

Same arguments, messages, exit codes and output bytes as the reference. As there, `tokenize -i`
reads the whole file as ONE string (cli.py:52-53); a long BPE / akshar row is cut at exact cut
points into tile-sized rows and stitched (akshar_amd/longrows.py), a SentencePiece row stays one
row. `preprocess` normalizes every stripped, non-empty line in one GPU batch (the reference's
train --no-preprocess=False step, cli.py:165-190) and writes them one per line. `train` is not
provided: training runs once, offline, with the reference's own trainer (tools/train_models.py).
"""
import argparse
import json
import sys
from pathlib import Path

from .tokenizer import aksharTokenizer


def tokenize_command(args):
    """cli.py:25-90."""
    if args.model and not Path(args.model).exists():
        print(f"Error: Model file not found: {args.model}", file=sys.stderr)
        print(f"  Current directory: {Path.cwd()}", file=sys.stderr)
        print("  To train a model: akshar train <corpus.txt> --output models/akshar --vocab-size 24000", file=sys.stderr)
        sys.exit(1)
    tokenizer = aksharTokenizer(model_path=args.model, model_type=args.model_type)
    if args.input:
        with open(args.input, "r", encoding="utf-8") as f:
            text = f.read()
    else:
        text = args.text
    if not text:
        print("Error: No text provided. Use --input or provide text as argument.", file=sys.stderr)
        sys.exit(1)
    if args.format == "id":
        if not args.model:
            print("Error: --model required for ID output", file=sys.stderr)
            sys.exit(1)
        if tokenizer.model is None:
            print(f"Error: Failed to load model from {args.model}", file=sys.stderr)
            print("  Make sure the model file exists and is valid.", file=sys.stderr)
            sys.exit(1)
        try:
            ids = tokenizer.encode(text)
            output = " ".join(map(str, ids))
        except ValueError as e:
            print(f"Error: {e}", file=sys.stderr)
            sys.exit(1)
    else:
        tokens = tokenizer.tokenize(text)
        if args.format == "json":
            output = json.dumps(tokens, ensure_ascii=False, indent=2)
        else:
            output = " ".join(tokens)
    if args.output:
        with open(args.output, "w", encoding="utf-8") as f:
            f.write(output)
    else:
        print(output)


def detokenize_command(args):
    """cli.py:93-128."""
    tokenizer = aksharTokenizer(model_path=args.model, model_type=args.model_type)
    if args.input:
        with open(args.input, "r", encoding="utf-8") as f:
            content = f.read()
            try:
                tokens = json.loads(content)
            except json.JSONDecodeError:
                tokens = content.split()
    else:
        tokens = args.tokens.split()
    text = tokenizer.detokenize(tokens)
    if args.output:
        with open(args.output, "w", encoding="utf-8") as f:
            f.write(text)
    else:
        print(text)


def explain_command(args):
    """cli.py:131-162."""
    tokenizer = aksharTokenizer(model_path=args.model, model_type=args.model_type)
    analysis = tokenizer.explain(args.text)
    print("\n=== akshar Analysis ===\n")
    print(f"Original: {analysis['original']}")
    print(f"Normalized: {analysis['normalized']}")
    print(f"\nakshars ({len(analysis['akshars'])}):")
    print("  " + " | ".join(analysis["akshars"]))
    print(f"\nCode Switches ({len(analysis['code_switches'])}):")
    for segment, script in analysis["code_switches"]:
        print(f"  [{script:12}] {segment!r}")
    print(f"\nTokens ({len(analysis['tokens'])}):")
    print("  " + " | ".join(analysis["tokens"]))
    print("\nStatistics:")
    for key, value in analysis["stats"].items():
        if isinstance(value, float):
            print(f"  {key}: {value:.2%}" if "ratio" in key else f"  {key}: {value:.2f}")
        else:
            print(f"  {key}: {value}")


def preprocess_corpus(input_file, output_file):
    """cli.py:165-190: normalize_text of every stripped non-empty line (one GPU batch)."""
    from .normalize import normalize_batch
    print(f"Preprocessing {input_file}...")
    with open(input_file, "r", encoding="utf-8") as f:
        lines = f.readlines()
    kept = [ln.strip() for ln in lines]
    kept = [ln for ln in kept if ln]
    processed = normalize_batch(kept)
    with open(output_file, "w", encoding="utf-8") as f:
        for line in processed:
            f.write(line + "\n")
    print(f"Wrote {len(processed)} lines to {output_file}")
    return str(output_file)


def preprocess_command(args):
    preprocess_corpus(args.input, args.output)


def build_parser():
    """cli.py:305-357 (the train subcommand excepted: offline, the reference's own trainer)."""
    parser = argparse.ArgumentParser(
        description="akshar: Linguistically-aware tokenizer for Hindi, Sanskrit, and Hinglish")
    sub = parser.add_subparsers(dest="command", help="Available commands")
    tp = sub.add_parser("tokenize", help="Tokenize text")
    tp.add_argument("text", nargs="?", help="Text to tokenize")
    tp.add_argument("-i", "--input", help="Input file")
    tp.add_argument("-o", "--output", help="Output file")
    tp.add_argument("-m", "--model", help="Path to trained model")
    tp.add_argument("--model-type", default="sentencepiece", choices=["sentencepiece", "bpe"])
    tp.add_argument("--format", default="text", choices=["text", "json", "id"],
                    help="Output format: text (tokens), json, or id (token IDs, requires --model)")
    dp = sub.add_parser("detokenize", help="Detokenize tokens")
    dp.add_argument("tokens", nargs="?", help="Space-separated tokens")
    dp.add_argument("-i", "--input", help="Input file (tokens)")
    dp.add_argument("-o", "--output", help="Output file")
    dp.add_argument("-m", "--model", help="Path to trained model")
    dp.add_argument("--model-type", default="sentencepiece", choices=["sentencepiece", "bpe"])
    ep = sub.add_parser("explain", help="Analyze text in detail")
    ep.add_argument("text", help="Text to analyze")
    ep.add_argument("-m", "--model", help="Path to trained model")
    ep.add_argument("--model-type", default="sentencepiece", choices=["sentencepiece", "bpe"])
    pp = sub.add_parser("preprocess", help="Normalize a corpus file line by line (the trainer's preprocessing)")
    pp.add_argument("input", help="Input corpus file")
    pp.add_argument("output", help="Output file")
    return parser


def main(argv=None):
    args = build_parser().parse_args(argv)
    if not args.command:
        build_parser().print_help()
        sys.exit(1)
    {"tokenize": tokenize_command, "detokenize": detokenize_command, "explain": explain_command,
     "preprocess": preprocess_command}[args.command](args)


if __name__ == "__main__":
    main()
