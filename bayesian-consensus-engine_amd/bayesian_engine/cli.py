"""``bayesian-engine`` command line -- a caller of the hot path (reference
src/bayesian_engine/cli.py:1-178 defines the surface this keeps).

Kept from the reference, byte for byte: the argparse surface (global --db/--dry-run/--input;
subcommands consensus, report-outcome, list-sources; no subcommand = the legacy consensus
path that never consults the store), the JSON on stdout (``json.dumps(indent=2)``), the
error text on stderr and exit status 1.  The reference quirk that a global ``--input``
placed before ``consensus`` is replaced by the subcommand's own default (cli.py:138) holds
too, because the subcommand declares its own ``--input``.

Added: ``consensus-batch`` -- a JSONL file of payloads, one engine launch for the batch
(SURVEY.md §8(f) f2), printing per line what ``consensus`` prints for that payload alone.

Structure: every consensus flavour goes through :func:`_consensus`; the store-backed
commands share :func:`_with_store`; the parser is built from the :data:`COMMANDS` table.
"""
from __future__ import annotations

import argparse
import json
import sys
from typing import Any, Callable, Dict, Iterable, List, Optional, Tuple

from .core import ValidationError, compute_consensus, validate_input_payload
from .reliability import SQLiteReliabilityStore


def _emit(obj: Any) -> None:
    print(json.dumps(obj, indent=2))


def _fail(message: str, cause: Optional[BaseException] = None) -> None:
    print(message, file=sys.stderr)
    raise SystemExit(1) from cause


def _read_payload(path: Optional[str]) -> Dict[str, Any]:
    """--input file, else JSON on a non-terminal stdin (cli.py:14-22)."""
    if path:
        with open(path, "r", encoding="utf-8") as fh:
            return json.load(fh)
    if sys.stdin.isatty():
        raise ValidationError("Input required: provide --input <file> or JSON via stdin")
    return json.load(sys.stdin)


def _store_reliability(db: str, payload: Dict[str, Any]) -> Dict[str, Dict[str, float]]:
    """Every signal's source looked up (decayed) in the store: cli.py:35-44."""
    market_id = payload["marketId"]
    table: Dict[str, Dict[str, float]] = {}
    with SQLiteReliabilityStore(db) as store:
        for signal in payload.get("signals", []):
            sid = signal.get("sourceId")
            if sid:
                rec = store.get_reliability(sid, market_id, apply_decay=True)
                table[sid] = {"reliability": rec.reliability, "confidence": rec.confidence}
    return table


def _consensus(args: argparse.Namespace, use_store: bool) -> None:
    """Load -> validate -> (store lookup) -> compute -> print, shared by the legacy path
    (use_store=False: the reference ignores --db there, cli.py:163-174) and ``consensus``."""
    try:
        payload = _read_payload(args.input)
        validate_input_payload(payload)
        reliability = _store_reliability(args.db, payload) if (use_store and args.db) else None
        result = compute_consensus(payload["signals"], reliability)
        if args.dry_run:
            result["diagnostics"]["dryRun"] = True
        _emit(result)
    except (json.JSONDecodeError, ValidationError) as exc:
        _fail(f"Validation error: {exc}", exc)


def _consensus_batch(args: argparse.Namespace) -> None:
    if args.input:
        with open(args.input, "r", encoding="utf-8") as fh:
            lines = fh.readlines()
    else:
        lines = sys.stdin.readlines()
    # the native front end (csrc/jsonl.cpp) renders every result; runs of results go to
    # stdout as bytes (they are ASCII: ids are \u-escaped), error lines through print() in
    # line order, as the per-line loop would write them
    from .jsonl import _consensus_jsonl_native

    texts, _ = _consensus_jsonl_native([ln for ln in lines if ln.strip()], None, dry_run=args.dry_run,
                                       mode="exact")
    failed = False
    run: list = []
    for ok, text in texts:
        if ok:
            run.append(text)
            continue
        if run:
            _write_out(run)
            run = []
        print(text.decode("utf-8", "surrogatepass"), file=sys.stderr)
        failed = True
    if run:
        _write_out(run)
    if failed:
        raise SystemExit(1)


def _write_out(texts: list) -> None:
    """The rendered results (ASCII bytes) to stdout: its byte buffer when it has one, else as
    text (a redirect_stdout(StringIO()) or an embedding host)."""
    data = b"\n".join(texts) + b"\n"
    out = sys.stdout
    if hasattr(out, "buffer"):
        out.flush()
        out.buffer.write(data)
        out.buffer.flush()
    else:
        out.write(data.decode("ascii"))


def _with_store(command: str, body: Callable[[argparse.Namespace, SQLiteReliabilityStore], Any]):
    """report-outcome / list-sources: --db required, any failure -> 'Error: ...', rc 1."""

    def run(args: argparse.Namespace) -> None:
        if not args.db:
            _fail(f"Error: --db is required for {command}")
        try:
            with SQLiteReliabilityStore(args.db) as store:
                out = body(args, store)
            _emit(out)
        except Exception as exc:  # noqa: BLE001 -- the reference catches everything (cli.py:79-81)
            _fail(f"Error: {exc}", exc)

    return run


def _record(rec, *, dry_run: Optional[bool] = None) -> Dict[str, Any]:
    d = {"sourceId": rec.source_id, "marketId": rec.market_id, "reliability": rec.reliability,
         "confidence": rec.confidence, "updatedAt": rec.updated_at}
    if dry_run is not None:
        d["dryRun"] = dry_run
    return d


def _report_outcome(args, store):
    rec = store.update_reliability(source_id=args.source_id, market_id=args.market_id,
                                   outcome_correct=args.correct, dry_run=args.dry_run)
    return _record(rec, dry_run=args.dry_run)


def _list_sources(args, store):
    rows = store.list_sources(market_id=args.market_id)
    return {"sources": [_record(r) for r in rows], "count": len(rows)}


Arg = Tuple[Tuple[str, ...], Dict[str, Any]]

GLOBAL_ARGS: List[Arg] = [
    (("--db",), dict(type=str, help="Path to SQLite database file (default: in-memory)")),
    (("--dry-run",), dict(action="store_true", help="Compute without persisting changes (zero DB writes)")),
    (("--input",), dict(type=str, help="Path to JSON input file (for consensus command)")),
]

# name -> (help, arguments, handler)
COMMANDS: Dict[str, Tuple[str, List[Arg], Callable[[argparse.Namespace], None]]] = {
    "consensus": ("Compute consensus from signals",
                  [(("--input",), dict(help="Path to JSON input file"))],
                  lambda a: _consensus(a, use_store=True)),
    "consensus-batch": ("Compute consensus for a JSONL batch of payloads",
                        [(("--input",), dict(help="Path to JSONL input file (one payload per line)"))],
                        _consensus_batch),
    "report-outcome": ("Report outcome and update reliability",
                       [(("--source-id",), dict(required=True, help="Source identifier")),
                        (("--market-id",), dict(required=True, help="Market identifier")),
                        (("--correct",), dict(action="store_true", help="Outcome was correct"))],
                       _with_store("report-outcome", _report_outcome)),
    "list-sources": ("List sources with reliability data",
                     [(("--market-id",), dict(help="Filter by market ID"))],
                     _with_store("list-sources", _list_sources)),
}


def _add(parser: argparse.ArgumentParser, specs: Iterable[Arg]) -> None:
    for flags, kw in specs:
        parser.add_argument(*flags, **kw)


def build_parser() -> argparse.ArgumentParser:
    parser = argparse.ArgumentParser(prog="bayesian-engine",
                                     description="Bayesian-weighted consensus engine with reliability tracking")
    _add(parser, GLOBAL_ARGS)
    sub = parser.add_subparsers(dest="command", help="Available commands")
    for name, (help_text, specs, handler) in COMMANDS.items():
        p = sub.add_parser(name, help=help_text)
        _add(p, specs)
        p.set_defaults(func=handler)
    return parser


def main(argv: Optional[List[str]] = None) -> None:
    args = build_parser().parse_args(argv)
    if args.command is None:
        _consensus(args, use_store=False)  # legacy path (cli.py:156-158)
    else:
        args.func(args)


if __name__ == "__main__":
    main()
