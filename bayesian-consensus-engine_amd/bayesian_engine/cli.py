"""Drop-in for ``bayesian_engine.cli`` (reference src/bayesian_engine/cli.py:1-178).

Same argparse surface (global --db/--dry-run/--input; subcommands consensus,
report-outcome, list-sources; no subcommand = legacy consensus), same JSON on stdout
(``json.dumps(indent=2)``) and the same error text on stderr / exit code 1.  It is a
caller of the hot path: validation, consensus, decay and outcome updates run in the
HIP engine through the drop-in modules.
"""
from __future__ import annotations

import argparse
import json
import sys
from typing import Any

from .core import ValidationError, compute_consensus, validate_input_payload
from .reliability import SQLiteReliabilityStore


def _load_input(input_path: str | None) -> dict[str, Any]:
    if input_path:
        with open(input_path, "r", encoding="utf-8") as f:
            return json.load(f)
    if sys.stdin.isatty():
        raise ValidationError("Input required: provide --input <file> or JSON via stdin")
    return json.load(sys.stdin)


def _cmd_consensus(args: argparse.Namespace) -> None:
    try:
        payload = _load_input(args.input)
        validate_input_payload(payload)
        source_reliability = None
        if args.db:
            with SQLiteReliabilityStore(args.db) as store:
                source_reliability = {}
                for signal in payload.get("signals", []):
                    source_id = signal.get("sourceId")
                    if source_id:
                        rec = store.get_reliability(source_id, payload["marketId"], apply_decay=True)
                        source_reliability[source_id] = {"reliability": rec.reliability,
                                                         "confidence": rec.confidence}
        result = compute_consensus(payload["signals"], source_reliability)
        if args.dry_run:
            result["diagnostics"]["dryRun"] = True
        print(json.dumps(result, indent=2))
    except (json.JSONDecodeError, ValidationError) as exc:
        print(f"Validation error: {exc}", file=sys.stderr)
        raise SystemExit(1) from exc


def _cmd_consensus_batch(args: argparse.Namespace) -> None:
    """Build-defined: a JSONL file of payloads, one consensus launch for all.
    Prints, per line, exactly what ``consensus`` prints for that payload alone (results on
    stdout, ``Validation error: ...`` on stderr); exit 1 if any line failed.  Sources are
    cold (no ``--db`` lookup), as in the legacy path."""
    from .jsonl import consensus_jsonl

    if args.input:
        with open(args.input, "r", encoding="utf-8") as f:
            lines = f.readlines()
    else:
        lines = sys.stdin.readlines()
    failed = False
    for ok, text in consensus_jsonl(lines, dry_run=args.dry_run):
        print(text, file=sys.stdout if ok else sys.stderr)
        failed |= not ok
    if failed:
        raise SystemExit(1)


def _cmd_report_outcome(args: argparse.Namespace) -> None:
    if not args.db:
        print("Error: --db is required for report-outcome", file=sys.stderr)
        raise SystemExit(1)
    try:
        with SQLiteReliabilityStore(args.db) as store:
            result = store.update_reliability(source_id=args.source_id, market_id=args.market_id,
                                              outcome_correct=args.correct, dry_run=args.dry_run)
        output = {"sourceId": result.source_id, "marketId": result.market_id, "reliability": result.reliability,
                  "confidence": result.confidence, "updatedAt": result.updated_at, "dryRun": args.dry_run}
        print(json.dumps(output, indent=2))
    except Exception as exc:  # noqa: BLE001  -- reference behaviour (cli.py:79-81)
        print(f"Error: {exc}", file=sys.stderr)
        raise SystemExit(1) from exc


def _cmd_list_sources(args: argparse.Namespace) -> None:
    if not args.db:
        print("Error: --db is required for list-sources", file=sys.stderr)
        raise SystemExit(1)
    try:
        with SQLiteReliabilityStore(args.db) as store:
            sources = store.list_sources(market_id=args.market_id)
        output = {"sources": [{"sourceId": s.source_id, "marketId": s.market_id, "reliability": s.reliability,
                               "confidence": s.confidence, "updatedAt": s.updated_at} for s in sources],
                  "count": len(sources)}
        print(json.dumps(output, indent=2))
    except Exception as exc:  # noqa: BLE001
        print(f"Error: {exc}", file=sys.stderr)
        raise SystemExit(1) from exc


def main() -> None:
    parser = argparse.ArgumentParser(prog="bayesian-engine",
                                     description="Bayesian-weighted consensus engine with reliability tracking")
    parser.add_argument("--db", type=str, help="Path to SQLite database file (default: in-memory)")
    parser.add_argument("--dry-run", action="store_true", help="Compute without persisting changes (zero DB writes)")
    parser.add_argument("--input", type=str, help="Path to JSON input file (for consensus command)")
    subparsers = parser.add_subparsers(dest="command", help="Available commands")
    consensus_parser = subparsers.add_parser("consensus", help="Compute consensus from signals")
    consensus_parser.add_argument("--input", help="Path to JSON input file")
    consensus_parser.set_defaults(func=_cmd_consensus)
    batch_parser = subparsers.add_parser("consensus-batch", help="Compute consensus for a JSONL batch of payloads")
    batch_parser.add_argument("--input", help="Path to JSONL input file (one payload per line)")
    batch_parser.set_defaults(func=_cmd_consensus_batch)
    outcome_parser = subparsers.add_parser("report-outcome", help="Report outcome and update reliability")
    outcome_parser.add_argument("--source-id", required=True, help="Source identifier")
    outcome_parser.add_argument("--market-id", required=True, help="Market identifier")
    outcome_parser.add_argument("--correct", action="store_true", help="Outcome was correct")
    outcome_parser.set_defaults(func=_cmd_report_outcome)
    list_parser = subparsers.add_parser("list-sources", help="List sources with reliability data")
    list_parser.add_argument("--market-id", help="Filter by market ID")
    list_parser.set_defaults(func=_cmd_list_sources)
    args = parser.parse_args()
    if args.command is None:
        _cmd_consensus_legacy(args)
    else:
        args.func(args)


def _cmd_consensus_legacy(args: argparse.Namespace) -> None:
    try:
        payload = _load_input(args.input)
        validate_input_payload(payload)
        result = compute_consensus(payload["signals"])
        if args.dry_run:
            result["diagnostics"]["dryRun"] = True
        print(json.dumps(result, indent=2))
    except (json.JSONDecodeError, ValidationError) as exc:
        print(f"Validation error: {exc}", file=sys.stderr)
        raise SystemExit(1) from exc


if __name__ == "__main__":
    main()
