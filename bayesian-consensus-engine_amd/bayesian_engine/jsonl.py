"""Batched JSON front end: many payloads -> one CSR -> one launch.

The reference handles one payload per CLI call (cli.py:25-52: ``json.load`` ->
``validate_input_payload`` -> ``compute_consensus`` -> ``json.dumps(indent=2)``).  Here a
whole JSONL batch goes through the same steps with the per-signal work batched:

* parse + structural checks on the host (core.py:34-58 via :func:`core.check_structure`);
* ONE ``bce_validate_csr`` launch for the range check of every payload (core.py:59-60);
* source ids of every valid payload interned once in code-point order (Python ``sorted``,
  core.py:103), so a market's ranks sort exactly like its ids;
* ONE consensus launch (length-binned plan) over the CSR of all markets;
* each result rendered as ``json.dumps(indent=2)`` would (:func:`render`, a fixed-shape
  formatter: byte-identical, ~10x faster than the pure-Python indenting encoder) -- what
  the single-payload CLI prints for that payload.

All payloads of a batch share one ``source_reliability`` dict (the CLI's no-``--db`` path
uses none: every source cold).  A non-numeric reliability/confidence in it raises the same
TypeError as compute_consensus would, for the whole batch.
"""
from __future__ import annotations

import json
from json.encoder import encode_basestring_ascii as _q
from typing import Any, Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _native as N
from . import batch
from .config import DEFAULT_CONFIDENCE, DEFAULT_RELIABILITY, SCHEMA_VERSION
from .core import ValidationError, _as_float, _check_number, _no_signals, check_structure

__all__ = ["consensus_many", "consensus_jsonl", "parse_batch", "render"]

_INF = float("inf")
_TOP = ["schemaVersion", "consensus", "confidence", "sourceWeights", "normalization", "diagnostics"]
_DIAG = ["status", "sources", "uniqueSources", "coldStartSources"]
_SW = ["sourceId", "weight", "normalizedWeight"]


def _num(x) -> str:
    """json.dumps' rendering of a number / None (json/encoder.py floatstr, allow_nan)."""
    if x is None:
        return "null"
    if x is True:
        return "true"
    if x is False:
        return "false"
    if isinstance(x, int):
        return int.__repr__(x)
    if x != x:
        return "NaN"
    if x == _INF:
        return "Infinity"
    if x == -_INF:
        return "-Infinity"
    return float.__repr__(x)


def render(r: dict) -> str:
    """``json.dumps(r, indent=2)`` for a compute_consensus result, byte for byte, without
    the pure-Python indenting encoder (it dominated the batch: ~80 us per payload).  Any
    dict not of the exact computed-result shape goes through json.dumps itself."""
    d = r.get("diagnostics")
    if (list(r) != _TOP or not isinstance(d, dict) or d.get("status") != "computed"
            or list(d)[:4] != _DIAG or len(d) > 5 or (len(d) == 5 and list(d)[4] != "dryRun")
            or list(r["normalization"]) != ["totalWeight", "sourceCount"] or r["schemaVersion"] != SCHEMA_VERSION):
        return json.dumps(r, indent=2)
    sw = r["sourceWeights"]
    if any(list(w) != _SW for w in sw):
        return json.dumps(r, indent=2)
    if sw:
        sws = "[\n" + ",\n".join(
            '    {\n      "sourceId": %s,\n      "weight": %s,\n      "normalizedWeight": %s\n    }'
            % (_q(w["sourceId"]), _num(w["weight"]), _num(w["normalizedWeight"])) for w in sw) + "\n  ]"
    else:
        sws = "[]"
    cold = d["coldStartSources"]
    cs = ("[\n" + ",\n".join("      " + _q(c) for c in cold) + "\n    ]") if cold else "[]"
    tail = (',\n    "dryRun": ' + _num(d["dryRun"])) if len(d) == 5 else ""
    nm = r["normalization"]
    return ('{\n  "schemaVersion": "%s",\n  "consensus": %s,\n  "confidence": %s,\n  "sourceWeights": %s,\n'
            '  "normalization": {\n    "totalWeight": %s,\n    "sourceCount": %s\n  },\n'
            '  "diagnostics": {\n    "status": "computed",\n    "sources": %s,\n    "uniqueSources": %s,\n'
            '    "coldStartSources": %s%s\n  }\n}'
            % (SCHEMA_VERSION, _num(r["consensus"]), _num(r["confidence"]), sws, _num(nm["totalWeight"]),
               _num(nm["sourceCount"]), _num(d["sources"]), _num(d["uniqueSources"]), cs, tail))


def consensus_many(signal_lists: Sequence[list], source_reliability: Optional[dict] = None, *,
                   mode: str = "exact") -> List[dict]:
    """``[compute_consensus(s, source_reliability) for s in signal_lists]`` in one launch."""
    M = len(signal_lists)
    if M == 0:
        return []
    sr = source_reliability or {}
    lens = np.fromiter((len(sig) for sig in signal_lists), np.int64, M)
    off = np.zeros(M + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    Ns = int(off[-1])
    if Ns == 0:
        return [_no_signals() for _ in range(M)]

    ids = [s["sourceId"] for sig in signal_lists for s in sig]
    raw = [s["probability"] for sig in signal_lists for s in sig]
    names = sorted(set(ids))
    rank = dict(zip(names, range(len(names))))
    sid = np.fromiter(map(rank.__getitem__, ids), np.int32, Ns)
    if set(map(type, raw)) == {float}:  # the JSON common case: one C-level conversion
        prob = np.array(raw, np.float64)
    else:
        for p in raw:
            if not isinstance(p, (int, float)):
                0 + p  # noqa: B018  -- builtin sum()'s TypeError (core.py:116)
        prob = np.fromiter((_as_float(p) for p in raw), np.float64, Ns)
    rel_objs = []
    for n in names:
        d = sr.get(n, {})
        r = d.get("reliability", DEFAULT_RELIABILITY)
        c = d.get("confidence", DEFAULT_CONFIDENCE)
        _check_number(r, None)
        if not isinstance(c, (int, float)):
            c * r  # noqa: B018  -- the reference's TypeError at core.py:142
        rel_objs.append(r)

    N.require_gpu()
    dev = N.device()
    T = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    table = batch.SourceTable.from_dict(names, sr, dev)
    max_len = int(lens.max())
    plan = None if max_len <= 64 else batch.Plan.build(off, dev)
    res = batch.consensus(T(off), T(sid), T(prob), table, plan=plan,
                          max_len=max_len if plan is None else None, mode=mode, validate=False,
                          check=True)
    # one device->host copy per array, then plain lists (numpy scalar/slice access per
    # market cost more than the whole launch)
    cons = res.consensus.cpu().tolist()
    conf = res.confidence.cpu().tolist()
    total = res.total_weight.cpu().tolist()
    nu = res.n_unique.cpu().tolist()
    usid = res.usid[:Ns].cpu().numpy()
    rank_all = (usid & 0x7FFFFFFF).tolist()
    cold_all = (usid < 0).tolist()
    nweight = res.nweight[:Ns].cpu().tolist()
    offl = off.tolist()

    out = []
    for m in range(M):
        o = offl[m]
        n = offl[m + 1] - o
        if n == 0:
            out.append(_no_signals())
            continue
        S = nu[m]
        rk = rank_all[o:o + S]
        null = total[m] == 0  # core.py:131
        out.append({
            "schemaVersion": SCHEMA_VERSION,
            "consensus": None if null else cons[m],
            "confidence": 0.0 if null else conf[m],
            "sourceWeights": [{"sourceId": names[r], "weight": rel_objs[r], "normalizedWeight": w}
                              for r, w in zip(rk, nweight[o:o + S])],
            "normalization": {"totalWeight": total[m], "sourceCount": S},
            "diagnostics": {
                "status": "computed",
                "sources": n,
                "uniqueSources": S,
                "coldStartSources": [names[r] for r, c in zip(rk, cold_all[o:o + S]) if c],
            },
        })
    return out


def parse_batch(lines: Iterable[str]) -> Tuple[List[Any], List[Optional[str]], List[list],
                                                 List[Optional[ValidationError]]]:
    """Host pass: per non-blank line the payload (or None), its header/JSON error text (or
    None), the probabilities to range-check and the first signal-level type error."""
    payloads, errors, probs, type_errors = [], [], [], []
    for line in lines:
        if not line.strip():
            continue
        try:
            payload = json.loads(line)
            p, te = check_structure(payload)
        except (json.JSONDecodeError, ValidationError, TypeError) as exc:
            # a JSON scalar (5, null, true) is not a payload: the reference's single-payload
            # CLI dies on it with this TypeError; the batch reports it for that line only
            payloads.append(None)
            errors.append(f"TypeError: {exc}" if isinstance(exc, TypeError) else f"Validation error: {exc}")
            probs.append([])
            type_errors.append(None)
            continue
        payloads.append(payload)
        errors.append(None)
        probs.append(p)
        type_errors.append(te)
    return payloads, errors, probs, type_errors


def consensus_jsonl(lines: Iterable[str], source_reliability: Optional[dict] = None, *,
                    dry_run: bool = False, mode: str = "exact") -> List[Tuple[bool, str]]:
    """One ``(ok, text)`` per non-blank JSONL line: ``text`` is what ``bayesian-engine
    consensus`` prints for that payload alone -- the ``json.dumps(indent=2)`` result on
    success, the ``Validation error: ...`` line otherwise (cli.py:46-52)."""
    payloads, errors, probs, type_errors = parse_batch(lines)
    M = len(payloads)
    lens = np.fromiter((len(p) for p in probs), np.int64, M)
    if M and lens.sum() > 0:  # one range-check launch for the whole batch (core.py:59-60)
        N.require_gpu()
        dev = N.device()
        off = np.zeros(M + 1, np.int64)
        np.cumsum(lens, out=off[1:])
        flat = np.fromiter((x for p in probs for x in p), np.float64, int(off[-1]))
        err = batch.validate(torch.from_numpy(off).to(dev), torch.from_numpy(flat).to(dev)).cpu().numpy()
        for i in range(M):
            if errors[i] is None and err[i] >= 0:
                errors[i] = f"Validation error: signals[{int(err[i])}].probability must be between 0 and 1"
    for i in range(M):
        if errors[i] is None and type_errors[i] is not None:
            errors[i] = f"Validation error: {type_errors[i]}"

    ok = [i for i in range(M) if errors[i] is None]
    results = consensus_many([payloads[i]["signals"] for i in ok], source_reliability, mode=mode)
    texts: List[Tuple[bool, str]] = [(False, e) if e is not None else (True, "") for e in errors]
    for i, r in zip(ok, results):
        if dry_run:
            r["diagnostics"]["dryRun"] = True
        texts[i] = (True, render(r))
    return texts
