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

__all__ = ["consensus_many", "consensus_jsonl", "consensus_jsonl_bytes", "parse_batch", "render"]

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
                    dry_run: bool = False, mode: str = "exact", native: bool = True) -> List[Tuple[bool, str]]:
    """One ``(ok, text)`` per non-blank JSONL line: ``text`` is what ``bayesian-engine
    consensus`` prints for that payload alone -- the ``json.dumps(indent=2)`` result on
    success, the ``Validation error: ...`` line otherwise (cli.py:46-52).

    ``native`` (default): parsing, structure checks, interning and rendering run in the
    library's C++ front end on host threads (csrc/jsonl.cpp); a line it does not reproduce
    exactly (malformed JSON, a non-object payload, a non-string schemaVersion, a line with
    an embedded newline) goes through the Python path below on its own.  Both paths give
    byte-identical texts."""
    lines = [ln for ln in lines if ln.strip()]  # parse_batch skips blank lines
    if not native:
        return _consensus_jsonl_py(lines, source_reliability, dry_run=dry_run, mode=mode)
    texts, _ = _consensus_jsonl_native(lines, source_reliability, dry_run=dry_run, mode=mode)
    return [(bool(ok), t.decode("utf-8", "surrogatepass")) for ok, t in texts]


def consensus_jsonl_bytes(lines: Sequence[str], source_reliability: Optional[dict] = None, *,
                          dry_run: bool = False, mode: str = "exact") -> Tuple[bytes, bytes, bool]:
    """What ``consensus-batch`` writes: (stdout bytes, stderr bytes, any line failed) -- each
    text plus a newline, in line order, without building a Python string per result."""
    lines = [ln for ln in lines if ln.strip()]
    texts, _ = _consensus_jsonl_native(lines, source_reliability, dry_run=dry_run, mode=mode)
    out = b"".join(t + b"\n" for ok, t in texts if ok)
    err = b"".join(t + b"\n" for ok, t in texts if not ok)
    return out, err, len(err) > 0


def _threads() -> int:
    import os
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


class _NativeBatch:
    """A parsed batch (bce_jsonl_parse) and its arrays on the host."""

    def __init__(self, text: bytes, threads: int):
        import ctypes as C
        self._L = N.lib()
        h = C.c_void_p()
        N.check(self._L.bce_jsonl_parse(text, len(text), threads, C.byref(h)), "bce_jsonl_parse")
        self.h = h
        cnt = np.zeros(4, np.int64)
        N.check(self._L.bce_jsonl_counts(h, N.ptr(cnt)), "bce_jsonl_counts")
        nl, nv, nn, nb = (int(x) for x in cnt)
        self.kind = np.empty(nl, np.int32)
        self.type_err = np.empty(nl, np.int32)
        self.n_signals = np.empty(nl, np.int32)
        self.voff = np.empty(nl + 1, np.int64)
        self.prob = np.empty(max(nv, 1), np.float64)
        self.sid = np.empty(max(nv, 1), np.int32)
        self._names = np.empty(max(nb, 1), np.uint8)
        self.name_off = np.empty(nn + 1, np.int64)
        N.check(self._L.bce_jsonl_arrays(h, N.ptr(self.kind), N.ptr(self.type_err), N.ptr(self.n_signals), None,
                                         N.ptr(self.voff), N.ptr(self.prob), N.ptr(self.sid), N.ptr(self._names),
                                         N.ptr(self.name_off)), "bce_jsonl_arrays")
        self.n_lines, self.n_checked, self.n_names = nl, nv, nn

    def names(self) -> List[str]:
        raw, o = self._names.tobytes(), self.name_off.tolist()
        return [raw[o[i]:o[i + 1]].decode("utf-8", "surrogatepass") for i in range(self.n_names)]

    def __del__(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self._L.bce_jsonl_free(self.h)
            self.h = None


def _weight_texts(nb: "_NativeBatch", sr: dict, used: np.ndarray):
    """Per interned name: json.dumps of its weight object (reliability, or the default 0.5 --
    an int stays an int, core.py:111,119), and the host table rows; the reference's
    TypeError for a non-numeric value of a name some computed market uses."""
    S = nb.n_names
    if not sr:
        return (b"0.5" * S, np.arange(S + 1, dtype=np.int64) * 3, np.full(S, DEFAULT_RELIABILITY),
                np.full(S, DEFAULT_CONFIDENCE), np.zeros(S, np.uint8), None)
    names = nb.names()
    rel, conf, present = np.empty(S), np.empty(S), np.zeros(S, np.uint8)
    parts = []
    usedset = set(used.tolist())
    for i, n in enumerate(names):
        d = sr.get(n, {})
        if i not in usedset and not isinstance(d, dict):
            # a name only failed lines use: the reference never looks it up (core.py:110 runs
            # for computed payloads only), so its entry's shape cannot raise
            d = {}
        r = d.get("reliability", DEFAULT_RELIABILITY)
        c = d.get("confidence", DEFAULT_CONFIDENCE)
        if i in usedset:
            _check_number(r, None)
            if not isinstance(c, (int, float)):
                c * r  # noqa: B018  -- the reference's TypeError at core.py:142
        ok_r, ok_c = isinstance(r, (int, float)), isinstance(c, (int, float))
        rel[i] = _as_float(r) if ok_r else DEFAULT_RELIABILITY
        conf[i] = _as_float(c) if ok_c else DEFAULT_CONFIDENCE
        present[i] = n in sr
        parts.append(_num(r).encode() if ok_r else b"null")
    off = np.zeros(S + 1, np.int64)
    np.cumsum([len(x) for x in parts], out=off[1:])
    return b"".join(parts), off, rel, conf, present, names


def _consensus_jsonl_native(lines: List[str], source_reliability: Optional[dict], *, dry_run: bool,
                            mode: str) -> Tuple[List[Tuple[bool, bytes]], int]:
    """The native front end over `lines` (non-blank); returns ((ok, text bytes) per line,
    number of lines the Python path handled)."""
    import ctypes as C
    M = len(lines)
    if M == 0:
        return [], 0
    bodies, py_idx = [], []
    for i, ln in enumerate(lines):
        b = ln[:-1] if ln.endswith("\n") else ln
        if "\n" in b:
            py_idx.append(i)  # a payload spanning lines: json.loads of the whole string
        else:
            bodies.append(b)
    skip = set(py_idx)
    nat_idx = [i for i in range(M) if i not in skip] if skip else list(range(M))
    text = "\n".join(bodies).encode("utf-8", "surrogatepass")
    T = _threads()
    nb = _NativeBatch(text, T)
    if nb.n_lines != len(bodies):
        raise RuntimeError(f"bce_jsonl_parse split {nb.n_lines} lines, expected {len(bodies)}")
    L = nb.n_lines
    err = np.full(L, -1, np.int32)
    if nb.n_checked > 0:  # one range-check launch for the whole batch (core.py:59-60)
        N.require_gpu()
        dev = N.device()
        err = batch.validate(torch.from_numpy(nb.voff).to(dev),
                             torch.from_numpy(nb.prob[:nb.n_checked]).to(dev)).cpu().numpy().astype(np.int32)
    rows = np.nonzero((nb.kind == 0) & (err < 0) & (nb.type_err < 0) & (nb.n_signals > 0))[0]
    res_of = np.full(L, -1, np.int64)
    res_of[rows] = np.arange(len(rows))
    lens = (nb.voff[rows + 1] - nb.voff[rows]).astype(np.int64)
    roff = np.zeros(len(rows) + 1, np.int64)
    np.cumsum(lens, out=roff[1:])
    Ns = int(roff[-1])
    flat = np.repeat(nb.voff[rows] - roff[:-1], lens) + np.arange(Ns, dtype=np.int64)
    sid = nb.sid[flat] if Ns else np.zeros(1, np.int32)
    sr = source_reliability or {}
    wtext, wtext_off, rel, conf, present, names = _weight_texts(nb, sr, np.unique(sid[:Ns]) if Ns else sid[:0])
    R = len(rows)
    f64, i32 = np.float64, np.int32
    cons, confd, total = np.zeros(max(R, 1), f64), np.zeros(max(R, 1), f64), np.zeros(max(R, 1), f64)
    nu = np.zeros(max(R, 1), i32)
    usid, nweight = np.zeros(max(Ns, 1), i32), np.zeros(max(Ns, 1), f64)
    if R:
        N.require_gpu()
        dev = N.device()
        Tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        table = batch.SourceTable.from_arrays(Tt(rel), Tt(conf), Tt(present), names)
        max_len = int(lens.max())
        plan = None if max_len <= 64 else batch.Plan.build(roff, dev)
        res = batch.consensus(Tt(roff), Tt(sid[:Ns]), Tt(nb.prob[flat]), table, plan=plan,
                              max_len=max_len if plan is None else None, mode=mode, validate=False, check=True)
        cons, confd, total = res.consensus.cpu().numpy(), res.confidence.cpu().numpy(), res.total_weight.cpu().numpy()
        nu = res.n_unique.cpu().numpy()
        usid, nweight = res.usid[:Ns].cpu().numpy(), res.nweight[:Ns].cpu().numpy()
    wt = np.frombuffer(wtext, np.uint8) if wtext else np.zeros(1, np.uint8)
    n_bytes = C.c_int64(0)
    args = [nb.h, N.ptr(err), N.ptr(res_of), N.ptr(cons), N.ptr(confd), N.ptr(total), N.ptr(nu), N.ptr(roff),
            N.ptr(usid), N.ptr(nweight), N.ptr(wt), N.ptr(wtext_off), int(bool(dry_run)), T]
    N.check(nb._L.bce_jsonl_render(*args, None, None, None, C.byref(n_bytes)), "bce_jsonl_render")
    buf = np.empty(max(n_bytes.value, 1), np.uint8)
    toff = np.empty(L + 1, np.int64)
    okf = np.empty(max(L, 1), np.uint8)
    N.check(nb._L.bce_jsonl_render(*args, N.ptr(buf), N.ptr(toff), N.ptr(okf), C.byref(n_bytes)),
            "bce_jsonl_render")
    raw = buf.tobytes()
    to = toff.tolist()
    out: List[Optional[Tuple[bool, bytes]]] = [None] * M
    fb = []
    for j, i in enumerate(nat_idx):
        if nb.kind[j] == 2:
            fb.append(i)
        else:
            out[i] = (bool(okf[j]), raw[to[j]:to[j + 1]])
    py = sorted(fb + py_idx)
    if py:  # lines the native parser hands over: the Python path, on their own
        for i, (ok, t) in zip(py, _consensus_jsonl_py([lines[i] for i in py], source_reliability,
                                                      dry_run=dry_run, mode=mode)):
            out[i] = (ok, t.encode("utf-8", "surrogatepass"))
    return out, len(py)


def _consensus_jsonl_py(lines: Iterable[str], source_reliability: Optional[dict] = None, *,
                        dry_run: bool = False, mode: str = "exact") -> List[Tuple[bool, str]]:
    """The Python path: json.loads + check_structure per line, one validation launch, one
    consensus launch (consensus_many), render per result."""
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
