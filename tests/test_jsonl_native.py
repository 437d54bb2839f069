"""CPU tests of the native JSONL front end (csrc/jsonl.cpp).

The C++ parser must see each line exactly as ``json.loads`` + ``check_structure``
(core.py:34-58) do -- same structure/type errors in the same order, the same probabilities
(float(str), float(int), bool, NaN / Infinity), the same sourceIds (escapes, surrogates,
duplicate keys: last wins) interned in Python ``sorted`` order -- and hand every line it does
not reproduce (malformed JSON, non-object payloads, non-string schemaVersion) to the Python
path.  The renderer must print what ``json.dumps(result, indent=2)`` prints, byte for byte.
Consensus numbers come from the oracle's C restatement here (no GPU); the GPU suite runs the
same comparison through the kernels (tests/test_gpu_jsonl.py).
"""
import ctypes as C
import json
import math
import random
import struct

import numpy as np
import pytest

from golden_util import load_json


def _lib():
    from bayesian_engine import _native as N
    return N.lib()


def test_float_repr_matches_python():
    """put_repr (float.__repr__) on random bit patterns, decimal-looking values and edges."""
    L = _lib()
    buf = C.create_string_buffer(64)
    rng = np.random.default_rng(1)
    xs = [struct.unpack("<d", struct.pack("<Q", int(b)))[0] for b in rng.integers(0, 2**63, 3000, dtype=np.uint64)]
    xs += list(rng.random(2000)) + [float(f"{rng.random():.{k}g}") for k in range(1, 18) for _ in range(20)]
    xs += [0.0, -0.0, 1.0, 0.1, 1e16, 1e15, 9999999999999998.0, 1e-4, 1e-5, 0.0001234, 123456789012345678.0, 5e-324,
           1.7976931348623157e308, 2.2250738585072014e-308, 0.6966666666666667, 0.3333333333333333, 1e22, 1e23,
           float("nan"), float("inf"), -float("inf")]
    xs += [-x for x in xs]
    bad = []
    for x in xs:
        n = L.bce_debug_float_repr(x, buf, 64)
        got = buf.raw[:n].decode()
        exp = json.dumps(x)  # float.__repr__, with NaN / Infinity as json writes them
        if got != exp:
            bad.append((x, got, exp))
    assert not bad, bad[:5]


def _py_expect(lines):
    """What the Python path decides per line: (kind, message or None, probs, type_err index)."""
    from bayesian_engine.jsonl import parse_batch
    out = []
    for ln in lines:
        try:
            json.loads(ln)
        except Exception:  # noqa: BLE001
            out.append(None)  # malformed: Python path's own message
            continue
        payloads, errors, probs, tes = parse_batch([ln])
        out.append((payloads[0], errors[0], probs[0], tes[0]))
    return out


def _rand_id(rnd):
    pool = ["src", "a", "B", "Ä", "é", "☃", "\U0001f600", "x\"y", "tab\t", "back\\slash", "ctl\x01", "del\x7f",
            " ", " sp", "sp ", "\ud800", "\udfff", "z" * 30]
    return "".join(rnd.choice(pool) for _ in range(rnd.randint(1, 3)))


def _rand_line(rnd):
    """A payload line with a random mix of valid and invalid features (json.dumps-encoded or
    hand-written to reach literals json.dumps never emits)."""
    n = rnd.choice([0, 1, 2, 5, 30, 70])
    sig = []
    for i in range(n):
        s = {"sourceId": _rand_id(rnd), "probability": rnd.choice(
            [rnd.random(), 0.0, 1.0, 0, 1, True, False, 0.5, 1.5, -0.25, float("nan"), float("inf"),
             12345678901234567890123, rnd.random() * 1e-310, -0.0])}
        r = rnd.random()
        if r < 0.02:
            s = rnd.choice([[1], "str", None, 3])
        elif r < 0.04:
            del s["sourceId"]
        elif r < 0.06:
            s["sourceId"] = rnd.choice(["", "   ", "　", 5, None, " x"])
        elif r < 0.08:
            del s["probability"]
        elif r < 0.10:
            s["probability"] = rnd.choice(["0.5", None, [0.5], {"p": 1}])
        elif r < 0.12:
            s["extra"] = {"nested": [1, 2, {"deep": None}]}
        sig.append(s)
    p = {"schemaVersion": "1.0.0", "marketId": rnd.choice(["m-1", "mkt é", " x "]), "signals": sig}
    r = rnd.random()
    if r < 0.03:
        del p["schemaVersion"]
    elif r < 0.06:
        p["schemaVersion"] = rnd.choice(["1.0", "2.0.0", "1.0.0 ", "é1"])
    elif r < 0.08:
        del p["marketId"]
    elif r < 0.10:
        p["marketId"] = rnd.choice(["", "  ", " ", 7, None])
    elif r < 0.12:
        del p["signals"]
    elif r < 0.14:
        p["signals"] = rnd.choice([{"a": 1}, "x", 5, None])
    text = json.dumps(p, ensure_ascii=rnd.random() < 0.5)
    r = rnd.random()
    if r < 0.05:  # duplicate keys: the last one wins
        text = text[:-1] + ', "marketId": "dup", "signals": []}'
    elif r < 0.08:
        text = "  " + text + " \t\r"
    elif r < 0.10:
        text = text[:-1]  # malformed
    elif r < 0.12:
        text = text.replace('"probability": 0.5', '"probability": 5e-1', 1).replace('"probability": 1,',
                                                                                  '"probability": 1E0,', 1)
    elif r < 0.14:
        text = text.replace('"probability": 0,', '"probability": -0,', 1)
    return text


def test_native_parse_matches_json_loads_and_check_structure():
    from bayesian_engine import jsonl
    rnd = random.Random(11)
    lines = [_rand_line(rnd) for _ in range(3000)]
    lines += [json.dumps(c["payload"]) for c in load_json("validate_cases.json")]
    lines += ["{not json", '{"schemaVersion": 1}', "[1, 2]", '"str"', "5", '{"a": 1} x', '{"a": [1,]}',
              '{"schemaVersion": "1.0.0", "marketId": "m", "signals": [{"sourceId": "a", "probability": 01}]}',
              '{"schemaVersion": "1.0.0", "marketId": "m", "signals": [{"sourceId": "a", "probability": 1.}]}',
              '{"schemaVersion": "1.0.0", "marketId": "m", "signals": [{"sourceId": "\\ud83d\\ude00", '
              '"probability": NaN}, {"sourceId": "\\ud83d", "probability": -Infinity}]}',
              '{"schemaVersion": "1.0.0", "marketId": "m", "signals": [{"sourceId": "a\\u0000b", "probability": 1e-400}]}',
              '{"schemaVersion": "1.0.0", "marketId": "m", "signals": [{"sourceId": "a", "probability": 1e400}]}']
    exp = _py_expect(lines)
    nb = jsonl._NativeBatch("\n".join(lines).encode("utf-8", "surrogatepass"), 4)
    assert nb.n_lines == len(lines)
    names = nb.names()
    assert names == sorted(set(names))
    bad = []
    for i, e in enumerate(exp):
        k = int(nb.kind[i])
        if e is None:
            if k != 2:
                bad.append((i, "malformed line not handed to Python", lines[i][:80]))
            continue
        payload, err, probs, te = e
        if k == 2:
            if payload is not None and isinstance(payload, dict) and isinstance(payload.get("schemaVersion"), str):
                bad.append((i, "unexpected fallback", lines[i][:80]))
            continue
        if (k == 1) != (err is not None):
            bad.append((i, "header error mismatch", err, k))
            continue
        if k == 1:
            continue
        v = nb.prob[nb.voff[i]:nb.voff[i + 1]].tolist()
        if len(v) != len(probs) or any(not ((a == b and math.copysign(1, a) == math.copysign(1, b))
                                            or (a != a and b != b)) for a, b in zip(v, map(float, probs))):
            bad.append((i, "probs", v[:4], probs[:4]))
        if (te is None) != (nb.type_err[i] < 0):
            bad.append((i, "type error", str(te), int(nb.type_err[i])))
        sigs = payload["signals"]
        if te is None and nb.n_signals[i] != len(sigs):
            bad.append((i, "n_signals", int(nb.n_signals[i]), len(sigs)))
        ids = [names[j] for j in nb.sid[nb.voff[i]:nb.voff[i + 1]]]
        if ids != [s["sourceId"] for s in sigs[:len(ids)]]:
            bad.append((i, "ids", ids[:3]))
    assert not bad, bad[:8]


@pytest.mark.parametrize("dry_run", [False, True])
def test_native_render_matches_json_dumps(dry_run):
    """Every line's text -- validation errors (header, range before type, type) and computed
    results (the oracle's numbers) -- against json.dumps(result, indent=2) built as
    consensus_many / the CLI would."""
    from bayesian_engine import jsonl
    from bayesian_engine.core import ValidationError  # noqa: F401
    from oracle import oracle as orc
    rnd = random.Random(23 + dry_run)
    lines = [_rand_line(rnd) for _ in range(1500)]
    lines += [json.dumps(c["payload"]) for c in load_json("validate_cases.json")]
    exp = _py_expect(lines)
    nb = jsonl._NativeBatch("\n".join(lines).encode("utf-8", "surrogatepass"), 3)
    names = nb.names()
    L = nb.n_lines
    # the GPU's range check, restated: first checked probability outside [0, 1] (NaN passes)
    err = np.full(L, -1, np.int32)
    for i in range(L):
        v = nb.prob[nb.voff[i]:nb.voff[i + 1]]
        badp = np.nonzero((v < 0) | (v > 1))[0]
        if len(badp):
            err[i] = badp[0]
    rows = np.nonzero((nb.kind == 0) & (err < 0) & (nb.type_err < 0) & (nb.n_signals > 0))[0]
    res_of = np.full(L, -1, np.int64)
    res_of[rows] = np.arange(len(rows))
    lens = nb.voff[rows + 1] - nb.voff[rows]
    roff = np.zeros(len(rows) + 1, np.int64)
    np.cumsum(lens, out=roff[1:])
    flat = np.repeat(nb.voff[rows] - roff[:-1], lens) + np.arange(int(roff[-1]))
    sid, prob = nb.sid[flat].astype(np.int32), nb.prob[flat]
    S = nb.n_names
    rel, conf, present = np.full(S, 0.5), np.full(S, 0.25), np.zeros(S, np.uint8)
    o = orc.consensus_csr(roff, sid, prob, rel, conf, present)
    wtext = b"0.5" * S
    woff = np.arange(S + 1, dtype=np.int64) * 3
    n = C.c_int64(0)
    Lb = _lib()
    u = o["usid"].astype(np.int32)
    args = [nb.h, err.ctypes.data, res_of.ctypes.data, o["consensus"].ctypes.data, o["confidence"].ctypes.data,
            o["total_weight"].ctypes.data, o["n_unique"].astype(np.int32).ctypes.data, roff.ctypes.data,
            u.ctypes.data, o["nweight"].ctypes.data, wtext, woff.ctypes.data, int(dry_run), 3]
    keep = [o, u]  # noqa: F841  (buffers alive through the calls)
    nu = o["n_unique"].astype(np.int32)
    args[6] = nu.ctypes.data
    assert Lb.bce_jsonl_render(*args, None, None, None, C.byref(n)) == 0
    buf = C.create_string_buffer(max(n.value, 1))
    toff = np.empty(L + 1, np.int64)
    okf = np.empty(L, np.uint8)
    assert Lb.bce_jsonl_render(*args, buf, toff.ctypes.data, okf.ctypes.data, C.byref(n)) == 0
    raw = buf.raw
    bad = []
    for i, e in enumerate(exp):
        if nb.kind[i] == 2:
            continue
        payload, perr, probs, te = e
        text = raw[toff[i]:toff[i + 1]].decode("utf-8", "surrogatepass")
        if perr is not None:
            want = perr
        elif err[i] >= 0:
            want = f"Validation error: signals[{err[i]}].probability must be between 0 and 1"
        elif te is not None:
            want = f"Validation error: {te}"
        else:
            sigs = payload["signals"]
            if not sigs:
                r = {"schemaVersion": "1.0.0", "consensus": None, "confidence": 0.0, "sourceWeights": [],
                     "normalization": {"totalWeight": 0.0, "sourceCount": 0},
                     "diagnostics": {"status": "no_signals", "sources": 0}}
            else:
                k = res_of[i]
                a, nuk = int(roff[k]), int(o["n_unique"][k])
                null = o["total_weight"][k] == 0
                r = {"schemaVersion": "1.0.0", "consensus": None if null else float(o["consensus"][k]),
                     "confidence": 0.0 if null else float(o["confidence"][k]),
                     "sourceWeights": [{"sourceId": names[int(u[a + j]) & 0x7FFFFFFF], "weight": 0.5,
                                        "normalizedWeight": float(o["nweight"][a + j])} for j in range(nuk)],
                     "normalization": {"totalWeight": float(o["total_weight"][k]), "sourceCount": nuk},
                     "diagnostics": {"status": "computed", "sources": len(sigs), "uniqueSources": nuk,
                                     "coldStartSources": [names[int(u[a + j]) & 0x7FFFFFFF] for j in range(nuk)
                                                          if u[a + j] < 0]}}
            if dry_run:
                r["diagnostics"]["dryRun"] = True
            want = json.dumps(r, indent=2)
        ok_want = not want.startswith("Validation error")
        if text != want or bool(okf[i]) != ok_want:
            bad.append((i, text[:120], want[:120]))
    assert not bad, bad[:4]
