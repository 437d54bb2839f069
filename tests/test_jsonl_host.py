"""Host half of the batched JSON front end (bayesian_engine/jsonl.py): parsing and the
structural checks run without a GPU and must report exactly what validate_input_payload
would (tests/golden/validate_cases.json, produced by the reference)."""
import json

from golden_util import load_json


def test_parse_batch_structure_errors_match_golden():
    from bayesian_engine.jsonl import parse_batch
    cases = load_json("validate_cases.json")
    lines = [json.dumps(c["payload"]) for c in cases]
    lines.insert(3, "   \n")  # blank lines are skipped
    payloads, errors, probs, type_errors = parse_batch(lines + ["[1, 2"])
    assert len(payloads) == len(cases) + 1
    for c, p, e, pr, te in zip(cases, payloads, errors, probs, type_errors):
        if c["error"] is None:
            assert e is None and te is None, c["name"]
            assert len(pr) == len(c["payload"]["signals"])
        elif e is not None:  # header error (schema/market/signals): raised on the host
            assert e == f"Validation error: {c['error']}", c["name"]
        elif te is not None and "between 0 and 1" not in c["error"]:
            assert str(te) == c["error"], c["name"]
        else:  # range errors are the GPU launch's to find
            assert "between 0 and 1" in c["error"], c["name"]
    assert payloads[-1] is None and errors[-1].startswith("Validation error: ")


def test_render_is_json_dumps_indent2():
    """render() must be byte-identical to json.dumps(indent=2) on every value kind a result
    can hold: NaN/inf, -0.0, int and bool weights, null consensus, unicode/escaped ids,
    empty and non-empty cold lists, dryRun; other shapes fall back to json.dumps."""
    import random
    from bayesian_engine.jsonl import render
    rnd = random.Random(5)
    vals = [0.0, -0.0, 1.0, 0.1, 1e-320, 1e300, float("nan"), float("inf"), -float("inf"), 0.6966666666666667,
            1, 0, -3, True, False]
    ids = ["a", "src-001", "Ä", "éé", "x\"y", "tab\t", "☃", "\U0001f600", " sp"]
    for i in range(400):
        S = rnd.randint(1, 6)
        sw = [{"sourceId": rnd.choice(ids), "weight": rnd.choice(vals), "normalizedWeight": rnd.choice(vals[:10])}
              for _ in range(S)]
        r = {"schemaVersion": "1.0.0", "consensus": rnd.choice([None, rnd.choice(vals[:10])]),
             "confidence": rnd.choice(vals[:10]), "sourceWeights": sw,
             "normalization": {"totalWeight": rnd.choice(vals[:10]), "sourceCount": S},
             "diagnostics": {"status": "computed", "sources": rnd.randint(1, 99), "uniqueSources": S,
                             "coldStartSources": rnd.sample(ids, rnd.randint(0, 3))}}
        if i % 3 == 0:
            r["diagnostics"]["dryRun"] = True
        assert render(r) == json.dumps(r, indent=2)
    no_sig = {"schemaVersion": "1.0.0", "consensus": None, "confidence": 0.0, "sourceWeights": [],
              "normalization": {"totalWeight": 0.0, "sourceCount": 0},
              "diagnostics": {"status": "no_signals", "sources": 0}}
    assert render(no_sig) == json.dumps(no_sig, indent=2)


def test_iso_to_us_many_matches_per_value():
    """Bulk stamp parsing (f1 load_table) == the per-value mirror of decay.py:125-141."""
    from datetime import datetime, timezone
    from bayesian_engine.timeutil import iso_to_us, iso_to_us_many
    vals = ["2026-03-01T12:34:56.123456+00:00", "2026-03-01T12:34:56+00:00", "1969-12-31T23:59:59.999999+00:00",
            "2026-02-30T00:00:00+00:00", "2026-03-01T12:34:56+02:00", "2026-03-01T12:34:56", "2026-03-01",
            "", None, "garbage", "2026-13-01T00:00:00+00:00", "2024-02-29T23:59:59.000001+00:00",
            datetime(2026, 1, 1, tzinfo=timezone.utc), "0001-01-01T00:00:00+00:00", "9999-12-31T23:59:59.999999+00:00"]
    want = [iso_to_us(v) for v in vals]
    assert iso_to_us_many(vals).tolist() == want
    good = [v for v in vals if isinstance(v, str) and v.endswith("+00:00") and "02-30" not in v and "-13-" not in v]
    assert iso_to_us_many(good).tolist() == [iso_to_us(v) for v in good]
    assert iso_to_us_many([]).tolist() == []


def test_parse_batch_scalar_lines_do_not_abort_the_batch():
    """A JSON scalar line (5, null, true) is reported for that line only; the payloads
    around it are still parsed (the reference's single CLI dies on it with this TypeError)."""
    from bayesian_engine.jsonl import parse_batch
    ok = json.dumps({"schemaVersion": "1.0.0", "marketId": "m", "signals": [{"sourceId": "a", "probability": 0.5}]})
    payloads, errors, probs, _ = parse_batch([ok, "5", "null", "true", ok, '"text"'])
    assert len(payloads) == 6
    assert errors[0] is None and errors[4] is None and probs[4] == [0.5]
    assert errors[1] == "TypeError: argument of type 'int' is not iterable"
    assert errors[2] == "TypeError: argument of type 'NoneType' is not iterable"
    assert errors[3] == "TypeError: argument of type 'bool' is not iterable"
    assert errors[5] == "Validation error: schemaVersion is required"
