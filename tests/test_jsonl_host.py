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
